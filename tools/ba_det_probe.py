import numpy as np, sys
sys.path.insert(0, '.')
from mageslam_amd import bundler, synth
g = synth.ba_graph(cameras=12, points=400, obs_per_point=8, fixed_cameras=3, seed=1)
res = []
for rep in range(4):
    b = bundler.BundlerLib(); b.set_graph(g)
    for _ in range(3): b.step([1.8], 7.25)
    res.append(b.state())
print("deterministic:", all(np.array_equal(r[0], res[0][0]) and np.array_equal(r[1], res[0][1]) for r in res))
