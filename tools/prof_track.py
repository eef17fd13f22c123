import cProfile, pstats, sys, time
sys.path.insert(0, '.')
import torch
from mageslam_amd import _lib, synth, tracking
T = 240
seq = synth.scene_sequence(T, 1280, 720)
cams = torch.from_numpy(seq.cams()).cuda()
frames = torch.empty((T, 720, 1280), dtype=torch.uint8, device='cuda')
_lib.check(_lib.load().mage_synth_scene_device(_lib.ptr(frames), T, 1280, 720, 1280 * 720, _lib.ptr(cams), seq.fx, seq.fy, seq.cx, seq.cy, synth.SCENE_PLANE_Z, synth.SCENE_TEXEL_SCALE, synth.SCENE_TEXEL_OFFSET, synth.FRAME_SEED, None))
K = (seq.fx, seq.fy, seq.cx, seq.cy)
p0 = tracking.Pose(seq.R[0], seq.t[0])
be = tracking.GpuBackend(2000, batch=64)
feats = be.extract(frames)
tracking.track(feats, K, p0, synth.SCENE_PLANE_Z, be)
torch.cuda.synchronize()
pr = cProfile.Profile()
t0 = time.perf_counter()
pr.enable()
tracking.track(feats, K, p0, synth.SCENE_PLANE_Z, be)
pr.disable()
print("track ms/frame", (time.perf_counter() - t0) / T * 1e3)
pstats.Stats(pr).sort_stats('tottime').print_stats(18)
