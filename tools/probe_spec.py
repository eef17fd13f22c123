"""Per-step BA probe (development tool): trials, lambda, chi2 and per-kernel times of each
StepBundleAdjustment on the C3 graph."""
import sys

sys.path.insert(0, '.')
import torch  # noqa: F401,E402

from mageslam_amd import _lib, bundler, synth  # noqa: E402

g = synth.ba_graph()
b = bundler.BundlerLib(device=0)
b.set_graph(g)
lib = _lib.load()
for it in range(int(sys.argv[1]) if len(sys.argv) > 1 else 70):
    s0 = b.stats()
    lib.mage_profile_reset()
    lib.mage_profile_enable(1)
    ms, out = b.step([1.8], 7.25)
    lib.mage_profile_enable(0)
    k = _lib.profile_report()
    s1 = b.stats()
    ch = k.get("ba.cholesky_solve", (0, 0))
    print(it, "trials", s1["trials"] - s0["trials"], "rej", s1["rejected"] - s0["rejected"], "outl", len(out),
          "lambda %.3g chi %.10g" % (s1["lambda_"], s1["chi2"]), "chol_ms %.4f" % (ch[1] / max(ch[0], 1)))
