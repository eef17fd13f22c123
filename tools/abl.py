"""Compile-time variants of one kernel source, timed on the C2 step (development tool, not part of
the product).

  python tools/abl.py build <source.hip> name:DEF=1+DEF2=3 [name:...]   # here (CPU): abl/<name>/libmage_hot.so
  python tools/abl.py run name[,name...]                                # on the GPU box

`run` extracts + matches one 256-frame C2 batch per iteration (as bench.py's step does), prints each
variant's per-kernel average launch time (the library's dispatch timestamps) and a checksum of the
keypoints, descriptors and matches, which must agree between variants of the same algorithm.
MAGE_ABLATE_GATE=<g> forces the FAST candidate gate of every timed batch.
"""
import ctypes as C
import hashlib
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def variant_source(stem):
    """csrc/<stem> with tools/patches/<name>_variants.patch applied (the ablation / experiment
    switches removed from the product sources in round 6) as csrc/.abl_variants_<stem>; the caller
    deletes it.  Without a patch for the file: the product source itself."""
    sys.path.insert(0, str(ROOT))
    from mageslam_amd import build as B

    patch = ROOT / "tools" / "patches" / (Path(stem).stem + "_variants.patch")
    if not patch.exists():
        return B.CSRC / stem, False
    with open(patch, "rb") as f:
        dry = subprocess.run(["patch", "-s", "--dry-run", str(B.CSRC / stem)], stdin=f, capture_output=True)
    if dry.returncode != 0:  # the product source moved on: its own switches only
        print(f"note: {patch.name} does not apply to the current {stem}; building the product source", flush=True)
        return B.CSRC / stem, False
    out = B.CSRC / f".abl_variants_{stem}"
    out.write_bytes((B.CSRC / stem).read_bytes())
    with open(patch, "rb") as f:
        subprocess.run(["patch", "-s", str(out)], stdin=f, check=True)
    return out, True


def build(src, specs):
    sys.path.insert(0, str(ROOT))
    from mageslam_amd import build as B
    B.build()
    stem = Path(src).name
    objs = [p for p in B.OBJ.glob("*.o") if p.name != stem + ".o"]
    for spec in specs:
        name, _, defs = spec.partition(":")
        # name@REV: the source as committed at git revision REV (a same-box baseline)
        name, _, rev = name.partition("@")
        out = ROOT / "abl" / name
        out.mkdir(parents=True, exist_ok=True)
        obj = out / (stem + ".o")
        flags = [f"-D{d}" for d in defs.split("+") if d]
        src_path, tmp = variant_source(stem)
        inc = []
        if rev:
            # the sources and headers as committed at REV (a same-box baseline), in a scratch tree
            import shutil
            import tempfile
            tree = Path(tempfile.mkdtemp(prefix="abl_rev_"))
            arch = subprocess.run(["git", "archive", rev, "mageslam_amd/csrc", "include"], cwd=ROOT, check=True,
                                  capture_output=True).stdout
            subprocess.run(["tar", "-x", "-C", str(tree)], input=arch, check=True)
            src_path = tree / "mageslam_amd" / "csrc" / stem
            inc = [f"-I{tree / 'include'}"]
        subprocess.run([B.hipcc(), "-x", "hip", f"--offload-arch={B.ARCH}", "-munsafe-fp-atomics", *inc, *B.COMMON, *flags,
                        "-c", str(src_path), "-o", str(obj)], check=True)
        if rev:
            shutil.rmtree(tree)
        elif tmp:
            src_path.unlink()
        subprocess.run([B.hipcc(), f"--offload-arch={B.ARCH}", "-shared", "-fPIC", "-o", str(out / "libmage_hot.so"),
                        str(obj), *map(str, objs)], check=True)
        print("built", out, flags, flush=True)


def run(names):
    import torch
    sys.path.insert(0, str(ROOT))
    from mageslam_amd import _lib, matcher, orb, synth
    W, H, B, N = 1280, 720, 256, 2000
    gate = int(os.environ["MAGE_ABLATE_GATE"]) if os.environ.get("MAGE_ABLATE_GATE") else None
    frames = torch.empty((B + 1, H, W), dtype=torch.uint8, device="cuda")
    kp = torch.zeros((B + 1, N * 28), dtype=torch.uint8, device="cuda")
    desc = torch.zeros((B + 1, N, 32), dtype=torch.uint8, device="cuda")
    cnt = torch.zeros(B + 1, dtype=torch.int32, device="cuda")
    mt = torch.zeros((B, N * 16), dtype=torch.uint8, device="cuda")
    nm = torch.zeros(B, dtype=torch.int32, device="cuda")
    for v in names:
        L = C.CDLL(str(ROOT / "abl" / v / "libmage_hot.so"))
        _lib._declare(L)
        _lib._lib = L
        orb.synth_frames_device(frames, B + 1, W, H, 0, synth.FRAME_SEED)
        det = orb.OrbDetector(nfeatures=N)

        def step():
            if gate is not None:
                det.set_fast_gate(gate)
            det.detect_and_compute_batch_device(frames, W, H, kp, desc, cnt, N)
            matcher.match_batch_device(desc[1:], N * 32, cnt[1:], desc[:-1], N * 32, cnt[:-1], B, 30, 1, mt, N, nm)

        for _ in range(3):
            step()
        torch.cuda.synchronize()
        L.mage_profile_reset()
        L.mage_profile_enable(1)
        for _ in range(10):
            step()
        torch.cuda.synchronize()
        rep = _lib.profile_report()
        L.mage_profile_enable(0)
        h = hashlib.sha256()
        for t in (kp, desc, cnt, nm):
            h.update(t.cpu().numpy().tobytes())
        mtn = mt.cpu().numpy()
        for b in range(B):
            h.update(mtn[b, : 16 * int(nm[b])].tobytes())
        ks = " ".join(f"{k} {ms / c:.4f}" for k, (c, ms) in sorted(rep.items()))
        print(f"{v:>10}: {ks}  | sha {h.hexdigest()[:12]} matches/frame {nm.float().mean().item():.1f}", flush=True)
        det.close()


if __name__ == "__main__":
    if sys.argv[1] == "build":
        build(sys.argv[2], sys.argv[3:])
    else:
        run(sys.argv[2].split(","))
