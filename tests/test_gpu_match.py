"""GPU parity: two-way Hamming matching through the C-ABI vs the CPU oracle (bit-exact)."""
import numpy as np
import pytest

from mageslam_amd import matcher, orb, synth

pytestmark = pytest.mark.gpu


def dm_bytes(m):
    return np.ascontiguousarray(m).view(np.uint8)


def test_hamming_distance_known_answers(gpu, oracle):
    a = np.zeros(32, np.uint8)
    b = np.full(32, 255, np.uint8)
    assert matcher.GetDescriptorDistance(a, b) == 256
    assert matcher.GetDescriptorDistance(a, a) == 0
    c = a.copy()
    c[0], c[31] = 0x81, 0x10
    assert matcher.GetDescriptorDistance(a, c) == 3
    rng = np.random.default_rng(1)
    for _ in range(100):
        x = rng.integers(0, 256, 32, dtype=np.uint8)
        y = rng.integers(0, 256, 32, dtype=np.uint8)
        assert matcher.GetDescriptorDistance(x, y) == oracle.hamming(x, y)


@pytest.mark.parametrize("na,nb", [(1, 1), (5, 300), (300, 5), (640, 700), (2000, 2000), (4096, 100), (513, 64)])
def test_match_random(gpu, oracle, na, nb):
    rng = np.random.default_rng(na * 7 + nb)
    base = rng.integers(0, 256, (max(na, nb), 32), dtype=np.uint8)
    # B = noisy copies of A's rows so that many pairs fall inside the radius
    A = base[:na].copy()
    flip = rng.integers(0, 256, (nb, 32), dtype=np.uint8) & rng.integers(0, 256, (nb, 32), dtype=np.uint8) \
        & rng.integers(0, 256, (nb, 32), dtype=np.uint8) & rng.integers(0, 256, (nb, 32), dtype=np.uint8)
    B = base[rng.integers(0, na, nb)] ^ flip
    for md, mdiff in ((30, 1), (64, 3), (255, 0), (0, 1)):
        g = matcher.Match(A, B, maxHammingDist=md, minHammingDifference=mdiff)
        o = oracle.match(A, B, max_distance=md, min_difference=mdiff)
        assert np.array_equal(dm_bytes(g), dm_bytes(o)), (na, nb, md, mdiff)


def test_match_masks_and_empty(gpu, oracle):
    rng = np.random.default_rng(3)
    A = rng.integers(0, 256, (400, 32), dtype=np.uint8)
    B = A[rng.permutation(400)] ^ (rng.integers(0, 256, (400, 32), dtype=np.uint8) & 0x11)
    ma = rng.random(400) < 0.6
    mb = rng.random(400) < 0.7
    g = matcher.Match(A, B, ma, mb, 40, 2)
    o = oracle.match(A, B, ma.astype(np.uint8), mb.astype(np.uint8), 40, 2)
    assert np.array_equal(dm_bytes(g), dm_bytes(o))
    assert len(matcher.Match(A, B, np.zeros(400, bool), mb)) == 0
    assert len(matcher.Match(A[:0], B)) == 0


def test_self_match_and_duplicates(gpu, oracle):
    det = orb.OrbDetector(nfeatures=2000)
    kp, d = det.DetectAndCompute(synth.frame(0, 640, 480))
    g = matcher.Match(d, d)
    assert len(g) == len(d) and (g["query_idx"] == g["train_idx"]).all()
    dd = np.concatenate([d[:100], d[:100]])  # exact duplicates: delta 0 -> rejected both ways
    g2 = matcher.Match(dd, dd)
    o2 = oracle.match(dd, dd)
    assert np.array_equal(dm_bytes(g2), dm_bytes(o2)) and len(g2) == 0


def test_frame_pair_matches_pan(gpu, oracle):
    det = orb.OrbDetector(nfeatures=2000)
    kp0, d0 = det.DetectAndCompute(synth.frame(0, 1280, 720))
    kp1, d1 = det.DetectAndCompute(synth.frame(1, 1280, 720))
    g = matcher.Match(d1, d0)
    o = oracle.match(d1, d0)
    assert np.array_equal(dm_bytes(g), dm_bytes(o))
    a, b = kp1[g["query_idx"]], kp0[g["train_idx"]]
    consistent = (np.abs(a["x"] + 3 - b["x"]) < 1e-3) & (np.abs(a["y"] + 2 - b["y"]) < 1e-3)
    assert consistent.mean() > 0.95


def test_batch_device(gpu, oracle):
    import torch

    rng = np.random.default_rng(11)
    pairs, cap = 5, 1500
    na = rng.integers(1, cap, pairs).astype(np.uint32)
    nb = rng.integers(1, cap, pairs).astype(np.uint32)
    A = rng.integers(0, 256, (pairs, cap, 32), dtype=np.uint8)
    B = A[:, rng.permutation(cap)] ^ (rng.integers(0, 256, (pairs, cap, 32), dtype=np.uint8) & 0x21)
    tA, tB = torch.from_numpy(A).cuda(), torch.from_numpy(B).cuda()
    tna, tnb = torch.from_numpy(na.view(np.int32)).cuda(), torch.from_numpy(nb.view(np.int32)).cuda()
    out = torch.zeros((pairs, cap * 16), dtype=torch.uint8, device="cuda")
    nout = torch.zeros(pairs, dtype=torch.int32, device="cuda")
    matcher.match_batch_device(tA, cap * 32, tna, tB, cap * 32, tnb, pairs, 30, 1, out, cap, nout)
    torch.cuda.synchronize()
    out_h, n_h = out.cpu().numpy(), nout.cpu().numpy()
    for p in range(pairs):
        o = oracle.match(A[p, : na[p]], B[p, : nb[p]])
        assert n_h[p] == len(o)
        assert np.array_equal(out_h[p, : 16 * n_h[p]], dm_bytes(o).reshape(-1))
