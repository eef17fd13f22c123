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


@pytest.mark.parametrize("na,nb", [(1, 1), (5, 300), (300, 5), (640, 700), (2000, 2000), (4096, 100), (513, 64),
                                   (1024, 97), (1025, 2048), (96, 2000)])  # fp4 passes of 1024 rows: exact, ragged, 3 row tiles
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


@pytest.mark.parametrize("na,nb", [(2048, 2048), (100, 2049), (2049, 100), (33, 2047)])
def test_match_fp4_path_boundaries(gpu, oracle, na, nb):
    """The packed-key fp4 MFMA path serves nb <= 2048 and maxDist < 128; nb = 2049 and maxDist
    >= 128 take the i8 path.  Both sides of each boundary, plus extreme distances (0 and 256:
    the accumulator's full range) and exact ties."""
    rng = np.random.default_rng(na + 3 * nb)
    base = rng.integers(0, 256, (max(na, nb), 32), dtype=np.uint8)
    base[:4] = 0
    base[4:8] = 255
    A = base[:na].copy()
    flip = rng.integers(0, 256, (nb, 32), dtype=np.uint8) & rng.integers(0, 256, (nb, 32), dtype=np.uint8) \
        & rng.integers(0, 256, (nb, 32), dtype=np.uint8)
    B = base[rng.integers(0, na, nb)] ^ flip
    B[:8] = base[:8]
    B[8:12] = B[12:16]  # duplicated columns: tied distances for every row
    for md, mdiff in ((30, 1), (127, 2), (128, 2), (0, 0)):
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
    # C1 (BASELINE configs[0]): the full self-match byte for byte against the oracle, and the
    # expected result — every keypoint matched to itself (no exact-duplicate descriptors here)
    assert np.array_equal(dm_bytes(g), dm_bytes(oracle.match(d, d)))
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


# ------------------------- RadiusMatch (FeatureMatcher.cpp:294-446) -------------


def _radius_pair(oracle, **kw):
    s = oracle.default_settings(2000, **kw)
    _, k0, d0 = oracle.orb_detect(synth.frame(0, 1280, 720), s)
    _, k1, d1 = oracle.orb_detect(synth.frame(1, 1280, 720), s)
    return k1, d1, k0, d0


@pytest.mark.parametrize("radius,md,mdiff", [(15.0, 30, 1), (4.0, 30, 1), (40.0, 64, 3), (2.5, 0, 0)])
def test_radius_match_frames(gpu, oracle, radius, md, mdiff):
    qk, qd, tk, td = _radius_pair(oracle)
    g = matcher.RadiusMatch(qk, qd, tk, td, radius, maxHammingDist=md, minHammingDifference=mdiff)
    o = oracle.radius_match(qk, qd, tk, td, radius, max_distance=md, min_difference=mdiff)
    assert len(o) > 0 or md == 0
    assert np.array_equal(dm_bytes(g), dm_bytes(o))


def test_radius_match_overrides_masks_octaves(gpu, oracle):
    qk, qd, tk, td = _radius_pair(oracle, nlevels=3, patch_size=31, use_orientation=True)
    rng = np.random.default_rng(5)
    pos = np.stack([qk["x"] + 3.0, qk["y"] + 2.0], 1).astype(np.float32)  # predicted positions (pan)
    qm = rng.random(len(qk)) < 0.8
    tm = rng.random(len(tk)) < 0.9
    for kw in (dict(), dict(qpos=pos), dict(qpos=pos, qmask=qm, tmask=tm)):
        g = matcher.RadiusMatch(qk, qd, tk, td, 3.0, queryKeypointPositionOverrides=kw.get("qpos"),
                                queryKeypointsMask=kw.get("qmask"), targetKeypointsMask=kw.get("tmask"))
        o = oracle.radius_match(qk, qd, tk, td, 3.0, **kw)
        assert np.array_equal(dm_bytes(g), dm_bytes(o)), kw
    assert len(o) > 100
    assert np.all(qk["octave"][o["query_idx"]] == tk["octave"][o["train_idx"]])


def test_radius_match_ties(gpu, oracle):
    # few distinct descriptors on a dense grid: exact ties everywhere exercise the "second best =
    # previous best" rule and the unique-minimum-per-target pass
    rng = np.random.default_rng(11)
    from mageslam_amd._lib import KP_DTYPE

    # set sizes around the 2048 targets staged in LDS and off the 1024-thread stride (the stage
    # hand-off audit)
    for nq, nt in ((500, 800), (1, 1), (3000, 4096), (1025, 2048), (2049, 2049), (64, 2047), (1023, 1025)):
        tk = np.zeros(nt, KP_DTYPE)
        tk["x"] = rng.integers(0, 60, nt).astype(np.float32)
        tk["y"] = rng.integers(0, 40, nt).astype(np.float32)
        tk["octave"] = rng.integers(0, 2, nt)
        qk = np.zeros(nq, KP_DTYPE)
        qk["x"] = rng.integers(0, 60, nq).astype(np.float32) + 0.5
        qk["y"] = rng.integers(0, 40, nq).astype(np.float32)
        qk["octave"] = rng.integers(0, 2, nq)
        pal = rng.integers(0, 256, (6, 32), dtype=np.uint8)
        td = pal[rng.integers(0, 6, nt)] ^ (rng.random((nt, 32)) < 0.02).astype(np.uint8)
        qd = pal[rng.integers(0, 6, nq)]
        for r, md, mdiff in ((1.5, 30, 1), (3.0, 256, 0), (0.5, 8, 2)):
            g = matcher.RadiusMatch(qk, qd, tk, td, r, maxHammingDist=md, minHammingDifference=mdiff)
            o = oracle.radius_match(qk, qd, tk, td, r, max_distance=md, min_difference=mdiff)
            assert np.array_equal(dm_bytes(g), dm_bytes(o)), (nq, nt, r, md, mdiff)


def test_radius_match_edges(gpu, oracle):
    from mageslam_amd._lib import KP_DTYPE, MageError

    qk, qd, tk, td = _radius_pair(oracle)
    assert len(matcher.RadiusMatch(qk[:0], qd[:0], tk, td, 10.0)) == 0
    assert len(matcher.RadiusMatch(qk, qd, tk[:0], td[:0], 10.0)) == 0
    big = np.zeros(4097, KP_DTYPE)
    with pytest.raises(MageError):
        matcher.RadiusMatch(qk, qd, big, np.zeros((4097, 32), np.uint8), 10.0)


@pytest.mark.parametrize("pairs", [3, 130])  # split (< 128 pairs: several workgroups per pair) and fused paths
def test_radius_match_batch_device(gpu, oracle, pairs):
    import torch

    from mageslam_amd._lib import KP_DTYPE

    pitch = 2000
    sets = []
    for t in range(4):
        _, k, d = oracle.orb_detect(synth.frame(t, 640, 480), oracle.default_settings(pitch))
        sets.append((k, d))
    kp = np.zeros((pairs + 1, pitch), KP_DTYPE)
    de = np.zeros((pairs + 1, pitch, 32), np.uint8)
    nn = np.zeros(pairs + 1, np.uint32)
    for i in range(pairs + 1):
        k, d = sets[i % 4]
        kp[i, : len(k)] = k
        de[i, : len(k)] = d
        nn[i] = len(k)
    dev = "cuda"
    kpt = torch.from_numpy(kp.view(np.uint8).reshape(pairs + 1, -1)).to(dev)
    det = torch.from_numpy(de).to(dev)
    nt = torch.from_numpy(nn.astype(np.int32)).to(dev)
    scratch = torch.zeros(pairs * pitch, dtype=torch.int32, device=dev)
    out = torch.zeros((pairs, pitch * 16), dtype=torch.uint8, device=dev)
    nout = torch.zeros(pairs, dtype=torch.int32, device=dev)
    status = torch.zeros(1, dtype=torch.int32, device=dev)
    # query set p + 1 against target set p
    matcher.radius_match_batch_device(kpt[1:], None, det[1:], pitch, nt[1:], kpt[:-1], det[:-1], pitch, nt[:-1],
                                      pairs, 12.0, 30, 1, scratch, out, pitch, nout, status)
    torch.cuda.synchronize()
    assert int(status[0]) == 0
    ref = {}
    for p in range(pairs):
        key = (p + 1) % 4, p % 4
        if key not in ref:
            ref[key] = oracle.radius_match(sets[key[0]][0], sets[key[0]][1], sets[key[1]][0], sets[key[1]][1], 12.0)
        o = ref[key]
        n = int(nout[p])
        assert n == len(o)
        assert np.array_equal(out[p, : 16 * n].cpu().numpy(), dm_bytes(o))
