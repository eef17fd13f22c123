"""CPU oracle self-checks: known answers, committed golden fixtures, finite differences.

The oracle is pinned only by these restated semantics and by the pattern tables extracted from
the reference (no reference fixtures exist) — "parity unpinned".
"""
import hashlib
import math
from pathlib import Path

import numpy as np
import pytest

from mageslam_amd import synth

GOLDEN = Path(__file__).resolve().parent / "golden"
DATA = Path(__file__).resolve().parent.parent / "mageslam_amd" / "data"

RING = [(0, 3), (1, 3), (2, 2), (3, 1), (3, 0), (3, -1), (2, -2), (1, -3), (0, -3), (-1, -3), (-2, -2),
        (-3, -1), (-3, 0), (-3, 1), (-2, 2), (-1, 3)]


def ring_image(values, center=100):
    img = np.full((7, 7), center, np.uint8)
    for (dx, dy), v in zip(RING, values):
        img[3 + dy, 3 + dx] = v
    return img


def test_pattern_tables_match_extraction():
    ref = (GOLDEN / "pattern_tables.sha256").read_text().split()
    for patch, digest in zip((15, 31), ref[::2]):
        data = (DATA / f"bit_pattern_{patch}_rotated.bin").read_bytes()
        assert len(data) == 30720
        assert hashlib.sha256(data).hexdigest() == digest


def test_gaussian_taps(oracle):
    assert oracle.gaussian_taps(7, 2.0).tolist() == [18, 34, 49, 55, 49, 34, 18]
    assert oracle.gaussian_taps(3, 2.0).sum() in (255, 256, 257)


def test_fast_known_answers(oracle):
    # 9 contiguous darker ring pixels: corner; score = (min over the best arc of v - x) - 1
    vals = [100] * 16
    for k in range(9):
        vals[k] = 100 - 10 - k
    s = oracle.fast_score_map(ring_image(vals), 4)
    assert s[3, 3] == 10 - 1
    # 8 contiguous: not a corner
    vals = [100] * 16
    for k in range(8):
        vals[k] = 50
    assert oracle.fast_score_map(ring_image(vals), 4)[3, 3] == 0
    # wrap-around run (15,0..7) brighter by 30 -> score 29
    vals = [100] * 16
    for k in [15] + list(range(8)):
        vals[k] = 130
    assert oracle.fast_score_map(ring_image(vals), 4)[3, 3] == 29
    # threshold boundary: difference exactly t is not a corner
    vals = [104] * 16
    assert oracle.fast_score_map(ring_image(vals), 4)[3, 3] == 0
    vals = [105] * 16
    assert oracle.fast_score_map(ring_image(vals), 4)[3, 3] == 4


def _verify_simd_frames(w, h):
    """Frames for the VERIFY_SIMD property: the synthetic stream, uniform noise, 0/255 binary
    noise (saturating adds / subs in the SIMD test), flat frames with isolated extreme pixels,
    low-contrast noise around a mid level, and ring-exact corners."""
    rng = np.random.default_rng(w * 7 + h)
    yield "synthetic", synth.frame(5, w, h)
    yield "uniform", rng.integers(0, 256, (h, w), dtype=np.uint8)
    yield "binary", (rng.integers(0, 2, (h, w), dtype=np.uint8) * 255).astype(np.uint8)
    for level in (0, 255):
        img = np.full((h, w), level, np.uint8)
        ys, xs = rng.integers(0, h, 3000), rng.integers(0, w, 3000)
        img[ys, xs] = 255 - level
        yield f"spikes{level}", img
    yield "lowcontrast", np.clip(128 + rng.integers(-6, 7, (h, w)), 0, 255).astype(np.uint8)
    img = np.full((h, w), 100, np.uint8)
    for k, (cy, cx) in enumerate(zip(range(10, h - 10, 17), range(10, w - 10, 23))):
        for j, (dx, dy) in enumerate(RING):  # arcs of 8 / 9 / 10 ring pixels, bright and dark
            if (j - k) % 16 < 8 + k % 3:
                img[cy + dy, cx + dx] = 100 + (60 if k % 2 else -60) + (j % 5)
    yield "rings", img


@pytest.mark.parametrize("shape", [(640, 480), (1280, 720)])
def test_verify_simd_sse2_build_equals_scalar_oracle(oracle, shape):
    """The reference's own self-check VERIFY_SIMD (OpenCVModified.cpp:1265-1271, 1408-1486), made
    stronger: the score map of the x64 SSE2 build — the 16-pixel SIMD row loop (:1278-1338), the
    scalar tail, and the SSE2 cornerScore<16> (:935-972) — restated in oracle/fast_sse2.c, equals
    the scalar oracle's map (scalar loop + scalar cornerScore, :1030-1064, :1415-1479) that the
    GPU parity tests use.  Equal score maps give equal keypoints: NMS and emission (:1489-1509)
    read only the score rows."""
    w, h = shape
    for name, img in _verify_simd_frames(w, h):
        for t in (0, 4, 20, 100, 254, 255):
            simd, cols = oracle.fast_score_map_sse2(img, t)
            scalar = oracle.fast_score_map(img, t)
            bad = np.argwhere(simd != scalar)
            assert len(bad) == 0, (name, t, bad[:5], simd[tuple(bad[0])], scalar[tuple(bad[0])])
            # the SIMD loop covered all but the row tail (< 16 + 3 columns, + 8 after a step back)
            assert (cols[3:h - 3] >= w - 16 - 3 - 8).all(), (name, t)
            if name == "synthetic" and t == 4:
                assert (scalar > 0).mean() > 0.1  # the comparison is over a dense corner map


def test_sse2_corner_score_ring_cases(oracle):
    """SSE2 cornerScore<16> vs the scalar branch on the ring known-answer cases, in the SIMD
    loop's columns (a 64-px wide frame puts them inside the 16-pixel blocks)."""
    for vals, center in (([90] * 9 + [100] * 7, 100), ([130] * 16, 100), ([105] * 16, 100),
                         ([0, 255] * 8, 128), ([255] * 9 + [0] * 7, 128)):
        img = np.full((7, 64), center, np.uint8)
        for off in (3, 20, 37):
            for (dx, dy), v in zip(RING, vals):
                img[3 + dy, off + dx] = v
        for t in (0, 4, 9, 100):
            assert np.array_equal(oracle.fast_score_map_sse2(img, t)[0], oracle.fast_score_map(img, t)), (vals, t)


def test_hamming_known(oracle):
    a = np.zeros(32, np.uint8)
    b = np.arange(32, dtype=np.uint8)
    assert oracle.hamming(a, b) == sum(bin(i).count("1") for i in range(32))
    assert oracle.hamming(a, np.full(32, 255, np.uint8)) == 256


def test_match_semantics(oracle):
    rng = np.random.default_rng(0)
    A = rng.integers(0, 256, (4, 32), dtype=np.uint8)
    B = A.copy()
    # exact copies -> all matched in A order
    m = oracle.match(A, B)
    assert m["query_idx"].tolist() == [0, 1, 2, 3] and m["train_idx"].tolist() == [0, 1, 2, 3]
    # ambiguous B (two identical candidates) -> delta 0 < 1 rejects A0
    B2 = np.concatenate([B, B[:1]])
    m2 = oracle.match(A, B2)
    assert 0 not in m2["query_idx"].tolist()
    # with minDiff 0 the tie resolves to the lowest index on both sides
    m3 = oracle.match(A, B2, min_difference=0)
    assert m3["train_idx"][0] == 0
    # radius is inclusive (OpenCV radiusMatch: distance <= maxDistance)
    C = A.copy()
    C[0, :4] ^= 0xFF  # distance 32
    assert 0 in oracle.match(A[:1], C[:1], max_distance=32)["query_idx"].tolist()
    assert len(oracle.match(A[:1], C[:1], max_distance=31)) == 0
    # masks select rows, outputs use original indices
    m4 = oracle.match(A, B, np.array([0, 1, 0, 1], np.uint8), None)
    assert m4["query_idx"].tolist() == [1, 3] and m4["train_idx"].tolist() == [1, 3]


def test_orb_golden_vga(oracle):
    g = np.load(GOLDEN / "orb_vga_t0.npz")
    img = synth.frame(0, 640, 480)
    assert hashlib.sha256(img.tobytes()).hexdigest() == str(g["frame_sha256"])
    st, kp, desc = oracle.orb_detect(img, oracle.default_settings(2000))
    assert st == 0
    assert np.array_equal(np.stack([kp["x"], kp["y"], kp["response"]], 1), g["kp_xyr"])
    assert np.array_equal(desc, g["desc"])


def test_match_golden(oracle):
    g = np.load(GOLDEN / "match_vga_t1_t0.npz")
    m = oracle.match(g["desc_a"], g["desc_b"], max_distance=30, min_difference=1)
    assert (m["img_idx"] == -1).all()  # cv::DMatch(int, int, float) (FeatureMatcher.cpp:159-162)
    assert np.array_equal(np.stack([m["query_idx"], m["train_idx"], m["distance"].astype(np.int32)], 1),
                          g["matches"])


def test_orb_invariants(oracle):
    img = synth.frame(4, 320, 180)
    st, kp, d = oracle.orb_detect(img, oracle.default_settings(440))
    assert st == 0 and len(kp) == 440
    assert (kp["x"] >= 7).all() and (kp["x"] < 320 - 7).all()
    # retained responses are bounded below by the fast threshold
    assert (kp["response"] >= 4).all()
    # oracle status codes: unsupported variants are reported, not approximated
    assert oracle.orb_detect(img, oracle.default_settings(440, nlevels=9))[0] == 4
    assert oracle.orb_detect(img, oracle.default_settings(440, patch_size=1))[0] == 1


def test_pyramid_known_answers(oracle):
    # level geometry and budgets of the rBRIEF-31 variant at 720p (ComputeKeyPoints :659-669)
    sc, lw, lh = oracle.level_geometry(1280, 720, 4, 1.5)
    assert sc.tolist() == [1.0, 1.5, 2.25, 3.375]
    assert lw.tolist() == [1280, 853, 569, 379] and lh.tolist() == [720, 480, 320, 213]
    assert oracle.features_per_level(2000, 1.5, 4).tolist() == [831, 554, 369, 246]
    assert oracle.features_per_level(440, 1.5, 1).tolist() == [440]
    # u_max of OpenCV ORB for halfPatchSize 15 (the circular patch of ICAngles)
    assert oracle.umax(15)[:16].tolist() == [15, 15, 15, 15, 14, 14, 14, 13, 13, 12, 11, 10, 9, 8, 6, 3]


def test_resize_linear_properties(oracle):
    rng = np.random.default_rng(11)
    img = rng.integers(0, 256, (37, 53), dtype=np.uint8)
    # same size: coefficients (2048, 0) reproduce the input through both fixed-point passes
    assert np.array_equal(oracle.resize_linear(img, 53, 37), img)
    # a constant image stays constant at any scale
    flat = np.full((40, 60), 173, np.uint8)
    assert (oracle.resize_linear(flat, 27, 17) == 173).all()
    # exact 2x downscale of a 2x2-block image returns the blocks
    blocks = rng.integers(0, 256, (20, 30), dtype=np.uint8)
    big = np.repeat(np.repeat(blocks, 2, 0), 2, 1)
    assert np.array_equal(oracle.resize_linear(big, 30, 20), blocks)
    # exact 2x takes cv::resize's INTER_AREA fast path: (sum + 2) >> 2 in the SSE2 8-wide blocks,
    # cvRound(sum * 0.25f) (half to even) in the tail — a 2x2 sum of 10 gives 3 there and 2 here
    tens = np.tile(np.array([[2, 3], [2, 3]], np.uint8), (1, 13))
    assert oracle.resize_linear(tens, 13, 1).tolist() == [[3] * 8 + [2] * 5]
    fourteen = np.tile(np.array([[3, 4], [3, 4]], np.uint8), (1, 13))  # 3.5: half-up and half-even agree
    assert oracle.resize_linear(fourteen, 13, 1).tolist() == [[4] * 13]


def test_fast_atan2_accuracy(oracle):
    rng = np.random.default_rng(5)
    for y, x in rng.integers(-5000, 5000, (200, 2)):
        a = oracle.fast_atan2(float(y), float(x))
        ref = np.degrees(np.arctan2(y, x)) % 360
        d = abs(a - ref)
        assert min(d, 360 - d) < 0.02
        assert 0.0 <= a <= 360.0
    assert oracle.fast_atan2(0.0, 1.0) == 0.0 and oracle.fast_atan2(1.0, 0.0) == 90.0


def test_ic_angle_direction(oracle):
    # a brightness ramp along +x has its intensity centroid at angle ~0, along +y at ~90
    x = np.arange(64, dtype=np.float64)
    ramp = np.tile(x * 3, (64, 1)).astype(np.uint8)
    assert abs(oracle.ic_angle(ramp, 32, 32, 15)) < 0.5 or abs(oracle.ic_angle(ramp, 32, 32, 15) - 360) < 0.5
    assert abs(oracle.ic_angle(ramp.T.copy(), 32, 32, 15) - 90) < 0.5


def test_orb_pyramid_invariants(oracle):
    img = synth.frame(2, 640, 480)
    s = oracle.default_settings(2000, nlevels=4, patch_size=31, use_orientation=1)
    st, kp, d = oracle.orb_detect(img, s)
    assert st == 0 and len(kp) == 2000
    per = oracle.features_per_level(2000, 1.5, 4)
    assert np.bincount(kp["octave"], minlength=4).tolist() == per.tolist()
    # level order, sizes and the oriented border (cvCeil(15 sqrt 2) = 22 in level coordinates)
    assert (np.diff(kp["octave"]) >= 0).all()
    sc = np.array([1.0, 1.5, 2.25, 3.375], np.float32)
    assert np.array_equal(kp["size"], np.float32(31) * sc[kp["octave"]])
    lx = np.rint(kp["x"] / sc[kp["octave"]])
    assert (lx >= 22).all()
    assert ((kp["angle"] >= 0) & (kp["angle"] <= 360)).all()


def test_blur_flat_and_border(oracle):
    flat = np.full((20, 30), 100, np.uint8)
    b = oracle.gaussian_blur(flat)
    # Q8 taps sum to 257: a flat 100 maps to (100*257*257 + 2^15) >> 16 = 101
    assert (b == (100 * 257 * 257 + 32768) // 65536).all()
    rng = np.random.default_rng(2)
    img = rng.integers(0, 256, (16, 16), dtype=np.uint8)
    b = oracle.gaussian_blur(img)
    # reflect-101 symmetry: mirrored image blurs to the mirrored result
    assert np.array_equal(oracle.gaussian_blur(img[:, ::-1].copy()), b[:, ::-1])


# ----------------------------- BA oracle -----------------------------------------------------


def small_graph(**kw):
    return synth.ba_graph(cameras=kw.pop("cameras", 10), points=kw.pop("points", 300),
                          obs_per_point=kw.pop("obs_per_point", 6), fixed_cameras=kw.pop("fixed_cameras", 2), **kw)


def test_ba_jacobians_finite_difference(oracle):
    g = small_graph(outlier_frac=0.0)
    b = oracle.BundlerOracle()
    b.set_graph(g)
    h = 1e-6
    for e in (0, 17, 123):
        err, jpt, jp = b.edge_linearization(e)
        c, p = int(g.cam[e]), int(g.pt[e])
        num_pt = np.zeros((2, 3))
        for k in range(3):
            u = np.zeros(3)
            u[k] = h
            b.perturb_point(p, u)
            ep, _, _ = b.edge_linearization(e)
            b.perturb_point(p, -u)
            num_pt[:, k] = (ep - err) / h
        assert np.allclose(num_pt, jpt, rtol=1e-3, atol=1e-3)
        num_pose = np.zeros((2, 6))
        for k in range(6):
            u = np.zeros(6)
            u[k] = h
            b.perturb_camera(c, u)
            ep, _, _ = b.edge_linearization(e)
            b.perturb_camera(c, -u)
            num_pose[:, k] = (ep - err) / h
        assert np.allclose(num_pose, jp, rtol=1e-3, atol=1e-2)


def test_ba_converges_and_reduces_error(oracle):
    g = small_graph(outlier_frac=0.0, noise_px=0.3)
    b = oracle.BundlerOracle()
    b.set_graph(g)
    first, _ = b.step([1.8], 1e9)
    for _ in range(8):
        last, outl = b.step([1.8], 1e9)
        assert len(outl) == 0
    assert last < first
    _, xyz = b.state()
    assert np.median(np.linalg.norm(xyz - g.true_points, axis=1)) < np.median(
        np.linalg.norm(g.points - g.true_points, axis=1))


def test_ba_outlier_report_order_and_lambda(oracle):
    g = small_graph(outlier_frac=0.05)
    b = oracle.BundlerOracle()
    b.set_graph(g)
    ms, outl = b.step([1.8], 7.25)
    assert len(outl) > 0 and np.all(np.diff(outl.astype(np.int64)) > 0)
    b.set_lambda(0.5)
    b.step([1.8], 7.25)
    assert b.stats()["iterations"] == 2


def test_ba_pose_only(oracle):
    g = small_graph(cameras=4, fixed_cameras=3, outlier_frac=0.0)
    b = oracle.BundlerOracle(points_fixed=True)
    b.set_graph(g)
    _, xyz0 = b.state()
    b.step([0.9, 0.9, 0.9], 1e9)
    _, xyz1 = b.state()
    assert np.array_equal(xyz0, xyz1)  # points untouched


def test_ba_golden(oracle):
    gold = np.load(GOLDEN / "ba_small.npz")
    g = synth.ba_graph(cameras=12, points=400, obs_per_point=8, fixed_cameras=3, seed=1)
    b = oracle.BundlerOracle()
    b.set_graph(g)
    outs = []
    for it in range(3):
        _, o = b.step([1.8], 7.25 * 0.9025 ** it)
        outs.append(o)
    qt, xyz = b.state()
    assert np.allclose(qt, gold["qt"], atol=1e-9)
    assert np.array_equal(np.concatenate(outs), gold["outliers"])


# ------------------------- random pattern (patch sizes other than 15 / 31) -------------------------


def _cv_rng_pattern(patch):
    """Independent restatement of MakeRandomPattern with OpenCV 3.4.0's cv::RNG (multiply-with-carry,
    core/operations.hpp): state = (uint32)state * 4164903690 + (state >> 32); uniform(a, b) =
    a + next() % (b - a)."""
    st = 0x34985739
    out = []
    for _ in range(1024):
        st = ((st & 0xFFFFFFFF) * 4164903690 + (st >> 32)) & 0xFFFFFFFFFFFFFFFF
        a, b = -(patch // 2), patch // 2 + 1
        out.append(a + (st & 0xFFFFFFFF) % (b - a))
    return np.array(out, np.int8)


@pytest.mark.parametrize("patch", [2, 9, 21, 25, 35])
def test_random_pattern_known_answer(oracle, patch):
    p = oracle.random_pattern(patch)
    assert np.array_equal(p, _cv_rng_pattern(patch))
    assert p.min() >= -(patch // 2) and p.max() <= patch // 2


def test_random_pattern_detect_runs(oracle):
    img = synth.frame(0, 320, 240)
    s = oracle.default_settings(500, patch_size=21, use_orientation=True)
    st, kp, d = oracle.orb_detect(img, s)
    assert st == 0 and len(kp) > 0
    assert d.any(axis=1).mean() > 0.9  # descriptors are not empty
    st2, kp2, d2 = oracle.orb_detect(img, s)
    assert np.array_equal(d, d2)


# ------------------------- RadiusMatch known answers (FeatureMatcher.cpp:294-446) ----------------


def _kp(xs, ys, octs=None):
    from mageslam_amd._lib import KP_DTYPE

    k = np.zeros(len(xs), KP_DTYPE)
    k["x"], k["y"] = xs, ys
    if octs is not None:
        k["octave"] = octs
    return k


def _desc_at_distance(base, d):
    out = base.copy()
    bits = np.unpackbits(out)
    bits[:d] ^= 1
    return np.packbits(bits)


def test_radius_match_known_answers(oracle):
    base = np.zeros(32, np.uint8)
    q = _kp([10.0], [10.0])
    qd = base[None]
    # candidates in index order with distances 10, 5, 7: best 5 (index 1), second = 10 (the best
    # before it) -> 10 - 5 > 1 accepted
    t = _kp([10.0, 11.0, 12.0], [10.0, 10.0, 10.0])
    td = np.stack([_desc_at_distance(base, d) for d in (10, 5, 7)])
    m = oracle.radius_match(q, qd, t, td, 5.0)
    assert len(m) == 1 and m[0]["train_idx"] == 1 and m[0]["distance"] == 5
    # distances 5, 6 in index order: best 5 found first, second = maxDist + 1 = 31 (the "second" is
    # only ever the previous best) -> accepted although 6 - 5 = 1 is not > 1
    td2 = np.stack([_desc_at_distance(base, d) for d in (5, 6, 40)])
    m = oracle.radius_match(q, qd, t, td2, 5.0)
    assert len(m) == 1 and m[0]["train_idx"] == 0
    # distances 6, 5: second = 6 -> 6 - 5 = 1 is not > minDiff = 1 -> rejected
    td3 = np.stack([_desc_at_distance(base, d) for d in (6, 5, 40)])
    assert len(oracle.radius_match(q, qd, t, td3, 5.0)) == 0
    # box is inclusive; other octaves never match
    t4 = _kp([15.0, 10.0], [15.0, 10.0], [0, 1])
    td4 = np.stack([_desc_at_distance(base, 3), base])
    m = oracle.radius_match(q, qd, t4, td4, 5.0)
    assert len(m) == 1 and m[0]["train_idx"] == 0
    # two queries with the same best distance to one target: neither survives the batch pass
    q2 = _kp([10.0, 10.5], [10.0, 10.0])
    t5 = _kp([10.0], [10.0])
    td5 = _desc_at_distance(base, 4)[None]
    assert len(oracle.radius_match(q2, np.stack([base, base]), t5, td5, 5.0)) == 0
    # ... but a single query keeps its match
    assert len(oracle.radius_match(q2[:1], base[None], t5, td5, 5.0)) == 1


# ------------------------- UndistortKeypoints (cv::undistortPoints restatement) -------------------


def _distort(pts, k, dist):
    """Forward OpenCV distortion model (cv::projectPoints): normalised -> distorted pixels."""
    fx, fy, cx, cy = k
    d = list(dist) + [0.0] * (8 - len(dist))
    k1, k2, p1, p2, k3, k4, k5, k6 = d
    x, y = pts[:, 0].astype(np.float64), pts[:, 1].astype(np.float64)
    r2 = x * x + y * y
    radial = (1 + ((k3 * r2 + k2) * r2 + k1) * r2) / (1 + ((k6 * r2 + k5) * r2 + k4) * r2)
    xd = x * radial + 2 * p1 * x * y + p2 * (r2 + 2 * x * x)
    yd = y * radial + p1 * (r2 + 2 * y * y) + 2 * p2 * x * y
    return np.stack([xd * fx + cx, yd * fy + cy], 1)


@pytest.mark.parametrize("dist", [(-0.12, 0.03, 1e-4, -2e-4, 0.0),
                                  (0.05, -0.01, -3e-4, 1e-4, 0.002, 0.02, -0.005, 0.001)])
def test_undistort_points_inverts_distortion(oracle, dist):
    rng = np.random.default_rng(2)
    kd = (900.0, 905.0, 640.0, 360.0)
    norm = np.stack([rng.uniform(-0.5, 0.5, 400), rng.uniform(-0.3, 0.3, 400)], 1)
    distorted = _distort(norm, kd, dist).astype(np.float32)
    out = oracle.undistort_points(distorted, kd, dist, kd)  # P = the same K: back to the ideal pixels
    ideal = np.stack([norm[:, 0] * kd[0] + kd[2], norm[:, 1] * kd[1] + kd[3]], 1)
    assert np.abs(out - ideal).max() < 0.02  # 5 fixed-point iterations on mild distortion
    assert np.array_equal(oracle.undistort_points(distorted, kd, (), kd), distorted)  # no coefficients


def _oracle_with_tethers(O, g, t):
    b = O.BundlerOracle()
    b.set_graph(g)
    for kind, tt in enumerate((t.distance, t.rotation, t.transform)):
        b.set_tethers(kind, *tt)
    return b


def test_ba_tether_jacobians_finite_difference(oracle):
    """BaseMultiEdge numeric Jacobians (distance / rotation) agree with wider central differences;
    EdgeSE3Expmap's adjoint Jacobians are exact at zero error (BundlerLib.cpp:22-88)."""
    from mageslam_amd import synth

    g = synth.ba_graph(cameras=12, points=400, obs_per_point=8, fixed_cameras=3)
    t = synth.ba_tethers(g)
    # transform measurements consistent with the current estimates: zero error
    R = g.rot.astype(np.float64)
    tt = g.pos.astype(np.float64)
    p7 = []
    for a, b_ in zip(t.transform[0], t.transform[1]):
        Rc = R[b_] @ R[a].T
        p7.append(np.concatenate([tt[b_] - Rc @ tt[a], synth.quat_from_rot(Rc)]))
    t.transform = (t.transform[0], t.transform[1], np.asarray(p7, np.float32), t.transform[3])
    b = _oracle_with_tethers(oracle, g, t)
    cams = [(int(c1), int(c2)) for tt_ in (t.distance, t.rotation, t.transform) for c1, c2 in zip(tt_[0], tt_[1])]
    checked = 0
    for i, pair in enumerate(cams):
        e, J1, J2 = b.tether_linearization(i)
        if len(e) == 0:
            assert g.fixed[pair[0]] and g.fixed[pair[1]]
            continue
        for v, J in enumerate((J1, J2)):
            c = pair[v]
            if g.fixed[c]:
                continue
            Jfd = np.zeros_like(J)
            h = 1e-6
            for d in range(6):
                u = np.zeros(6)
                u[d] = h
                b.perturb_camera(c, u)
                ep, _, _ = b.tether_linearization(i)
                u[d] = -2 * h
                b.perturb_camera(c, u)
                em, _, _ = b.tether_linearization(i)
                u[d] = h
                b.perturb_camera(c, u)
                Jfd[:, d] = (ep - em) / (2 * h)
            tol = 2e-5 * max(1.0, np.abs(J).max()) if len(e) == 1 else 1e-3
            assert np.abs(J - Jfd).max() < tol, (i, v, np.abs(J - Jfd).max())
            checked += 1
    assert checked >= 12


def test_ba_tethers_pull_cameras(oracle):
    """A distance tether with a longer measurement pulls the two translations towards it (against
    the photogrammetric evidence): closer to the measurement than the untethered solution."""
    from mageslam_amd import synth

    g = synth.ba_graph(cameras=12, points=400, obs_per_point=8, fixed_cameras=3, seed=4)
    none = (np.zeros(0, np.uint32),) * 2
    d0 = float(np.linalg.norm(g.pos[8].astype(np.float64) - g.pos[5]))
    t = synth.Tethers(distance=(np.array([5], np.uint32), np.array([8], np.uint32),
                                np.array([d0 * 1.05], np.float32), np.array([200.0], np.float32)),
                      rotation=none + (np.zeros((0, 4), np.float32), np.zeros(0, np.float32)),
                      transform=none + (np.zeros((0, 7), np.float32), np.zeros(0, np.float32)))
    b = _oracle_with_tethers(oracle, g, t)
    for _ in range(10):
        b.step([1.8], 7.25)
    qt, _ = b.state()
    d1 = float(np.linalg.norm(qt[8, 4:] - qt[5, 4:]))
    # without the tether the pair keeps its photogrammetric distance
    b2 = oracle.BundlerOracle()
    b2.set_graph(g)
    for _ in range(10):
        b2.step([1.8], 7.25)
    qt2, _ = b2.state()
    assert abs(float(np.linalg.norm(qt2[8, 4:] - qt2[5, 4:])) - d0 * 1.05) > abs(d1 - d0 * 1.05)


def test_ba_tether_only_camera_joins_system(oracle):
    """An unobserved free camera with a transform tether is optimised (it moves onto the tether)."""
    from tests.test_gpu_ba import tethered_extra_camera
    from mageslam_amd import synth

    g = tethered_extra_camera()
    C = len(g.pos)
    none = (np.zeros(0, np.uint32),) * 2
    t = synth.Tethers(distance=none + (np.zeros((0, 1), np.float32), np.zeros(0, np.float32)),
                      rotation=none + (np.zeros((0, 4), np.float32), np.zeros(0, np.float32)),
                      transform=(np.array([C - 2], np.uint32), np.array([C - 1], np.uint32),
                                 g.extra_tether[None, :], np.array([50.0], np.float32)))
    b = _oracle_with_tethers(oracle, g, t)
    before = b.state()[0][C - 1].copy()
    for _ in range(10):  # lambda starts large against the tether's Hessian: LM closes slowly
        b.step([1.8], 7.25)
    qt, _ = b.state()
    assert np.abs(qt[C - 1] - before).max() > 1e-3
    # the constraint holds: log(T2^-1 C T1) ~ 0
    e, _, _ = b.tether_linearization(0)
    assert np.abs(e).max() < 1e-4


def _tiny_tree():
    """root -> {1, 2}; 1 -> {3, 4}; 2 -> {5}: node descriptors chosen for tie cases."""
    nd = np.zeros((6, 32), np.uint8)
    nd[1, 0] = 0x0F
    nd[2, 0] = 0xF0
    nd[3, 1] = 0x01
    nd[4, 1] = 0x02
    nd[5, 2] = 0xFF
    cs = np.array([0, 2, 4, 5, 5, 5, 5], np.uint32)
    ch = np.array([1, 2, 3, 4, 5], np.uint32)
    return nd, cs, ch


def test_bow_find_leaf_known_answers(oracle):
    """OnlineBow::FindLeafNode (OnlineBow.cpp:289-311): strictly-smaller updates, so the first
    child wins ties; descent stops at a node without children."""
    tree = _tiny_tree()
    q = np.zeros((4, 32), np.uint8)
    # q0: d(1) = 4, d(2) = 4 -> child 1 (first); then d(3) = d(4) = 1 -> 3
    q[1, 1] = 0x02  # d(3) = 2, d(4) = 0 -> 4 (under 1: d(1) = d(2) = 4)
    q[2, 0] = 0xF0  # -> 2, then its only child 5
    q[3, 0] = 0x0F
    q[3, 1] = 0x03  # -> 1, then d(3) = 1, d(4) = 1 -> 3
    assert list(oracle.bow_find_leaves(tree, q)) == [3, 4, 5, 3]


def test_bow_tree_builder_shape(oracle):
    from mageslam_amd import synth

    g = np.load(GOLDEN / "match_vga_t1_t0.npz")
    nd, cs, ch = synth.bow_tree(np.concatenate([g["desc_a"], g["desc_b"]]))
    assert len(nd) == 1 + 6 + 36 and cs[0] == 0 and cs[-1] == len(ch) == len(nd) - 1
    # children follow their parent (OnlineBow::Kmean appends)
    for i in range(len(nd)):
        assert all(c > i for c in ch[cs[i]:cs[i + 1]])
    leaves = oracle.bow_find_leaves((nd, cs, ch), g["desc_a"])
    assert all(cs[l] == cs[l + 1] for l in np.unique(leaves))


def test_mt19937_known_answers(oracle):
    """std::mt19937 as InitializeTraining default-constructs it (seed 5489): first output and the
    10000th output required by the C++ standard ([rand.predef])."""
    assert oracle.mt19937_output(5489, 1) == 3499211612
    assert oracle.mt19937_output(5489, 10000) == 4123659995


def test_msvc_shuffle_two_restatements(oracle):
    from mageslam_amd import synth

    for n in (0, 1, 2, 7, 1000, 30001):
        a, b = oracle.msvc_shuffle(n), synth.msvc_shuffle(n)
        assert np.array_equal(a, b) and sorted(a.tolist()) == list(range(n))


@pytest.mark.parametrize("levels,branching,max_iter", [(2, 6, 12), (3, 4, 3), (1, 6, 12), (2, 6, 1), (2, 2, 12)])
def test_bow_train_two_restatements(oracle, levels, branching, max_iter):
    """CreateTree / Kmean (OnlineBow.cpp:325-614): the C oracle (literal recursive loops) against
    the numpy restatement (matrix distances, vectorised majority), on ORB descriptors of two
    golden frames, random descriptors and a degenerate set (duplicates -> empty clusters)."""
    from mageslam_amd import synth

    g = np.load(GOLDEN / "match_vga_t1_t0.npz")
    rng = np.random.default_rng(7)
    sets = [np.concatenate([g["desc_a"], g["desc_b"]]), rng.integers(0, 256, (900, 32), dtype=np.uint8),
            np.repeat(rng.integers(0, 256, (3, 32), dtype=np.uint8), 40, axis=0), g["desc_a"][:5]]
    for d in sets:
        a = oracle.bow_train(d, levels, branching, max_iter)
        b = synth.bow_tree(d, levels, branching, max_iter)
        assert all(np.array_equal(x, y) for x, y in zip(a, b))
        nd, cs, ch = a
        for i in range(len(nd)):  # ids grow downwards (Kmean appends children after the parent)
            assert all(c > i for c in ch[cs[i]:cs[i + 1]])


def test_indexed_match_semantics(oracle):
    """IndexedMatch (FeatureMatcher.cpp:192-292) on hand-made sets in one leaf: TrackMatch's
    second best keeps ties, the min-difference test, masks and the reverse check."""
    tree = _tiny_tree()
    base = np.zeros(32, np.uint8)
    base[0] = 0x0F  # leaf 3 region
    base[1] = 0x01

    def with_bits(k):
        d = base.copy()
        for b in k:
            d[4 + b // 8] |= 1 << (b % 8)
        return d

    A = np.stack([with_bits([]), with_bits([0, 1, 2]), with_bits(range(20, 40))])
    B = np.stack([with_bits([5]), with_bits([0, 1]), with_bits([0, 1, 2, 3]), with_bits([6])])
    # A0: d(B0)=1, d(B1)=2, d(B2)=4, d(B3)=1 -> best B0 (first), second 1 -> diff 0 < 1: rejected
    # A1: d(B0)=4, d(B1)=1, d(B2)=1, d(B3)=4 -> tie again: rejected
    m = oracle.indexed_match(tree, A, B, max_distance=30, min_difference=1)
    assert len(m) == 0
    # min_difference 0 accepts ties: A0 -> B0; reverse of B0 over A: d(A0)=1 best -> kept
    m = oracle.indexed_match(tree, A, B, max_distance=30, min_difference=0)
    assert [(r["query_idx"], r["train_idx"], r["distance"], r["img_idx"]) for r in m] == [(0, 0, 1.0, -1), (1, 1, 1.0, -1)]
    # mask B0 out: A0 -> B3 (d = 1), second B1 (d = 2): diff 1 >= 1 accepted; B3's reverse -> A0
    m = oracle.indexed_match(tree, A, B, mask_b=np.array([0, 1, 1, 1], np.uint8), min_difference=1)
    assert [(r["query_idx"], r["train_idx"]) for r in m] == [(0, 3)]
    # max_distance: A2 is 20 bits away from everything: only a max above 20 lets it compete
    assert all(r["query_idx"] != 2 for r in oracle.indexed_match(tree, A, B, max_distance=19, min_difference=0))
    # empty mask -> 0 matches
    assert len(oracle.indexed_match(tree, A, B, mask_a=np.zeros(3, np.uint8))) == 0


def test_pose_batch_oracle_converges(oracle):
    """The batched pose-only oracle (fresh BundlerLib per frame, TrackLocalMap.cpp:421-501) recovers
    the true poses and flags the planted outliers."""
    from mageslam_amd import synth

    pb = synth.pose_batch(problems=16, obs=300, outlier_frac=0.05)
    r = oracle.pose_batch(pb, 3, 4.0, 36.0)
    r = oracle.pose_batch(pb, 4, 0.9, 4.5 ** 2)
    assert np.abs(r["qt7"][:, 4:] - pb.true_pos).max() < 0.01
    assert (r["stats"][:, 0] >= 1).all()
    assert 0.02 < r["outlier"].mean() < 0.1


def test_undistort_image_pure_shift(oracle):
    """With no distortion the map is a translation by (cx - w/2, cy - h/2): an integer offset moves
    the frame exactly (the remap table's saturated (0, 0) entry cannot change a pixel), with the
    constant-0 border outside (ImagePreprocessor.cpp:71-120)."""
    from mageslam_amd import synth

    img = synth.frame(2, 160, 120)
    out, mx, my, kn = oracle.undistort_image(img, (200.0, 210.0, 80.0 + 3, 60.0 - 2), np.zeros(5, np.float32))
    assert kn[2] == 80.0 and kn[3] == 60.0
    # the inverse of K' carries rounding (cv::invert's cofactors / det): maps are ~integers
    assert np.allclose(mx[0, :4], [3, 4, 5, 6], atol=1e-5) and np.allclose(my[:3, 0], [-2, -1, 0], atol=1e-5)
    ref = np.zeros_like(img)
    ref[2:, :-3] = img[:-2, 3:]
    assert np.array_equal(out, ref)


@pytest.mark.parametrize("dist", [[-0.28, 0.07, 0.001, -0.0005, 0.0],
                                  [0.9, -0.3, 0.0007, 0.0002, 0.02, 1.2, -0.2, 0.05]])
def test_undistort_map_inverts_points(oracle, dist):
    """initUndistortRectifyMap sends undistorted pixel p to a distorted position q; undistortPoints
    (the keypoint path, OrbFeatureDetector.cpp:30-62) maps q back to p (two independent
    restatements of OpenCV's model agree to its 5 fixed-point iterations)."""
    from mageslam_amd import synth

    img = synth.frame(0, 200, 150)
    kd = np.float32([180.0, 185.0, 97.5, 77.0])
    out, mx, my, kn = oracle.undistort_image(img, kd, np.float32(dist))
    ys, xs = np.mgrid[20:130:11, 20:180:13]
    q = np.stack([mx[ys, xs].ravel(), my[ys, xs].ravel()], 1).astype(np.float32)
    back = oracle.undistort_points(q, kd, np.float32(dist), kn)
    err = np.hypot(back[:, 0] - xs.ravel(), back[:, 1] - ys.ravel())
    assert err.max() < 0.05, err.max()


def test_online_bow_oracle_database(oracle):
    """The oracle's OnlineBow database on random descriptors: IDF weights (a leaf every training
    image reaches gets log((n + 1) / n)), an image queried with its own descriptors scores 1 and
    ranks first, QueryFeatures returns the inserted index, removed keyframes drop out."""
    rng = np.random.default_rng(5)
    train = rng.integers(0, 256, (6 * 200, 32), dtype=np.uint8)
    o = oracle.OnlineBowOracle(oracle.bow_train(train, levels=2, branching=4, max_iter=6))
    o.SetNodeWeights(train, [200] * 6)
    w = np.array(o.nodes_weight, np.float32)
    leaves = oracle.bow_find_leaves(o.tree, train)
    for leaf in set(leaves.tolist()):
        n_img = len({i // 200 for i in np.flatnonzero(leaves == leaf)})
        assert w[leaf] == np.float32(math.log(float(np.float32(7) / np.float32(n_img))))
    imgs = {kf: rng.integers(0, 256, (150, 32), dtype=np.uint8) for kf in range(4)}
    for kf, d in imgs.items():
        o.InsertDescriptors(kf, d)
    r = o.QueryUnknownImage(imgs[2], 3)
    assert r[0][0] == 2 and abs(r[0][1] - 1.0) < 1e-5
    assert 11 in o.QueryFeatures(imgs[1][11], 1)
    o.RemoveImage(2)
    assert all(kf != 2 for kf, _ in o.QueryUnknownImage(imgs[2], 4))


def test_bow_train_kmedoid_oracle(oracle):
    """The oracle's Kmedoid tree: every node a training descriptor and, once the loop has
    converged, each medoid minimises the summed distances over the group assigned to it (numpy)."""
    rng = np.random.default_rng(9)
    d = rng.integers(0, 256, (400, 32), dtype=np.uint8)
    nd, cs, ch = oracle.bow_train(d, levels=1, branching=5, max_iter=100, kmedoid=True)
    rows = [bytes(r) for r in d]
    assert all(bytes(r) in set(rows) for r in nd[1:])
    bits = np.unpackbits(d, axis=1).astype(np.int64)
    dist = (bits[:, None, :] != np.unpackbits(nd[1:], axis=1)[None, :, :]).sum(2)
    g = dist.argmin(1)  # FindCluster: first smallest distance
    for c in range(len(nd) - 1):
        mem = np.flatnonzero(g == c)
        if len(mem) == 0:
            continue
        sums = (bits[mem][:, None, :] != bits[mem][None, :, :]).sum((1, 2))
        med = [k for k, m in enumerate(mem) if rows[m] == bytes(nd[1 + c])]
        assert med and sums[med[0]] == sums.min()
