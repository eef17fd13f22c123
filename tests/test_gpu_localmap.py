"""TrackLocalMap's per-map-point matching (TrackLocalMap.cpp:175-256; mage_local_map_match) against
the oracle's literal sequential loop (oracle/orb_oracle.c oracle_local_map_match): identical
results and final masks.  The GPU resolves the points 64 at a time with conflict restarts, so the
cases below force what makes the sequential order matter: many points competing for the same
keypoints (duplicate map points), hidden keypoints of pose-estimation outliers, keypoints already
associated at the start, dense clusters that overflow a point's kept candidates, several octaves."""
import numpy as np
import pytest

from mageslam_amd import matcher
from mageslam_amd._lib import KP_DTYPE

pytestmark = pytest.mark.gpu


def frame(rng, n, w=1280, h=720, octaves=1, cluster=None):
    kp = np.zeros(n, KP_DTYPE)
    kp["x"] = rng.uniform(0, w, n).astype(np.float32)
    kp["y"] = rng.uniform(0, h, n).astype(np.float32)
    if cluster:  # a dense blob: more than 8 candidates inside one 16 x 16 box
        c = cluster
        kp["x"][:c] = np.float32(640) + rng.uniform(-6, 6, c).astype(np.float32)
        kp["y"][:c] = np.float32(360) + rng.uniform(-6, 6, c).astype(np.float32)
    kp["octave"] = rng.integers(0, octaves, n)
    kp["size"] = 15
    desc = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    return kp, desc


def queries(rng, kp, desc, nq, dup=3, noise_bits=0.04, jitter=3.0):
    """Map points near keypoints, each physical point repeated `dup` times (different keyframes)."""
    base = rng.integers(0, len(kp), nq // dup + 1)
    src = np.repeat(base, dup)[:nq]
    pos = np.stack([kp["x"][src], kp["y"][src]], 1) + rng.uniform(-jitter, jitter, (nq, 2)).astype(np.float32)
    flip = (rng.random((nq, 256)) < noise_bits)
    bits = np.unpackbits(desc[src], axis=1) ^ flip
    qd = np.packbits(bits.astype(np.uint8), axis=1)
    return pos.astype(np.float32), kp["octave"][src].astype(np.int32), qd, src


def run_both(qp, qo, qd, kp, desc, mask, hide=None, radius=8.0, md=30, mdiff=1):
    from oracle import oracle as O

    g, gm = matcher.LocalMapMatch(qp, qo, qd, kp, desc, mask, radius, md, mdiff, queryHidden=hide)
    o, om = O.local_map_match(qp, qo, qd, hide, kp, desc, mask.astype(np.uint8), radius, md, mdiff)
    return g, gm, o, om.astype(bool)


@pytest.mark.parametrize("seed,nt,nq,dup,octaves", [(0, 2000, 3000, 3, 1), (1, 4096, 8000, 4, 1), (2, 500, 2000, 6, 2),
                                                    (3, 2000, 64, 2, 1), (4, 2000, 65, 1, 1), (5, 3000, 6000, 2, 3)])
def test_local_map_match_matches_oracle(gpu, seed, nt, nq, dup, octaves):
    rng = np.random.default_rng(seed)
    kp, desc = frame(rng, nt, octaves=octaves)
    qp, qo, qd, src = queries(rng, kp, desc, nq, dup=dup)
    mask = rng.random(nt) < 0.7  # 30 % already associated by the pose-estimation matches
    hide = np.where(rng.random(nq) < 0.2, rng.integers(0, nt, nq), -1).astype(np.int32)
    g, gm, o, om = run_both(qp, qo, qd, kp, desc, mask, hide)
    assert np.array_equal(g, o)
    assert np.array_equal(gm, om)
    assert (o >= 0).sum() > nq // (4 * dup)  # the case really associates keypoints


def test_local_map_match_conflicts_and_overflow(gpu):
    """A dense blob of 40 keypoints with near-identical descriptors inside one search box and 200 map
    points all projecting into it: every point sees > 8 candidates (overflow rescans) and each success
    changes the next points' results."""
    rng = np.random.default_rng(7)
    kp, desc = frame(rng, 1000, cluster=40)
    desc[:40] = desc[0] ^ (rng.random((40, 32)) < 0.05).astype(np.uint8)
    nq = 200
    qp = np.float32([640, 360]) + rng.uniform(-2, 2, (nq, 2)).astype(np.float32)
    qo = np.zeros(nq, np.int32)
    qd = np.repeat(desc[:1], nq, 0) ^ (rng.random((nq, 32)) < 0.03).astype(np.uint8)
    for mdiff in (0, 1, 3):
        g, gm, o, om = run_both(qp, qo, qd, kp, desc, np.ones(1000, bool), None, 8.0, 30, mdiff)
        assert np.array_equal(g, o) and np.array_equal(gm, om), mdiff
    assert (o >= 0).sum() >= 5


def test_local_map_match_edges(gpu):
    rng = np.random.default_rng(9)
    kp, desc = frame(rng, 300)
    qp, qo, qd, _ = queries(rng, kp, desc, 100)
    # nothing available, empty target set, empty query set, radius 0, maxDist -1
    g, gm, o, om = run_both(qp, qo, qd, kp, desc, np.zeros(300, bool))
    assert (g == -1).all() and np.array_equal(g, o)
    g, _ = matcher.LocalMapMatch(qp, qo, qd, kp[:0], desc[:0], np.zeros(0, bool))
    assert (g == -1).all()
    g, gm = matcher.LocalMapMatch(qp[:0], qo[:0], qd[:0], kp, desc, np.ones(300, bool))
    assert len(g) == 0 and gm.all()
    for radius, md in ((0.0, 30), (8.0, -1), (30.0, 256)):
        g, gm, o, om = run_both(qp, qo, qd, kp, desc, np.ones(300, bool), None, radius, md, 1)
        assert np.array_equal(g, o) and np.array_equal(gm, om), (radius, md)
