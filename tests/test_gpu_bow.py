"""GPU parity: vocabulary-tree descent and IndexedMatch through the C-ABI vs the CPU oracle.

Bit-exact: leaf ids, and the full cv::DMatch records (queryIdx, trainIdx, imgIdx = -1, distance)
in the same order.  The oracle runs the reference's sequential TrackMatch loops
(FeatureMatcher.cpp:192-292); the kernel uses order-free reductions.
"""
import numpy as np
import pytest

from mageslam_amd import bow, synth
from mageslam_amd._lib import DM_DTYPE, MAGE_EINVAL, MageError

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def frames(oracle):
    from mageslam_amd import orb

    det = orb.OrbDetector(nfeatures=2000)
    descs = [det.DetectAndCompute(synth.frame(t, 640, 480))[1] for t in range(4)]
    tree = synth.bow_tree(np.concatenate(descs[:2]))
    return descs, tree


def test_find_leaves(gpu, oracle, frames):
    descs, tree = frames
    t = bow.OnlineBowTree(*tree)
    for d in descs:
        assert np.array_equal(t.find_leaves(d), oracle.bow_find_leaves(tree, d))
    # a deeper, narrower tree (levels 3, branching 3) and a single-node tree (root is the leaf)
    deep = synth.bow_tree(descs[2], levels=3, branching=3)
    assert np.array_equal(bow.OnlineBowTree(*deep).find_leaves(descs[3]), oracle.bow_find_leaves(deep, descs[3]))
    single = (np.zeros((1, 32), np.uint8), np.zeros(2, np.uint32), np.zeros(0, np.uint32))
    assert (bow.OnlineBowTree(*single).find_leaves(descs[0][:10]) == 0).all()


@pytest.mark.parametrize("maxd,mind", [(30, 1), (50, 0), (64, 5), (10, 1)])
def test_indexed_match_parity(gpu, oracle, frames, maxd, mind):
    descs, tree = frames
    t = bow.OnlineBowTree(*tree)
    for a, b in [(1, 0), (2, 1), (3, 0)]:
        g = bow.IndexedMatch(t, descs[a], descs[b], maxHammingDist=maxd, minHammingDifference=mind)
        o = oracle.indexed_match(tree, descs[a], descs[b], max_distance=maxd, min_difference=mind)
        assert np.array_equal(g.view(np.uint8), o.view(np.uint8)), (a, b, len(g), len(o))


def test_indexed_match_masks_ties_and_edges(gpu, oracle, frames):
    descs, tree = frames
    t = bow.OnlineBowTree(*tree)
    rng = np.random.default_rng(3)
    a, b = descs[1], descs[0]
    ma = rng.random(len(a)) < 0.6
    mb = rng.random(len(b)) < 0.7
    g = bow.IndexedMatch(t, a, b, ma, mb)
    o = oracle.indexed_match(tree, a, b, ma.astype(np.uint8), mb.astype(np.uint8))
    assert np.array_equal(g.view(np.uint8), o.view(np.uint8))
    # exact duplicates in B create best-distance ties (rejected for min_difference >= 1, the lower
    # index wins at 0)
    bd = np.concatenate([b, b[::3]])
    for mind in (0, 1):
        g = bow.IndexedMatch(t, a, bd, minHammingDifference=mind)
        o = oracle.indexed_match(tree, a, bd, min_difference=mind)
        assert np.array_equal(g.view(np.uint8), o.view(np.uint8))
    # self match, one-element sets, empty masks
    g = bow.IndexedMatch(t, a, a)
    assert np.array_equal(g.view(np.uint8), oracle.indexed_match(tree, a, a).view(np.uint8))
    assert len(bow.IndexedMatch(t, a[:1], a[:1])) == 1
    assert len(bow.IndexedMatch(t, a, b, np.zeros(len(a), bool))) == 0
    assert len(bow.IndexedMatch(t, a[:0], b)) == 0


def test_indexed_match_batch_device(gpu, oracle, frames):
    import torch

    descs, tree = frames
    t = bow.OnlineBowTree(*tree)
    pitch = 2048
    n = len(descs)
    D = torch.zeros((n, pitch, 32), dtype=torch.uint8, device="cuda")
    L = torch.zeros((n, pitch), dtype=torch.int32, device="cuda")
    M = torch.zeros((n, pitch), dtype=torch.uint8, device="cuda")
    rng = np.random.default_rng(9)
    masks = [rng.random(len(d)) < 0.8 for d in descs]
    for i, d in enumerate(descs):
        D[i, : len(d)] = torch.from_numpy(d).cuda()
        M[i, : len(d)] = torch.from_numpy(masks[i].astype(np.uint8)).cuda()
        t.find_leaves_device(D[i], len(d), L[i])
    counts = torch.tensor([len(d) for d in descs], dtype=torch.int32, device="cuda")
    # pairs (i + 1, i): A = frames 1..3, B = frames 0..2
    out = torch.zeros((n - 1, pitch * 16), dtype=torch.uint8, device="cuda")
    nout = torch.zeros(n - 1, dtype=torch.int32, device="cuda")
    status = torch.zeros(1, dtype=torch.int32, device="cuda")
    bow.indexed_match_batch_device(D[1:], L[1:], M[1:], pitch, counts[1:], D[:-1], L[:-1], M[:-1], pitch, counts[:-1],
                                   n - 1, 30, 1, out, pitch, nout, status)
    torch.cuda.synchronize()
    assert int(status.item()) == 0
    for p in range(n - 1):
        o = oracle.indexed_match(tree, descs[p + 1], descs[p], masks[p + 1].astype(np.uint8), masks[p].astype(np.uint8))
        k = int(nout[p].item())
        g = out[p, : 16 * k].cpu().numpy().view(DM_DTYPE)
        assert np.array_equal(g.view(np.uint8), o.view(np.uint8)), p


def test_tree_validation(gpu):
    nd = np.zeros((3, 32), np.uint8)
    with pytest.raises(MageError) as e:
        bow.OnlineBowTree(nd, np.array([0, 1, 2, 2], np.uint32), np.array([2, 1], np.uint32))  # 1 -> 1: a cycle
    assert e.value.status == MAGE_EINVAL
    with pytest.raises(MageError):
        bow.OnlineBowTree(nd, np.array([0, 1, 1, 1], np.uint32), np.array([7], np.uint32))  # out of range


@pytest.mark.parametrize("levels,branching,max_iter", [(2, 6, 12), (3, 4, 3), (1, 6, 12), (2, 6, 1), (2, 16, 12)])
def test_create_tree_parity(gpu, oracle, frames, levels, branching, max_iter):
    """OnlineBow::CreateTree on the GPU (mage_bow_train) vs the oracle's literal recursion: the
    whole tree (node descriptors, child lists, ids) bit-exact."""
    descs, _ = frames
    rng = np.random.default_rng(11)
    sets = [np.concatenate(descs), rng.integers(0, 256, (2500, 32), dtype=np.uint8),
            np.repeat(rng.integers(0, 256, (3, 32), dtype=np.uint8), 40, axis=0), descs[0][:1], descs[0][:4]]
    for d in sets:
        t = bow.OnlineBowTree.CreateTree(d, levels, branching, max_iter)
        ref = oracle.bow_train(d, levels, branching, max_iter)
        for x, y in zip(t.tree(), ref):
            assert np.array_equal(x, y)
        assert np.array_equal(t.find_leaves(descs[3]), oracle.bow_find_leaves(ref, descs[3]))


def test_create_tree_training_frames(gpu, oracle):
    """BagOfWordsSettings::TrainingFrames (15) x 2000 features of 720p frames: the reference's
    training set size."""
    from mageslam_amd import orb

    det = orb.OrbDetector(nfeatures=2000)
    d = np.concatenate([det.DetectAndCompute(synth.frame(t, 1280, 720))[1] for t in range(15)])
    t = bow.OnlineBowTree.CreateTree(d)
    for x, y in zip(t.tree(), oracle.bow_train(d)):
        assert np.array_equal(x, y)


def test_create_tree_empty_and_errors(gpu):
    t = bow.OnlineBowTree.CreateTree(np.zeros((0, 32), np.uint8))
    nd, cs, ch = t.tree()
    assert len(nd) == 1 and list(cs) == [0, 0] and len(ch) == 0
    with pytest.raises(MageError):
        bow.OnlineBowTree.CreateTree(np.zeros((10, 32), np.uint8), branching=17)
    with pytest.raises(MageError):
        bow.OnlineBowTree.CreateTree(np.zeros((10, 32), np.uint8), levels=0)


@pytest.mark.parametrize("na,nb", [(2048, 2048), (2049, 2049), (1025, 2047), (3000, 1023), (1, 2049)])
def test_indexed_match_stage_boundaries(gpu, oracle, na, nb):
    """B sets at and around the 2048 descriptors indexed_match_kernel stages in LDS, and counts off
    the 1024-thread stride (the stage hand-off audit): bit-exact, with and
    without masks (the staged count is the masked count)."""
    from mageslam_amd import orb

    det = orb.OrbDetector(nfeatures=3200)
    da = det.DetectAndCompute(synth.frame(0, 1280, 720))[1]
    db = det.DetectAndCompute(synth.frame(1, 1280, 720))[1]
    assert len(da) >= na and len(db) >= nb
    da, db = da[:na], db[:nb]
    tree = synth.bow_tree(np.concatenate([da[:1000], db[:1000]]))
    t = bow.OnlineBowTree(*tree)
    got = bow.IndexedMatch(t, da, db)
    ref = oracle.indexed_match(tree, da, db)
    assert np.array_equal(got.view(np.uint8), ref.view(np.uint8))
    mb = np.ones(nb, bool)
    mb[::7] = False  # a masked B count below the stage size
    got = bow.IndexedMatch(t, da, db, None, mb)
    ref = oracle.indexed_match(tree, da, db, None, mb.astype(np.uint8))
    assert np.array_equal(got.view(np.uint8), ref.view(np.uint8))


def test_indexed_and_radius_large_sets(gpu, oracle):
    """Sets above the 2048 entries staged in LDS (the kernels' global-memory path): 3000-feature
    frames through IndexedMatch and RadiusMatch, bit-exact vs the oracle."""
    from mageslam_amd import matcher, orb

    det = orb.OrbDetector(nfeatures=3000)
    (ka, da), (kb, db) = (det.DetectAndCompute(synth.frame(t, 1280, 720)) for t in (0, 1))
    assert len(da) > 2048 and len(db) > 2048
    tree = synth.bow_tree(np.concatenate([da, db]))
    got = bow.IndexedMatch(bow.OnlineBowTree(*tree), da, db)
    ref = oracle.indexed_match(tree, da, db)
    assert np.array_equal(got.view(np.uint8), ref.view(np.uint8))
    got = matcher.RadiusMatch(kb, db, ka, da, 15.0)
    ref = oracle.radius_match(kb, db, ka, da, 15.0)
    assert len(got) > 0 and np.array_equal(got.view(np.uint8), ref.view(np.uint8))


def test_online_bow_weights_insert_query_parity(gpu, oracle):
    """OnlineBow's keyframe database (SetNodeWeights, InsertDescriptors, QueryFeatures,
    QueryUnknownImage, RemoveImage) with GPU leaf descent vs the oracle's literal restatement:
    identical IDF weights, node values, query results and scores (float32, canonical orders)."""
    from mageslam_amd import orb

    det = orb.OrbDetector(nfeatures=2000)
    train = [det.DetectAndCompute(synth.frame(t, 640, 480))[1] for t in range(15)]
    counts = [len(d) for d in train]
    g = bow.OnlineBow.CreateTree(np.concatenate(train), counts)
    o = oracle.OnlineBowOracle(oracle.bow_train(np.concatenate(train)))
    o.SetNodeWeights(np.concatenate(train), counts)
    assert np.array_equal(g.weights, np.array(o.nodes_weight, np.float32))
    assert (g.weights > 0).sum() > 10
    kfs = {kf: det.DetectAndCompute(synth.frame(40 + 7 * kf, 640, 480))[1] for kf in range(6)}
    for kf, d in kfs.items():
        g.InsertDescriptors(kf, d)
        o.InsertDescriptors(kf, d)
    for leaf, entries in o.m_NodeKeyframeMap.items():
        for kf, e in entries.items():
            assert g.node_kf[leaf][kf][0] == e["nodeValue"] and g.node_kf[leaf][kf][1] == e["indexes"]
    for kf in (0, 3, 5):
        rg = g.QueryUnknownImage(kfs[kf], 4)
        ro = o.QueryUnknownImage(kfs[kf], 4)
        assert rg == ro and rg[0][0] == kf and abs(rg[0][1] - 1.0) < 1e-4, (kf, rg)
        q = kfs[kf][17]
        assert g.QueryFeatures(q, kf) == o.QueryFeatures(q, kf) and 17 in g.QueryFeatures(q, kf)
    g.RemoveImage(3)
    o.RemoveImage(3)
    assert g.QueryUnknownImage(kfs[3], 6) == o.QueryUnknownImage(kfs[3], 6)
    assert all(kf != 3 for kf, _ in g.QueryUnknownImage(kfs[3], 6))


@pytest.mark.parametrize("levels,branching,max_iter", [(2, 6, 12), (3, 4, 8), (1, 16, 5)])
def test_create_tree_kmedoid_parity(gpu, oracle, frames, levels, branching, max_iter):
    """OnlineBow::Kmedoid (OnlineBow.cpp:487-521): the GPU's linear medoid selection (per-bit
    member counts) gives the same tree as the oracle's literal O(g^2) IterateClusteringKmedoid."""
    descs, _ = frames
    d = np.concatenate(descs[:2])
    t = bow.OnlineBowTree.CreateTree(d, levels, branching, max_iter, kmedoid=True)
    ref = oracle.bow_train(d, levels, branching, max_iter, kmedoid=True)
    for x, y in zip(t.tree(), ref):
        assert np.array_equal(x, y)
    rows = {bytes(r) for r in d}
    assert all(bytes(r) in rows for r in t.tree()[0][1:])  # every node is a training descriptor


def test_create_tree_kmedoid_training_frames(gpu, oracle):
    from mageslam_amd import orb

    det = orb.OrbDetector(nfeatures=2000)
    d = np.concatenate([det.DetectAndCompute(synth.frame(t, 640, 480))[1] for t in range(6)])
    t = bow.OnlineBowTree.CreateTree(d, kmedoid=True)
    for x, y in zip(t.tree(), oracle.bow_train(d, kmedoid=True)):
        assert np.array_equal(x, y)


def test_online_bow_query_edges(gpu, oracle, frames):
    """QueryUnknownImage edge cases against the oracle: an empty query, maxResults truncation, the
    QualifyingCandidateScore filter, and a keyframe inserted twice (only the first call's entries
    are normalised, as in the reference)."""
    descs, tree = frames
    train = np.concatenate(descs[:2])
    counts = [len(descs[0]), len(descs[1])]
    g = bow.OnlineBow(bow.OnlineBowTree(*tree), qualifying_candidate_score=0.3)
    o = oracle.OnlineBowOracle(tree, qualifying_candidate_score=0.3)
    g.SetNodeWeights(train, counts)
    o.SetNodeWeights(train, counts)
    assert g.QueryUnknownImage(descs[2][:0], 5) == o.QueryUnknownImage(descs[2][:0], 5) == []
    for kf, d in enumerate(descs):
        g.InsertDescriptors(kf, d)
        o.InsertDescriptors(kf, d)
    g.InsertDescriptors(1, descs[3][:50])
    o.InsertDescriptors(1, descs[3][:50])
    for q in (descs[0], descs[3][:300]):
        for m in (1, 2, 10):
            assert g.QueryUnknownImage(q, m) == o.QueryUnknownImage(q, m)
    assert len(g.QueryUnknownImage(descs[0], 1)) == 1
