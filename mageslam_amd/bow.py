"""Vocabulary tree + IndexedMatch — host mirror of OnlineBow's feature lookup and IndexedMatch.

`OnlineBowTree` holds the tree OnlineBow::CreateTree builds (Core/MAGESLAM/Source/BoW/OnlineBow.cpp:
325-411) on the GPU; `FindLeafNode` mirrors OnlineBow::FindLeafNode (:289-311).  `IndexedMatch`
mirrors `IndexedMatch(bagOfWords, matcherA, matcherB, idA, idB, imageA, imageB, maskA, maskB, countA,
countB, maxHammingDist, minHammingDifference, memory, goodMatches)` (Tracking/FeatureMatcher.h:30-62,
FeatureMatcher.cpp:192-292) for the BoW candidate source every caller uses — OnlineBowFeatureMatcher
or OnlineBow::QueryFeatures, both "the other image's features in the query's leaf" — with the
descriptors passed directly.
"""
from __future__ import annotations

import ctypes as C
import math

import numpy as np

from . import _lib
from ._lib import DM_DTYPE, check, ptr


class OnlineBowTree:
    def __init__(self, node_desc, child_start, children, device: int = 0):
        self._nd = np.ascontiguousarray(node_desc, np.uint8).reshape(-1, 32)
        self._cs = np.ascontiguousarray(child_start, np.uint32)
        self._ch = np.ascontiguousarray(children, np.uint32)
        if len(self._cs) != len(self._nd) + 1:
            raise ValueError("child_start needs n_nodes + 1 entries")
        self._h = C.c_void_p()
        check(_lib.load().mage_bow_create(ptr(self._nd), ptr(self._cs), ptr(self._ch), len(self._nd), device,
                                          C.byref(self._h)))

    @classmethod
    def from_tuple(cls, tree, device: int = 0) -> "OnlineBowTree":
        return cls(*tree, device=device)

    @classmethod
    def CreateTree(cls, descriptors, levels: int = 2, branching: int = 6, max_iter: int = 12,
                   device: int = 0, kmedoid: bool = False) -> "OnlineBowTree":
        """OnlineBow::CreateTree (OnlineBow.cpp:325-337) on the GPU: hierarchical Kmean over the
        training descriptors with BagOfWordsSettings TrainingTreeLevels / TrainingTreeBranchingFactor
        / MaxTrainingIteration (MageSettings.h:230-232); kmedoid: the Kmedoid recursion (:487-521)."""
        d = np.ascontiguousarray(descriptors, np.uint8).reshape(-1, 32)
        self = cls.__new__(cls)
        self._h = C.c_void_p()
        train = _lib.load().mage_bow_train_kmedoid if kmedoid else _lib.load().mage_bow_train
        check(train(ptr(d), len(d), levels, branching, max_iter, device, C.byref(self._h)))
        self._nd, self._cs, self._ch = self.tree()
        return self

    def tree(self):
        """(node_desc (n, 32) u8, child_start (n + 1,) u32, children (n - 1,) u32) of the device tree."""
        n = C.c_uint32(0)
        L = _lib.load()
        L.mage_bow_get_tree(self._h, None, None, None, 0, C.byref(n))
        nd = np.zeros((n.value, 32), np.uint8)
        cs = np.zeros(n.value + 1, np.uint32)
        ch = np.zeros(max(n.value, 1), np.uint32)
        check(L.mage_bow_get_tree(self._h, ptr(nd), ptr(cs), ptr(ch), n.value, C.byref(n)))
        return nd, cs, ch[: int(cs[-1])]

    @property
    def handle(self):
        return self._h

    def close(self) -> None:
        if getattr(self, "_h", None) and self._h.value:
            _lib.load().mage_bow_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def find_leaves(self, descriptors) -> np.ndarray:
        d = np.ascontiguousarray(descriptors, np.uint8).reshape(-1, 32)
        out = np.zeros(len(d), np.uint32)
        check(_lib.load().mage_bow_find_leaves(self._h, ptr(d), len(d), ptr(out)))
        return out

    def FindLeafNode(self, descriptor) -> int:
        return int(self.find_leaves(descriptor)[0])

    def find_leaves_device(self, desc, n: int, leaf, stream=None) -> None:
        """Device form over n descriptors (torch device tensors)."""
        check(_lib.load().mage_bow_find_leaves_device(self._h, ptr(desc), n, ptr(leaf),
                                                      C.c_void_p(stream) if stream else None))


def IndexedMatch(tree: OnlineBowTree, descA, descB, maskA=None, maskB=None, maxHammingDist: int = 30,
                 minHammingDifference: int = 1) -> np.ndarray:
    """Two-way BoW-indexed match on the GPU; DMatch records (imgIdx -1) in ascending A index."""
    da = np.ascontiguousarray(descA, np.uint8).reshape(-1, 32)
    db = np.ascontiguousarray(descB, np.uint8).reshape(-1, 32)
    ma = None if maskA is None else np.ascontiguousarray(np.asarray(maskA, bool), np.uint8)
    mb = None if maskB is None else np.ascontiguousarray(np.asarray(maskB, bool), np.uint8)
    if ma is not None and len(ma) != len(da):
        raise ValueError("maskA length must equal the number of A descriptors")
    if mb is not None and len(mb) != len(db):
        raise ValueError("maskB length must equal the number of B descriptors")
    cap = max(len(da), 1)
    out = np.zeros(cap, DM_DTYPE)
    n = C.c_uint32(0)
    check(_lib.load().mage_indexed_match(tree.handle, ptr(da), len(da), ptr(ma), ptr(db), len(db), ptr(mb),
                                         int(maxHammingDist), int(minHammingDifference), ptr(out), cap, C.byref(n)))
    return out[: n.value].copy()


def indexed_match_batch_device(desc_a, leaf_a, mask_a, a_pitch: int, n_a, desc_b, leaf_b, mask_b, b_pitch: int, n_b,
                               pairs: int, max_distance: int, min_difference: int, out, capacity: int, n_out, status,
                               stream=None) -> None:
    """Batched device IndexedMatch over `pairs` (A_p, B_p) sets (torch device tensors; masks may be None)."""
    check(_lib.load().mage_indexed_match_batch_device(
        ptr(desc_a), ptr(leaf_a), ptr(mask_a), a_pitch, ptr(n_a), ptr(desc_b), ptr(leaf_b), ptr(mask_b), b_pitch,
        ptr(n_b), pairs, max_distance, min_difference, ptr(out), capacity, ptr(n_out), ptr(status),
        C.c_void_p(stream) if stream else None))


class OnlineBow:
    """OnlineBow's keyframe database over a vocabulary tree (Core/MAGESLAM/Source/BoW/OnlineBow.cpp):
    the IDF node weights CreateTree ends with (SetNodeWeights :340-394), AddImage / InsertDescriptors
    (:94-98, :413-449), RemoveImage (:100-113), QueryFeatures (:115-133) and QueryUnknownImage
    (:155-271).  The descriptor -> leaf descent (FindLeafNode, the Hamming part) runs on the GPU
    (mage_bow_find_leaves); the bookkeeping is host code, as in the reference, in float32 with the
    reference's expression order.  The reference iterates unordered_maps (node -> keyframe entries,
    query node values), so its float sums and its std::sort tie order are implementation-defined:
    here nodes and keyframes are visited in ascending id and equal scores keep ascending keyframe id.
    The root's weight is left 0 (the reference leaves it uninitialised; no descriptor reaches it)."""

    def __init__(self, tree: OnlineBowTree, qualifying_candidate_score: float = 0.75):
        self.tree = tree
        self.weights = np.zeros(len(tree._nd), np.float32)
        self.node_kf: dict = {}  # leaf -> {keyframe id: [nodeValue (f32), feature indexes]}
        self.image_set: set = set()
        self.qualifying = np.float32(qualifying_candidate_score)  # BagOfWordsSettings (MageSettings.h:226)

    @classmethod
    def CreateTree(cls, training, descriptors_count, levels: int = 2, branching: int = 6, max_iter: int = 12,
                   device: int = 0, qualifying_candidate_score: float = 0.75) -> "OnlineBow":
        """OnlineBow::CreateTree (:325-338) over the training set AddTrainingDescriptors collected
        (`descriptors_count` = descriptors per training image, m_descriptorsCount)."""
        t = OnlineBowTree.CreateTree(training, levels, branching, max_iter, device)
        self = cls(t, qualifying_candidate_score)
        self.SetNodeWeights(training, descriptors_count)
        return self

    def SetNodeWeights(self, training, descriptors_count) -> None:
        leaves = self.tree.find_leaves(training).tolist()
        images = {}  # leaf -> training images with a descriptor in it
        start = 0
        for c in descriptors_count:
            for leaf in set(leaves[start:start + int(c)]):
                images[leaf] = images.get(leaf, 0) + 1
            start += int(c)
        n_images = len(descriptors_count)
        for leaf, cnt in images.items():  # log((float)(nImages + 1) / (float)count), std::log(float)
            self.weights[leaf] = np.float32(math.log(float(np.float32(n_images + 1) / np.float32(cnt))))  # logf, correctly rounded

    def InsertDescriptors(self, kf_id: int, descriptors) -> None:
        leaves = self.tree.find_leaves(descriptors).tolist()
        fresh = []  # entries created by this call: normalised at the end (the reference's pts)
        total = np.float32(0)
        for i, leaf in enumerate(leaves):
            entries = self.node_kf.setdefault(leaf, {})
            e = entries.get(kf_id)
            if e is None:
                e = entries[kf_id] = [np.float32(0), []]
                fresh.append(e)
            e[1].append(i)
            e[0] = np.float32(e[0] + self.weights[leaf])
            total = np.float32(total + self.weights[leaf])
        if total == 0:
            return
        for e in fresh:
            e[0] = np.float32(e[0] / total)
        self.image_set.add(kf_id)

    AddImage = InsertDescriptors

    def RemoveImage(self, kf_id: int) -> None:
        for entries in self.node_kf.values():
            entries.pop(kf_id, None)
        self.image_set.discard(kf_id)

    def QueryFeatures(self, descriptor, kf_id: int) -> list:
        """Feature indexes of keyframe kf_id in the descriptor's leaf."""
        if kf_id not in self.image_set:
            raise KeyError("QueryFeatures for a keyframe that is not in the BoW")
        leaf = int(self.tree.find_leaves(descriptor)[0])
        e = self.node_kf.get(leaf, {}).get(kf_id)
        return [] if e is None else list(e[1])

    def QueryUnknownImage(self, descriptors, max_results: int) -> list:
        """[(keyframe id, score)] most similar first: L1 scoring of the normalised node values."""
        leaves = self.tree.find_leaves(descriptors).tolist()
        cur: dict = {}
        total = np.float32(0)
        for leaf in leaves:
            w = self.weights[leaf]
            cur[leaf] = np.float32(cur[leaf] + w) if leaf in cur else w
            total = np.float32(total + w)
        if total == 0:
            return []
        for leaf in cur:
            cur[leaf] = np.float32(cur[leaf] / total)
        score: dict = {}
        for leaf in sorted(cur):
            a = cur[leaf]
            entries = self.node_kf.get(leaf, {})
            for kf in sorted(entries):
                b = entries[kf][0]
                v = np.float32(np.float32(np.abs(np.float32(a - b)) - np.abs(a)) - np.abs(b))
                score[kf] = np.float32(score[kf] + v) if kf in score else v
        best = np.float32(0)
        for kf in score:
            score[kf] = np.float32(-score[kf] / np.float32(2.0))
            if score[kf] > best:
                best = score[kf]
        q = np.float32(best * self.qualifying)
        out = sorted(((kf, s) for kf, s in score.items() if s >= q), key=lambda t: (-t[1], t[0]))
        return [(int(kf), float(s)) for kf, s in out[:max_results]]
