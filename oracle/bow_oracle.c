/*
 * bow_oracle.c — CPU restatement of the OnlineBow vocabulary-tree descent and IndexedMatch
 * (TEST INFRASTRUCTURE ONLY: used by tests/ and smoke(), never by the product).
 *
 * Follows Core/MAGESLAM/Source/BoW/OnlineBow.cpp:289-311 (FindLeafNode),
 * BoW/OnlineBowFeatureMatcher.cpp:8-31 (leaf -> feature lists in insertion order, QueryFeatures),
 * OnlineBow.cpp:115-133 / 413-440 (QueryFeatures of a keyframe: same leaf lists) and
 * Tracking/FeatureMatcher.cpp:22-55 (TrackMatch), 192-292 (IndexedMatch), written sequentially
 * exactly as the reference loops (candidate order = ascending feature index), so that the GPU's
 * order-free reductions are checked against the literal loop.  Parity unpinned (no reference
 * fixtures exist for this path).
 */
#include <limits.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/mage_hot.h"

int oracle_hamming(const uint8_t* a, const uint8_t* b);

/* OnlineBow::FindLeafNode: from the root, repeatedly take the child with the strictly smallest
 * GetDescriptorDistance (first child wins ties) until a node without children. */
uint32_t oracle_bow_find_leaf(const uint8_t* node_desc, const uint32_t* child_start, const uint32_t* children,
                              const uint8_t* desc)
{
    uint32_t cur = 0;
    while (child_start[cur + 1] > child_start[cur]) {
        const uint32_t node = cur; /* the range-for binds m_nodes[curId].childrenIDs once */
        int best_d = INT_MAX;
        for (uint32_t k = child_start[node]; k < child_start[node + 1]; k++) {
            const uint32_t child = children[k];
            const int d = oracle_hamming(desc, node_desc + 32 * (size_t)child);
            if (d < best_d) {
                best_d = d;
                cur = child;
            }
        }
    }
    return cur;
}

typedef struct {
    size_t idx;
    int d;
} track_result;

/* TrackMatch (FeatureMatcher.cpp:28-54) */
static void track_match(const uint8_t* left, const uint8_t* right_desc, size_t idx_right, const uint8_t* right_mask,
                        track_result* best, track_result* second, int max_hamming)
{
    if (right_mask && !right_mask[idx_right]) return;
    const int d = oracle_hamming(left, right_desc + 32 * idx_right);
    if (d < max_hamming) {
        if (d < best->d) {
            *second = *best;
            best->idx = idx_right;
            best->d = d;
        } else if (d < second->d) {
            second->idx = idx_right;
            second->d = d;
        }
    }
}

/* QueryFeatures: the features of the other image assigned to `leaf`, ascending index */
static size_t query_features(const uint32_t* leaves, uint32_t n, uint32_t leaf, uint32_t* out)
{
    size_t k = 0;
    for (uint32_t i = 0; i < n; i++)
        if (leaves[i] == leaf) out[k++] = i;
    return k;
}

/* IndexedMatch (FeatureMatcher.cpp:192-292) with BoW candidates; leaves from FindLeafNode.
 * Masks may be NULL (all true).  Returns the number of matches (<= cap written). */
uint32_t oracle_indexed_match(const uint8_t* node_desc, const uint32_t* child_start, const uint32_t* children,
                              const uint8_t* da, uint32_t na, const uint8_t* ma, const uint8_t* db, uint32_t nb,
                              const uint8_t* mb, int max_hamming_dist, int min_hamming_difference,
                              mage_dmatch* out, uint32_t cap)
{
    uint32_t cnt_a = 0, cnt_b = 0;
    for (uint32_t i = 0; i < na; i++) cnt_a += !ma || ma[i];
    for (uint32_t i = 0; i < nb; i++) cnt_b += !mb || mb[i];
    if (cnt_a == 0 || cnt_b == 0) return 0;
    const int max_hamming = max_hamming_dist + 1;
    uint32_t* la = (uint32_t*)malloc(sizeof(uint32_t) * (na + 1));
    uint32_t* lb = (uint32_t*)malloc(sizeof(uint32_t) * (nb + 1));
    uint32_t* cand = (uint32_t*)malloc(sizeof(uint32_t) * ((na > nb ? na : nb) + 1));
    uint32_t* fa = (uint32_t*)malloc(sizeof(uint32_t) * (na + 1));
    uint32_t* fb = (uint32_t*)malloc(sizeof(uint32_t) * (na + 1));
    /* CreateFeatureMatcher / AddImage assign every feature of an image to its leaf */
    for (uint32_t i = 0; i < na; i++) la[i] = oracle_bow_find_leaf(node_desc, child_start, children, da + 32 * (size_t)i);
    for (uint32_t i = 0; i < nb; i++) lb[i] = oracle_bow_find_leaf(node_desc, child_start, children, db + 32 * (size_t)i);
    uint32_t nf = 0;
    for (uint32_t ia = 0; ia < na; ia++) {
        if (ma && !ma[ia]) continue;
        const uint8_t* desc_a = da + 32 * (size_t)ia;
        const size_t nc = query_features(lb, nb, oracle_bow_find_leaf(node_desc, child_start, children, desc_a), cand);
        track_result best = {SIZE_MAX, max_hamming}, second = {SIZE_MAX, max_hamming};
        for (size_t j = 0; j < nc; j++) track_match(desc_a, db, cand[j], mb, &best, &second, max_hamming);
        if (best.d < max_hamming &&
            (second.d >= max_hamming || second.d - best.d >= min_hamming_difference)) {
            fa[nf] = ia;
            fb[nf] = (uint32_t)best.idx;
            nf++;
        }
    }
    uint32_t n = 0;
    for (uint32_t m = 0; m < nf; m++) {
        const uint32_t ib = fb[m];
        const uint8_t* desc_b = db + 32 * (size_t)ib;
        const size_t nc = query_features(la, na, oracle_bow_find_leaf(node_desc, child_start, children, desc_b), cand);
        track_result best = {SIZE_MAX, max_hamming}, second = {SIZE_MAX, max_hamming};
        for (size_t j = 0; j < nc; j++) track_match(desc_b, da, cand[j], ma, &best, &second, max_hamming);
        if (best.d < max_hamming && best.idx == fa[m] &&
            (second.d >= max_hamming || second.d - best.d >= min_hamming_difference)) {
            if (n < cap) {
                out[n].query_idx = (int32_t)best.idx;
                out[n].train_idx = (int32_t)ib;
                out[n].img_idx = -1;
                out[n].distance = (float)best.d;
            }
            n++;
        }
    }
    free(la);
    free(lb);
    free(cand);
    free(fa);
    free(fb);
    return n;
}
