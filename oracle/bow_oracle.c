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

/* ---------------------------------------------------------------------------------------------
 * Vocabulary training: OnlineBow::CreateTree (OnlineBow.cpp:325-337) -> Kmean (:451-485),
 * InitializeTraining (:396-411), IterateClusteringKmean (:587-614), KmeanCenter (:551-585),
 * FindCluster (:631-638).  Literal recursive restatement.
 *
 * InitializeTraining shuffles the descriptor refs with std::shuffle(…, mt19937{}) — a FRESH
 * default-seeded engine (seed 5489) per call, so the first `branching` positions depend only on
 * the subset size.  std::shuffle's algorithm is the standard library's: the reference is built
 * with MSVC, whose _Random_shuffle1 walks targets 1..n-1 and swaps target t with position
 * _Rng_from_urng(t + 1) (one 32-bit draw per target for sizes < 2^32; a draw r is kept when
 * r / (t+1) < 0xFFFFFFFF / (t+1) or 0xFFFFFFFF % (t+1) == t, and yields r % (t+1)).  Restated from
 * the published MSVC STL algorithm; no reference fixture pins it (parity unpinned).
 * --------------------------------------------------------------------------------------------- */
typedef struct {
    uint32_t mt[624];
    int idx;
} mt19937_t;

static void mt_seed(mt19937_t* m, uint32_t s)
{
    m->mt[0] = s;
    for (int i = 1; i < 624; i++) m->mt[i] = 1812433253u * (m->mt[i - 1] ^ (m->mt[i - 1] >> 30)) + (uint32_t)i;
    m->idx = 624;
}

static uint32_t mt_next(mt19937_t* m)
{
    if (m->idx >= 624) {
        for (int i = 0; i < 624; i++) {
            const uint32_t y = (m->mt[i] & 0x80000000u) | (m->mt[(i + 1) % 624] & 0x7FFFFFFFu);
            m->mt[i] = m->mt[(i + 397) % 624] ^ (y >> 1) ^ ((y & 1u) ? 0x9908B0DFu : 0u);
        }
        m->idx = 0;
    }
    uint32_t y = m->mt[m->idx++];
    y ^= y >> 11;
    y ^= (y << 7) & 0x9D2C5680u;
    y ^= (y << 15) & 0xEFC60000u;
    y ^= y >> 18;
    return y;
}

uint32_t oracle_mt19937_first(uint32_t seed, uint32_t k) /* k-th output (1-based), for the known answer */
{
    mt19937_t m;
    mt_seed(&m, seed);
    uint32_t v = 0;
    for (uint32_t i = 0; i < k; i++) v = mt_next(&m);
    return v;
}

/* positions of the first `k` refs after shuffle(refs[0..n), mt19937{}) — perm[] gets all n */
void oracle_msvc_shuffle(uint32_t n, uint32_t* perm)
{
    mt19937_t m;
    mt_seed(&m, 5489u);
    for (uint32_t i = 0; i < n; i++) perm[i] = i;
    for (uint32_t t = 1; t < n; t++) {
        const uint64_t index = (uint64_t)t + 1, mask = 0xFFFFFFFFull;
        uint64_t off;
        for (;;) {
            const uint64_t r = mt_next(&m);
            if (r / index < mask / index || mask % index == index - 1) {
                off = r % index;
                break;
            }
        }
        if (off != t) {
            const uint32_t tmp = perm[t];
            perm[t] = perm[off];
            perm[off] = tmp;
        }
    }
}

typedef struct {
    uint8_t* desc;  /* node descriptors, 32 B each */
    uint32_t** kids;
    uint32_t* nkids;
    uint32_t n, cap;
} bow_tree_t;

static uint32_t tree_add(bow_tree_t* t, const uint8_t* d)
{
    if (t->n == t->cap) {
        t->cap = t->cap ? 2 * t->cap : 64;
        t->desc = (uint8_t*)realloc(t->desc, 32ull * t->cap);
        t->kids = (uint32_t**)realloc(t->kids, sizeof(uint32_t*) * t->cap);
        t->nkids = (uint32_t*)realloc(t->nkids, sizeof(uint32_t) * t->cap);
    }
    memcpy(t->desc + 32ull * t->n, d, 32);
    t->kids[t->n] = NULL;
    t->nkids[t->n] = 0;
    return t->n++;
}

static int find_cluster(const uint8_t* d, const uint8_t* centers, uint32_t k)
{
    /* min_element with d(c1) < d(c2): the first smallest */
    uint32_t best = 0;
    int bd = oracle_hamming(centers, d);
    for (uint32_t g = 1; g < k; g++) {
        const int dd = oracle_hamming(centers + 32 * g, d);
        if (dd < bd) {
            bd = dd;
            best = g;
        }
    }
    return (int)best;
}

static void kmean_center(const uint8_t* descs, const uint32_t* idx, uint32_t cnt, uint8_t* c)
{
    uint32_t sum[256] = {0};
    for (uint32_t i = 0; i < cnt; i++)
        for (int j = 0; j < 32; j++)
            for (int k = 0; k < 8; k++) sum[j * 8 + k] += (descs[32ull * idx[i] + j] >> k) & 1u;
    const uint32_t half = (cnt + 1) / 2;
    for (int j = 0; j < 32; j++)
        for (int k = 0; k < 8; k++) {
            if (sum[j * 8 + k] >= half) c[j] |= (uint8_t)(1u << k);
            else c[j] &= (uint8_t)~(1u << k);
        }
}

/* IterateClusteringKmedoid's update (OnlineBow.cpp:608-637), literally: the member with the
 * first smallest sum of distances to all members of its group becomes the medoid.  An empty
 * group (the reference would read groups[g][0] of an empty vector) keeps its medoid. */
static int kmedoid_update(const uint8_t* descs, const uint32_t* idx, uint32_t cnt, uint8_t* c)
{
    if (cnt == 0) return 0;
    long long minD = 0x7FFFFFFFFFFFFFFFll;
    uint32_t minI = 0;
    for (uint32_t i = 0; i < cnt; i++) {
        long long distance = 0;
        for (uint32_t k = 0; k < cnt; k++) distance += oracle_hamming(descs + 32ull * idx[i], descs + 32ull * idx[k]);
        if (distance < minD) {
            minD = distance;
            minI = i;
        }
    }
    if (oracle_hamming(descs + 32ull * idx[minI], c) != 0) {
        memcpy(c, descs + 32ull * idx[minI], 32);
        return 1;
    }
    return 0;
}

/* Kmean (OnlineBow.cpp:451-485) or, with medoid, Kmedoid (:487-521): the same recursion */
static void kmean(bow_tree_t* t, uint32_t parent, const uint8_t* descs, uint32_t n, uint32_t level, uint32_t levels,
                  uint32_t branching, uint32_t max_iter, int medoid)
{
    uint32_t* perm = (uint32_t*)malloc(sizeof(uint32_t) * (n ? n : 1));
    oracle_msvc_shuffle(n, perm);
    const uint32_t k = branching < n ? branching : n;
    uint8_t* centers = (uint8_t*)malloc(32ull * (k ? k : 1));
    for (uint32_t g = 0; g < k; g++) memcpy(centers + 32 * g, descs + 32ull * perm[g], 32);
    /* groups: members of cluster g in ascending descriptor order */
    uint32_t* assign = (uint32_t*)malloc(sizeof(uint32_t) * (n ? n : 1));
    uint32_t* gidx = (uint32_t*)malloc(sizeof(uint32_t) * (n ? n : 1));
    uint32_t* gstart = (uint32_t*)calloc(k + 1, sizeof(uint32_t));
    uint32_t iter = 0, changed;
    do {
        changed = 0;
        iter++;
        memset(gstart, 0, sizeof(uint32_t) * (k + 1));
        for (uint32_t i = 0; i < n; i++) {
            assign[i] = (uint32_t)find_cluster(descs + 32ull * i, centers, k);
            gstart[assign[i] + 1]++;
        }
        for (uint32_t g = 0; g < k; g++) gstart[g + 1] += gstart[g];
        {
            uint32_t* fill = (uint32_t*)malloc(sizeof(uint32_t) * (k + 1));
            memcpy(fill, gstart, sizeof(uint32_t) * (k + 1));
            for (uint32_t i = 0; i < n; i++) gidx[fill[assign[i]]++] = i;
            free(fill);
        }
        for (uint32_t g = 0; g < k; g++) {
            if (medoid) {
                changed += (uint32_t)kmedoid_update(descs, gidx + gstart[g], gstart[g + 1] - gstart[g], centers + 32 * g);
                continue;
            }
            uint8_t pre[32];
            memcpy(pre, centers + 32 * g, 32);
            kmean_center(descs, gidx + gstart[g], gstart[g + 1] - gstart[g], centers + 32 * g);
            if (oracle_hamming(pre, centers + 32 * g) != 0) changed++;
        }
    } while (iter < max_iter && changed > 0);
    uint32_t* ids = (uint32_t*)malloc(sizeof(uint32_t) * (k ? k : 1));
    for (uint32_t g = 0; g < k; g++) {
        ids[g] = tree_add(t, centers + 32 * g);
        t->kids[parent] = (uint32_t*)realloc(t->kids[parent], sizeof(uint32_t) * (t->nkids[parent] + 1));
        t->kids[parent][t->nkids[parent]++] = ids[g];
    }
    if (level < levels) {
        for (uint32_t g = 0; g < k; g++) {
            const uint32_t cnt = gstart[g + 1] - gstart[g];
            if (cnt > 1) {
                uint8_t* sub = (uint8_t*)malloc(32ull * cnt);
                for (uint32_t i = 0; i < cnt; i++) memcpy(sub + 32ull * i, descs + 32ull * gidx[gstart[g] + i], 32);
                kmean(t, ids[g], sub, cnt, level + 1, levels, branching, max_iter, medoid);
                free(sub);
            }
        }
    }
    free(ids);
    free(perm);
    free(centers);
    free(assign);
    free(gidx);
    free(gstart);
}

/* CreateTree over n descriptors: fills node_desc (cap nodes), child_start (n_nodes + 1) and
 * children (n_nodes - 1); returns the node count (0 when it exceeds cap). */
uint32_t oracle_bow_train2(const uint8_t* desc, uint32_t n, uint32_t levels, uint32_t branching, uint32_t max_iter,
                           uint8_t* node_desc, uint32_t* child_start, uint32_t* children, uint32_t cap, int medoid)
{
    bow_tree_t t = {0};
    static const uint8_t zero[32] = {0};
    tree_add(&t, zero); /* Node(0): the root's descriptor is never compared */
    if (n > 0) kmean(&t, 0, desc, n, 1, levels, branching, max_iter, medoid);
    uint32_t out = 0;
    if (t.n <= cap) {
        uint32_t c = 0;
        for (uint32_t i = 0; i < t.n; i++) {
            memcpy(node_desc + 32ull * i, t.desc + 32ull * i, 32);
            child_start[i] = c;
            for (uint32_t k = 0; k < t.nkids[i]; k++) children[c++] = t.kids[i][k];
        }
        child_start[t.n] = c;
        out = t.n;
    }
    for (uint32_t i = 0; i < t.n; i++) free(t.kids[i]);
    free(t.kids);
    free(t.nkids);
    free(t.desc);
    return out;
}

uint32_t oracle_bow_train(const uint8_t* desc, uint32_t n, uint32_t levels, uint32_t branching, uint32_t max_iter,
                          uint8_t* node_desc, uint32_t* child_start, uint32_t* children, uint32_t cap)
{
    return oracle_bow_train2(desc, n, levels, branching, max_iter, node_desc, child_start, children, cap, 0);
}
