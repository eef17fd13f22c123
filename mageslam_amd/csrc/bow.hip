// bow.hip — OnlineBow vocabulary-tree descent and IndexedMatch on MI355X (gfx950).
//
// Replaces OnlineBow::FindLeafNode (Core/MAGESLAM/Source/BoW/OnlineBow.cpp:289-311), the leaf ->
// feature lists of OnlineBowFeatureMatcher / OnlineBow::QueryFeatures (OnlineBowFeatureMatcher.cpp:
// 8-31, OnlineBow.cpp:115-133) and IndexedMatch (Tracking/FeatureMatcher.cpp:192-292).
//
//   bow_leaves_kernel     thread per descriptor: descend from the root, first child with the
//                         strictly smallest Hamming distance per level (the tree is tiny and
//                         stays in L2 / the scalar cache: 6^2 leaves by default, MageSettings.h:230)
//   indexed_match_kernel  one 1024-thread workgroup per (A, B) feature-set pair:
//     1. masked features of each side -> 64-bit keys (leaf, index) sorted ascending in LDS (the
//        shared hybrid bitonic sort): a leaf's candidates are one contiguous run in ascending
//        index order — exactly QueryFeatures' lists, which hold every feature of that leaf in
//        insertion order (the masks only filter inside TrackMatch);
//     2. a 16-lane group per A feature: lanes stride over B's run of its leaf.  TrackMatch
//        (:28-54) visited in ascending order is order-free: best = min (d, index) over d <
//        maxHamming, second = the second smallest such d (the strict-< updates keep ties as
//        second); merged with four shuffle steps.  The reverse check of an accepted pair (i, j)
//        (:255-276) needs only B_j and A's run of the same leaf (leaf(B_j) = leaf(A_i) since j came
//        from that run), so the same group runs it immediately — no barrier between the passes;
//     3. ordered compaction in A order (the reference appends in forward-match order).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <functional>
#include <cstring>
#include <vector>

#include "common.hpp"
#include "lds_sort.hpp"

struct mage_bow {
    int device = 0;
    uint32_t n_nodes = 0;
    mage::DeviceBuffer nodes, child_start, children;
    mage::DeviceBuffer scratch;
    hipStream_t st = nullptr;
};

namespace mage {
namespace {

constexpr int IM_MAX = 4096;  // features per side held in LDS (NumFeatures-sized sets)
constexpr int IM_GROUP = 16;  // lanes per A feature
constexpr int IM_GROUPS = SORT_THREADS / IM_GROUP;

struct IndexedParams {
    const uint8_t* da;
    const uint32_t* la;
    const uint8_t* ma;  // optional
    const uint32_t* na;
    long long a_pitch;
    const uint8_t* db;
    const uint32_t* lb;
    const uint8_t* mb;  // optional
    const uint32_t* nb;
    long long b_pitch;
    int max_dist, min_diff;
    unsigned cap;
    mage_dmatch* out;
    uint32_t* n_out;
    uint32_t* status;  // bit 0: a feature set exceeded IM_MAX
};

__device__ __forceinline__ unsigned hamming32(const uint4& qa, const uint4& qb, const uint8_t* t)
{
    const uint4 ta = *reinterpret_cast<const uint4*>(t);
    const uint4 tb = *reinterpret_cast<const uint4*>(t + 16);
    return __popc(qa.x ^ ta.x) + __popc(qa.y ^ ta.y) + __popc(qa.z ^ ta.z) + __popc(qa.w ^ ta.w) +
           __popc(qb.x ^ tb.x) + __popc(qb.y ^ tb.y) + __popc(qb.z ^ tb.z) + __popc(qb.w ^ tb.w);
}

__global__ __launch_bounds__(256) void bow_leaves_kernel(const uint8_t* __restrict__ nodes,
                                                         const uint32_t* __restrict__ child_start,
                                                         const uint32_t* __restrict__ children,
                                                         const uint8_t* __restrict__ desc, uint32_t n,
                                                         uint32_t* __restrict__ leaf)
{
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const uint4 qa = *reinterpret_cast<const uint4*>(desc + 32ull * i);
    const uint4 qb = *reinterpret_cast<const uint4*>(desc + 32ull * i + 16);
    uint32_t cur = 0;
    for (;;) {
        const uint32_t c0 = child_start[cur], c1 = child_start[cur + 1];
        if (c0 == c1) break;
        unsigned best = UINT_MAX;
        uint32_t next = cur;
        for (uint32_t k = c0; k < c1; k++) {
            const uint32_t c = children[k];
            const unsigned d = hamming32(qa, qb, nodes + 32ull * c);
            if (d < best) {
                best = d;
                next = c;
            }
        }
        cur = next;  // children have larger ids than their parent (checked at creation): terminates
    }
    leaf[i] = cur;
}

// first position in keys[0, n) (ascending) with keys[pos] >= k
__device__ __forceinline__ int lower_bound_u64(const unsigned long long* keys, int n, unsigned long long k)
{
    int lo = 0, hi = n;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (keys[mid] < k) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// TrackMatch over a run keys[lo, hi) of one leaf (indices in the low 32 bits) against query
// (qa, qb): returns best (d << 12 | index) and the second smallest d, both capped at max_h.
__device__ __forceinline__ void track_run(const unsigned long long* keys, int lo, int hi, int sub,
                                          const uint8_t* __restrict__ desc, const uint4& qa, const uint4& qb,
                                          unsigned max_h, unsigned& bestk, unsigned& second)
{
    unsigned m1 = max_h << 12 | 0xFFFu, m2 = max_h;
    for (int k = lo + sub; k < hi; k += IM_GROUP) {
        const unsigned idx = (unsigned)(keys[k] & 0xFFFFFFFFull);
        const unsigned d = hamming32(qa, qb, desc + 32ull * idx);
        if (d >= max_h) continue;
        const unsigned key = d << 12 | idx;
        if (key < m1) {
            m2 = min(m2, m1 >> 12);
            m1 = key;
        } else {
            m2 = min(m2, d);
        }
    }
#pragma unroll
    for (int off = IM_GROUP / 2; off > 0; off >>= 1) {
        const unsigned o1 = (unsigned)__shfl_xor((int)m1, off), o2 = (unsigned)__shfl_xor((int)m2, off);
        // two smallest of the union of {m1 <= m2} and {o1 <= o2}
        m2 = min(max(m1 >> 12, o1 >> 12), min(m2, o2));
        m1 = min(m1, o1);
    }
    bestk = m1;
    second = m2;
}

// the same over B's run with B's descriptors staged in LDS in key order (position k holds the
// descriptor of keys[k]): a 16-lane group reads 16 consecutive 32-byte entries
constexpr int IM_STAGE = 2048;  // B sets up to NumFeatures-sized 2048 are staged (64 KB of LDS)

__device__ __forceinline__ void track_run_lds(const unsigned long long* keys, int lo, int hi, int sub,
                                              const uint4* __restrict__ sdesc, const uint4& qa, const uint4& qb,
                                              unsigned max_h, unsigned& bestk, unsigned& second)
{
    unsigned m1 = max_h << 12 | 0xFFFu, m2 = max_h;
    for (int k = lo + sub; k < hi; k += IM_GROUP) {
        const unsigned idx = (unsigned)(keys[k] & 0xFFFFFFFFull);
        const uint4 ta = sdesc[2 * k], tb = sdesc[2 * k + 1];
        const unsigned d = __popc(qa.x ^ ta.x) + __popc(qa.y ^ ta.y) + __popc(qa.z ^ ta.z) + __popc(qa.w ^ ta.w) +
                           __popc(qb.x ^ tb.x) + __popc(qb.y ^ tb.y) + __popc(qb.z ^ tb.z) + __popc(qb.w ^ tb.w);
        if (d >= max_h) continue;
        const unsigned key = d << 12 | idx;
        if (key < m1) {
            m2 = min(m2, m1 >> 12);
            m1 = key;
        } else {
            m2 = min(m2, d);
        }
    }
#pragma unroll
    for (int off = IM_GROUP / 2; off > 0; off >>= 1) {
        const unsigned o1 = (unsigned)__shfl_xor((int)m1, off), o2 = (unsigned)__shfl_xor((int)m2, off);
        m2 = min(max(m1 >> 12, o1 >> 12), min(m2, o2));
        m1 = min(m1, o1);
    }
    bestk = m1;
    second = m2;
}

__global__ __launch_bounds__(SORT_THREADS) void indexed_match_kernel(IndexedParams p)
{
    __shared__ unsigned long long keysA[IM_MAX], keysB[IM_MAX];
    __shared__ uint4 sdescB[2 * IM_STAGE];
    __shared__ int res[IM_MAX];
    __shared__ int wsum[SORT_THREADS / kWave];
    __shared__ int s_cnt[2], s_base;
    const int pr = blockIdx.x, tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int na = (int)p.na[pr], nb = (int)p.nb[pr];
    const uint8_t* da = p.da + pr * p.a_pitch * 32;
    const uint8_t* db = p.db + pr * p.b_pitch * 32;
    const uint32_t* la = p.la + pr * p.a_pitch;
    const uint32_t* lb = p.lb + pr * p.b_pitch;
    const uint8_t* ma = p.ma ? p.ma + pr * p.a_pitch : nullptr;
    const uint8_t* mb = p.mb ? p.mb + pr * p.b_pitch : nullptr;
    if (na > IM_MAX || nb > IM_MAX) {
        if (tid == 0) {
            p.n_out[pr] = 0;
            atomicOr(p.status, 1u);
        }
        return;
    }
    // 1. masked (leaf, index) keys of both sides, ascending (descending sort of complements)
    if (tid < 2) s_cnt[tid] = 0;
    __syncthreads();
    for (int i = tid; i < na; i += SORT_THREADS)
        if (!ma || ma[i]) keysA[atomicAdd(&s_cnt[0], 1)] = ~((unsigned long long)la[i] << 32 | (unsigned)i);
    for (int i = tid; i < nb; i += SORT_THREADS)
        if (!mb || mb[i]) keysB[atomicAdd(&s_cnt[1], 1)] = ~((unsigned long long)lb[i] << 32 | (unsigned)i);
    __syncthreads();
    const int ca = s_cnt[0], cb = s_cnt[1];
    if (ca == 0 || cb == 0) {  // IndexedMatch returns 0 when either mask count is 0 (:209)
        if (tid == 0) p.n_out[pr] = 0;
        return;
    }
    int PA = 1, PB = 1;
    while (PA < ca) PA <<= 1;
    while (PB < cb) PB <<= 1;
    for (int i = ca + tid; i < max(PA, SORT_THREADS); i += SORT_THREADS) keysA[i] = 0ull;
    for (int i = cb + tid; i < max(PB, SORT_THREADS); i += SORT_THREADS) keysB[i] = 0ull;
    __syncthreads();
    sort_desc(keysA, PA);
    sort_desc(keysB, PB);
    for (int i = tid; i < ca; i += SORT_THREADS) keysA[i] = ~keysA[i];
    for (int i = tid; i < cb; i += SORT_THREADS) keysB[i] = ~keysB[i];
    __syncthreads();
    // B's descriptors in key order into LDS (each is read by ~all A features of its leaf)
    const bool staged = cb <= IM_STAGE;
    if (staged) {
        for (int i = tid; i < 2 * cb; i += SORT_THREADS) {
            const unsigned idx = (unsigned)(keysB[i >> 1] & 0xFFFFFFFFull);
            sdescB[i] = reinterpret_cast<const uint4*>(db + 32ull * idx)[i & 1];
        }
        __syncthreads();
    }

    // 2. forward TrackMatch over B's run of the leaf, then the reverse check over A's run
    const unsigned max_h = (unsigned)(p.max_dist + 1);
    const int group = tid / IM_GROUP, sub = tid % IM_GROUP;
    // A features are visited in (leaf, index) order: neighbouring groups scan the same B run and,
    // for the reverse check, the same A run (its descriptors stay in the CU's L1); masked-out
    // features are not in keysA and keep -1
    for (int i = tid; i < na; i += SORT_THREADS) res[i] = -1;
    __syncthreads();
    for (int pos = group; pos < ca; pos += IM_GROUPS) {
        const int i = (int)(keysA[pos] & 0xFFFFFFFFull);
        int r = -1;
        {
            const unsigned long long leaf = keysA[pos] >> 32;
            const uint4 qa = *reinterpret_cast<const uint4*>(da + 32ll * i);
            const uint4 qb = *reinterpret_cast<const uint4*>(da + 32ll * i + 16);
            const int lo = lower_bound_u64(keysB, cb, leaf << 32), hi = lower_bound_u64(keysB, cb, (leaf + 1) << 32);
            unsigned bk, sd;
            if (staged)
                track_run_lds(keysB, lo, hi, sub, sdescB, qa, qb, max_h, bk, sd);
            else
                track_run(keysB, lo, hi, sub, db, qa, qb, max_h, bk, sd);
            const unsigned bd = bk >> 12;
            if (bd < max_h && (sd >= max_h || (int)(sd - bd) >= p.min_diff)) {
                const int j = (int)(bk & 0xFFFu);
                const uint4 ra = *reinterpret_cast<const uint4*>(db + 32ll * j);
                const uint4 rb = *reinterpret_cast<const uint4*>(db + 32ll * j + 16);
                const unsigned long long lj = leaf;  // j is in B's run of this leaf
                const int lo2 = lower_bound_u64(keysA, ca, lj << 32), hi2 = lower_bound_u64(keysA, ca, (lj + 1) << 32);
                unsigned bk2, sd2;
                track_run(keysA, lo2, hi2, sub, da, ra, rb, max_h, bk2, sd2);
                const unsigned bd2 = bk2 >> 12;
                if (bd2 < max_h && (int)(bk2 & 0xFFFu) == i && (sd2 >= max_h || (int)(sd2 - bd2) >= p.min_diff))
                    r = j << 9 | (int)bd2;
            }
        }
        if (sub == 0) res[i] = r;
    }
    if (tid == 0) s_base = 0;
    __syncthreads();

    // 3. ordered compaction in A order
    for (int q0 = 0; q0 < na; q0 += SORT_THREADS) {
        const int q = q0 + tid;
        const int v = q < na ? res[q] : -1;
        const bool keep = v >= 0;
        const unsigned long long b = __ballot(keep);
        const int before = __popcll(b & ((1ull << lane) - 1ull));
        if (lane == 0) wsum[wave] = __popcll(b);
        __syncthreads();
        int off = s_base;
        for (int w = 0; w < wave; w++) off += wsum[w];
        if (keep) {
            const int pos = off + before;
            if (pos < (int)p.cap) {
                mage_dmatch m;
                m.query_idx = q;
                m.train_idx = v >> 9;
                m.img_idx = -1;  // cv::DMatch(int, int, float) (FeatureMatcher.cpp:274)
                m.distance = (float)(v & 0x1FF);
                p.out[(long long)pr * p.cap + pos] = m;
            }
        }
        __syncthreads();
        if (tid == 0) {
            int tot = 0;
            for (int w = 0; w < SORT_THREADS / kWave; w++) tot += wsum[w];
            s_base += tot;
        }
        __syncthreads();
    }
    if (tid == 0) p.n_out[pr] = (uint32_t)s_base;
}

mage_status leaves_launch(const mage_bow* b, const uint8_t* d_desc, uint32_t n, uint32_t* d_leaf, hipStream_t st)
{
    if (n == 0) return MAGE_OK;
    launch("bow.leaves", bow_leaves_kernel, dim3((n + 255) / 256), dim3(256), 0, st, b->nodes.as<const uint8_t>(),
           b->child_start.as<const uint32_t>(), b->children.as<const uint32_t>(), d_desc, n, d_leaf);
    MAGE_HIP(hipGetLastError());
    return MAGE_OK;
}

mage_status indexed_launch(const IndexedParams& p, uint32_t pairs, hipStream_t st)
{
    launch("match.indexed", indexed_match_kernel, dim3(pairs), dim3(SORT_THREADS), 0, st, p);
    MAGE_HIP(hipGetLastError());
    return MAGE_OK;
}


// ---------------------------------------------------------------------------------------------
// Vocabulary training (OnlineBow::CreateTree, OnlineBow.cpp:325-337): the Kmean of every node of
// one tree level runs concurrently.  The host keeps the control flow of Kmean (subsets, the
// InitializeTraining shuffle, node numbering); the GPU runs IterateClusteringKmean (:587-614):
//   km_assign_kernel  FindCluster of every entry (first smallest distance) + the KmeanCenter bit
//                     sums: per wave 256 ballots (one per bit) are kept in LDS, each lane then
//                     counts 4 bits for every cluster present in the wave (popc of ballot &
//                     cluster mask), LDS sums per block, one global atomic per nonzero counter;
//   km_update_kernel  per node: majority bits (count >= (members + 1) / 2, an empty cluster
//                     becomes all ones as in the reference), the changed test, iteration count and
//                     the loop's exit condition — after it, both kernels are no-ops for the node,
//                     so the host launches MaxTrainingIteration rounds without reading anything back.
// ---------------------------------------------------------------------------------------------
constexpr int KM_THREADS = 1024;
constexpr int KM_MAXB = 16;  // branching factors handled on the GPU

struct KmParams {
    const uint8_t* desc;        // training descriptors, 32 B each
    const uint32_t* entry_desc; // entry -> descriptor index (entries grouped by slot, ascending)
    const uint32_t* blk_slot;   // block -> slot
    const uint32_t* blk_start;  // block -> first entry
    const uint32_t* slot_end;   // slot -> end entry (exclusive)
    const uint32_t* ncent;      // slot -> number of clusters
    uint8_t* centers;           // slot x KM_MAXB x 32
    uint32_t* counts;           // slot x KM_MAXB x 256
    uint32_t* members;          // slot x KM_MAXB
    uint32_t* assign;           // entry -> cluster
    uint32_t* state;            // slot -> {iterations, done}
    uint32_t max_iter;
};

__global__ __launch_bounds__(KM_THREADS) void km_assign_kernel(KmParams p)
{
    __shared__ unsigned long long wbal[KM_THREADS / kWave][256];
    __shared__ uint32_t lcnt[KM_MAXB * 256];
    __shared__ uint32_t lmem[KM_MAXB];
    __shared__ uint4 cen[KM_MAXB * 2];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t s = p.blk_slot[blockIdx.x];
    if (p.state[2 * s + 1]) return;  // this node's loop has ended
    const int k = (int)p.ncent[s];
    const uint32_t e = p.blk_start[blockIdx.x] + tid;
    const bool valid = e < p.slot_end[s];
    for (int i = tid; i < k * 256; i += KM_THREADS) lcnt[i] = 0;
    if (tid < k) lmem[tid] = 0;
    if (tid < 2 * k) cen[tid] = reinterpret_cast<const uint4*>(p.centers + (size_t)s * KM_MAXB * 32)[tid];
    __syncthreads();
    uint32_t d[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    int g = -1;
    if (valid) {
        const uint4* dp = reinterpret_cast<const uint4*>(p.desc + 32ull * p.entry_desc[e]);
        const uint4 a = dp[0], b = dp[1];
        d[0] = a.x, d[1] = a.y, d[2] = a.z, d[3] = a.w, d[4] = b.x, d[5] = b.y, d[6] = b.z, d[7] = b.w;
        int best = INT_MAX;
        for (int c = 0; c < k; c++) {
            const uint4 ca = cen[2 * c], cb = cen[2 * c + 1];
            const int dist = __popc(d[0] ^ ca.x) + __popc(d[1] ^ ca.y) + __popc(d[2] ^ ca.z) + __popc(d[3] ^ ca.w) +
                             __popc(d[4] ^ cb.x) + __popc(d[5] ^ cb.y) + __popc(d[6] ^ cb.z) + __popc(d[7] ^ cb.w);
            if (dist < best) {  // FindCluster: min_element keeps the first smallest
                best = dist;
                g = c;
            }
        }
        p.assign[e] = (uint32_t)g;
    }
    // one ballot per bit (bit j*8+b of the descriptor = bit b of byte j: KmeanCenter's order)
#pragma unroll
    for (int w = 0; w < 8; w++)
        for (int b = 0; b < 32; b++) {
            const unsigned long long bal = __ballot((d[w] >> b) & 1u);
            if (lane == 0) wbal[wave][w * 32 + b] = bal;
        }
    __syncthreads();
    for (int c = 0; c < k; c++) {
        const unsigned long long m = __ballot(g == c);
        if (m == 0) continue;
        if (lane == 0) atomicAdd(&lmem[c], (uint32_t)__popcll(m));
#pragma unroll
        for (int r = 0; r < 4; r++) {
            const int bit = lane + 64 * r;
            const uint32_t cnt = (uint32_t)__popcll(m & wbal[wave][bit]);
            if (cnt) atomicAdd(&lcnt[c * 256 + bit], cnt);
        }
    }
    __syncthreads();
    uint32_t* gc = p.counts + (size_t)s * KM_MAXB * 256;
    for (int i = tid; i < k * 256; i += KM_THREADS)
        if (lcnt[i]) atomicAdd(&gc[i], lcnt[i]);
    if (tid < k && lmem[tid]) atomicAdd(&p.members[s * KM_MAXB + tid], lmem[tid]);
}

__global__ __launch_bounds__(256) void km_update_kernel(KmParams p)
{
    __shared__ uint32_t changed[KM_MAXB];
    const int s = blockIdx.x, t = threadIdx.x, lane = t & 63, wave = t >> 6;
    if (p.state[2 * s + 1]) return;
    const int k = (int)p.ncent[s];
    if (t < KM_MAXB) changed[t] = 0;
    __syncthreads();
    uint32_t* gc = p.counts + (size_t)s * KM_MAXB * 256;
    unsigned long long* cen = reinterpret_cast<unsigned long long*>(p.centers + (size_t)s * KM_MAXB * 32);
    for (int c = 0; c < k; c++) {
        const uint32_t half = (p.members[s * KM_MAXB + c] + 1) / 2;
        const unsigned long long nb = __ballot(gc[c * 256 + t] >= half);  // bits 64*wave .. +63
        if (lane == 0) {
            if (nb != cen[4 * c + wave]) changed[c] = 1;
            cen[4 * c + wave] = nb;
        }
        gc[c * 256 + t] = 0;
    }
    __syncthreads();
    if (t == 0) {
        uint32_t ch = 0;
        for (int c = 0; c < k; c++) {
            ch += changed[c];
            p.members[s * KM_MAXB + c] = 0;
        }
        const uint32_t it = p.state[2 * s] + 1;
        p.state[2 * s] = it;
        // do { ... } while (iterationCounter < MaxTrainingIteration && changedKmeanCounter > 0)
        if (!(it < p.max_iter && ch > 0)) p.state[2 * s + 1] = 1;
    }
}


// Kmedoid's update (IterateClusteringKmedoid, OnlineBow.cpp:608-637): the member of a group with
// the first smallest sum of Hamming distances to all members becomes the medoid.  The reference's
// O(g^2) scan is linear here: with c_b the number of members with bit b set (km_assign_kernel's
// KmeanCenter counts) and m the group size, member i's sum is sum_b (bit_ib ? m - c_b : c_b) =
// sum_b c_b + sum over its set bits of (m - 2 c_b), exact in integers.  Entries of a slot are in
// group order, so the smallest (sum, entry) key is the reference's first minimum.  An empty group
// (the reference reads groups[g][0] of an empty vector) keeps its medoid.  Then the same
// bookkeeping as km_update_kernel: counts reset, changed test, iteration count and exit rule.
__global__ __launch_bounds__(256) void km_medoid_kernel(KmParams p)
{
    __shared__ int wtab[KM_MAXB][256];
    __shared__ int base[KM_MAXB];
    __shared__ unsigned long long best[KM_MAXB][4];
    __shared__ uint32_t changed;
    const int s = blockIdx.x, t = threadIdx.x, lane = t & 63, wave = t >> 6;
    if (p.state[2 * s + 1]) return;
    const int k = (int)p.ncent[s];
    uint32_t* gc = p.counts + (size_t)s * KM_MAXB * 256;
    for (int c = 0; c < k; c++) {
        const int m = (int)p.members[s * KM_MAXB + c], cb = (int)gc[c * 256 + t];
        wtab[c][t] = m - 2 * cb;
        // base[c] = sum_b c_b: one wave-reduced partial per wave
        int v = cb;
        for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
        if (lane == 0) best[c][wave] = (unsigned long long)(uint32_t)v;  // reuse as scratch
    }
    if (t == 0) changed = 0;
    __syncthreads();
    if (t < k) base[t] = (int)(best[t][0] + best[t][1] + best[t][2] + best[t][3]);
    __syncthreads();
    unsigned long long mine[KM_MAXB];
#pragma unroll
    for (int c = 0; c < KM_MAXB; c++) mine[c] = ~0ull;
    const uint32_t e0 = s ? p.slot_end[s - 1] : 0, e1 = p.slot_end[s];
    for (uint32_t e = e0 + t; e < e1; e += 256) {
        const int c = (int)p.assign[e];
        const uint32_t* d = reinterpret_cast<const uint32_t*>(p.desc + 32ull * p.entry_desc[e]);
        int cost = base[c];
        for (int w = 0; w < 8; w++) {
            uint32_t x = d[w];
            while (x) {
                cost += wtab[c][32 * w + __builtin_ctz(x)];
                x &= x - 1u;
            }
        }
        const unsigned long long key = ((unsigned long long)(uint32_t)cost << 32) | (e - e0);
#pragma unroll
        for (int g = 0; g < KM_MAXB; g++)
            if (g == c && key < mine[g]) mine[g] = key;
    }
    __syncthreads();  // best[] was scratch above
#pragma unroll
    for (int c = 0; c < KM_MAXB; c++) {
        if (c >= k) break;
        unsigned long long v = mine[c];
        for (int o = 32; o >= 1; o >>= 1) {
            const unsigned long long u = __shfl_xor(v, o);
            v = u < v ? u : v;
        }
        if (lane == 0) best[c][wave] = v;
    }
    __syncthreads();
    unsigned long long* cen = reinterpret_cast<unsigned long long*>(p.centers + (size_t)s * KM_MAXB * 32);
    if (t < k) {
        unsigned long long v = best[t][0];
        for (int w = 1; w < 4; w++) v = best[t][w] < v ? best[t][w] : v;
        if (p.members[s * KM_MAXB + t] > 0 && v != ~0ull) {
            const uint32_t e = e0 + (uint32_t)(v & 0xFFFFFFFFull);
            const unsigned long long* d = reinterpret_cast<const unsigned long long*>(p.desc + 32ull * p.entry_desc[e]);
            bool diff = false;
            for (int q = 0; q < 4; q++) diff |= d[q] != cen[4 * t + q];
            if (diff) {
                for (int q = 0; q < 4; q++) cen[4 * t + q] = d[q];
                atomicAdd(&changed, 1u);
            }
        }
    }
    __syncthreads();
    for (int c = 0; c < k; c++) gc[c * 256 + t] = 0;
    if (t == 0) {
        for (int c = 0; c < k; c++) p.members[s * KM_MAXB + c] = 0;
        const uint32_t it = p.state[2 * s] + 1;
        p.state[2 * s] = it;
        if (!(it < p.max_iter && changed > 0)) p.state[2 * s + 1] = 1;
    }
}

// std::shuffle(refs, mt19937{}) as the reference's MSVC STL computes it (InitializeTraining,
// OnlineBow.cpp:404): a fresh default-seeded engine per call, target t swapped with a draw in
// [0, t] from _Rng_from_urng (one 32-bit output per draw for sizes < 2^32, rejection of the biased
// tail).  Host-side: the positions of the first `branching` refs of an n-element subset.
struct Mt19937 {
    uint32_t mt[624];
    int idx = 624;
    explicit Mt19937(uint32_t seed) {
        mt[0] = seed;
        for (int i = 1; i < 624; i++) mt[i] = 1812433253u * (mt[i - 1] ^ (mt[i - 1] >> 30)) + (uint32_t)i;
    }
    uint32_t operator()() {
        if (idx >= 624) {
            for (int i = 0; i < 624; i++) {
                const uint32_t y = (mt[i] & 0x80000000u) | (mt[(i + 1) % 624] & 0x7FFFFFFFu);
                mt[i] = mt[(i + 397) % 624] ^ (y >> 1) ^ ((y & 1u) ? 0x9908B0DFu : 0u);
            }
            idx = 0;
        }
        uint32_t y = mt[idx++];
        y ^= y >> 11;
        y ^= (y << 7) & 0x9D2C5680u;
        y ^= (y << 15) & 0xEFC60000u;
        return y ^ (y >> 18);
    }
};

std::vector<uint32_t> shuffled_head(uint32_t n, uint32_t k)
{
    std::vector<uint32_t> perm(n);
    for (uint32_t i = 0; i < n; i++) perm[i] = i;
    Mt19937 rng(5489u);
    for (uint32_t t = 1; t < n; t++) {
        const uint64_t index = (uint64_t)t + 1, mask = 0xFFFFFFFFull;
        uint64_t r;
        do r = rng();
        while (!(r / index < mask / index || mask % index == index - 1));
        const uint32_t off = (uint32_t)(r % index);
        if (off != t) std::swap(perm[t], perm[off]);
    }
    perm.resize(k < n ? k : n);
    return perm;
}

}  // namespace
}  // namespace mage

extern "C" {

mage_status mage_bow_create(const uint8_t* node_desc, const uint32_t* child_start, const uint32_t* children,
                            uint32_t n_nodes, int device, mage_bow** out)
{
    using namespace mage;
    MAGE_REQUIRE(out, MAGE_EINVAL, "null output");
    *out = nullptr;
    MAGE_REQUIRE(n_nodes >= 1 && node_desc && child_start, MAGE_EINVAL, "empty tree");
    MAGE_REQUIRE(child_start[0] == 0, MAGE_EINVAL, "child_start[0] must be 0");
    const uint32_t nc = child_start[n_nodes];
    MAGE_REQUIRE(nc == 0 || children, MAGE_EINVAL, "null children");
    for (uint32_t i = 0; i < n_nodes; i++) {
        MAGE_REQUIRE(child_start[i + 1] >= child_start[i], MAGE_EINVAL, "child_start must be non-decreasing");
        for (uint32_t k = child_start[i]; k < child_start[i + 1]; k++)
            // OnlineBow::Kmean appends children after their parent: ids grow downwards, which
            // also guarantees that every descent terminates
            MAGE_REQUIRE(children[k] > i && children[k] < n_nodes, MAGE_EINVAL,
                         "child ids must exceed their parent's and be < n_nodes");
    }
    mage_status r = bind_device(device);
    if (r != MAGE_OK) return r;
    auto* b = new mage_bow();
    b->device = device;
    b->n_nodes = n_nodes;
    auto fail = [&](mage_status s) {
        b->nodes.release();
        b->child_start.release();
        b->children.release();
        if (b->st) (void)hipStreamDestroy(b->st);
        delete b;
        return s;
    };
    if ((r = b->nodes.reserve(32ull * n_nodes)) != MAGE_OK) return fail(r);
    if ((r = b->child_start.reserve(4ull * (n_nodes + 1))) != MAGE_OK) return fail(r);
    if ((r = b->children.reserve(4ull * (nc + 1))) != MAGE_OK) return fail(r);
    if (hipStreamCreateWithFlags(&b->st, hipStreamNonBlocking) != hipSuccess ||
        hipMemcpy(b->nodes.ptr, node_desc, 32ull * n_nodes, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(b->child_start.ptr, child_start, 4ull * (n_nodes + 1), hipMemcpyHostToDevice) != hipSuccess ||
        (nc > 0 && hipMemcpy(b->children.ptr, children, 4ull * nc, hipMemcpyHostToDevice) != hipSuccess)) {
        set_error("tree upload failed");
        return fail(MAGE_EDEVICE);
    }
    *out = b;
    return MAGE_OK;
}

mage_status mage_bow_destroy(mage_bow* b)
{
    if (!b) return MAGE_OK;
    (void)hipSetDevice(b->device);
    b->nodes.release();
    b->child_start.release();
    b->children.release();
    b->scratch.release();
    if (b->st) (void)hipStreamDestroy(b->st);
    delete b;
    return MAGE_OK;
}

mage_status mage_bow_find_leaves_device(mage_bow* b, const uint8_t* d_desc, uint32_t n, uint32_t* d_leaf,
                                        mage_stream stream)
{
    using namespace mage;
    MAGE_REQUIRE(b && (n == 0 || (d_desc && d_leaf)), MAGE_EINVAL, "null argument");
    return leaves_launch(b, d_desc, n, d_leaf, (hipStream_t)stream);
}

mage_status mage_bow_find_leaves(mage_bow* b, const uint8_t* desc, uint32_t n, uint32_t* leaf)
{
    using namespace mage;
    MAGE_REQUIRE(b && (n == 0 || (desc && leaf)), MAGE_EINVAL, "null argument");
    if (n == 0) return MAGE_OK;
    MAGE_HIP(hipSetDevice(b->device));
    mage_status r = b->scratch.reserve(36ull * n);
    if (r != MAGE_OK) return r;
    uint8_t* d = b->scratch.as<uint8_t>();
    uint32_t* dl = reinterpret_cast<uint32_t*>(d + 32ull * n);
    MAGE_HIP(hipMemcpyAsync(d, desc, 32ull * n, hipMemcpyHostToDevice, b->st));
    if ((r = leaves_launch(b, d, n, dl, b->st)) != MAGE_OK) return r;
    MAGE_HIP(hipMemcpyAsync(leaf, dl, 4ull * n, hipMemcpyDeviceToHost, b->st));
    MAGE_HIP(hipStreamSynchronize(b->st));
    return MAGE_OK;
}

mage_status mage_indexed_match(mage_bow* b, const uint8_t* desc_a, uint32_t n_a, const uint8_t* mask_a,
                               const uint8_t* desc_b, uint32_t n_b, const uint8_t* mask_b, int32_t max_distance,
                               int32_t min_difference, mage_dmatch* out, uint32_t cap, uint32_t* n)
{
    using namespace mage;
    MAGE_REQUIRE(b && n && (cap == 0 || out), MAGE_EINVAL, "null argument");
    *n = 0;
    MAGE_REQUIRE((n_a == 0 || desc_a) && (n_b == 0 || desc_b), MAGE_EINVAL, "null input");
    MAGE_REQUIRE(n_a <= (uint32_t)IM_MAX && n_b <= (uint32_t)IM_MAX, MAGE_EUNSUPPORTED, "more than 4096 features");
    MAGE_REQUIRE(max_distance >= -1 && max_distance <= 256, MAGE_EINVAL, "maxHammingDist must be in [-1, 256]");
    if (n_a == 0 || n_b == 0) return MAGE_OK;
    MAGE_HIP(hipSetDevice(b->device));
    // device layout: [da][db][la][lb][ma][mb][out][counts]
    auto al = [](size_t v) { return (v + 255) & ~(size_t)255; };
    const size_t oda = 0, odb = al(32ull * n_a), ola = al(odb + 32ull * n_b), olb = al(ola + 4ull * n_a),
                 oma = al(olb + 4ull * n_b), omb = al(oma + n_a), oout = al(omb + n_b), ocnt = al(oout + 16ull * n_a),
                 total = ocnt + 32;
    mage_status r = b->scratch.reserve(total);
    if (r != MAGE_OK) return r;
    char* d = b->scratch.as<char>();
    MAGE_HIP(hipMemcpyAsync(d + oda, desc_a, 32ull * n_a, hipMemcpyHostToDevice, b->st));
    MAGE_HIP(hipMemcpyAsync(d + odb, desc_b, 32ull * n_b, hipMemcpyHostToDevice, b->st));
    if (mask_a) MAGE_HIP(hipMemcpyAsync(d + oma, mask_a, n_a, hipMemcpyHostToDevice, b->st));
    if (mask_b) MAGE_HIP(hipMemcpyAsync(d + omb, mask_b, n_b, hipMemcpyHostToDevice, b->st));
    const uint32_t counts[4] = {n_a, n_b, 0, 0};
    MAGE_HIP(hipMemcpyAsync(d + ocnt, counts, 16, hipMemcpyHostToDevice, b->st));
    // CreateFeatureMatcher / AddImage: every feature of both images to its leaf
    if ((r = leaves_launch(b, reinterpret_cast<const uint8_t*>(d + oda), n_a, reinterpret_cast<uint32_t*>(d + ola),
                           b->st)) != MAGE_OK)
        return r;
    if ((r = leaves_launch(b, reinterpret_cast<const uint8_t*>(d + odb), n_b, reinterpret_cast<uint32_t*>(d + olb),
                           b->st)) != MAGE_OK)
        return r;
    IndexedParams p{};
    p.da = reinterpret_cast<const uint8_t*>(d + oda);
    p.la = reinterpret_cast<const uint32_t*>(d + ola);
    p.ma = mask_a ? reinterpret_cast<const uint8_t*>(d + oma) : nullptr;
    p.na = reinterpret_cast<const uint32_t*>(d + ocnt);
    p.a_pitch = n_a;
    p.db = reinterpret_cast<const uint8_t*>(d + odb);
    p.lb = reinterpret_cast<const uint32_t*>(d + olb);
    p.mb = mask_b ? reinterpret_cast<const uint8_t*>(d + omb) : nullptr;
    p.nb = reinterpret_cast<const uint32_t*>(d + ocnt) + 1;
    p.b_pitch = n_b;
    p.max_dist = max_distance;
    p.min_diff = min_difference;
    p.cap = n_a;
    p.out = reinterpret_cast<mage_dmatch*>(d + oout);
    p.n_out = reinterpret_cast<uint32_t*>(d + ocnt) + 2;
    p.status = reinterpret_cast<uint32_t*>(d + ocnt) + 3;
    if ((r = indexed_launch(p, 1, b->st)) != MAGE_OK) return r;
    uint32_t got = 0;
    MAGE_HIP(hipMemcpyAsync(&got, d + ocnt + 8, 4, hipMemcpyDeviceToHost, b->st));
    MAGE_HIP(hipStreamSynchronize(b->st));
    if (got > 0 && cap > 0) MAGE_HIP(hipMemcpy(out, d + oout, 16ull * (got < cap ? got : cap), hipMemcpyDeviceToHost));
    *n = got < cap ? got : cap;
    MAGE_REQUIRE(got <= cap, MAGE_ECAPACITY, "output capacity too small");
    return MAGE_OK;
}

mage_status mage_indexed_match_batch_device(const uint8_t* d_desc_a, const uint32_t* d_leaf_a, const uint8_t* d_mask_a,
                                            int64_t a_pitch, const uint32_t* d_n_a, const uint8_t* d_desc_b,
                                            const uint32_t* d_leaf_b, const uint8_t* d_mask_b, int64_t b_pitch,
                                            const uint32_t* d_n_b, uint32_t pairs, int32_t max_distance,
                                            int32_t min_difference, mage_dmatch* d_out, uint32_t cap, uint32_t* d_n,
                                            uint32_t* d_status, mage_stream stream)
{
    using namespace mage;
    if (pairs == 0) return MAGE_OK;
    MAGE_REQUIRE(d_desc_a && d_leaf_a && d_n_a && d_desc_b && d_leaf_b && d_n_b && d_out && d_n && d_status,
                 MAGE_EINVAL, "null buffer");
    MAGE_REQUIRE(a_pitch > 0 && b_pitch > 0, MAGE_EINVAL, "pitches must be positive");
    MAGE_REQUIRE(max_distance >= -1 && max_distance <= 256, MAGE_EINVAL, "maxHammingDist must be in [-1, 256]");
    IndexedParams p{};
    p.da = d_desc_a;
    p.la = d_leaf_a;
    p.ma = d_mask_a;
    p.na = d_n_a;
    p.a_pitch = a_pitch;
    p.db = d_desc_b;
    p.lb = d_leaf_b;
    p.mb = d_mask_b;
    p.nb = d_n_b;
    p.b_pitch = b_pitch;
    p.max_dist = max_distance;
    p.min_diff = min_difference;
    p.cap = cap;
    p.out = d_out;
    p.n_out = d_n;
    p.status = d_status;
    return indexed_launch(p, pairs, (hipStream_t)stream);
}

}  // extern "C"

namespace mage {
namespace {

// OnlineBow::CreateTree's recursion with Kmean (medoid = false) or Kmedoid (medoid = true)
mage_status bow_train(const uint8_t* desc, uint32_t n, uint32_t levels, uint32_t branching, uint32_t max_iter,
                      int device, bool medoid, mage_bow** out)
{
    MAGE_REQUIRE(out, MAGE_EINVAL, "null output");
    *out = nullptr;
    MAGE_REQUIRE(n == 0 || desc, MAGE_EINVAL, "null descriptors");
    MAGE_REQUIRE(levels >= 1, MAGE_EINVAL, "TrainingTreeLevels must be >= 1");
    MAGE_REQUIRE(branching >= 1 && branching <= (uint32_t)KM_MAXB, MAGE_EUNSUPPORTED,
                 "TrainingTreeBranchingFactor must be in [1, 16]");
    mage_status r = bind_device(device);
    if (r != MAGE_OK) return r;
    struct HNode {
        uint8_t d[32];
        std::vector<uint32_t> kids;
    };
    std::vector<HNode> nodes(1);
    std::memset(nodes[0].d, 0, 32);
    struct Slot {
        uint32_t node;
        std::vector<uint32_t> idx;  // descriptor indices, ascending (child_features keep the order)
    };
    std::vector<Slot> slots;
    if (n > 0) {
        Slot s0{0, std::vector<uint32_t>(n)};
        for (uint32_t i = 0; i < n; i++) s0.idx[i] = i;
        slots.push_back(std::move(s0));
    }
    hipStream_t st = nullptr;
    MAGE_HIP(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    DeviceBuffer d_desc, d_work;
    auto fail = [&](mage_status e) {
        (void)hipStreamDestroy(st);
        return e;
    };
    if (n > 0) {
        if ((r = d_desc.reserve(32ull * n)) != MAGE_OK) return fail(r);
        if (hipMemcpyAsync(d_desc.ptr, desc, 32ull * n, hipMemcpyHostToDevice, st) != hipSuccess)
            return fail(MAGE_EDEVICE);
    }
    for (uint32_t level = 1; !slots.empty(); level++) {
        const uint32_t S = (uint32_t)slots.size();
        std::vector<uint32_t> entry, blk_slot, blk_start, slot_end(S), ncent(S);
        std::vector<uint8_t> centers((size_t)S * KM_MAXB * 32, 0);
        for (uint32_t si = 0; si < S; si++) {
            const Slot& sl = slots[si];
            const uint32_t base = (uint32_t)entry.size(), cnt = (uint32_t)sl.idx.size();
            for (uint32_t b = 0; b < cnt; b += KM_THREADS) {
                blk_slot.push_back(si);
                blk_start.push_back(base + b);
            }
            entry.insert(entry.end(), sl.idx.begin(), sl.idx.end());
            slot_end[si] = (uint32_t)entry.size();
            // InitializeTraining: the first min(branching, n) refs after the shuffle
            const std::vector<uint32_t> head = shuffled_head(cnt, branching);
            ncent[si] = (uint32_t)head.size();
            for (size_t g = 0; g < head.size(); g++)
                std::memcpy(&centers[((size_t)si * KM_MAXB + g) * 32], desc + 32ull * sl.idx[head[g]], 32);
        }
        const uint32_t E = (uint32_t)entry.size(), B = (uint32_t)blk_slot.size();
        auto al = [](size_t v) { return (v + 255) & ~(size_t)255; };
        const size_t o_entry = 0, o_bs = al(4ull * E), o_bst = al(o_bs + 4ull * B), o_se = al(o_bst + 4ull * B),
                     o_nc = al(o_se + 4ull * S), o_cen = al(o_nc + 4ull * S), o_cnt = al(o_cen + centers.size()),
                     o_mem = al(o_cnt + 4ull * S * KM_MAXB * 256), o_st = al(o_mem + 4ull * S * KM_MAXB),
                     o_as = al(o_st + 8ull * S), total = o_as + 4ull * E;
        if ((r = d_work.reserve(total)) != MAGE_OK) return fail(r);
        char* w = d_work.as<char>();
        if (hipMemcpyAsync(w + o_entry, entry.data(), 4ull * E, hipMemcpyHostToDevice, st) != hipSuccess ||
            hipMemcpyAsync(w + o_bs, blk_slot.data(), 4ull * B, hipMemcpyHostToDevice, st) != hipSuccess ||
            hipMemcpyAsync(w + o_bst, blk_start.data(), 4ull * B, hipMemcpyHostToDevice, st) != hipSuccess ||
            hipMemcpyAsync(w + o_se, slot_end.data(), 4ull * S, hipMemcpyHostToDevice, st) != hipSuccess ||
            hipMemcpyAsync(w + o_nc, ncent.data(), 4ull * S, hipMemcpyHostToDevice, st) != hipSuccess ||
            hipMemcpyAsync(w + o_cen, centers.data(), centers.size(), hipMemcpyHostToDevice, st) != hipSuccess ||
            hipMemsetAsync(w + o_cnt, 0, o_as - o_cnt, st) != hipSuccess)
            return fail(MAGE_EDEVICE);
        KmParams p{d_desc.as<const uint8_t>(),
                   reinterpret_cast<const uint32_t*>(w + o_entry),
                   reinterpret_cast<const uint32_t*>(w + o_bs),
                   reinterpret_cast<const uint32_t*>(w + o_bst),
                   reinterpret_cast<const uint32_t*>(w + o_se),
                   reinterpret_cast<const uint32_t*>(w + o_nc),
                   reinterpret_cast<uint8_t*>(w + o_cen),
                   reinterpret_cast<uint32_t*>(w + o_cnt),
                   reinterpret_cast<uint32_t*>(w + o_mem),
                   reinterpret_cast<uint32_t*>(w + o_as),
                   reinterpret_cast<uint32_t*>(w + o_st),
                   max_iter};
        // the do-while body runs at least once
        for (uint32_t it = 0; it < std::max(max_iter, 1u); it++) {
            launch("bow.km_assign", km_assign_kernel, dim3(B), dim3(KM_THREADS), 0, st, p);
            if (hipGetLastError() != hipSuccess) return fail(MAGE_EDEVICE);
            if (medoid)
                launch("bow.km_medoid", km_medoid_kernel, dim3(S), dim3(256), 0, st, p);
            else
                launch("bow.km_update", km_update_kernel, dim3(S), dim3(256), 0, st, p);
            if (hipGetLastError() != hipSuccess) return fail(MAGE_EDEVICE);
        }
        std::vector<uint32_t> assign(E);
        if (hipMemcpyAsync(assign.data(), w + o_as, 4ull * E, hipMemcpyDeviceToHost, st) != hipSuccess ||
            hipMemcpyAsync(centers.data(), w + o_cen, centers.size(), hipMemcpyDeviceToHost, st) != hipSuccess ||
            hipStreamSynchronize(st) != hipSuccess)
            return fail(MAGE_EDEVICE);
        // Kmean: the centers become children of the node (in cluster order); groups recurse
        std::vector<Slot> next;
        for (uint32_t si = 0; si < S; si++) {
            const uint32_t k = ncent[si], base = si ? slot_end[si - 1] : 0;
            std::vector<std::vector<uint32_t>> groups(k);
            for (uint32_t e = base; e < slot_end[si]; e++) groups[assign[e]].push_back(entry[e]);
            for (uint32_t g = 0; g < k; g++) {
                HNode c;
                std::memcpy(c.d, &centers[((size_t)si * KM_MAXB + g) * 32], 32);
                nodes.push_back(c);
                const uint32_t id = (uint32_t)nodes.size() - 1;
                nodes[slots[si].node].kids.push_back(id);
                if (level < levels && groups[g].size() > 1) next.push_back(Slot{id, std::move(groups[g])});
            }
        }
        slots = std::move(next);
    }
    (void)hipStreamDestroy(st);
    // ids as the recursive Kmean hands them out: a node's children consecutively, then each
    // child's subtree in order (depth first)
    std::vector<uint32_t> nid(nodes.size(), 0);
    uint32_t next_id = 1;
    std::function<void(uint32_t)> number = [&](uint32_t v) {
        for (uint32_t c : nodes[v].kids) nid[c] = next_id++;
        for (uint32_t c : nodes[v].kids)
            if (!nodes[c].kids.empty()) number(c);
    };
    number(0);
    const uint32_t N = (uint32_t)nodes.size();
    std::vector<uint8_t> nd(32ull * N);
    std::vector<std::vector<uint32_t>> kids(N);
    for (uint32_t v = 0; v < N; v++) {
        std::memcpy(&nd[32ull * nid[v]], nodes[v].d, 32);
        for (uint32_t c : nodes[v].kids) kids[nid[v]].push_back(nid[c]);
    }
    std::vector<uint32_t> cs(N + 1, 0), ch;
    for (uint32_t v = 0; v < N; v++) {
        cs[v] = (uint32_t)ch.size();
        ch.insert(ch.end(), kids[v].begin(), kids[v].end());
    }
    cs[N] = (uint32_t)ch.size();
    return mage_bow_create(nd.data(), cs.data(), ch.empty() ? nullptr : ch.data(), N, device, out);
}

}  // namespace
}  // namespace mage

extern "C" {

mage_status mage_bow_train(const uint8_t* desc, uint32_t n, uint32_t levels, uint32_t branching, uint32_t max_iter,
                           int device, mage_bow** out)
{
    return mage::bow_train(desc, n, levels, branching, max_iter, device, false, out);
}

mage_status mage_bow_train_kmedoid(const uint8_t* desc, uint32_t n, uint32_t levels, uint32_t branching,
                                   uint32_t max_iter, int device, mage_bow** out)
{
    return mage::bow_train(desc, n, levels, branching, max_iter, device, true, out);
}

mage_status mage_bow_get_tree(mage_bow* b, uint8_t* node_desc, uint32_t* child_start, uint32_t* children,
                              uint32_t cap_nodes, uint32_t* n_nodes)
{
    using namespace mage;
    MAGE_REQUIRE(b && n_nodes, MAGE_EINVAL, "null argument");
    *n_nodes = b->n_nodes;
    if (cap_nodes < b->n_nodes) return MAGE_ECAPACITY;
    MAGE_REQUIRE(node_desc && child_start && children, MAGE_EINVAL, "null output");
    MAGE_HIP(hipSetDevice(b->device));
    MAGE_HIP(hipMemcpy(node_desc, b->nodes.ptr, 32ull * b->n_nodes, hipMemcpyDeviceToHost));
    MAGE_HIP(hipMemcpy(child_start, b->child_start.ptr, 4ull * (b->n_nodes + 1), hipMemcpyDeviceToHost));
    const uint32_t nc = child_start[b->n_nodes];
    if (nc) MAGE_HIP(hipMemcpy(children, b->children.ptr, 4ull * nc, hipMemcpyDeviceToHost));
    return MAGE_OK;
}

}  // extern "C"
