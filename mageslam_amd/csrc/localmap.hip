// localmap.hip — TrackLocalMap's per-map-point matching on MI355X (gfx950).
//
// TrackLocalMap::RunTrackLocalMap (Core/MAGESLAM/Source/Tracking/TrackLocalMap.cpp:175-256) walks the
// connected keyframes' map points in order and, for every point that projects well, runs the
// single-query RadiusMatch (FeatureMatcher.cpp:386-446) against the frame's still-unassociated
// keypoints; a success associates the keypoint (unassociatedMask[t] = false, :252), so every later
// point sees it taken.  The work is a sequential scan in the reference; here it is exact and
// parallel in three launches:
//   lm_keys_kernel     the frame's band index (band_index.hpp) sorted once;
//   lm_cand_kernel     a 16-lane group per point: every box candidate (same octave, f32 box) that
//                      is unassociated at the start, is not the point's hidden keypoint and lies
//                      within maxHammingDist — only those can ever change the point's result
//                      (the best starts at maxDist + 1 and only strictly smaller distances count);
//   lm_resolve_kernel  the points in order: 1024 threads compact the points with candidates into
//                      LDS, one wave resolves them 64 at a time against the LDS mask — each lane's
//                      result under the current mask, the keypoints the lanes would take marked
//                      with the lowest taking lane (LDS atomicMin), and the lanes before the first
//                      one that sees an earlier lane's keypoint among its candidates are final;
//                      they commit and the chunk restarts at that lane.  Exactly the sequential
//                      outcome: a lane's result depends on earlier lanes only through keypoints
//                      they take from its candidate set.
// The reference's "second best = the previous best" rule (:425-437) is taken in ascending keypoint
// order (the R*-tree's visiting order is unspecified), where it is order-free:
// best = min (distance, index), second = min(maxDist + 1, min distance over lower indices).
// Hiding a pose-estimation outlier's old keypoint from its own point (:192-229) is equivalent to
// never offering that keypoint to the point: hidden or already taken, it is unavailable either way.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cstring>

#include "band_index.hpp"
#include "common.hpp"
#include "lds_sort.hpp"

namespace mage {
namespace {

constexpr int LM_MAXT = 4096;   // frame keypoints (mask bits in LDS)
constexpr int LM_CAP = 8;       // candidates kept per point (more: the point rescans its band)
constexpr int LM_GROUP = 16;    // lanes per point in lm_cand_kernel

struct LmRec {
    int n;       // candidates (> LM_CAP: overflow, the entries are not all kept)
    int lo, hi;  // the point's band run in the sorted keys
    int pad;
    uint32_t e[LM_CAP];  // target << 9 | distance
};

__device__ __forceinline__ uint32_t hamming32(const uint8_t* a, const uint8_t* b)
{
    const uint4 a0 = *reinterpret_cast<const uint4*>(a), a1 = *reinterpret_cast<const uint4*>(a + 16);
    const uint4 b0 = *reinterpret_cast<const uint4*>(b), b1 = *reinterpret_cast<const uint4*>(b + 16);
    return __popc(a0.x ^ b0.x) + __popc(a0.y ^ b0.y) + __popc(a0.z ^ b0.z) + __popc(a0.w ^ b0.w) +
           __popc(a1.x ^ b1.x) + __popc(a1.y ^ b1.y) + __popc(a1.z ^ b1.z) + __popc(a1.w ^ b1.w);
}

__global__ __launch_bounds__(SORT_THREADS) void lm_keys_kernel(LocalMapArgs a, unsigned long long* __restrict__ gkeys)
{
    __shared__ unsigned long long keys[LM_MAXT];
    const int n = (int)*a.nt, tid = threadIdx.x;
    if (*a.nq == 0) return;  // the tracker's frames without local-map queries
    if (n > LM_MAXT) {
        if (tid == 0) atomicOr(a.status, 1u);
        return;
    }
    int P = 1;
    while (P < n) P <<= 1;
    for (int i = tid; i < max(P, SORT_THREADS); i += SORT_THREADS)
        keys[i] = i < n ? ~band_key(a.tkp[i].octave, a.tkp[i].y, (unsigned)i) : 0ull;
    __syncthreads();
    sort_desc(keys, P);
    for (int i = tid; i < n; i += SORT_THREADS) gkeys[i] = ~keys[i];
}

// The candidates of point q under the starting mask: box, octave, availability, not hidden,
// distance <= maxDist.  `visit(t, d)` for each; returns nothing.
template <typename F>
__device__ __forceinline__ void scan_band(const LocalMapArgs& a, const unsigned long long* keys, int q, int lo, int hi,
                                          int first, int step, F visit)
{
    const float r = a.radius, px = a.qpos[2 * q], py = a.qpos[2 * q + 1];
    const float x0 = px - r, x1 = px + r, y0 = py - r, y1 = py + r;
    const int hide = a.qhide ? a.qhide[q] : -1;
    const uint8_t* qd = a.qdesc + 32ll * q;
    for (int i = lo + first; i < hi; i += step) {
        const int t = (int)(keys[i] & 0xFFFFFFu);
        const float tx = a.tkp[t].x, ty = a.tkp[t].y;
        if (!(tx >= x0 && tx <= x1 && ty >= y0 && ty <= y1) || t == hide) continue;
        const uint32_t d = hamming32(qd, a.tdesc + 32ll * t);
        if ((int)d <= a.max_dist) visit(t, (int)d);
    }
}

__global__ __launch_bounds__(1024) void lm_cand_kernel(LocalMapArgs a, const unsigned long long* __restrict__ keys,
                                                       LmRec* __restrict__ recs)
{
    const int nq = (int)*a.nq, nt = (int)*a.nt;
    if (nt > LM_MAXT || nq > (int)a.q_cap) return;
    const int q = (int)((blockIdx.x * 1024 + threadIdx.x) / LM_GROUP), sub = threadIdx.x % LM_GROUP;
    const int lane = threadIdx.x & 63, gbase = lane & ~(LM_GROUP - 1);
    const bool live = q < nq;
    int lo = 0, hi = 0;
    if (live) {
        const float py = a.qpos[2 * q + 1], r = a.radius;
        const int oq = a.qoct[q];
        lo = lower_bound_keys(keys, nt, band_key(oq, py - r, 0u));
        hi = lower_bound_keys(keys, nt, band_key(oq, py + r, 0xFFFFFFu) + 1ull);
    }
    // the group walks its run 16 entries at a time; found candidates are compacted with a ballot
    int n = 0;
    for (int i0 = lo; __any(live && i0 < hi); i0 += LM_GROUP) {
        bool f = false;
        uint32_t ent = 0;
        if (live && i0 + sub < hi) {
            const int i = i0 + sub;
            const int t = (int)(keys[i] & 0xFFFFFFu);
            const bool avail = (a.mask_words[t >> 5] >> (t & 31)) & 1u;
            if (avail)
                scan_band(a, keys, q, i, i + 1, 0, 1, [&](int tt, int d) {
                    f = true;
                    ent = (uint32_t)tt << 9 | (uint32_t)d;
                });
        }
        const uint64_t b = __ballot(f);
        const uint32_t gb = (uint32_t)(b >> gbase) & 0xFFFFu;
        const int pos = n + __popc(gb & ((1u << sub) - 1u));
        if (f && pos < LM_CAP) recs[q].e[pos] = ent;
        n += __popc(gb);
    }
    if (live && sub == 0) {
        recs[q].n = n;
        recs[q].lo = lo;
        recs[q].hi = hi;
    }
}

__device__ __forceinline__ bool bit(const uint32_t* w, int t) { return (w[t >> 5] >> (t & 31)) & 1u; }

__global__ __launch_bounds__(1024) void lm_resolve_kernel(LocalMapArgs a, const unsigned long long* __restrict__ keys,
                                                          const LmRec* __restrict__ recs)
{
    __shared__ uint32_t m[LM_MAXT / 32];
    __shared__ int taker[LM_MAXT];
    __shared__ int list[1024];
    __shared__ uint32_t ent[64][LM_CAP];
    __shared__ uint32_t wsum[16];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int nq = (int)*a.nq, nt = (int)*a.nt;
    if (nt > LM_MAXT || nq > (int)a.q_cap) {
        if (tid == 0) atomicOr(a.status, 2u);
        return;
    }
    for (int i = tid; i < LM_MAXT / 32; i += 1024) m[i] = i < (nt + 31) / 32 ? a.mask_words[i] : 0u;
    for (int i = tid; i < LM_MAXT; i += 1024) taker[i] = 64;
    __syncthreads();
    for (int b0 = 0; b0 < nq; b0 += 1024) {
        // ordered compaction of this block's points that have candidates
        const int q = b0 + tid;
        const bool has = q < nq && recs[q].n > 0;
        if (q < nq) a.result[q] = -1;
        const uint64_t bal = __ballot(has);
        if (lane == 0) wsum[wave] = (uint32_t)__popcll(bal);
        __syncthreads();
        int off = 0, cnt = 0;
        for (int w = 0; w < 16; w++) {
            off += w < wave ? (int)wsum[w] : 0;
            cnt += (int)wsum[w];
        }
        if (has) list[off + __popcll(bal & ((1ull << lane) - 1ull))] = q;
        __syncthreads();
        if (wave == 0) {
            int c0 = 0;
            while (c0 < cnt) {
                const int k = c0 + lane;
                const bool act = k < cnt;
                const int qq = act ? list[k] : 0;
                int n = 0, lo = 0, hi = 0;
                if (act) {
                    n = recs[qq].n;
                    lo = recs[qq].lo;
                    hi = recs[qq].hi;
                    for (int e = 0; e < LM_CAP && e < n; e++) ent[lane][e] = recs[qq].e[e];
                }
                const bool over = n > LM_CAP;
                // every available candidate of the lane (overflow: the band rescanned)
                auto each = [&](auto fn) {
                    if (!act) return;
                    if (!over) {
                        for (int e = 0; e < n; e++) {
                            const uint32_t v = ent[lane][e];
                            const int t = (int)(v >> 9);
                            if (bit(m, t)) fn(t, (int)(v & 0x1FFu));
                        }
                    } else {
                        scan_band(a, keys, qq, lo, hi, 0, 1, [&](int t, int d) {
                            if (bit(m, t)) fn(t, d);
                        });
                    }
                };
                uint32_t bestk = 0xFFFFFFFFu;
                each([&](int t, int d) { bestk = min(bestk, (uint32_t)d << 12 | (uint32_t)t); });
                const int tb = (int)(bestk & 0xFFFu), best = (int)(bestk >> 12);
                int sec = a.max_dist + 1;
                each([&](int t, int d) {
                    if (t < tb) sec = min(sec, d);
                });
                const bool ok = bestk != 0xFFFFFFFFu && sec - best > a.min_diff;
                if (ok) atomicMin(&taker[tb], lane);
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                bool conflict = false;
                each([&](int t, int) {
                    if (taker[t] < lane) conflict = true;
                });
                const uint64_t cb = __ballot(conflict);
                const int f = cb ? __builtin_ctzll(cb) : 64;
                if (ok && lane < f) {
                    atomicAnd(&m[tb >> 5], ~(1u << (tb & 31)));
                    a.result[qq] = tb;
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                if (ok) taker[tb] = 64;
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                c0 += f;
            }
        }
        __syncthreads();
    }
    for (int i = tid; i < (nt + 31) / 32; i += 1024) a.mask_words[i] = m[i];
}

}  // namespace

size_t local_map_scratch_bytes(uint32_t q_cap)
{
    return ((size_t)LM_MAXT * 8 + 255) / 256 * 256 + (size_t)std::max(q_cap, 1u) * sizeof(LmRec);
}

mage_status local_map_match_launch(const LocalMapArgs& a, void* scratch, hipStream_t st)
{
    unsigned long long* keys = static_cast<unsigned long long*>(scratch);
    LmRec* recs = reinterpret_cast<LmRec*>(static_cast<char*>(scratch) + ((size_t)LM_MAXT * 8 + 255) / 256 * 256);
    if (a.keys)  // the frame's band index is built already (the tracker's, shared with RadiusMatch)
        keys = const_cast<unsigned long long*>(a.keys);
    else
        launch("localmap.keys", lm_keys_kernel, dim3(1), dim3(SORT_THREADS), 0, st, a, keys);
    const unsigned groups = (unsigned)(((size_t)std::max(a.q_cap, 1u) * LM_GROUP + 1023) / 1024);
    launch("localmap.cand", lm_cand_kernel, dim3(groups), dim3(1024), 0, st, a, (const unsigned long long*)keys, recs);
    launch("localmap.resolve", lm_resolve_kernel, dim3(1), dim3(1024), 0, st, a, (const unsigned long long*)keys,
           (const LmRec*)recs);
    MAGE_HIP(hipGetLastError());
    return MAGE_OK;
}

}  // namespace mage

extern "C" mage_status mage_local_map_match(const float* query_pos, const int32_t* query_octave, const uint8_t* query_desc,
                                            const int32_t* query_hide, uint32_t n_query, const mage_keypoint* target_kp,
                                            const uint8_t* target_desc, uint32_t n_target, uint8_t* mask, float radius,
                                            int32_t max_distance, int32_t min_difference, int32_t* result, int device)
{
    using namespace mage;
    MAGE_REQUIRE(mask && (n_target == 0 || (target_kp && target_desc)) &&
                     (n_query == 0 || (query_pos && query_octave && query_desc && result)),
                 MAGE_EINVAL, "null argument");
    MAGE_REQUIRE(n_target <= (uint32_t)LM_MAXT, MAGE_EUNSUPPORTED, "more than 4096 target keypoints");
    MAGE_REQUIRE(max_distance >= -1 && max_distance <= 256, MAGE_EINVAL, "maxHammingDist must be in [-1, 256]");
    if (n_query == 0) return MAGE_OK;
    mage_status r = bind_device(device);
    if (r != MAGE_OK) return r;
    HostScratch* sp = host_scratch(device, SCRATCH_LOCALMAP);
    if (!sp) return MAGE_EDEVICE;
    HostScratch& S = *sp;
    // device layout [qpos][qoct][qhide][qdesc][tkp][tdesc][counts][mask words][result][status] + scratch;
    // inputs in one H2D copy, [mask words, status] back in one D2H copy
    auto al = [](size_t v) { return (v + 255) & ~(size_t)255; };
    const size_t oqp = 0, oqo = al(oqp + 8ull * n_query), oqh = al(oqo + 4ull * n_query), oqd = al(oqh + 4ull * n_query),
                 otk = al(oqd + 32ull * n_query), otd = al(otk + 28ull * std::max(n_target, 1u)),
                 ocnt = al(otd + 32ull * std::max(n_target, 1u)), omw = al(ocnt + 8), ores = al(omw + 4 * (LM_MAXT / 32)),
                 ost = al(ores + 4ull * n_query), oscr = al(ost + 4), total = oscr + local_map_scratch_bytes(n_query);
    if ((r = S.buf.reserve(total)) != MAGE_OK || (r = S.host.reserve(oscr)) != MAGE_OK) return r;
    char* b = S.buf.as<char>();
    char* h = S.host.as<char>();
    std::memcpy(h + oqp, query_pos, 8ull * n_query);
    std::memcpy(h + oqo, query_octave, 4ull * n_query);
    if (query_hide) std::memcpy(h + oqh, query_hide, 4ull * n_query);
    else std::memset(h + oqh, 0xFF, 4ull * n_query);
    std::memcpy(h + oqd, query_desc, 32ull * n_query);
    if (n_target) {
        std::memcpy(h + otk, target_kp, 28ull * n_target);
        std::memcpy(h + otd, target_desc, 32ull * n_target);
    }
    const uint32_t counts[2] = {n_query, n_target};
    std::memcpy(h + ocnt, counts, 8);
    uint32_t* mw = reinterpret_cast<uint32_t*>(h + omw);
    std::memset(mw, 0, 4 * (LM_MAXT / 32));
    for (uint32_t t = 0; t < n_target; t++)
        if (mask[t]) mw[t >> 5] |= 1u << (t & 31);
    std::memset(h + ost, 0, 4);
    MAGE_HIP(hipMemcpyAsync(b, h, oscr, hipMemcpyHostToDevice, S.st));
    LocalMapArgs a{};
    a.qpos = reinterpret_cast<const float*>(b + oqp);
    a.qoct = reinterpret_cast<const int*>(b + oqo);
    a.qhide = reinterpret_cast<const int*>(b + oqh);
    a.qdesc = reinterpret_cast<const uint8_t*>(b + oqd);
    a.nq = reinterpret_cast<const uint32_t*>(b + ocnt);
    a.q_cap = n_query;
    a.tkp = reinterpret_cast<const mage_keypoint*>(b + otk);
    a.tdesc = reinterpret_cast<const uint8_t*>(b + otd);
    a.nt = reinterpret_cast<const uint32_t*>(b + ocnt) + 1;
    a.mask_words = reinterpret_cast<uint32_t*>(b + omw);
    a.radius = radius;
    a.max_dist = max_distance;
    a.min_diff = min_difference;
    a.result = reinterpret_cast<int*>(b + ores);
    a.status = reinterpret_cast<uint32_t*>(b + ost);
    if ((r = local_map_match_launch(a, b + oscr, S.st)) != MAGE_OK) return r;
    MAGE_HIP(hipMemcpyAsync(h + omw, b + omw, oscr - omw, hipMemcpyDeviceToHost, S.st));
    MAGE_HIP(hipStreamSynchronize(S.st));
    MAGE_REQUIRE(*reinterpret_cast<const uint32_t*>(h + ost) == 0, MAGE_EDEVICE, "local map match: bad counts");
    std::memcpy(result, h + ores, 4ull * n_query);
    for (uint32_t t = 0; t < n_target; t++) mask[t] = (mw[t >> 5] >> (t & 31)) & 1u;
    return MAGE_OK;
}
