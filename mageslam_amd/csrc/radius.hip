// radius.hip — RadiusMatch on MI355X (gfx950): spatially gated Hamming matching of a query keypoint
// set against a target set (Core/MAGESLAM/Source/Tracking/FeatureMatcher.cpp:294-446) with the
// target KeypointSpatialIndex (Image/KeypointSpatialIndex.cpp:46-106) replaced by an LDS-sorted
// band index.
//
// One 1024-thread workgroup per (query set, target set) pair (or several, see radius_match_kernel):
//   1. targets -> 64-bit keys (octave, orderable f32 y, index), sorted ascending in LDS (the
//      shared hybrid bitonic sort); the R-tree box query |x - qx| <= r, |y - qy| <= r, same
//      octave becomes a binary search for the y band of the query's octave plus an exact f32
//      box test on each band entry;
//   2. a 16-lane group per query: lanes scan the band (positions and descriptors staged in LDS in
//      band order), mask, 32-byte Hamming distance.  The reference
//      visits candidates in R-tree order and keeps "second best" = the previous best at the last
//      improvement (:425-437).  With the deterministic ascending-index order
//      that is order-free: best = min d (lowest index on ties, only if d <= maxDist) and
//      second = min(maxDist + 1, min d over candidates with a lower index) — two group reductions;
//      accepted when second - best > minDiff (:441);
//   3. batch post-pass (:342-371): a match survives when its distance is the unique minimum among
//      the matches to its target (LDS atomicMin, then a count of the minima), ordered compaction in
//      query order.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cstring>

#include "common.hpp"
#include "band_index.hpp"
#include "lds_sort.hpp"

namespace mage {
namespace {

constexpr int RM_MAXT = 4096;   // targets per pair held in LDS (NumFeatures-sized sets)
constexpr int RM_STAGE = 2048;  // target sets up to this size also get positions + descriptors in LDS

struct RadiusParams {
    const mage_keypoint* qkp;
    const float* qpos;  // optional query positions (queryKeypointPositionOverrides), 2 floats each
    const uint8_t* qmask;
    const uint8_t* qdesc;
    const uint32_t* nq;
    long long q_pitch;  // query entries between pairs
    const mage_keypoint* tkp;
    const uint8_t* tmask;
    const uint8_t* tdesc;
    const uint32_t* nt;
    long long t_pitch;
    float radius;
    int max_dist, min_diff;
    unsigned cap;
    int* res;  // per query: target << 9 | distance, or -1 (pairs x q_pitch)
    mage_dmatch* out;
    uint32_t* n_out;
    uint32_t* status;  // bit 0: a target set exceeded RM_MAXT; bit 1: a count exceeded its pitch
    // optional band index built once per target set (radius_band_index_kernel, t_pitch entries per
    // pair): keys ascending, positions and descriptors in key order; no target mask with it
    const unsigned long long* bkeys;
    const float2* bxy;
    const uint4* bdesc;
    RadiusFollow follow;  // follow.exec == nullptr: none
};

// The match count of pair pr is final (thread 0): the optional fallback decision (RadiusFollow).
__device__ __forceinline__ void radius_done(const RadiusParams& p, int pr, uint32_t n)
{
    p.n_out[pr] = n;
    const RadiusFollow& g = p.follow;
    if (!g.exec) return;
    const uint32_t ns = *g.ns;
    const bool weak = n < g.min_matches || (double)n / (double)max(ns, 1u) < g.ratio;
    const uint32_t run = g.exec[g.k] && weak;
    g.exec[g.k + 1] = run;
    *g.nq_next = run ? ns : 0u;
}

constexpr int RM_GROUP = 16;  // lanes per query (a band holds ~20-150 candidates)
constexpr int RM_GROUPS = SORT_THREADS / RM_GROUP;

__device__ __forceinline__ unsigned group_min(unsigned v)
{
#pragma unroll
    for (int off = RM_GROUP / 2; off > 0; off >>= 1) v = min(v, (unsigned)__shfl_xor((int)v, off));
    return v;
}

// 3. batch post-pass of pair pr: unique minimum per target, then ordered compaction in query order
__device__ void radius_post(const RadiusParams& p, int pr, const int* res, int nq, int ntr, int* bestD, int* cnt,
                            int* wsum, int& s_base)
{
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    for (int i = tid; i < ntr; i += SORT_THREADS) {
        bestD[i] = INT_MAX;
        cnt[i] = 0;
    }
    __syncthreads();
    for (int q = tid; q < nq; q += SORT_THREADS) {
        const int v = res[q];
        if (v >= 0) atomicMin(&bestD[v >> 9], v & 0x1FF);
    }
    __syncthreads();
    for (int q = tid; q < nq; q += SORT_THREADS) {
        const int v = res[q];
        if (v >= 0 && (v & 0x1FF) == bestD[v >> 9]) atomicAdd(&cnt[v >> 9], 1);
    }
    if (tid == 0) s_base = 0;
    __syncthreads();
    for (int q0 = 0; q0 < nq; q0 += SORT_THREADS) {
        const int q = q0 + tid;
        const int v = q < nq ? res[q] : -1;
        const bool keep = v >= 0 && (v & 0x1FF) == bestD[v >> 9] && cnt[v >> 9] == 1;
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
                m.img_idx = 0;
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
    if (tid == 0) radius_done(p, pr, (uint32_t)s_base);
}

// blockIdx.y of gridDim.y workgroups handles every gridDim.y-th group slot of the pair's queries
// (gridDim.y > 1 spreads one pair over many CUs: the per-frame tracking call is a single pair);
// FUSED (gridDim.y == 1) runs the post-pass in the same workgroup, otherwise radius_post_kernel does
template <bool FUSED>
__global__ __launch_bounds__(SORT_THREADS) void radius_match_kernel(RadiusParams p)
{
    __shared__ unsigned long long keys[RM_MAXT];
    __shared__ float2 sxy[RM_STAGE];
    __shared__ uint4 sdesc[2 * RM_STAGE];
    __shared__ int wsum[SORT_THREADS / kWave];
    __shared__ int s_base;
    const int pr = blockIdx.x, tid = threadIdx.x;
    const int nq = (int)p.nq[pr], ntr = (int)p.nt[pr];
    const mage_keypoint* qkp = p.qkp + pr * p.q_pitch;
    const mage_keypoint* tkp = p.tkp + pr * p.t_pitch;
    const uint8_t* qdesc = p.qdesc + pr * p.q_pitch * 32;
    const uint8_t* tdesc = p.tdesc + pr * p.t_pitch * 32;
    const uint8_t* qmask = p.qmask ? p.qmask + pr * p.q_pitch : nullptr;
    const uint8_t* tmask = p.tmask ? p.tmask + pr * p.t_pitch : nullptr;
    const float* qpos = p.qpos ? p.qpos + 2 * pr * p.q_pitch : nullptr;
    int* res = p.res + pr * p.q_pitch;
    if (nq == 0) {  // no queries (the tracker's skipped fallback passes): no target sort either
        if (FUSED && tid == 0) radius_done(p, pr, 0);
        return;
    }
    // a count above its pair's pitch would read the next pair's (or unallocated) entries
    if (ntr > RM_MAXT || ntr > p.t_pitch || nq > p.q_pitch) {
        if (tid == 0 && blockIdx.y == 0) {
            radius_done(p, pr, 0);
            atomicOr(p.status, ntr > RM_MAXT ? 1u : 2u);
        }
        return;
    }
    const bool staged = ntr <= RM_STAGE;
    if (p.bkeys) {
        // 1'. the band index of this target set is built already: contiguous copies into LDS
        const long long tb = pr * p.t_pitch;
        for (int i = tid; i < ntr; i += SORT_THREADS) keys[i] = p.bkeys[tb + i];
        if (staged)
            for (int i = tid; i < 2 * ntr; i += SORT_THREADS) {
                sdesc[i] = p.bdesc[2 * tb + i];
                if (!(i & 1)) sxy[i >> 1] = p.bxy[tb + (i >> 1)];
            }
        __syncthreads();
    } else {
    // 1. band index: ascending keys via the descending sort of their complements (zero padding
    //    sorts last)
    int P = 1;
    while (P < ntr) P <<= 1;
    for (int i = tid; i < max(P, SORT_THREADS); i += SORT_THREADS)
        keys[i] = i < ntr ? ~band_key(tkp[i].octave, tkp[i].y, (unsigned)i) : 0ull;
    __syncthreads();
    sort_desc(keys, P);
    for (int i = tid; i < ntr; i += SORT_THREADS) keys[i] = ~keys[i];
    __syncthreads();
    // targets in key order into LDS: a band is then a contiguous run of positions + descriptors;
    // a masked target gets a NaN position, which fails the box test exactly like the mask check
    if (staged) {
        for (int i = tid; i < 2 * ntr; i += SORT_THREADS) {
            const int t = (int)(keys[i >> 1] & 0xFFFFFFu);
            sdesc[i] = reinterpret_cast<const uint4*>(tdesc + 32 * (long long)t)[i & 1];
            if (!(i & 1)) {
                const bool off = tmask && !tmask[t];
                sxy[i >> 1] = off ? make_float2(__int_as_float(0x7FC00000), 0.f) : make_float2(tkp[t].x, tkp[t].y);
            }
        }
        __syncthreads();
    }
    }

    // 2. a 16-lane group per query (four queries per wave)
    const float r = p.radius;
    const int group = tid / RM_GROUP, sub = tid % RM_GROUP;
    for (int q = (int)blockIdx.y * RM_GROUPS + group; q < nq; q += RM_GROUPS * (int)gridDim.y) {
        if (qmask && !qmask[q]) {
            if (sub == 0) res[q] = -1;
            continue;
        }
        const float px = qpos ? qpos[2 * q] : qkp[q].x, py = qpos ? qpos[2 * q + 1] : qkp[q].y;
        const int oq = qkp[q].octave;
        const float x0 = px - r, x1 = px + r, y0 = py - r, y1 = py + r;
        const int lo = lower_bound_keys(keys, ntr, band_key(oq, y0, 0u));
        const int hi = lower_bound_keys(keys, ntr, band_key(oq, y1, 0xFFFFFFu) + 1ull);
        uint4 qa = *reinterpret_cast<const uint4*>(qdesc + 32 * (long long)q);
        uint4 qb = *reinterpret_cast<const uint4*>(qdesc + 32 * (long long)q + 16);
        // pass 1: best = min (d << 12 | t) over the box candidates
        unsigned bestk = 0xFFFFFFFFu;
        for (int i = lo + sub; i < hi; i += RM_GROUP) {
            const int t = (int)(keys[i] & 0xFFFFFFu);
            uint4 ta, tb;
            if (staged) {
                const float2 xy = sxy[i];
                if (!(xy.x >= x0 && xy.x <= x1 && xy.y >= y0 && xy.y <= y1)) continue;
                ta = sdesc[2 * i];
                tb = sdesc[2 * i + 1];
            } else {
                const float tx = tkp[t].x, ty = tkp[t].y;
                if (!(tx >= x0 && tx <= x1 && ty >= y0 && ty <= y1)) continue;
                if (tmask && !tmask[t]) continue;
                ta = *reinterpret_cast<const uint4*>(tdesc + 32 * (long long)t);
                tb = *reinterpret_cast<const uint4*>(tdesc + 32 * (long long)t + 16);
            }
            const unsigned d = __popc(qa.x ^ ta.x) + __popc(qa.y ^ ta.y) + __popc(qa.z ^ ta.z) + __popc(qa.w ^ ta.w) +
                               __popc(qb.x ^ tb.x) + __popc(qb.y ^ tb.y) + __popc(qb.z ^ tb.z) + __popc(qb.w ^ tb.w);
            bestk = min(bestk, d << 12 | (unsigned)t);
        }
        bestk = group_min(bestk);
        const int best = bestk == 0xFFFFFFFFu ? INT_MAX : (int)(bestk >> 12), tbest = (int)(bestk & 0xFFFu);
        if (best > p.max_dist) {
            if (sub == 0) res[q] = -1;
            continue;
        }
        // pass 2: second = min(maxDist + 1, min d over candidates with a lower target index)
        unsigned sec = (unsigned)(p.max_dist + 1);
        for (int i = lo + sub; i < hi; i += RM_GROUP) {
            const int t = (int)(keys[i] & 0xFFFFFFu);
            if (t >= tbest) continue;
            uint4 ta, tb;
            if (staged) {
                const float2 xy = sxy[i];
                if (!(xy.x >= x0 && xy.x <= x1 && xy.y >= y0 && xy.y <= y1)) continue;
                ta = sdesc[2 * i];
                tb = sdesc[2 * i + 1];
            } else {
                const float tx = tkp[t].x, ty = tkp[t].y;
                if (!(tx >= x0 && tx <= x1 && ty >= y0 && ty <= y1)) continue;
                if (tmask && !tmask[t]) continue;
                ta = *reinterpret_cast<const uint4*>(tdesc + 32 * (long long)t);
                tb = *reinterpret_cast<const uint4*>(tdesc + 32 * (long long)t + 16);
            }
            const unsigned d = __popc(qa.x ^ ta.x) + __popc(qa.y ^ ta.y) + __popc(qa.z ^ ta.z) + __popc(qa.w ^ ta.w) +
                               __popc(qb.x ^ tb.x) + __popc(qb.y ^ tb.y) + __popc(qb.z ^ tb.z) + __popc(qb.w ^ tb.w);
            sec = min(sec, d);
        }
        sec = group_min(sec);
        if (sub == 0) res[q] = ((int)sec - best > p.min_diff) ? (tbest << 9 | best) : -1;
    }
    if constexpr (FUSED) {
        __syncthreads();
        // LDS of the band keys is reused for the post-pass arrays
        int* bestD = reinterpret_cast<int*>(keys);
        radius_post(p, pr, res, nq, ntr, bestD, bestD + RM_MAXT, wsum, s_base);
    }
}

__global__ __launch_bounds__(SORT_THREADS) void radius_post_kernel(RadiusParams p)
{
    __shared__ int bestD[RM_MAXT];
    __shared__ int cnt[RM_MAXT];
    __shared__ int wsum[SORT_THREADS / kWave];
    __shared__ int s_base;
    const int pr = blockIdx.x;
    const int nq = (int)p.nq[pr], ntr = (int)p.nt[pr];
    if (nq == 0) {
        if (threadIdx.x == 0) radius_done(p, pr, 0);
        return;
    }
    if (ntr > RM_MAXT || ntr > p.t_pitch || nq > p.q_pitch) return;
    radius_post(p, pr, p.res + pr * p.q_pitch, nq, ntr, bestD, cnt, wsum, s_base);
}

// The band index of each target set once (one workgroup per set): the keys sorted as
// radius_match_kernel sorts them, then positions and descriptors in key order, so every RadiusMatch
// against the set (the tracker's passes over one frame, each spread over ~64 workgroups) starts
// from contiguous copies instead of its own sort and gather.
__global__ __launch_bounds__(SORT_THREADS) void radius_band_index_kernel(const mage_keypoint* __restrict__ tkp,
                                                                         const uint8_t* __restrict__ tdesc,
                                                                         const uint32_t* __restrict__ nt, long long t_pitch,
                                                                         unsigned long long* __restrict__ bkeys,
                                                                         float2* __restrict__ bxy, uint4* __restrict__ bdesc)
{
    __shared__ unsigned long long keys[RM_MAXT];
    const int set = blockIdx.x, tid = threadIdx.x;
    const int ntr = (int)nt[set];
    if (ntr > RM_MAXT || ntr > t_pitch) return;  // radius_match_kernel reports it
    const long long tb = set * t_pitch;
    const mage_keypoint* k = tkp + tb;
    int P = 1;
    while (P < ntr) P <<= 1;
    for (int i = tid; i < max(P, SORT_THREADS); i += SORT_THREADS)
        keys[i] = i < ntr ? ~band_key(k[i].octave, k[i].y, (unsigned)i) : 0ull;
    __syncthreads();
    sort_desc(keys, P);
    for (int i = tid; i < ntr; i += SORT_THREADS) {
        const unsigned long long key = ~keys[i];
        const int t = (int)(key & 0xFFFFFFu);
        bkeys[tb + i] = key;
        bxy[tb + i] = make_float2(k[t].x, k[t].y);
        const uint4* d = reinterpret_cast<const uint4*>(tdesc + 32 * (tb + t));
        bdesc[2 * (tb + i)] = d[0];
        bdesc[2 * (tb + i) + 1] = d[1];
    }
}

}  // namespace

mage_status radius_band_index_launch(const mage_keypoint* d_target_kp, const uint8_t* d_target_desc,
                                     const uint32_t* d_n_target, int64_t target_pitch, uint32_t sets,
                                     unsigned long long* d_keys, float* d_xy, uint32_t* d_desc, hipStream_t st)
{
    if (sets == 0) return MAGE_OK;
    launch("match.radius_index", radius_band_index_kernel, dim3(sets), dim3(SORT_THREADS), 0, st, d_target_kp,
           d_target_desc, d_n_target, (long long)target_pitch, d_keys, reinterpret_cast<float2*>(d_xy),
           reinterpret_cast<uint4*>(d_desc));
    MAGE_HIP(hipGetLastError());
    return MAGE_OK;
}

mage_status radius_match_launch(const RadiusParams& p, uint32_t pairs, hipStream_t st)
{
    // a few pairs (the tracker's per-frame call) are spread over ~256 workgroups; batches of
    // >= 128 pairs already fill the chip with one fused workgroup per pair
    const uint32_t split = pairs >= 128 ? 1u : std::min(64u, (256u + pairs - 1) / pairs);
    if (split == 1) {
        launch("match.radius", radius_match_kernel<true>, dim3(pairs), dim3(SORT_THREADS), 0, st, p);
    } else {
        launch("match.radius", radius_match_kernel<false>, dim3(pairs, split), dim3(SORT_THREADS), 0, st, p);
        MAGE_HIP(hipGetLastError());
        launch("match.radius_post", radius_post_kernel, dim3(pairs), dim3(SORT_THREADS), 0, st, p);
    }
    MAGE_HIP(hipGetLastError());
    return MAGE_OK;
}

}  // namespace mage

extern "C" {

mage_status mage_radius_match(const mage_keypoint* query_kp, const float* query_pos, const uint8_t* query_mask,
                              const uint8_t* query_desc, uint32_t n_query, const mage_keypoint* target_kp,
                              const uint8_t* target_mask, const uint8_t* target_desc, uint32_t n_target,
                              float radius, int32_t max_distance, int32_t min_difference, mage_dmatch* out,
                              uint32_t cap, uint32_t* n)
{
    using namespace mage;
    MAGE_REQUIRE(n && (cap == 0 || out), MAGE_EINVAL, "null output");
    *n = 0;
    MAGE_REQUIRE((n_query == 0 || (query_kp && query_desc)) && (n_target == 0 || (target_kp && target_desc)),
                 MAGE_EINVAL, "null input");
    MAGE_REQUIRE(n_target <= (uint32_t)RM_MAXT, MAGE_EUNSUPPORTED, "more than 4096 target keypoints");
    MAGE_REQUIRE(max_distance >= -1 && max_distance <= 256, MAGE_EINVAL, "maxHammingDist must be in [-1, 256]");
    if (n_query == 0 || n_target == 0) return MAGE_OK;
    int dev = 0;
    MAGE_HIP(hipGetDevice(&dev));
    mage_status r = bind_device(dev);
    if (r != MAGE_OK) return r;
    HostScratch* sp = host_scratch(dev, SCRATCH_RADIUS);
    if (!sp) return MAGE_EDEVICE;
    HostScratch& S = *sp;
    // device layout: [qkp][tkp][qdesc][tdesc][qpos][qmask][tmask][counts] (inputs, one H2D copy)
    // [res][out]; the D2H copy takes [counts, end)
    auto al = [](size_t v) { return (v + 255) & ~(size_t)255; };
    const size_t oqk = 0, otk = al(oqk + 28ull * n_query), oqd = al(otk + 28ull * n_target),
                 otd = al(oqd + 32ull * n_query), oqp = al(otd + 32ull * n_target), oqm = al(oqp + 8ull * n_query),
                 otm = al(oqm + n_query), ocnt = al(otm + n_target), ores = al(ocnt + 16),
                 oout = al(ores + 4ull * n_query), total = oout + 16ull * n_query;
    if ((r = S.buf.reserve(total)) != MAGE_OK || (r = S.host.reserve(total)) != MAGE_OK) return r;
    char* b = S.buf.as<char>();
    char* h = S.host.as<char>();
    // inputs packed at their device offsets in pinned memory: one H2D copy of [0, ores)
    std::memcpy(h + oqk, query_kp, 28ull * n_query);
    std::memcpy(h + otk, target_kp, 28ull * n_target);
    std::memcpy(h + oqd, query_desc, 32ull * n_query);
    std::memcpy(h + otd, target_desc, 32ull * n_target);
    if (query_pos) std::memcpy(h + oqp, query_pos, 8ull * n_query);
    if (query_mask) std::memcpy(h + oqm, query_mask, n_query);
    if (target_mask) std::memcpy(h + otm, target_mask, n_target);
    const uint32_t counts[4] = {n_query, n_target, 0, 0};
    std::memcpy(h + ocnt, counts, 16);
    MAGE_HIP(hipMemcpyAsync(b, h, ores, hipMemcpyHostToDevice, S.st));
    RadiusParams p{};
    p.qkp = reinterpret_cast<const mage_keypoint*>(b + oqk);
    p.qpos = query_pos ? reinterpret_cast<const float*>(b + oqp) : nullptr;
    p.qmask = query_mask ? reinterpret_cast<const uint8_t*>(b + oqm) : nullptr;
    p.qdesc = reinterpret_cast<const uint8_t*>(b + oqd);
    p.nq = reinterpret_cast<const uint32_t*>(b + ocnt);
    p.q_pitch = n_query;
    p.tkp = reinterpret_cast<const mage_keypoint*>(b + otk);
    p.tmask = target_mask ? reinterpret_cast<const uint8_t*>(b + otm) : nullptr;
    p.tdesc = reinterpret_cast<const uint8_t*>(b + otd);
    p.nt = reinterpret_cast<const uint32_t*>(b + ocnt) + 1;
    p.t_pitch = n_target;
    p.radius = radius;
    p.max_dist = max_distance;
    p.min_diff = min_difference;
    p.cap = n_query;
    p.res = reinterpret_cast<int*>(b + ores);
    p.out = reinterpret_cast<mage_dmatch*>(b + oout);
    p.n_out = reinterpret_cast<uint32_t*>(b + ocnt) + 2;
    p.status = reinterpret_cast<uint32_t*>(b + ocnt) + 3;
    if ((r = radius_match_launch(p, 1, S.st)) != MAGE_OK) return r;
    // matches + counts come back in one copy
    MAGE_HIP(hipMemcpyAsync(h + ocnt, b + ocnt, total - ocnt, hipMemcpyDeviceToHost, S.st));
    MAGE_HIP(hipStreamSynchronize(S.st));
    const uint32_t m = reinterpret_cast<const uint32_t*>(h + ocnt)[2];
    if (m > 0 && cap > 0) std::memcpy(out, h + oout, 16ull * (m < cap ? m : cap));
    *n = m < cap ? m : cap;
    MAGE_REQUIRE(m <= cap, MAGE_ECAPACITY, "output capacity too small");
    return MAGE_OK;
}

mage_status mage_radius_match_batch_device(const mage_keypoint* d_query_kp, const float* d_query_pos,
                                           const uint8_t* d_query_desc, int64_t query_pitch,
                                           const uint32_t* d_n_query, const mage_keypoint* d_target_kp,
                                           const uint8_t* d_target_desc, int64_t target_pitch,
                                           const uint32_t* d_n_target, uint32_t pairs, float radius,
                                           int32_t max_distance, int32_t min_difference, int32_t* d_scratch,
                                           mage_dmatch* d_out, uint32_t cap, uint32_t* d_n, uint32_t* d_status,
                                           mage_stream stream)
{
    using namespace mage;
    if (pairs == 0) return MAGE_OK;
    MAGE_REQUIRE(d_query_kp && d_query_desc && d_n_query && d_target_kp && d_target_desc && d_n_target &&
                     d_scratch && d_out && d_n && d_status,
                 MAGE_EINVAL, "null buffer");
    MAGE_REQUIRE(query_pitch > 0 && target_pitch > 0, MAGE_EINVAL, "pitches must be positive");
    MAGE_REQUIRE(max_distance >= -1 && max_distance <= 256, MAGE_EINVAL, "maxHammingDist must be in [-1, 256]");
    RadiusParams p{};
    p.qkp = d_query_kp;
    p.qpos = d_query_pos;
    p.qdesc = d_query_desc;
    p.nq = d_n_query;
    p.q_pitch = query_pitch;
    p.tkp = d_target_kp;
    p.tdesc = d_target_desc;
    p.nt = d_n_target;
    p.t_pitch = target_pitch;
    p.radius = radius;
    p.max_dist = max_distance;
    p.min_diff = min_difference;
    p.cap = cap;
    p.res = d_scratch;
    p.out = d_out;
    p.n_out = d_n;
    p.status = d_status;
    return radius_match_launch(p, pairs, (hipStream_t)stream);
}

}  // extern "C"

namespace mage {
// mage_radius_match_batch_device against target sets indexed by radius_band_index_launch (same
// pitch); the results are those of the plain call.
mage_status radius_match_indexed(const mage_keypoint* d_query_kp, const float* d_query_pos, const uint8_t* d_query_desc,
                                 int64_t query_pitch, const uint32_t* d_n_query, const mage_keypoint* d_target_kp,
                                 const uint8_t* d_target_desc, int64_t target_pitch, const uint32_t* d_n_target,
                                 const unsigned long long* d_keys, const float* d_xy, const uint32_t* d_desc,
                                 uint32_t pairs, float radius, int32_t max_distance, int32_t min_difference,
                                 int32_t* d_scratch, mage_dmatch* d_out, uint32_t cap, uint32_t* d_n, uint32_t* d_status,
                                 hipStream_t st, const RadiusFollow* follow)
{
    if (pairs == 0) return MAGE_OK;
    MAGE_REQUIRE(!follow || pairs == 1, MAGE_EINVAL, "a RadiusFollow decision is per single pair");
    MAGE_REQUIRE(max_distance >= -1 && max_distance <= 256, MAGE_EINVAL, "maxHammingDist must be in [-1, 256]");
    RadiusParams p{};
    p.qkp = d_query_kp;
    p.qpos = d_query_pos;
    p.qdesc = d_query_desc;
    p.nq = d_n_query;
    p.q_pitch = query_pitch;
    p.tkp = d_target_kp;
    p.tdesc = d_target_desc;
    p.nt = d_n_target;
    p.t_pitch = target_pitch;
    p.radius = radius;
    p.max_dist = max_distance;
    p.min_diff = min_difference;
    p.cap = cap;
    p.res = d_scratch;
    p.out = d_out;
    p.n_out = d_n;
    p.status = d_status;
    p.bkeys = d_keys;
    p.bxy = reinterpret_cast<const float2*>(d_xy);
    p.bdesc = reinterpret_cast<const uint4*>(d_desc);
    if (follow) p.follow = *follow;
    return radius_match_launch(p, pairs, st);
}
}  // namespace mage
