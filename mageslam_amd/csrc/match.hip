// match.hip — two-way brute-force Hamming matching on MI355X (gfx950).  Replaces Match and
// GetDescriptorDistance (Core/MAGESLAM/Source/Tracking/FeatureMatcher.cpp:61-190, 453-504); the
// reference builds two N x N float distance matrices with cv::BFMatcher::radiusMatch twice.
//
// One workgroup (8 waves) per (A, B) frame pair, nothing materialised in HBM.
//   * Each lane owns RPL = 4 A rows (32 B each, in VGPRs); B is staged in LDS in 1024-row
//     tiles, split into first and second 16-byte halves.
//   * Only pairs with d <= maxDist can change "best and second best within the radius"
//     (radiusMatch keeps d <= maxDist; FeatureMatcher.cpp:117-156), so the reductions are a rare
//     branch instead of per-pair work.  The first-half popcount (4 x v_xor + v_bcnt) is a lower
//     bound of d: if it exceeds maxDist for every lane and row of the wave (one ballot), the
//     second half is never read.  For random 256-bit descriptors and maxDist = 30 the branch is
//     taken only around true matches.
//   * Row best / second live in registers as packed keys (d << 16 | j); column best / second
//     live in LDS and are updated by 64-bit compare-and-swap (order-independent: the two
//     smallest keys of a set).  The cross-check (best(a) = b and best(b) = a,
//     FeatureMatcher.cpp:158) and the ordered DMatch compaction run in the same launch.
// Ties at the best distance are rejected by the delta test for minDifference >= 1 and
// otherwise resolve to the lowest index (canonical).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <vector>

#include "common.hpp"

namespace mage {
namespace {

constexpr int MW = 8;              // waves per workgroup
constexpr int MT = MW * kWave;     // threads per workgroup
constexpr int RPL = 4;             // A rows per lane
constexpr int ROWS = MT * RPL;     // A rows per pass
constexpr int BT = 1024;           // B rows per LDS tile
constexpr int NMAX = 4096;         // max descriptors per side (column state in LDS)
constexpr uint32_t INF = 0xFFFFFFFFu;

struct MatchParams {
    int max_dist, min_diff;
    unsigned out_cap;
    long long a_pitch, b_pitch;  // bytes between pairs
    uint32_t* row_scratch;       // per pair NMAX x 2 u32 (row states between passes)
};

__device__ __forceinline__ void push2(uint32_t& m1, uint32_t& m2, uint32_t key)
{
    m2 = min(m2, max(m1, key));
    m1 = min(m1, key);
}

// Row/column acceptance of FeatureMatcher.cpp:125-137 on (best, second) keys.
__device__ __forceinline__ bool accept(uint32_t m1, uint32_t m2, int maxDist, int minDiff)
{
    if (m1 == INF) return false;
    const int d0 = (int)(m1 >> 16);
    if (d0 > maxDist) return false;
    if (m2 != INF) {
        const int d1 = (int)(m2 >> 16);
        if (d1 <= maxDist && d1 - d0 < minDiff) return false;
    }
    return true;
}

__device__ __forceinline__ uint32_t popc4(const uint4& a, const uint4& b)
{
    return __popc(a.x ^ b.x) + __popc(a.y ^ b.y) + __popc(a.z ^ b.z) + __popc(a.w ^ b.w);
}

__device__ __forceinline__ void col_push(unsigned long long* cell, uint32_t key)
{
    unsigned long long old = *cell, assumed;
    do {
        assumed = old;
        uint32_t m1 = (uint32_t)assumed, m2 = (uint32_t)(assumed >> 32);
        push2(m1, m2, key);
        const unsigned long long nw = (unsigned long long)m1 | ((unsigned long long)m2 << 32);
        if (nw == assumed) return;
        old = atomicCAS(cell, assumed, nw);
    } while (old != assumed);
}

__global__ __launch_bounds__(MT) void match_kernel(const uint8_t* __restrict__ A,
                                                   const uint32_t* __restrict__ nA,
                                                   const uint8_t* __restrict__ B,
                                                   const uint32_t* __restrict__ nB, MatchParams p,
                                                   mage_dmatch* __restrict__ out,
                                                   uint32_t* __restrict__ n_out,
                                                   uint32_t* __restrict__ status)
{
    __shared__ uint4 Blo[BT], Bhi[BT];
    __shared__ unsigned long long colstate[NMAX];
    __shared__ uint32_t wsum[MW];

    const int pair = blockIdx.x;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int na = (int)nA[pair], nb = (int)nB[pair];
    if (na > NMAX || nb > NMAX) {
        if (tid == 0) {
            atomicOr(status, 1u);
            n_out[pair] = 0;
        }
        return;
    }
    const int maxDist = p.max_dist;
    const uint4* Ap = reinterpret_cast<const uint4*>(A + pair * p.a_pitch);
    const uint4* Bp = reinterpret_cast<const uint4*>(B + pair * p.b_pitch);
    uint32_t* rows = p.row_scratch + (long long)pair * NMAX * 2;
    for (int j = tid; j < nb; j += MT) colstate[j] = ~0ull;

    uint32_t m1[RPL], m2[RPL];
    for (int rb = 0; rb < na; rb += ROWS) {
        uint4 alo[RPL], ahi[RPL];
        bool valid[RPL];
#pragma unroll
        for (int r = 0; r < RPL; r++) {
            const int i = rb + r * MT + tid;
            valid[r] = i < na;
            alo[r] = valid[r] ? Ap[2 * i] : make_uint4(0, 0, 0, 0);
            ahi[r] = valid[r] ? Ap[2 * i + 1] : make_uint4(0, 0, 0, 0);
            m1[r] = INF;
            m2[r] = INF;
        }
        for (int cb = 0; cb < nb; cb += BT) {
            const int ncol = min(BT, nb - cb);
            __syncthreads();  // previous tile consumed (and colstate initialised)
            for (int j = tid; j < ncol; j += MT) {
                Blo[j] = Bp[2 * (cb + j)];
                Bhi[j] = Bp[2 * (cb + j) + 1];
            }
            __syncthreads();
            for (int c = 0; c < ncol; c++) {
                const uint4 b0 = Blo[c];
                uint32_t h[RPL];
                bool close = false;
#pragma unroll
                for (int r = 0; r < RPL; r++) {
                    h[r] = valid[r] ? popc4(alo[r], b0) : 1024u;
                    close |= h[r] <= (uint32_t)maxDist;
                }
                if (__any(close)) {
                    const uint4 b1 = Bhi[c];
                    const int j = cb + c;
#pragma unroll
                    for (int r = 0; r < RPL; r++) {
                        if (h[r] <= (uint32_t)maxDist) {
                            const uint32_t d = h[r] + popc4(ahi[r], b1);
                            if (d <= (uint32_t)maxDist) {
                                push2(m1[r], m2[r], (d << 16) | (uint32_t)j);
                                col_push(&colstate[j], (d << 16) | (uint32_t)(rb + r * MT + tid));
                            }
                        }
                    }
                }
            }
        }
        if (na > ROWS) {  // more passes follow: park this pass's rows (read back by this thread)
#pragma unroll
            for (int r = 0; r < RPL; r++) {
                const int i = rb + r * MT + tid;
                if (i < na) {
                    rows[2 * i] = m1[r];
                    rows[2 * i + 1] = m2[r];
                }
            }
        }
    }
    __syncthreads();

    // cross-check + ordered compaction (ascending A index, FeatureMatcher.cpp:142-167)
    uint32_t base = 0;
    mage_dmatch* o = out + (long long)pair * p.out_cap;
    for (int rb = 0; rb < na; rb += ROWS) {
#pragma unroll
        for (int r = 0; r < RPL; r++) {
            const int i = rb + r * MT + tid;
            bool ok = false;
            uint32_t j = 0, d = 0;
            if (i < na) {
                uint32_t r1 = m1[r], r2 = m2[r];
                if (na > ROWS) {
                    r1 = rows[2 * i];
                    r2 = rows[2 * i + 1];
                }
                if (accept(r1, r2, maxDist, p.min_diff)) {
                    j = r1 & 0xFFFFu;
                    d = r1 >> 16;
                    const unsigned long long c = colstate[j];
                    ok = accept((uint32_t)c, (uint32_t)(c >> 32), maxDist, p.min_diff) &&
                         ((uint32_t)c & 0xFFFFu) == (uint32_t)i;
                }
            }
            const unsigned long long m = __ballot(ok);
            const uint32_t before = (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
            if (lane == 0) wsum[wave] = (uint32_t)__popcll(m);
            __syncthreads();
            uint32_t woff = 0, total = 0;
            for (int w = 0; w < MW; w++) {
                if (w < wave) woff += wsum[w];
                total += wsum[w];
            }
            if (ok) {
                const uint32_t pos = base + woff + before;
                if (pos < p.out_cap) {
                    mage_dmatch mm;
                    mm.query_idx = i;
                    mm.train_idx = (int32_t)j;
                    mm.img_idx = 0;
                    mm.distance = (float)d;
                    o[pos] = mm;
                }
            }
            base += total;
            __syncthreads();
        }
    }
    if (tid == 0) n_out[pair] = base;
}

struct MatchScratch {
    DeviceBuffer a, b, n, out, status, rows;
};
thread_local MatchScratch g_match;

}  // namespace

mage_status match_batch(const uint8_t* dA, long long aPitch, const uint32_t* dnA, const uint8_t* dB,
                        long long bPitch, const uint32_t* dnB, uint32_t pairs, int maxDist,
                        int minDiff, mage_dmatch* dOut, uint32_t cap, uint32_t* dN,
                        uint32_t* dStatus, hipStream_t st)
{
    mage_status r = g_match.rows.reserve((size_t)pairs * NMAX * 2 * 4);
    if (r != MAGE_OK) return r;
    MatchParams mp{};
    mp.max_dist = maxDist;
    mp.min_diff = minDiff;
    mp.out_cap = cap;
    mp.a_pitch = aPitch;
    mp.b_pitch = bPitch;
    mp.row_scratch = g_match.rows.as<uint32_t>();
    {
        KernelTimer _kt("match.two_way", st);
        hipLaunchKernelGGL(match_kernel, dim3(pairs), dim3(MT), 0, st, dA, dnA, dB, dnB, mp, dOut, dN, dStatus);
    }
    MAGE_HIP(hipGetLastError());
    return MAGE_OK;
}

}  // namespace mage

extern "C" {

int32_t mage_hamming_distance(const uint8_t* a, const uint8_t* b)
{
    int32_t d = 0;
    for (int k = 0; k < 32; k++) d += __builtin_popcount((unsigned)(a[k] ^ b[k]));
    return d;
}

mage_status mage_hamming_match_batch_device(const uint8_t* d_desc_a, int64_t a_pitch,
                                            const uint32_t* d_n_a, const uint8_t* d_desc_b,
                                            int64_t b_pitch, const uint32_t* d_n_b,
                                            uint32_t pairs, int32_t max_distance,
                                            int32_t min_difference, mage_dmatch* d_out,
                                            uint32_t cap, uint32_t* d_n, mage_stream stream)
{
    MAGE_REQUIRE(d_desc_a && d_desc_b && d_n_a && d_n_b && d_out && d_n, MAGE_EINVAL, "null buffer");
    MAGE_REQUIRE(a_pitch % 16 == 0 && b_pitch % 16 == 0, MAGE_EINVAL, "pair pitch must be a multiple of 16");
    if (pairs == 0) return MAGE_OK;
    auto& s = mage::g_match;
    mage_status r = s.status.reserve(4);
    if (r != MAGE_OK) return r;
    return mage::match_batch(d_desc_a, a_pitch, d_n_a, d_desc_b, b_pitch, d_n_b, pairs, max_distance,
                             min_difference, d_out, cap, d_n, s.status.as<uint32_t>(), (hipStream_t)stream);
}

mage_status mage_hamming_match(const uint8_t* desc_a, uint32_t n_a, const uint8_t* mask_a,
                               const uint8_t* desc_b, uint32_t n_b, const uint8_t* mask_b,
                               int32_t max_distance, int32_t min_difference, mage_dmatch* out,
                               uint32_t cap, uint32_t* n)
{
    MAGE_REQUIRE(n && (cap == 0 || out), MAGE_EINVAL, "null output");
    *n = 0;
    // Masked rows are compacted first, exactly like the reference's descriptorMatrixA/B
    // (FeatureMatcher.cpp:84-108); indices are mapped back on output.
    std::vector<uint32_t> ia, ib;
    for (uint32_t i = 0; i < n_a; i++)
        if (!mask_a || mask_a[i]) ia.push_back(i);
    for (uint32_t i = 0; i < n_b; i++)
        if (!mask_b || mask_b[i]) ib.push_back(i);
    if (ia.empty() || ib.empty()) return MAGE_OK;  // FeatureMatcher.cpp:72-77
    MAGE_REQUIRE(desc_a && desc_b, MAGE_EINVAL, "null descriptors");
    MAGE_REQUIRE(ia.size() <= 4096 && ib.size() <= 4096, MAGE_EUNSUPPORTED, "more than 4096 descriptors per side");
    int dev = 0;
    MAGE_HIP(hipGetDevice(&dev));
    mage_status r = mage::bind_device(dev);
    if (r != MAGE_OK) return r;
    std::vector<uint8_t> ha(ia.size() * 32), hb(ib.size() * 32);
    for (size_t k = 0; k < ia.size(); k++) std::copy(desc_a + 32 * (size_t)ia[k], desc_a + 32 * (size_t)ia[k] + 32, &ha[32 * k]);
    for (size_t k = 0; k < ib.size(); k++) std::copy(desc_b + 32 * (size_t)ib[k], desc_b + 32 * (size_t)ib[k] + 32, &hb[32 * k]);
    auto& s = mage::g_match;
    const uint32_t ocap = (uint32_t)ia.size();
    if ((r = s.a.reserve(ha.size())) != MAGE_OK) return r;
    if ((r = s.b.reserve(hb.size())) != MAGE_OK) return r;
    if ((r = s.n.reserve(16)) != MAGE_OK) return r;
    if ((r = s.out.reserve(sizeof(mage_dmatch) * ocap)) != MAGE_OK) return r;
    if ((r = s.status.reserve(4)) != MAGE_OK) return r;
    uint32_t counts[3] = {(uint32_t)ia.size(), (uint32_t)ib.size(), 0};
    MAGE_HIP(hipMemcpy(s.a.ptr, ha.data(), ha.size(), hipMemcpyHostToDevice));
    MAGE_HIP(hipMemcpy(s.b.ptr, hb.data(), hb.size(), hipMemcpyHostToDevice));
    MAGE_HIP(hipMemcpy(s.n.ptr, counts, 12, hipMemcpyHostToDevice));
    MAGE_HIP(hipMemset(s.status.ptr, 0, 4));
    uint32_t* dn = s.n.as<uint32_t>();
    r = mage::match_batch(s.a.as<uint8_t>(), 0, dn, s.b.as<uint8_t>(), 0, dn + 1, 1, max_distance,
                          min_difference, s.out.as<mage_dmatch>(), ocap, dn + 2, s.status.as<uint32_t>(), nullptr);
    if (r != MAGE_OK) return r;
    uint32_t total = 0;
    MAGE_HIP(hipMemcpy(&total, dn + 2, 4, hipMemcpyDeviceToHost));
    std::vector<mage_dmatch> tmp(std::min(total, ocap));
    if (!tmp.empty()) MAGE_HIP(hipMemcpy(tmp.data(), s.out.ptr, sizeof(mage_dmatch) * tmp.size(), hipMemcpyDeviceToHost));
    const uint32_t nw = std::min<uint32_t>((uint32_t)tmp.size(), cap);
    for (uint32_t k = 0; k < nw; k++) {
        out[k] = tmp[k];
        out[k].query_idx = (int32_t)ia[tmp[k].query_idx];
        out[k].train_idx = (int32_t)ib[tmp[k].train_idx];
    }
    *n = nw;
    return total > cap ? MAGE_ECAPACITY : MAGE_OK;
}

}  // extern "C"
