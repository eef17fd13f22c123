// match.hip — two-way brute-force Hamming matching on MI355X (gfx950).  Replaces Match and
// GetDescriptorDistance (Core/MAGESLAM/Source/Tracking/FeatureMatcher.cpp:61-190, 453-504); the
// reference builds two N x N float distance matrices with cv::BFMatcher::radiusMatch twice.
//
// One workgroup (8 waves) per (A, B) frame pair, nothing materialised in HBM:
//   * each lane owns one A row (32 B in 8 VGPRs) and walks 64-column B tiles staged in LDS,
//     d = sum popc(a ^ b) (v_xor + v_bcnt with accumulate), keeping the row's best and second
//     best as packed keys (d << 16 | j) with two min and one max per pair;
//   * the 64x64 distance tile is transposed through LDS (2 distances per dword, 65-dword row
//     pitch: conflict-free) so that lane c then owns column c and reduces it in registers;
//   * wave column partials merge in LDS; the final cross-check (best(a) = b and best(b) = a,
//     FeatureMatcher.cpp:158) and the ordered DMatch compaction run in the same launch.
// Radius semantics follow OpenCV radiusMatch (distance <= maxDist); ties at the best distance
// are rejected by the delta test for minDifference >= 1, and otherwise resolve to the lowest
// index (canonical).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <vector>

#include "common.hpp"

namespace mage {
namespace {

constexpr int MW = 8;               // waves per workgroup
constexpr int MT = MW * kWave;      // rows per pass
constexpr int NMAX = 4096;          // max descriptors per side (row/column state in LDS)
constexpr uint32_t INF = 0xFFFFFFFFu;

struct MatchParams {
    int max_dist, min_diff;
    unsigned out_cap;
    long long a_pitch, b_pitch;  // bytes between pairs
};

__device__ __forceinline__ void push2(uint32_t& m1, uint32_t& m2, uint32_t key)
{
    m2 = min(m2, max(m1, key));
    m1 = min(m1, key);
}

__device__ __forceinline__ void merge2(uint32_t& a1, uint32_t& a2, uint32_t b1, uint32_t b2)
{
    uint32_t n1 = min(a1, b1);
    a2 = min(max(a1, b1), min(a2, b2));
    a1 = n1;
}

// Row/column acceptance of FeatureMatcher.cpp:125-137 on (best, second) keys.
__device__ __forceinline__ bool accept(uint32_t m1, uint32_t m2, int maxDist, int minDiff)
{
    if (m1 == INF) return false;
    int d0 = (int)(m1 >> 16);
    if (d0 > maxDist) return false;
    if (m2 != INF) {
        int d1 = (int)(m2 >> 16);
        if (d1 <= maxDist && d1 - d0 < minDiff) return false;
    }
    return true;
}

__device__ __forceinline__ uint32_t hamming(const uint4& a0, const uint4& a1, const uint4& b0, const uint4& b1)
{
    uint32_t d = __popc(a0.x ^ b0.x);
    d += __popc(a0.y ^ b0.y);
    d += __popc(a0.z ^ b0.z);
    d += __popc(a0.w ^ b0.w);
    d += __popc(a1.x ^ b1.x);
    d += __popc(a1.y ^ b1.y);
    d += __popc(a1.z ^ b1.z);
    d += __popc(a1.w ^ b1.w);
    return d;
}

__global__ __launch_bounds__(MT) void match_kernel(const uint8_t* __restrict__ A,
                                                   const uint32_t* __restrict__ nA,
                                                   const uint8_t* __restrict__ B,
                                                   const uint32_t* __restrict__ nB, MatchParams p,
                                                   mage_dmatch* __restrict__ out,
                                                   uint32_t* __restrict__ n_out,
                                                   uint32_t* __restrict__ status)
{
    __shared__ uint4 Bt[64][2];
    __shared__ uint32_t T[MW][32][65];
    __shared__ uint2 colpart[MW][64];
    __shared__ uint2 colstate[NMAX];
    __shared__ uint2 rowstate[NMAX];
    __shared__ uint32_t wsum[MW];

    const int pair = blockIdx.x;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    int na = (int)nA[pair], nb = (int)nB[pair];
    if (na > NMAX || nb > NMAX) {
        if (tid == 0) {
            atomicOr(status, 1u);
            n_out[pair] = 0;
        }
        return;
    }
    const uint4* Ap = reinterpret_cast<const uint4*>(A + pair * p.a_pitch);
    const uint4* Bp = reinterpret_cast<const uint4*>(B + pair * p.b_pitch);
    for (int j = tid; j < nb; j += MT) colstate[j] = make_uint2(INF, INF);

    for (int rb = 0; rb < na; rb += MT) {
        const int i = rb + tid;
        const bool valid = i < na;
        uint4 a0 = make_uint4(0, 0, 0, 0), a1 = a0;
        if (valid) {
            a0 = Ap[2 * i];
            a1 = Ap[2 * i + 1];
        }
        uint32_t rm1 = INF, rm2 = INF;
        const int waveRow0 = rb + wave * kWave;
        const int rowsValid = min(kWave, na - waveRow0);
        for (int cb = 0; cb < nb; cb += 64) {
            __syncthreads();  // previous tile fully consumed
            if (tid < 128) {
                int j = cb + (tid >> 1);
                Bt[tid >> 1][tid & 1] = j < nb ? Bp[2 * j + (tid & 1)] : make_uint4(0, 0, 0, 0);
            }
            __syncthreads();
            const int ncol = min(64, nb - cb);
#pragma unroll 4
            for (int c = 0; c < 64; c += 2) {
                const uint32_t d0 = hamming(a0, a1, Bt[c][0], Bt[c][1]);
                const uint32_t d1 = hamming(a0, a1, Bt[c + 1][0], Bt[c + 1][1]);
                if (valid && c < ncol) push2(rm1, rm2, (d0 << 16) | (uint32_t)(cb + c));
                if (valid && c + 1 < ncol) push2(rm1, rm2, (d1 << 16) | (uint32_t)(cb + c + 1));
                T[wave][c >> 1][lane] = d0 | (d1 << 16);
            }
            __syncthreads();
            // lane = column: reduce the wave's 64 rows of this column
            uint32_t cm1 = INF, cm2 = INF;
            if (rowsValid > 0) {
                const int cp = lane >> 1, sh = (lane & 1) * 16;
                for (int r = 0; r < rowsValid; r++) {
                    uint32_t d = (T[wave][cp][r] >> sh) & 0xFFFFu;
                    push2(cm1, cm2, (d << 16) | (uint32_t)(waveRow0 + r));
                }
            }
            colpart[wave][lane] = make_uint2(cm1, cm2);
            __syncthreads();
            if (tid < 64 && cb + tid < nb) {
                uint2 s = colstate[cb + tid];
#pragma unroll
                for (int w = 0; w < MW; w++) merge2(s.x, s.y, colpart[w][tid].x, colpart[w][tid].y);
                colstate[cb + tid] = s;
            }
        }
        if (valid) rowstate[i] = make_uint2(rm1, rm2);
    }
    __syncthreads();

    // cross-check + ordered compaction (ascending A index, FeatureMatcher.cpp:142-167)
    uint32_t base = 0;
    mage_dmatch* o = out + (long long)pair * p.out_cap;
    for (int rb = 0; rb < na; rb += MT) {
        const int i = rb + tid;
        bool ok = false;
        uint32_t j = 0, d = 0;
        if (i < na) {
            uint2 r = rowstate[i];
            if (accept(r.x, r.y, p.max_dist, p.min_diff)) {
                j = r.x & 0xFFFFu;
                d = r.x >> 16;
                uint2 c = colstate[j];
                ok = accept(c.x, c.y, p.max_dist, p.min_diff) && (c.x & 0xFFFFu) == (uint32_t)i;
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
            uint32_t pos = base + woff + before;
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
    if (tid == 0) n_out[pair] = base;
}

}  // namespace

mage_status match_batch(const uint8_t* dA, long long aPitch, const uint32_t* dnA, const uint8_t* dB,
                        long long bPitch, const uint32_t* dnB, uint32_t pairs, int maxDist,
                        int minDiff, mage_dmatch* dOut, uint32_t cap, uint32_t* dN,
                        uint32_t* dStatus, hipStream_t st)
{
    MatchParams mp{};
    mp.max_dist = maxDist;
    mp.min_diff = minDiff;
    mp.out_cap = cap;
    mp.a_pitch = aPitch;
    mp.b_pitch = bPitch;
    {
        KernelTimer _kt("match.two_way", st);
        hipLaunchKernelGGL(match_kernel, dim3(pairs), dim3(MT), 0, st, dA, dnA, dB, dnB, mp, dOut, dN, dStatus);
    }
    MAGE_HIP(hipGetLastError());
    return MAGE_OK;
}

namespace {
struct MatchScratch {
    DeviceBuffer a, b, n, out, status;
};
thread_local MatchScratch g_match;
}  // namespace

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
