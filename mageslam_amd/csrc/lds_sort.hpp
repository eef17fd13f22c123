// lds_sort.hpp — workgroup-wide descending sort of 64-bit keys in LDS (1024 threads), shared by
// the ORB select kernel (ANMS ranking) and the radius matcher (target ordering).
#pragma once

#include <hip/hip_runtime.h>

namespace mage {

constexpr int SORT_THREADS = 1024;

// The 32-bit value of lane (l ^ LM), all on the VALU (no LDS crossbar round trip): quad_perm for
// LM = 1, 2; DPP row_shl:4 / row_shr:4 on alternate banks for 4; row_ror:8 for 8;
// v_permlane16_swap / v_permlane32_swap for 16 / 32 (the swap returns (own, partner) in lanes
// without bit LM, (partner, own) in lanes with it).
template <int LM>
__device__ __forceinline__ unsigned xor_lanes32(unsigned v)
{
    if constexpr (LM == 1) return (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);
    if constexpr (LM == 2) return (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false);
    if constexpr (LM == 4) {
        const int r = __builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xA, false);  // banks 1, 3: lane - 4
        return (unsigned)__builtin_amdgcn_update_dpp(r, (int)v, 0x104, 0xF, 0x5, false);   // banks 0, 2: lane + 4
    }
    if constexpr (LM == 8) return (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x128, 0xF, 0xF, false);
    if constexpr (LM == 16) {
        const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
        return (threadIdx.x & 16) ? r[0] : r[1];
    }
    if constexpr (LM == 32) {
        const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
        return (threadIdx.x & 32) ? r[0] : r[1];
    }
    return v;
}
template <int LM>
__device__ __forceinline__ unsigned long long xor_lanes(unsigned long long v)
{
    const unsigned lo = xor_lanes32<LM>((unsigned)v), hi = xor_lanes32<LM>((unsigned)(v >> 32));
    return ((unsigned long long)hi << 32) | lo;
}
// One bitonic level (block size K) of sort_desc_e, unrolled at compile time so every lane
// exchange has a constant pattern.  Strides J >= 64E go through LDS (one barrier each), strides
// E <= J < 64E exchange between lanes of one wave, strides J < E stay in the thread's registers.
template <int E, int K, int J>
__device__ __forceinline__ void bitonic_lane_steps(unsigned long long (&v)[E])
{
    if constexpr (J >= E) {
        constexpr int LM = J / E;
        // i = tid E + e: (i & J) is (tid & LM) and (i & K) is (tid & K / E) for every e
        const bool keep_big = ((threadIdx.x & LM) == 0) == ((threadIdx.x & (K / E)) == 0);
#pragma unroll
        for (int e = 0; e < E; e++) {
            const unsigned long long o = xor_lanes<LM>(v[e]);
            // keep the larger key where keep_big, else the smaller: one compare, one select
            v[e] = ((v[e] > o) == keep_big) ? v[e] : o;
        }
        bitonic_lane_steps<E, K, J / 2>(v);
    }
}
template <int E, int K>
__device__ __forceinline__ void bitonic_level(unsigned long long (&v)[E], unsigned long long* keys)
{
    constexpr int P = SORT_THREADS * E;
    const int tid = threadIdx.x;
    if constexpr ((K >> 1) >= 64 * E) {
#pragma unroll
        for (int e = 0; e < E; e++) keys[tid * E + e] = v[e];
        __syncthreads();
        for (int j = K >> 1; j >= 64 * E; j >>= 1) {
            for (int i = tid; i < P; i += SORT_THREADS) {
                const int ixj = i ^ j;
                if (ixj > i) {
                    const unsigned long long a = keys[i], b = keys[ixj];
                    if (((i & K) == 0) ? (a < b) : (a > b)) {
                        keys[i] = b;
                        keys[ixj] = a;
                    }
                }
            }
            __syncthreads();
        }
#pragma unroll
        for (int e = 0; e < E; e++) v[e] = keys[tid * E + e];
    }
    bitonic_lane_steps<E, K, ((K >> 1) < 32 * E ? (K >> 1) : 32 * E)>(v);
    for (int j = E / 2; j >= 1; j >>= 1) {  // (constant trip count: unrolled without a pragma)
        if (j > (K >> 1)) continue;
#pragma unroll
        for (int e = 0; e < E; e++) {
            if (e & j) continue;
            const int i = tid * E + e;
            const unsigned long long a = v[e], b = v[e | j];
            if (((i & K) == 0) ? (a < b) : (a > b)) {
                v[e] = b;
                v[e | j] = a;
            }
        }
    }
    if constexpr (K < P) bitonic_level<E, 2 * K>(v, keys);
}

// Descending bitonic sort of P = 1024 * E keys held in LDS, thread t owning keys [tE, tE + E).
// Compare-exchange strides j < E stay in registers, E <= j < 64E cross lanes of one wave
// (VALU lane exchanges, xor_lanes: no barrier, no LDS round trip) and only j >= 64E go through
// LDS with a workgroup barrier: for P = 4096, 10 barrier steps instead of the 78 of a plain LDS
// bitonic network.
template <int E>
__device__ inline void sort_desc_e(unsigned long long* keys)
{
    const int tid = threadIdx.x;
    unsigned long long v[E];
#pragma unroll
    for (int e = 0; e < E; e++) v[e] = keys[tid * E + e];
    bitonic_level<E, 2>(v, keys);
    __syncthreads();
#pragma unroll
    for (int e = 0; e < E; e++) keys[tid * E + e] = v[e];
    __syncthreads();
}

// Descending sort of keys[0..P), P a power of two <= KMAX; pads with zero keys to >= 1024.
__device__ inline void sort_desc(unsigned long long* keys, int P)
{
    const int Pp = max(P, SORT_THREADS);
    for (int i = P + (int)threadIdx.x; i < Pp; i += SORT_THREADS) keys[i] = 0ull;
    __syncthreads();
    switch (Pp / SORT_THREADS) {
    case 1: sort_desc_e<1>(keys); break;
    case 2: sort_desc_e<2>(keys); break;
    case 4: sort_desc_e<4>(keys); break;
    default: sort_desc_e<8>(keys); break;
    }
}

}  // namespace mage
