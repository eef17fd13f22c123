// lds_sort.hpp — workgroup-wide descending sort of 64-bit keys in LDS (1024 threads), shared by
// the ORB select kernel (ANMS ranking) and the radius matcher (target ordering).
#pragma once

#include <hip/hip_runtime.h>

namespace mage {

constexpr int SORT_THREADS = 1024;

// Descending bitonic sort of P = 1024 * E keys held in LDS, thread t owning keys [tE, tE + E).
// Compare-exchange strides j < E stay in registers, E <= j < 64E cross lanes of one wave
// (__shfl_xor, no barrier) and only j >= 64E go through LDS with a workgroup barrier: for
// P = 4096, 10 barrier steps instead of the 78 of a plain LDS bitonic network.
template <int E>
__device__ inline void sort_desc_e(unsigned long long* keys)
{
    constexpr int P = SORT_THREADS * E;
    const int tid = threadIdx.x;
    unsigned long long v[E];
#pragma unroll
    for (int e = 0; e < E; e++) v[e] = keys[tid * E + e];
    for (int k = 2; k <= P; k <<= 1) {
        if ((k >> 1) >= 64 * E) {
#pragma unroll
            for (int e = 0; e < E; e++) keys[tid * E + e] = v[e];
            __syncthreads();
            for (int j = k >> 1; j >= 64 * E; j >>= 1) {
                for (int i = tid; i < P; i += SORT_THREADS) {
                    const int ixj = i ^ j;
                    if (ixj > i) {
                        const unsigned long long a = keys[i], b = keys[ixj];
                        if (((i & k) == 0) ? (a < b) : (a > b)) {
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
        for (int j = min(k >> 1, 32 * E); j >= E; j >>= 1) {
            const int lm = j / E;
#pragma unroll
            for (int e = 0; e < E; e++) {
                const int i = tid * E + e;
                const unsigned long long o = __shfl_xor(v[e], lm);
                const bool keep_big = ((i & j) == 0) == ((i & k) == 0);
                v[e] = keep_big ? (v[e] > o ? v[e] : o) : (v[e] < o ? v[e] : o);
            }
        }
#pragma unroll
        for (int j = E / 2; j >= 1; j >>= 1) {
            if (j > (k >> 1)) continue;
#pragma unroll
            for (int e = 0; e < E; e++) {
                if (e & j) continue;
                const int i = tid * E + e;
                const unsigned long long a = v[e], b = v[e | j];
                if (((i & k) == 0) ? (a < b) : (a > b)) {
                    v[e] = b;
                    v[e | j] = a;
                }
            }
        }
    }
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
