// Micro-benchmark for the matcher's MFMA skeleton (development tool).
// mode 0: 8-MFMA chains on register operands; mode 1: B operands via ds_read_b128 from LDS;
// mode 2: mode 1 + __syncthreads every 4 chains; mode 3: mode 1 with 2 independent chains
// interleaved (two tiles in flight).  Reports cycles per MFMA per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

template <int MODE>
__global__ void probe(const v4i* __restrict__ src, int iters, int* __restrict__ sink, long long* cyc)
{
    __shared__ v4i lds[4][8][64];
    const int lane = threadIdx.x & 63;
    for (int i = threadIdx.x; i < 4 * 8 * 64; i += blockDim.x) (&lds[0][0][0])[i] = src[i];
    __syncthreads();
    v4i a[8];
    for (int s = 0; s < 8; s++) a[s] = src[s * 64 + lane];
    int accum = 0;
    long long t0 = clock64();
    for (int it = 0; it < iters; it++) {
        if (MODE == 3) {
            v16i x = {}, y = {};
#pragma unroll
            for (int s = 0; s < 8; s++) {
                x = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[s], lds[it & 3][s][lane], x, 0, 0, 0);
                y = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[s], lds[(it + 1) & 3][s][lane], y, 0, 0, 0);
            }
#pragma unroll
            for (int g = 0; g < 16; g++) accum = max(accum, x[g] ^ y[g]);
            it++;
        } else {
            v16i x = {};
#pragma unroll
            for (int s = 0; s < 8; s++) {
                const v4i b = MODE == 0 ? a[(s + it) & 7] : lds[it & 3][s][lane];
                x = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[s], b, x, 0, 0, 0);
            }
#pragma unroll
            for (int g = 0; g < 16; g++) accum = max(accum, x[g]);
            if (MODE == 2 && (it & 3) == 3) __syncthreads();
        }
    }
    long long t1 = clock64();
    sink[blockIdx.x * blockDim.x + threadIdx.x] = accum;
    if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}

template <int MODE>
void run(int threads, const v4i* src, int* sink, long long* cyc)
{
    const int iters = 2000, blocks = 256;
    hipLaunchKernelGGL(probe<MODE>, dim3(blocks), dim3(threads), 0, 0, src, iters, sink, cyc);
    hipDeviceSynchronize();
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL(probe<MODE>, dim3(blocks), dim3(threads), 0, 0, src, iters, sink, cyc);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    long long c = 0;
    hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
    const double mfma_per_simd = (double)iters * 8 * (threads / 64) / 4;
    printf("mode %d waves/SIMD %d: %.3f ms, clock64 %lld -> %.1f cyc/MFMA/SIMD (clock64), %.1f ns/MFMA\n", MODE,
           threads / 256, ms, c, c / mfma_per_simd, ms * 1e6 / mfma_per_simd);
}

int main()
{
    v4i* src;
    int* sink;
    long long* cyc;
    hipMalloc(&src, 4 * 8 * 64 * 16);
    hipMemset(src, 1, 4 * 8 * 64 * 16);
    hipMalloc(&sink, 256 * 1024 * 4);
    hipMalloc(&cyc, 8);
    for (int w : {1, 2, 3, 4}) {
        run<0>(256 * w, src, sink, cyc);
        run<1>(256 * w, src, sink, cyc);
        run<2>(256 * w, src, sink, cyc);
        run<3>(256 * w, src, sink, cyc);
    }
    return 0;
}
