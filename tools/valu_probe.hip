// Issue-rate probe for the VALU forms the ORB kernels use (development tool).
// Each kernel runs 8 independent dependency chains of one instruction form; reports ns per
// wave-instruction per SIMD at 4 waves/SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef _Float16 h2 __attribute__((ext_vector_type(2)));
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

template <int OP>
__global__ void probe(const unsigned* __restrict__ src, unsigned* __restrict__ dst, int iters)
{
    unsigned x[8];
    for (int i = 0; i < 8; i++) x[i] = src[(threadIdx.x + i) & 255];
    const unsigned a = src[256], b = src[257];
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int i = 0; i < 8; i++) {
            if (OP == 0) x[i] = min(min(x[i], a), b);  // v_min3_u32
            if (OP == 1) {
                h2 v = __builtin_bit_cast(h2, x[i]);
                v = __builtin_elementwise_minimum(__builtin_elementwise_minimum(v, __builtin_bit_cast(h2, a)), __builtin_bit_cast(h2, b));
                x[i] = __builtin_bit_cast(unsigned, v);
            }
            if (OP == 2) x[i] = __builtin_bit_cast(unsigned, __builtin_bit_cast(h2, x[i]) - __builtin_bit_cast(h2, a));
            if (OP == 3) x[i] = __builtin_amdgcn_perm(x[i], a, b);
            if (OP == 4) x[i] = __builtin_amdgcn_udot4(x[i], a, b, false);
            if (OP == 5) x[i] = __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, x[i]), __builtin_bit_cast(u16x2, a), b, false);
            if (OP == 6) x[i] = x[i] + a;
        }
    }
    unsigned s = 0;
    for (int i = 0; i < 8; i++) s ^= x[i];
    dst[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int OP>
void run(const char* name, const unsigned* src, unsigned* dst)
{
    const int iters = 4000, blocks = 256, threads = 1024;
    hipLaunchKernelGGL(probe<OP>, dim3(blocks), dim3(threads), 0, 0, src, dst, iters);
    hipDeviceSynchronize();
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL(probe<OP>, dim3(blocks), dim3(threads), 0, 0, src, dst, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    const double per_simd = (double)iters * 8 * (threads / 64) / 4;
    printf("%-22s %.3f ns per wave-instruction per SIMD (%.2f cycles at 2.1 GHz)\n", name, ms * 1e6 / per_simd,
           ms * 1e6 / per_simd * 2.1);
}

int main()
{
    unsigned *src, *dst;
    hipMalloc(&src, 4096);
    hipMemset(src, 0x3c, 4096);
    hipMalloc(&dst, 256 * 1024 * 4);
    run<0>("v_min3_u32", src, dst);
    run<1>("v_pk_minimum3_f16", src, dst);
    run<2>("v_pk_add_f16", src, dst);
    run<3>("v_perm_b32", src, dst);
    run<4>("v_dot4_u32_u8", src, dst);
    run<5>("v_dot2_u32_u16", src, dst);
    run<6>("v_add_u32", src, dst);
    return 0;
}
