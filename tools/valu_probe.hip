// VALU issue-rate probe (development tool, round 5 rewrite).
//
// Every form is emitted by inline asm (no compiler folding, no extra instructions), as 8
// independent accumulation chains unrolled 16x per loop iteration (128 instructions per
// iteration).  Each wave stamps s_memtime around its loop (after an s_barrier so the
// workgroup's waves start together); throughput per SIMD = waves_per_simd x instructions /
// per-wave cycles.  Waves per SIMD = workgroup size / 256 (one workgroup per CU: the grid is
// 256 workgroups and each uses 96 KB of LDS so no second one fits).  The in-kernel clock comes
// from s_memrealtime (100 MHz) over the same window.
//
// Build: hipcc -O3 --offload-arch=gfx950 tools/valu_probe.hip -o tools/valu_probe
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>

#define CHAINS 8
#define UNROLL 16

#define OP_LIST(X)  \
    X(0, "v_fma_f32", "v_fma_f32 %0, %1, %2, %0") \
    X(1, "v_add_f32", "v_add_f32 %0, %1, %0") \
    X(2, "v_mul_f32", "v_mul_f32 %0, %1, %0") \
    X(3, "v_max_f32", "v_max_f32 %0, %1, %0") \
    X(4, "v_min_f32", "v_min_f32 %0, %1, %0") \
    X(5, "v_max3_f32", "v_max3_f32 %0, %1, %2, %0") \
    X(6, "v_med3_f32", "v_med3_f32 %0, %1, %2, %0") \
    X(7, "v_add_u32", "v_add_u32 %0, %1, %0") \
    X(8, "v_sub_u32", "v_sub_u32 %0, %1, %0") \
    X(9, "v_add3_u32", "v_add3_u32 %0, %1, %2, %0") \
    X(10, "v_lshl_add_u32", "v_lshl_add_u32 %0, %0, 1, %1") \
    X(11, "v_mad_u32_u24", "v_mad_u32_u24 %0, %0, %1, %2") \
    X(12, "v_mul_u32_u24", "v_mul_u32_u24 %0, %1, %0") \
    X(13, "v_and_b32", "v_and_b32 %0, %1, %0") \
    X(14, "v_or_b32", "v_or_b32 %0, %1, %0") \
    X(15, "v_xor_b32", "v_xor_b32 %0, %1, %0") \
    X(16, "v_or3_b32", "v_or3_b32 %0, %1, %2, %0") \
    X(17, "v_bitop3_b32", "v_bitop3_b32 %0, %1, %2, %0 bitop3:0x96") \
    X(18, "v_lshlrev_b32", "v_lshlrev_b32 %0, 1, %0") \
    X(19, "v_lshrrev_b32", "v_lshrrev_b32 %0, 1, %0") \
    X(20, "v_bfe_u32", "v_bfe_u32 %0, %0, %1, 8") \
    X(21, "v_max_u32", "v_max_u32 %0, %1, %0") \
    X(22, "v_max_i32", "v_max_i32 %0, %1, %0") \
    X(23, "v_min3_u32", "v_min3_u32 %0, %1, %2, %0") \
    X(24, "v_max_u16", "v_max_u16 %0, %1, %0") \
    X(25, "v_sub_u16", "v_sub_u16 %0, %1, %0") \
    X(26, "v_add_f16", "v_add_f16 %0, %1, %0") \
    X(27, "v_max_f16", "v_max_f16 %0, %1, %0") \
    X(28, "v_pk_add_f16", "v_pk_add_f16 %0, %1, %0") \
    X(29, "v_pk_mul_f16", "v_pk_mul_f16 %0, %1, %0") \
    X(30, "v_pk_max_f16", "v_pk_max_f16 %0, %1, %0") \
    X(31, "v_pk_minimum3_f16", "v_pk_minimum3_f16 %0, %1, %2, %0") \
    X(32, "v_pk_max_i16", "v_pk_max_i16 %0, %1, %0") \
    X(33, "v_pk_min_u16", "v_pk_min_u16 %0, %1, %0") \
    X(34, "v_pk_sub_u16", "v_pk_sub_u16 %0, %1, %0") \
    X(35, "v_pk_add_u16", "v_pk_add_u16 %0, %1, %0") \
    X(36, "v_perm_b32", "v_perm_b32 %0, %1, %2, %0") \
    X(37, "v_alignbyte_b32", "v_alignbyte_b32 %0, %1, %0, %2") \
    X(38, "v_dot4_u32_u8", "v_dot4_u32_u8 %0, %1, %2, %0") \
    X(39, "v_dot2_u32_u16", "v_dot2_u32_u16 %0, %1, %2, %0") \
    X(40, "v_sad_u8", "v_sad_u8 %0, %1, %2, %0") \
    X(41, "v_bcnt_u32_b32", "v_bcnt_u32_b32 %0, %1, %0") \
    X(42, "v_ffbl_b32", "v_ffbl_b32 %0, %0") \
    X(43, "v_mov_b32", "v_mov_b32 %0, %1") \
    X(44, "v_cndmask_b32 s", "v_cndmask_b32 %0, %0, %1, s[0:1]") \
    X(45, "v_cvt_f32_u32", "v_cvt_f32_u32 %0, %0") \
    X(46, "v_mbcnt_lo", "v_mbcnt_lo_u32_b32 %0, %1, %0")

template <int OP>
__device__ __forceinline__ void step(unsigned& x, unsigned a, unsigned b);

#define DEF_STEP(ID, NAME, ASM)                                                         \
    template <>                                                                         \
    __device__ __forceinline__ void step<ID>(unsigned& x, unsigned a, unsigned b)       \
    {                                                                                   \
        asm volatile(ASM : "+v"(x) : "v"(a), "v"(b));                                   \
    }
OP_LIST(DEF_STEP)

template <int OP>
__global__ void __launch_bounds__(1024) probe(const unsigned* __restrict__ src, unsigned* __restrict__ dst,
                                              unsigned long long* __restrict__ stamps, int iters)
{
    __shared__ unsigned pad[24 * 1024];  // 96 KB: one workgroup per CU
    unsigned x[CHAINS];
    for (int i = 0; i < CHAINS; i++) x[i] = src[(threadIdx.x + i) & 255];
    const unsigned a = src[256 + (threadIdx.x & 7)], b = src[264 + (threadIdx.x & 7)];
    if (threadIdx.x == 0) pad[blockIdx.x & 1023] = a;
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int u = 0; u < UNROLL; u++) {
#pragma unroll
            for (int i = 0; i < CHAINS; i++) step<OP>(x[i], a, b);
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    unsigned s = pad[(threadIdx.x * 7) & 1023];
    for (int i = 0; i < CHAINS; i++) s ^= x[i];
    dst[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if ((threadIdx.x & 63) == 0) {
        const int w = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
        stamps[2 * w] = t1 - t0;
        stamps[2 * w + 1] = r1 - r0;
    }
}

template <int OP>
void run(const char* name, const unsigned* src, unsigned* dst, unsigned long long* stamps)
{
    const int iters = 2000, blocks = 256;
    printf("%-22s", name);
    for (int wps : {1, 2, 4}) {
        const int threads = 256 * wps;
        hipLaunchKernelGGL(probe<OP>, dim3(blocks), dim3(threads), 0, 0, src, dst, stamps, iters);
        hipEvent_t e0, e1;
        hipEventCreate(&e0);
        hipEventCreate(&e1);
        hipEventRecord(e0);
        hipLaunchKernelGGL(probe<OP>, dim3(blocks), dim3(threads), 0, 0, src, dst, stamps, iters);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        const int nw = blocks * threads / 64;
        std::vector<unsigned long long> h(2 * nw);
        hipMemcpy(h.data(), stamps, 16 * nw, hipMemcpyDeviceToHost);
        std::vector<double> cyc(nw), ghz(nw);
        for (int w = 0; w < nw; w++) {
            cyc[w] = (double)h[2 * w];
            ghz[w] = (double)h[2 * w] / ((double)h[2 * w + 1] * 10.0);
        }
        std::sort(cyc.begin(), cyc.end());
        std::sort(ghz.begin(), ghz.end());
        const double n_per_wave = (double)iters * UNROLL * CHAINS;
        const double cpi = cyc[nw - 1] / (n_per_wave * wps);  // SIMD cycles per wave-instruction (slowest wave)
        const double wall_ns = ms * 1e6 / (n_per_wave * wps);
        printf("  w%d: %.2f cyc (%.2f GHz, wall %.3f ns)", wps, cpi, ghz[nw / 2], wall_ns);
        hipEventDestroy(e0);
        hipEventDestroy(e1);
    }
    printf("\n");
}

// Does ds_read_u8_d16 keep the register's other half (it does not with SRAM ECC enabled)?
__global__ void d16_check(unsigned* out)
{
    __shared__ unsigned char b[64];
    b[threadIdx.x] = (unsigned char)(threadIdx.x + 1);
    __syncthreads();
    unsigned r = 0xABCD1234u, q = 0xABCD1234u;
    const unsigned a = (unsigned)(uintptr_t)(__attribute__((address_space(3))) void*)&b[threadIdx.x];
    asm volatile("ds_read_u8_d16 %0, %2\n\tds_read_u8_d16_hi %1, %2\n\ts_waitcnt lgkmcnt(0)" : "+v"(r), "+v"(q) : "v"(a) : "memory");
    if (threadIdx.x == 5) { out[0] = r; out[1] = q; }
}

int main()
{
    unsigned *src, *dst;
    unsigned long long* stamps;
    hipMalloc(&src, 4096);
    std::vector<unsigned> hs(1024);
    for (int i = 0; i < 1024; i++) hs[i] = 0x3c003c00u ^ (i * 0x01010101u & 0x00ff00ffu);
    hipMemcpy(src, hs.data(), 4096, hipMemcpyHostToDevice);
    hipMalloc(&dst, 256 * 1024 * 4);
    hipMalloc(&stamps, 256 * 16 * 16);
    {
        unsigned* o;
        hipMalloc(&o, 8);
        hipLaunchKernelGGL(d16_check, dim3(1), dim3(64), 0, 0, o);
        unsigned ho[2];
        hipMemcpy(ho, o, 8, hipMemcpyDeviceToHost);
        printf("ds_read_u8_d16 on 0xABCD1234 -> 0x%08x, _hi -> 0x%08x (byte 6)\n", ho[0], ho[1]);
    }
    printf("SIMD cycles per wave64 instruction (slowest wave; s_memtime), waves per SIMD w1/w2/w4\n");
#define RUN(ID, NAME, ASM) run<ID>(NAME, src, dst, stamps);
    OP_LIST(RUN)
    return 0;
}
