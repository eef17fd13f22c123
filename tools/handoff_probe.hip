// Cross-CU hand-off latency probe for the multi-CU Cholesky question (development tool, not part of
// the product; DESIGN.md §2 Local BA, "Round 6").  Two workgroups on different CUs pass a payload
// back and forth R times: the sender writes the payload with agent-scope relaxed stores (sc1,
// write-through), drains its stores (s_waitcnt vmcnt(0)), then stores the round number into a flag;
// the receiver polls the flag with agent-scope relaxed loads, reads the payload with the same loads,
// checks every word, and answers with its own payload + flag.  One-way hop = elapsed / (2 R).
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/handoff_probe tools/handoff_probe.hip
//   ./tools/handoff_probe   # one JSON line per (workgroup size, payload bytes, partner block) case
//
// Payload sizes: one 16x16 f64 tile (2 KB: the chain tile a step of chol_tiles hands over) and a
// block row of the factor (up to 15 tiles, 30 KB: what every CU holding trailing tiles would read per
// step).  The partner block is 1 (the next XCD under round-robin dispatch) or 8 (the same XCD).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>

#define CHECK(x)                                                                       \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                              \
        }                                                                              \
    } while (0)

__device__ __forceinline__ void st_agent(unsigned long long* p, unsigned long long v)
{
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned long long ld_agent(const unsigned long long* p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_flag(unsigned* p, unsigned v)
{
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned ld_flag(const unsigned* p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// blocks 0 and `partner` play; every other block exits at once.  buf: [2][words] payloads,
// flags: [2] (one line each), out: [0] errors, [1] cycles of block 0.
__global__ __launch_bounds__(1024) void pingpong(unsigned long long* buf, unsigned* flags, int words, int rounds,
                                               int partner, unsigned long long* out)
{
    const int b = blockIdx.x;
    if (b != 0 && b != partner) return;
    const int me = b == 0 ? 0 : 1, other = 1 - me;
    unsigned long long* mine = buf + (long long)me * words;
    const unsigned long long* theirs = buf + (long long)other * words;
    unsigned* myflag = flags + 32 * me;
    const unsigned* theirflag = flags + 32 * other;
    unsigned long long errors = 0;
    const long long t0 = wall_clock64();
    for (int r = 1; r <= rounds; r++) {
        if (me == 1 || r > 1) {
            // wait for the partner's round (block 1 answers round r, block 0 waits for round r - 1)
            const unsigned want = me == 1 ? (unsigned)r : (unsigned)(r - 1);
            if (threadIdx.x == 0)
                while (ld_flag(theirflag) != want) __builtin_amdgcn_s_sleep(0);
            __syncthreads();
            const unsigned long long tag = (unsigned long long)want << 32;
            for (int i = threadIdx.x; i < words; i += blockDim.x)
                if (ld_agent(theirs + i) != (tag | (unsigned)i)) errors++;
        }
        if (me == 0 || r <= rounds) {
            const unsigned long long tag = (unsigned long long)r << 32;
            for (int i = threadIdx.x; i < words; i += blockDim.x) st_agent(mine + i, tag | (unsigned)i);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (threadIdx.x == 0) st_flag(myflag, (unsigned)r);
        }
    }
    if (me == 0) {
        // the last answer
        if (threadIdx.x == 0)
            while (ld_flag(theirflag) != (unsigned)rounds) __builtin_amdgcn_s_sleep(0);
        __syncthreads();
    }
    const long long t1 = wall_clock64();
    if (errors) atomicAdd(out, errors);
    if (me == 0 && threadIdx.x == 0) out[1] = (unsigned long long)(t1 - t0);
}

int main()
{
    int wall_khz = 0;
    CHECK(hipDeviceGetAttribute(&wall_khz, hipDeviceAttributeWallClockRate, 0));
    const int rounds = 2000;
    unsigned long long *buf, *out;
    unsigned* flags;
    const int max_words = 30 * 1024 / 8;
    CHECK(hipMalloc(&buf, 2 * max_words * sizeof(unsigned long long)));
    CHECK(hipMalloc(&flags, 64 * sizeof(unsigned)));
    CHECK(hipMalloc(&out, 2 * sizeof(unsigned long long)));
    const int sizes[] = {8, 2048, 30 * 1024};
    const int partners[] = {1, 8};
    const int threads[] = {64, 1024};
    for (int nt : threads)
    for (int s : sizes)
        for (int partner : partners) {
            const int words = s / 8;
            for (int rep = 0; rep < 2; rep++) {  // the first run warms the code object and the lines
                CHECK(hipMemset(flags, 0, 64 * sizeof(unsigned)));
                CHECK(hipMemset(out, 0, 2 * sizeof(unsigned long long)));
                CHECK(hipMemset(buf, 0, 2 * max_words * sizeof(unsigned long long)));
                pingpong<<<dim3(16), dim3(nt)>>>(buf, flags, words, rounds, partner, out);
                CHECK(hipGetLastError());
                CHECK(hipDeviceSynchronize());
            }
            unsigned long long h[2];
            CHECK(hipMemcpy(h, out, sizeof(h), hipMemcpyDeviceToHost));
            const double us = (double)h[1] / (wall_khz * 1e-3) / (2.0 * rounds);
            std::printf("{\"threads\": %d, \"payload_bytes\": %d, \"partner_block\": %d, \"one_way_hop_us\": %.3f, \"errors\": %llu}\n",
                        nt, s, partner, us, h[0]);
            std::fflush(stdout);
        }
    CHECK(hipFree(buf));
    CHECK(hipFree(flags));
    CHECK(hipFree(out));
    return 0;
}
