// match.hip — two-way brute-force Hamming matching on MI355X (gfx950).  Replaces Match and
// GetDescriptorDistance (Core/MAGESLAM/Source/Tracking/FeatureMatcher.cpp:61-190, 453-504); the
// reference builds two N x N float distance matrices with cv::BFMatcher::radiusMatch twice.
//
// The distance matrix is a GEMM: with s(x) = 1 - 2x per bit, sum_k s(a_k) s(b_k) = 256 - 2 d(a, b).
// Descriptors are expanded to +-1 int8 and multiplied with v_mfma_i32_32x32x32_i8 (8 MFMAs per
// 32 x 32 block of pairs, K = 256); the VALU only turns each result into packed keys and keeps
// the two best per row and per column.  One workgroup (8 waves) per (A, B) frame pair, nothing
// materialised in HBM:
//   * 8 waves; each owns two 32-row tiles per pass, their +-1 operands stay in VGPRs; the MFMAs
//     of one row tile are in flight while the VALU folds the other (software pipeline);
//   * B is expanded in 64-column stages into LDS (double buffered, one barrier per stage) in the
//     exact per-lane operand order, so every wave reads it with conflict-free ds_read_b128;
//   * keys are (D << 15 | 0x7FFF - index) with D = 256 - 2d, so "larger key" = smaller distance,
//     then lower index (the canonical tie order); the two largest keys over ALL
//     columns give radiusMatch's best and second best whenever they lie within the radius
//     (FeatureMatcher.cpp:117-137), so no per-pair radius mask is needed;
//   * row (best, second) live per lane and register and are reduce-scattered across the 32
//     lanes of a half-wave once per pass; column (best, second) are reduced over the lane's 16
//     rows and its partner half, then merged across waves with two LDS atomicMax (no CAS loop:
//     every key that loses or is displaced in the best slot is pushed into the second slot).
// The cross-check (best(a) = b and best(b) = a, FeatureMatcher.cpp:158) and the ordered DMatch
// compaction run in the same launch.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cstring>
#include <vector>

#include "common.hpp"

namespace mage {
namespace {

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v8i __attribute__((ext_vector_type(8)));
typedef int v16i __attribute__((ext_vector_type(16)));
typedef float v16f __attribute__((ext_vector_type(16)));

constexpr int MW = 8;          // waves per workgroup (2 per SIMD)
constexpr int MT = MW * kWave; // threads per workgroup
constexpr int RT = 2;          // 32-row tiles per wave per pass
constexpr int ROWS = MW * RT * 32;  // A rows per pass
constexpr int SC = MT / 8;     // B columns per LDS stage (32-column tiles, one fill item per thread)
constexpr int NMAX = 4096;     // max descriptors per side (states in LDS)
constexpr int NBUF = 3;        // B stage buffers
constexpr int NONE = INT_MIN;  // empty key
static_assert(SC * 8 == MT, "one stage-fill item per thread");

struct MatchParams {
    int max_dist, min_diff;
    unsigned out_cap;
    long long a_pitch, b_pitch;  // bytes between pairs
    int2* rows;                  // per pair NMAX (best, second) row keys
};

__device__ __forceinline__ int med3(int a, int b, int c)
{
    int r;
    asm volatile("v_med3_i32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

// (m1, m2) = the two largest keys seen; m1 >= m2 always.
__device__ __forceinline__ void push2(int& m1, int& m2, int k)
{
    m2 = med3(m1, m2, k);
    m1 = max(m1, k);
}

__device__ __forceinline__ void merge2(int& m1, int& m2, int o1, int o2)
{
    const int lo = min(m1, o1);
    m1 = max(m1, o1);
    m2 = max(max(lo, m2), o2);
}

__device__ __forceinline__ int key_dist(int k) { return (256 - (k >> 15)) >> 1; }
__device__ __forceinline__ int key_index(int k) { return 0x7FFF - (k & 0x7FFF); }

// Row/column acceptance of FeatureMatcher.cpp:125-137 on (best, second) keys.
__device__ __forceinline__ bool accept(int m1, int m2, int maxDist, int minDiff)
{
    if (m1 == NONE) return false;
    const int d0 = key_dist(m1);
    if (d0 > maxDist) return false;
    if (m2 != NONE) {
        const int d1 = key_dist(m2);
        if (d1 <= maxDist && d1 - d0 < minDiff) return false;
    }
    return true;
}

// 16 descriptor bits -> 16 bytes of c * s(bit), s = +1 / -1; byte b <-> bit b.  TAB holds the
// two byte values (+c in byte 0, -c in byte 1) that v_perm_b32 selects from.
template <uint32_t TAB>
__device__ __forceinline__ v4i expand16(uint32_t w)
{
    v4i r;
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const uint32_t t = (w >> (4 * q)) & 0xFu;
        const uint32_t x = (t * 0x00204081u) & 0x01010101u;  // bit i -> byte i
        r[q] = (int)__builtin_amdgcn_perm(0u, TAB, x);
    }
    return r;
}

// 32 descriptor bits -> 32 fp4 (e2m1) elements s(bit) = +1 (0x2) / -1 (0xA), element j in
// nibble j (low nibble first) of the 16 bytes.  Per output dword (byte q of w): the even and odd
// bits of the byte are spread to the byte LSBs (multiply by 1 + 2^6 + 2^12 + 2^18: bit 2m lands at
// 8m, the colliding sums at 6 / 12 / 18 carry only into bits the mask drops), and v_perm picks
// one of the four two-element bytes {0x22, 0x2A, 0xA2, 0xAA}.
__device__ __forceinline__ v4i expand32_fp4(uint32_t w)
{
    const uint32_t E = w & 0x55555555u, O = (w >> 1) & 0x55555555u;
    v4i r;
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const uint32_t xe = (((E >> (8 * q)) & 0xFFu) * 0x00041041u) & 0x01010101u;
        const uint32_t xo = (((O >> (8 * q)) & 0xFFu) * 0x00041041u) & 0x01010101u;
        r[q] = (int)__builtin_amdgcn_perm(0u, 0xAAA22A22u, xe | (xo << 1));
    }
    return r;
}

// Row offset (within a 32-row tile, lane half 0) of accumulator register g of a 32x32 MFMA.
__host__ __device__ constexpr int acc_row(int g) { return (g & 3) + 8 * (g >> 2); }

// D = 256 - 2d for the wave's 32 rows x one 32-column B tile: 8 chained i8 MFMAs over K = 256.
__device__ __forceinline__ v16i tile_mfma_i8(const v4i (&a)[8], const v4i (&b)[8])
{
    v16i acc = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int s = 0; s < 8; s++) acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[s], b[s], acc, 0, 0, 0);
    return acc;
}

// The same product on the MX fp4 MFMA (K = 64 per instruction: 4 instead of 8, half the matrix
// cycles).  Elements are +-1 with E8M0 block scales 2^-11 (A) and 2^-10 (B), so each bit
// contributes +-2^-21 and the sum is x = 2^-20 (128 - d).  The accumulator starts at the inline
// constant C0 = 1/(2 pi) (f32 0x3E22F983, no register set to initialise per tile): C0 + x stays in
// C0's binade [1/8, 1/4) (|x| <= 2^-13), whose ulp is 2^-26, and every partial sum is C0 plus a
// multiple of 2^-21, so the result is exact and its bit pattern is 0x3E22F983 + 64 (128 - d).
// The low 16 bits, read as i16, are 64 (128 - d - FP4_K0) + 3 (0xF983 + [-8192, 8192] stays
// within [32768, 98304), so the wrap is the same for every d): monotone in d, low 6 bits = 3.
constexpr int FP4_K0 = 26;  // (0x10000 - 0xF983 + 3) / 64
__device__ __forceinline__ v16i tile_mfma_fp4(const v4i (&a)[8], const v4i (&b)[8])
{
    v16f acc;
#pragma unroll
    for (int g = 0; g < 16; g++) acc[g] = 0.15915494309189535f;  // 1 / (2 pi): inline constant
#pragma unroll
    for (int s = 0; s < 4; s++) {
        const v8i av = {a[s][0], a[s][1], a[s][2], a[s][3], 0, 0, 0, 0};
        const v8i bv = {b[s][0], b[s][1], b[s][2], b[s][3], 0, 0, 0, 0};
        acc = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(av, bv, acc, 4, 4, 0, 127 - 11, 0, 127 - 10);
    }
    return __builtin_bit_cast(v16i, acc);
}

template <int KS>
__device__ __forceinline__ void load_frags(v4i (&b)[8], const v4i* __restrict__ bt, int lane)
{
#pragma unroll
    for (int s = 0; s < KS; s++) b[s] = bt[s * kWave + lane];
}

// The value of lane l ^ 32 (v_permlane32_swap: a VALU exchange, no LDS round trip).
__device__ __forceinline__ int xor32(int x, int lane)
{
    const auto r = __builtin_amdgcn_permlane32_swap((unsigned)x, (unsigned)x, false, false);
    return (int)(lane < 32 ? r[1] : r[0]);
}

// A column flush whose second atomic is still to be issued (flush_finish).
struct PendingCol {
    int j, c1, c2, old;
    bool live;
};

// Column partial of one B tile, as global keys (D << 15 | 0x7FFF - i), merged with the partner
// half-wave, then into the workgroup's column top-2 with two LDS atomicMax (no CAS loop: a key
// that loses, or is displaced from, the best slot is pushed into the second slot).  The second
// atomic needs the first one's return value; it is issued later (flush_finish, after the next
// fold) so the LDS round trip overlaps VALU work.
__device__ __forceinline__ PendingCol flush_global(int c1, int c2, int lane, int colbase, int nb, int* colM1)
{
    merge2(c1, c2, xor32(c1, lane), xor32(c2, lane));
    PendingCol pc;
    pc.j = colbase + (lane & 31);
    pc.c1 = c1;
    pc.c2 = c2;
    pc.live = (lane >> 5) == 0 && pc.j < nb && c1 != NONE;
    pc.old = pc.live ? atomicMax(&colM1[pc.j], c1) : NONE;
    return pc;
}

__device__ __forceinline__ void flush_finish(PendingCol& pc, int* colM2)
{
    if (pc.live) atomicMax(&colM2[pc.j], pc.old > pc.c1 ? pc.c1 : max(pc.old, pc.c2));
    pc.live = false;
}

// 32-bit keys: operands s = +-1, D = 256 - 2d.  Row keys (D << 15 | 0x7FFF - j); column
// partials hold local keys (D << 6 | 63 - wave row).  Any nb <= NMAX.  PADMASK: padding rows and
// columns are masked (needed only when maxDist >= 128, see fold_any).
template <bool PADMASK>
struct Keys32 {
    // i8 operands: k-step s = descriptor dword s, lane half h = its 16-bit half h
    static constexpr int KS = 8;
    static __device__ __forceinline__ v4i a_frag(const uint32_t (&dw)[8], int half, int s)
    {
        return expand16<0x0000FF01u>(half ? (dw[s] >> 16) : (dw[s] & 0xFFFFu));
    }
    static __device__ __forceinline__ void fill(v4i (*tile)[kWave], int fs, int c, uint32_t dw, bool ok)
    {
        const v4i zero = {0, 0, 0, 0};
        tile[fs][c] = ok ? expand16<0x0000FF01u>(dw & 0xFFFFu) : zero;
        tile[fs][32 + c] = ok ? expand16<0x0000FF01u>(dw >> 16) : zero;
    }
    static __device__ __forceinline__ v16i tile_mfma(const v4i (&a)[8], const v4i (&b)[8]) { return tile_mfma_i8(a, b); }
    struct Rows {
        int r1[RT][16], r2[RT][16];
    };
    struct Part {
        int c1, c2;
    };
    static __device__ __forceinline__ void init(Rows& r)
    {
#pragma unroll
        for (int rt = 0; rt < RT; rt++)
#pragma unroll
            for (int g = 0; g < 16; g++) r.r1[rt][g] = r.r2[rt][g] = NONE;
    }
    static __device__ __forceinline__ void reset(Part& c) { c.c1 = c.c2 = NONE; }

    template <bool MASK>
    static __device__ __forceinline__ void fold_m(const v16i& acc, int rt, int lane, int colbase, int nb, int rowbase,
                                                  int na, Rows& R, Part& C)
    {
        const int h = lane >> 5;
        const int j = colbase + (lane & 31);
        const int jc = 0x7FFF - j;
#pragma unroll
        for (int g = 0; g < 16; g++) {
            const int D = acc[g];
            int kr = (D << 15) | jc;
            int kc = (D << 6) | (63 - (rt * 32 + acc_row(g)));
            if (MASK) {
                if (j >= nb) kr = NONE;
                if (rowbase + rt * 32 + acc_row(g) + 4 * h >= na) kc = NONE;
            }
            push2(R.r1[rt][g], R.r2[rt][g], kr);
            push2(C.c1, C.c2, kc);
        }
    }
    // Padding rows and columns have zero operands, so D = 0 (d = 128) there: such a key can
    // neither be accepted (d0 <= maxDist) nor hide an in-radius second best while maxDist <
    // 128, so for those radii (every practical one) the fold needs no masks.
    static __device__ __forceinline__ void fold(const v16i& acc, int rt, int lane, int colbase, int nb, int rowbase,
                                                int na, Rows& R, Part& C)
    {
        if (PADMASK && (colbase + 32 > nb || rowbase + RT * 32 > na))
            fold_m<true>(acc, rt, lane, colbase, nb, rowbase, na, R, C);
        else
            fold_m<false>(acc, rt, lane, colbase, nb, rowbase, na, R, C);
    }
    static __device__ __forceinline__ PendingCol flush(const Part& C, int lane, int colbase, int nb, int rowbase,
                                                       int* colM1)
    {
        const int ib = rowbase + 4 * (lane >> 5) + 63;
        int c1 = C.c1, c2 = C.c2;
        if (c1 != NONE) c1 = ((c1 >> 6) << 15) | (0x7FFF - (ib - (c1 & 63)));
        if (c2 != NONE) c2 = ((c2 >> 6) << 15) | (0x7FFF - (ib - (c2 & 63)));
        return flush_global(c1, c2, lane, colbase, nb, colM1);
    }
    // row state q = rt * 16 + g as global keys
    static __device__ __forceinline__ void export_rows(const Rows& R, int lane, int (&s1)[RT * 16], int (&s2)[RT * 16])
    {
#pragma unroll
        for (int q = 0; q < RT * 16; q++) {
            s1[q] = R.r1[q >> 4][q & 15];
            s2[q] = R.r2[q >> 4][q & 15];
        }
    }
};

// Packed 16-bit keys, two accumulator registers per VGPR: the low 16 bits of the fp4 MFMA result
// (tile_mfma_fp4) are (128 - d - FP4_K0) << 6 | 3.  Row keys ((128 - d - FP4_K0) << 6 | 63 - tile),
// column keys ((128 - d - FP4_K0) << 6 | 63 - wave row): the index replaces the 3 by one XOR;
// both top-2 updates are v_pk_max_i16 / v_pk_min_i16 on two elements at once.  Requires nb <= 2048 (64 tiles) and maxDist < 128.
struct Keys16 {
    // fp4 operands: k-step s = descriptor dwords 2s (lane half 0) and 2s + 1 (half 1)
    static constexpr int KS = 4;
    static __device__ __forceinline__ v4i a_frag(const uint32_t (&dw)[8], int half, int s)
    {
        return expand32_fp4(half ? dw[2 * s + 1] : dw[2 * s]);
    }
    static __device__ __forceinline__ void fill(v4i (*tile)[kWave], int fs, int c, uint32_t dw, bool ok)
    {
        const v4i zero = {0, 0, 0, 0};
        tile[fs >> 1][32 * (fs & 1) + c] = ok ? expand32_fp4(dw) : zero;
    }
    static __device__ __forceinline__ v16i tile_mfma(const v4i (&a)[8], const v4i (&b)[8]) { return tile_mfma_fp4(a, b); }
    static constexpr uint32_t NONE2 = 0x80008000u;
    struct Rows {
        uint32_t r1[RT][8], r2[RT][8];
    };
    struct Part {
        uint32_t c1, c2;
    };
    typedef short s16x2 __attribute__((ext_vector_type(2)));
    static __device__ __forceinline__ uint32_t pmax(uint32_t a, uint32_t b)
    {
        return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(s16x2, a), __builtin_bit_cast(s16x2, b)));
    }
    static __device__ __forceinline__ uint32_t pmin(uint32_t a, uint32_t b)
    {
        return __builtin_bit_cast(uint32_t, __builtin_elementwise_min(__builtin_bit_cast(s16x2, a), __builtin_bit_cast(s16x2, b)));
    }
    static __device__ __forceinline__ void init(Rows& r)
    {
#pragma unroll
        for (int rt = 0; rt < RT; rt++)
#pragma unroll
            for (int q = 0; q < 8; q++) r.r1[rt][q] = r.r2[rt][q] = NONE2;
    }
    static __device__ __forceinline__ void reset(Part& c) { c.c1 = c.c2 = NONE2; }
    static __device__ __forceinline__ void fold(const v16i& acc, int rt, int lane, int colbase, int nb, int rowbase,
                                                int na, Rows& R, Part& C)
    {
        const uint32_t tpair = ((uint32_t)(63 - (colbase >> 5)) ^ 3u) * 0x00010001u;
#pragma unroll
        for (int q = 0; q < 8; q++) {
            const uint32_t P = __builtin_amdgcn_perm((uint32_t)acc[2 * q + 1], (uint32_t)acc[2 * q], 0x05040100u);
            const uint32_t kr = P ^ tpair;
            R.r2[rt][q] = pmax(R.r2[rt][q], pmin(R.r1[rt][q], kr));
            R.r1[rt][q] = pmax(R.r1[rt][q], kr);
            const uint32_t rc = ((uint32_t)(63 - (rt * 32 + acc_row(2 * q))) ^ 3u) |
                                (((uint32_t)(63 - (rt * 32 + acc_row(2 * q + 1))) ^ 3u) << 16);
            const uint32_t kc = P ^ rc;
            C.c2 = pmax(C.c2, pmin(C.c1, kc));
            C.c1 = pmax(C.c1, kc);
        }
    }
    static __device__ __forceinline__ int lo16(uint32_t v) { return (int)(short)(v & 0xFFFFu); }
    static __device__ __forceinline__ int hi16(uint32_t v) { return (int)v >> 16; }
    static __device__ __forceinline__ PendingCol flush(const Part& C, int lane, int colbase, int nb, int rowbase,
                                                       int* colM1)
    {
        // merge the even / odd register halves, then local -> global keys
        int m1 = lo16(C.c1), m2 = lo16(C.c2);
        merge2(m1, m2, hi16(C.c1), hi16(C.c2));
        const int ib = rowbase + 4 * (lane >> 5) + 63;
        int c1 = m1 == -32768 ? NONE : (((m1 >> 6) + FP4_K0) << 16) | (0x7FFF - (ib - (m1 & 63)));
        int c2 = m2 == -32768 ? NONE : (((m2 >> 6) + FP4_K0) << 16) | (0x7FFF - (ib - (m2 & 63)));
        return flush_global(c1, c2, lane, colbase, nb, colM1);
    }
    static __device__ __forceinline__ int row_global(int k, int lane)
    {
        if (k == -32768) return NONE;
        const int j = (63 - (k & 63)) * 32 + (lane & 31);
        return (((k >> 6) + FP4_K0) << 16) | (0x7FFF - j);
    }
    static __device__ __forceinline__ void export_rows(const Rows& R, int lane, int (&s1)[RT * 16], int (&s2)[RT * 16])
    {
#pragma unroll
        for (int rt = 0; rt < RT; rt++)
#pragma unroll
            for (int q = 0; q < 8; q++) {
                s1[rt * 16 + 2 * q] = row_global(lo16(R.r1[rt][q]), lane);
                s1[rt * 16 + 2 * q + 1] = row_global(hi16(R.r1[rt][q]), lane);
                s2[rt * 16 + 2 * q] = row_global(lo16(R.r2[rt][q]), lane);
                s2[rt * 16 + 2 * q + 1] = row_global(hi16(R.r2[rt][q]), lane);
            }
    }
};

// All row passes of one (A, B) pair.  RES: the packed B descriptors are resident in LDS (Bres),
// so the stage loop issues no global loads (hipcc drains vmcnt(0) at the first use of any
// global-load result, which would expose a full L2/HBM round trip per stage); otherwise each
// stage's B words are fetched from global one stage ahead (nb > NRES only).
template <class K, bool RES>
__device__ __forceinline__ void row_passes(const uint32_t* __restrict__ Aw, const uint32_t* __restrict__ Bw,
                                           const uint32_t* Bres, int na, int nb,
                                           v4i (*stage)[SC / 32][8][kWave], int* colM1, int* colM2,
                                           int2* __restrict__ rows)
{
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int nstages = (nb + SC - 1) / SC;
    // stage-fill item of this thread: k-step s, column c of the stage
    const int fs = tid / SC, fc = tid % SC;
    auto fetch = [&](int st) -> uint32_t {
        const int j = min(st * SC + fc, nb - 1);
        return RES ? Bres[8 * j + fs] : Bw[8 * j + fs];
    };
    auto fill = [&](int buf, int st, uint32_t dw) {
        // padding columns: zero operands
        K::fill(stage[buf][fc >> 5], fs, fc & 31, dw, st * SC + fc < nb);
    };

    for (int pb = 0; pb < na; pb += ROWS) {
        const int rowbase = pb + wave * (RT * 32);
        const bool active = rowbase < na;
        v4i a[RT][8];
        typename K::Rows R;
        K::init(R);
#pragma unroll
        for (int rt = 0; rt < RT; rt++) {
            const int i = rowbase + rt * 32 + (lane & 31);
            const int ic = min(i, na - 1);
            uint32_t dw[8];
#pragma unroll
            for (int s = 0; s < 8; s++) dw[s] = Aw[8 * ic + s];
#pragma unroll
            for (int s = 0; s < K::KS; s++) {
                a[rt][s] = K::a_frag(dw, lane >> 5, s);
                if (i >= na) a[rt][s] = v4i{0, 0, 0, 0};  // padding rows: zero operands
            }
        }
        {
            const uint32_t w0 = fetch(0), w1 = nstages > 1 ? fetch(1) : 0u;
            __syncthreads();  // column states / Bres ready; previous pass done with the stages
            fill(0, 0, w0);
            if (nstages > 1) fill(1, 1, w1);
            __syncthreads();
        }
        // Software pipeline over the pass's B tiles t (stage st + 2 is filled during stage st,
        // three buffers):  MFMA(t, rows 0-31) | fold(t-1, rows 32-63) + column flush(t-1) |
        // MFMA(t, rows 32-63) | fragments of t+1 | fold(t, rows 0-31).
        v4i bf[8];
        load_frags<K::KS>(bf, &stage[0][0][0][0], lane);
        v16i acc1;
        int cbp = -1;
        PendingCol pc{0, 0, 0, 0, false};
        typename K::Part C;
        K::reset(C);
        for (int st = 0; st < nstages; st++) {
            const int buf = st % NBUF;
            uint32_t nxt = 0;
            if (st + 2 < nstages) nxt = fetch(st + 2);
            if (active) {
#pragma unroll
                for (int ct = 0; ct < SC / 32; ct++) {
                    const int colbase = st * SC + ct * 32;
                    if (colbase >= nb) break;
                    const v16i acc0 = K::tile_mfma(a[0], bf);
                    if (cbp >= 0) {
                        K::fold(acc1, 1, lane, cbp, nb, rowbase, na, R, C);
                        pc = K::flush(C, lane, cbp, nb, rowbase, colM1);
                    }
                    acc1 = K::tile_mfma(a[1], bf);
                    if (ct + 1 < SC / 32 && colbase + 32 < nb)
                        load_frags<K::KS>(bf, &stage[buf][ct + 1][0][0], lane);
                    else if (st + 1 < nstages)
                        load_frags<K::KS>(bf, &stage[(st + 1) % NBUF][0][0][0], lane);
                    K::reset(C);
                    K::fold(acc0, 0, lane, colbase, nb, rowbase, na, R, C);
                    flush_finish(pc, colM2);
                    cbp = colbase;
                }
            }
            if (st + 2 < nstages) fill((st + 2) % NBUF, st + 2, nxt);
            __syncthreads();
        }
        if (active) {
            if (cbp >= 0) {
                K::fold(acc1, 1, lane, cbp, nb, rowbase, na, R, C);
                pc = K::flush(C, lane, cbp, nb, rowbase, colM1);
                flush_finish(pc, colM2);
            }
            // reduce-scatter the 32 row states (row tile q >> 4, register q & 15) over the 32
            // lanes of each half: lane c ends with state q = c.
            int s1[RT * 16], s2[RT * 16];
            K::export_rows(R, lane, s1, s2);
#pragma unroll
            for (int m = 16, n = 32; m >= 1; m >>= 1, n >>= 1) {
                const bool up = (lane & m) != 0;
                const int hf = n / 2;
#pragma unroll
                for (int k = 0; k < hf; k++) {
                    const int send1 = up ? s1[k] : s1[k + hf], send2 = up ? s2[k] : s2[k + hf];
                    int m1 = up ? s1[k + hf] : s1[k], m2 = up ? s2[k + hf] : s2[k];
                    merge2(m1, m2, __shfl_xor(send1, m), __shfl_xor(send2, m));
                    s1[k] = m1;
                    s2[k] = m2;
                }
            }
            const int c = lane & 31;
            const int i = rowbase + (c >> 4) * 32 + acc_row(c & 15) + 4 * (lane >> 5);
            if (i < na) rows[i] = make_int2(s1[0], s2[0]);
        }
    }
}

constexpr int NRES = 2560;  // B descriptors kept resident in LDS up to this count

// ------------------------------------------------------------------------------------------
// fp4 matcher (nb <= 2048, maxDist < 128, minDiff >= 1: every practical call, C2 included).
//
// 8 waves (2 per SIMD, 249 VGPRs), four 32-row A tiles each per pass; one column flush (partner
// half, LDS atomics) per two tiles (64 rows: the 6-bit row code).  2000 rows are 63 row tiles:
// 8 waves x 4 run them in 2 passes with one wave slot idle (98 % of the slots busy), 12 x 2 in 3
// passes with 9 idle (88 %).  Measured on C2 (tools/abl.py, 256 pairs, one box): 12 x 2 0.234-0.240
// ms, 8 x 4 0.227-0.229 (8 x 4 with 4 / 1 fill columns per thread 0.229 / 0.230, 16 x 2 0.288
// (4 waves per SIMD: spills), 4 x 8 0.341); round 5: 16 x 1 0.277, 8 x 2 0.261.  Per 32x32 tile a
// lane folds 16 accumulator values:
//   * the accumulator starts at C = 1/8 + (0x2400 + code) ulp (per-lane constant registers, code =
//     63 - the lane's row in the tile), so the result's low 16 bits are the packed key
//     64 (272 - d) + code, a positive i16 (and positive normal f16), exact: see tile_mfma_fp4;
//   * column keys need the row -> the code is already there (no XOR);
//   * row states keep only the two best *distances* (the code is the same constant for every
//     tile a register sees), so the row side needs no index at all: with minDiff >= 1 an
//     accepted row has a unique best column, and (i, j) is a match iff row i is accepted with
//     best distance d0, column j is accepted with best row i, and d(i, j) = d0 — the column
//     states (which carry the row index) identify j.  Same result as the reference's two
//     radiusMatch calls + cross-check (FeatureMatcher.cpp:117-167) whenever ties are rejected.
// ------------------------------------------------------------------------------------------
#ifndef MAGE_FP4_WAVES
#define MAGE_FP4_WAVES 8
#endif
constexpr int FW = MAGE_FP4_WAVES;   // waves
constexpr int FT = FW * kWave;       // 512 threads
#ifndef MAGE_FP4_RT
#define MAGE_FP4_RT 4
#endif
constexpr int FRT = MAGE_FP4_RT;     // 32-row A tiles per wave per pass (the column flush serves all)
constexpr int FROWS = FW * 32 * FRT; // A rows per pass
#ifndef MAGE_FP4_FCOLS
#define MAGE_FP4_FCOLS 2  // B columns filled per thread per stage: 2 = twice the columns per barrier, two
                          // stage buffers (C2 match 0.235 -> 0.231 ms; LDS 127 -> 139 KB)
#endif
constexpr int FCOLS = MAGE_FP4_FCOLS;
constexpr int FSC1 = FT / 8;         // columns one fill dword per thread covers
constexpr int FSC = FCOLS * FSC1;    // B columns per LDS stage
constexpr int FNT = FSC / 32;        // column tiles per stage
constexpr int FNB = 2048;            // max B descriptors
constexpr int FNA = 4096;            // max A descriptors
constexpr int FBUF = FCOLS == 1 ? 3 : 2;  // stage buffers (LDS: 160 KB per CU)
constexpr int FPF = FBUF - 1;        // stages filled ahead
constexpr uint32_t K16_BASE = 0x2400u;  // low-16 mantissa offset of the accumulator start
constexpr int K16_D = 272;           // key >> 6 = K16_D - d
constexpr uint32_t NONE16 = 0x80008000u;
#ifndef MAGE_FP4_GATE
// 1: skip the fold of 32x32 tiles with no key within maxDist (a v_max3 tree + one ballot per
// tile), adaptively: a wave stops gating once more than a quarter of its tiles (after 64) held a
// candidate.  Exact either way, but off: measured (tools/abl.py, 256 C2 pairs) the always-on gate
// costs 0.229 -> 0.267 ms, the adaptive one 0.253 (half-density cut-off) / 0.256 (quarter) — the
// fold is not what bounds the kernel once the gate's branch breaks the overlap of the MFMAs with
// the fold — while rBRIEF-31's sparser candidates would gain 0.23 -> 0.16 ms.
#define MAGE_FP4_GATE 0
#endif

typedef short s16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pkmax(uint32_t a, uint32_t b)
{
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(s16x2, a), __builtin_bit_cast(s16x2, b)));
}
__device__ __forceinline__ uint32_t pkmin(uint32_t a, uint32_t b)
{
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_min(__builtin_bit_cast(s16x2, a), __builtin_bit_cast(s16x2, b)));
}
// Three-input max of packed keys on the f16 path (v_pk_maximum3_f16): keys are positive normal
// f16 values and NONE16 is -0, so the f16 order is the i16 order on every value that occurs.
typedef _Float16 h16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pkmax3(uint32_t a, uint32_t b, uint32_t c)
{
    const h16x2 m = __builtin_elementwise_maximum(__builtin_bit_cast(h16x2, a), __builtin_bit_cast(h16x2, b));
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_maximum(m, __builtin_bit_cast(h16x2, c)));
}
__device__ __forceinline__ int lo16s(uint32_t v) { return (int)(short)(v & 0xFFFFu); }
__device__ __forceinline__ int hi16s(uint32_t v) { return (int)v >> 16; }

// The fp4 product of the wave's 32 rows and one 32-column B tile, accumulated onto cc (the
// per-lane code registers).  Elements are +-1 with E8M0 scales 2^-11 (A) and 2^-10 (B): each bit
// adds +-2^-21 = +-32 ulp of the binade [1/8, 1/4), the total is (128 - d) 64 ulp with |.| <=
// 2^-13, and cc = 1/8 + (0x2400 + code) ulp keeps every partial sum inside the binade: exact, and
// the low 16 bits are 0x2400 + code + 64 (128 - d) = 64 (272 - d) + code in [0x0400, 0x643F].
__device__ __forceinline__ v16f tile_mfma_k16(const v4i (&a)[4], const v4i (&b)[4], const v16f& cc)
{
    v16f acc = cc;
#pragma unroll
    for (int s = 0; s < 4; s++) {
        const v8i av = {a[s][0], a[s][1], a[s][2], a[s][3], 0, 0, 0, 0};
        const v8i bv = {b[s][0], b[s][1], b[s][2], b[s][3], 0, 0, 0, 0};
        acc = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(av, bv, acc, 4, 4, 0, 127 - 11, 0, 127 - 10);
    }
    return acc;
}

// A pending column flush (the second LDS atomic needs the first one's return value; it is issued
// after the next tile's fold so the round trip overlaps VALU work).
struct PendingCol16 {
    int j, c1, c2, old;
    bool live;
};

__global__ __launch_bounds__(FT) void match_fp4_kernel(const uint8_t* __restrict__ A, const uint32_t* __restrict__ nA,
                                                       const uint8_t* __restrict__ B, const uint32_t* __restrict__ nB,
                                                       MatchParams p, mage_dmatch* __restrict__ out,
                                                       uint32_t* __restrict__ n_out, uint32_t* __restrict__ status)
{
    __shared__ v4i stage[FBUF][FNT][4][kWave];          // [buffer][tile][k-step][lane] fp4 operands
    __shared__ __attribute__((aligned(16))) uint32_t bres[FNB * 8];  // packed B
    __shared__ int colM1[FNB], colM2[FNB];             // column (best, second) global keys
    __shared__ uint16_t rowd[FNA];                     // accepted row: best distance, else 0xFFFF
    __shared__ uint32_t wsum[FW];
    uint16_t* matchOf = reinterpret_cast<uint16_t*>(&stage[0][0][0][0]);  // after the passes
    static_assert(sizeof(stage) >= FNA * sizeof(uint16_t), "matchOf aliases the stages");

    const int pair = blockIdx.x;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int na = (int)nA[pair], nb = (int)nB[pair];
    if (na > FNA || nb > FNB) {
        if (tid == 0) {
            atomicOr(status, 1u);
            n_out[pair] = 0;
        }
        return;
    }
    const int maxDist = p.max_dist, minDiff = p.min_diff;
    const uint32_t* Aw = reinterpret_cast<const uint32_t*>(A + pair * p.a_pitch);
    const uint32_t* Bw = reinterpret_cast<const uint32_t*>(B + pair * p.b_pitch);
    for (int j = tid; j < nb; j += FT) {
        colM1[j] = NONE;
        colM2[j] = NONE;
    }
    if (na > 0 && nb > 0) {
        for (int k = tid; k < 2 * nb; k += FT) reinterpret_cast<uint4*>(bres)[k] = reinterpret_cast<const uint4*>(Bw)[k];
    }
    // B resident before the first pass's stage fetches read it (other threads' rows; without this
    // barrier a fetch could read a row not yet written: test_match_random[513-64] caught it)
    __syncthreads();
    // per-lane accumulator start: register g holds tile row acc_row(g) + 4 h, code 63 - row
    v16f cc;
#pragma unroll
    for (int g = 0; g < 16; g++)
        cc[g] = __builtin_bit_cast(float, (124u << 23) | (K16_BASE + (uint32_t)(63 - acc_row(g) - 4 * (lane >> 5))));
    const int nstages = (nb + FSC - 1) / FSC;
    const int fs = tid / FSC1, fc0 = tid % FSC1;  // stage-fill items: descriptor dword fs of columns fc0 + k FSC1
    struct Fetch {
        uint32_t dw[FCOLS];
    };
    auto fetch = [&](int st) -> Fetch {
        Fetch f;
#pragma unroll
        for (int k = 0; k < FCOLS; k++) f.dw[k] = bres[8 * min(st * FSC + fc0 + k * FSC1, nb - 1) + fs];
        return f;
    };
    auto fill = [&](int buf, int st, const Fetch& f) {
        const v4i zero = {0, 0, 0, 0};
#pragma unroll
        for (int k = 0; k < FCOLS; k++) {
            const int fc = fc0 + k * FSC1;
            stage[buf][fc >> 5][fs >> 1][32 * (fs & 1) + (fc & 31)] = st * FSC + fc < nb ? expand32_fp4(f.dw[k]) : zero;
        }
    };

    // the maxDist gate's per-wave statistics (wave-uniform: scalar registers)
    bool gating = MAGE_FP4_GATE != 0;
    int g_tiles = 0, g_hits = 0;
    for (int pb = 0; pb < (nb > 0 ? na : 0); pb += FROWS) {
        const int rowbase = pb + wave * 32 * FRT;
        const bool active = rowbase < na;
        v4i a[FRT][4];
#pragma unroll
        for (int rt = 0; rt < FRT; rt++) {
            const int i = rowbase + 32 * rt + (lane & 31);
            const uint32_t* ar = Aw + 8 * min(i, na - 1);
            const v4i zero = {0, 0, 0, 0};
#pragma unroll
            for (int s = 0; s < 4; s++) a[rt][s] = i < na ? expand32_fp4(ar[2 * s + (lane >> 5)]) : zero;
        }
        uint32_t r1[FRT][8], r2[FRT][8];
#pragma unroll
        for (int rt = 0; rt < FRT; rt++)
#pragma unroll
            for (int q = 0; q < 8; q++) r1[rt][q] = r2[rt][q] = NONE16;
        {
            Fetch w[FPF];
#pragma unroll
            for (int j = 0; j < FPF; j++)
                if (j < nstages) w[j] = fetch(j);
            __syncthreads();  // B resident / column states ready; the previous pass is done with the stages
#pragma unroll
            for (int j = 0; j < FPF; j++)
                if (j < nstages) fill(j, j, w[j]);
            __syncthreads();
        }
        // global key of a local column key (code = 63 - row in the wave's 64 rows):
        // (64 (272 - d) + code) -> ((272 - d) << 16 | 0x7FFF - row)
        const int kadd = 0x7FFF - rowbase - 63;
        // accumulator bits of the smallest key with d <= maxDist: (124 << 23) | 64 (272 - maxDist)
        const uint32_t gate_bits = (124u << 23) | (uint32_t)(64 * (K16_D - min(max(maxDist, -1), 127)));
        PendingCol16 pc{0, 0, 0, 0, false};
        for (int st = 0; st < nstages; st++) {
            const int buf = st % FBUF;
            Fetch nxt{};
            if (st + FPF < nstages) nxt = fetch(st + FPF);
            if (active) {
#pragma unroll
                for (int ct = 0; ct < FNT; ct++) {
                    const int colbase = st * FSC + ct * 32;
                    if (colbase >= nb) break;
                    v4i bf[4];
#pragma unroll
                    for (int s = 0; s < 4; s++) bf[s] = stage[buf][ct][s][lane];
#pragma unroll
                    for (int grp = 0; grp < FRT; grp += 2) {  // one column flush per 64 rows (6-bit codes)
                        uint32_t c1 = NONE16, c2 = NONE16;
                        bool any = false;
#pragma unroll
                        for (int rt = grp; rt < min(grp + 2, FRT); rt++) {
                            const v16i acc = __builtin_bit_cast(v16i, tile_mfma_k16(a[rt], bf, cc));
                            if (MAGE_FP4_GATE && gating) {
                                // maxDist gate: radiusMatch keeps only d <= maxDist, and a top-2 state over
                                // a superset of those values decides exactly as one over them alone, so a
                                // tile whose 1024 keys all lie below the gate key (d > maxDist) is skipped
                                uint32_t mx = (uint32_t)acc[15];  // v_max3_u32 tree (key order = bit order)
#pragma unroll
                                for (int g = 0; g < 15; g += 3)
                                    mx = max(mx, max(max((uint32_t)acc[g], (uint32_t)acc[g + 1]), (uint32_t)acc[g + 2]));
                                const bool hit = __ballot(mx >= gate_bits) != 0;  // wave-uniform
                                g_tiles++;
                                g_hits += hit ? 1 : 0;
                                if (!hit) continue;
                            }
                            any = true;
                            uint32_t P[8];
#pragma unroll
                            for (int q = 0; q < 8; q++)
                                P[q] = __builtin_amdgcn_perm((uint32_t)acc[2 * q + 1], (uint32_t)acc[2 * q], 0x05040100u);
                            // row states: the two best distances over the tiles (same code per register)
#pragma unroll
                            for (int q = 0; q < 8; q++) {
                                r2[rt][q] = pkmax(r2[rt][q], pkmin(r1[rt][q], P[q]));
                                r1[rt][q] = pkmax(r1[rt][q], P[q]);
                            }
                            // column: the two best (distance, row) keys of the lane's 16 rows of this tile
                            // a knock-out tournament: every key but the winner loses exactly one
                            // comparison, so the second best is the best of the 7 losers (3 max3s)
                            uint32_t h[4], l[4];
#pragma unroll
                            for (int q = 0; q < 4; q++) {
                                h[q] = pkmax(P[2 * q], P[2 * q + 1]);
                                l[q] = pkmin(P[2 * q], P[2 * q + 1]);
                            }
                            const uint32_t hh0 = pkmax(h[0], h[1]), hl0 = pkmin(h[0], h[1]);
                            const uint32_t hh1 = pkmax(h[2], h[3]), hl1 = pkmin(h[2], h[3]);
                            uint32_t t1 = pkmax(hh0, hh1);
                            uint32_t t2 = pkmax3(pkmax3(l[0], l[1], l[2]), pkmax3(l[3], hl0, hl1), pkmin(hh0, hh1));
                            if (rt & 1) {  // rows 32..63 of the group: codes 32..63 -> 0..31 (bit 5 cleared)
                                t1 ^= 0x00200020u;
                                t2 ^= 0x00200020u;
                            }
                            const uint32_t lo = pkmin(c1, t1);
                            c1 = pkmax(c1, t1);
                            c2 = pkmax3(lo, c2, t2);
                        }
                        if (gating && g_tiles >= 64 && 4 * g_hits > g_tiles) gating = false;  // dense: fold all
                        if (!any) continue;  // no key of the column tile within maxDist: no flush
                        const int kg = kadd - 64 * (grp / 2);
                        // the partner half-wave holds the same column (rows + 4)
                        {
                            const uint32_t o1 = (uint32_t)xor32((int)c1, lane), o2 = (uint32_t)xor32((int)c2, lane);
                            const uint32_t lo = pkmin(c1, o1);
                            c1 = pkmax(c1, o1);
                            c2 = pkmax3(lo, c2, o2);
                        }
                        const int a1 = lo16s(c1), b1 = hi16s(c1);
                        const int m1 = max(a1, b1), m2 = max(min(a1, b1), max(lo16s(c2), hi16s(c2)));
                        const int g1 = ((m1 >> 6) << 16) | ((m1 & 63) + kg);
                        const int g2 = ((m2 >> 6) << 16) | ((m2 & 63) + kg);
                        if (pc.live) atomicMax(&colM2[pc.j], pc.old > pc.c1 ? pc.c1 : max(pc.old, pc.c2));
                        pc.j = colbase + (lane & 31);
                        pc.c1 = g1;
                        pc.c2 = g2;
                        pc.live = lane < 32 && pc.j < nb;
                        pc.old = pc.live ? atomicMax(&colM1[pc.j], g1) : NONE;
                    }
                }
            }
            if (st + FPF < nstages) fill((st + FPF) % FBUF, st + FPF, nxt);
            __syncthreads();
        }
        if (pc.live) atomicMax(&colM2[pc.j], pc.old > pc.c1 ? pc.c1 : max(pc.old, pc.c2));
        if (active) {
#pragma unroll
            for (int rt = 0; rt < FRT; rt++) {
                // reduce-scatter the 8 packed row states over lane bits 4, 3, 2, then all-reduce
                // over bits 1, 0: lane (lane & 31) ends with packed state k = (lane & 31) >> 2
                uint32_t* R1 = r1[rt];
                uint32_t* R2 = r2[rt];
#pragma unroll
                for (int m = 16, n = 8; m >= 4; m >>= 1, n >>= 1) {
                    const bool up = (lane & m) != 0;
                    const int hf = n / 2;
#pragma unroll
                    for (int k = 0; k < hf; k++) {
                        const uint32_t s1 = up ? R1[k] : R1[k + hf], s2 = up ? R2[k] : R2[k + hf];
                        const uint32_t x1 = up ? R1[k + hf] : R1[k], x2 = up ? R2[k + hf] : R2[k];
                        const uint32_t o1 = (uint32_t)__shfl_xor((int)s1, m), o2 = (uint32_t)__shfl_xor((int)s2, m);
                        const uint32_t lo = pkmin(x1, o1);
                        R1[k] = pkmax(x1, o1);
                        R2[k] = pkmax(pkmax(lo, x2), o2);
                    }
                }
#pragma unroll
                for (int m = 2; m >= 1; m >>= 1) {
                    const uint32_t o1 = (uint32_t)__shfl_xor((int)R1[0], m), o2 = (uint32_t)__shfl_xor((int)R2[0], m);
                    const uint32_t lo = pkmin(R1[0], o1);
                    R1[0] = pkmax(R1[0], o1);
                    R2[0] = pkmax(pkmax(lo, R2[0]), o2);
                }
                if ((lane & 3) == 0) {
                    const int k = (lane & 31) >> 2;
#pragma unroll
                    for (int e = 0; e < 2; e++) {
                        const int i = rowbase + 32 * rt + acc_row(2 * k + e) + 4 * (lane >> 5);
                        const int k1 = e ? hi16s(R1[0]) : lo16s(R1[0]), k2 = e ? hi16s(R2[0]) : lo16s(R2[0]);
                        const int d0 = K16_D - (k1 >> 6), d1 = K16_D - (k2 >> 6);  // NONE -> d > 511
                        const bool ok = d0 <= maxDist && !(d1 <= maxDist && d1 - d0 < minDiff);
                        if (i < na) rowd[i] = ok ? (uint16_t)d0 : (uint16_t)0xFFFFu;
                    }
                }
            }
        }
    }
    __syncthreads();
    // pair the accepted columns with their rows (see the section comment)
    for (int i = tid; i < na; i += FT) matchOf[i] = 0xFFFFu;
    __syncthreads();
    for (int j = tid; j < (na > 0 ? nb : 0); j += FT) {
        const int k1 = colM1[j], k2 = colM2[j];
        if (k1 == NONE) continue;
        const int dc = K16_D - (k1 >> 16);
        const int d2 = k2 == NONE ? INT_MAX : K16_D - (k2 >> 16);
        if (dc > maxDist || (d2 <= maxDist && d2 - dc < minDiff)) continue;
        const int i = 0x7FFF - (k1 & 0x7FFF);
        if (i < na && rowd[i] == (uint16_t)dc) matchOf[i] = (uint16_t)j;
    }
    __syncthreads();
    // ordered compaction (ascending A index, FeatureMatcher.cpp:142-167)
    uint32_t base = 0;
    mage_dmatch* o = out + (long long)pair * p.out_cap;
    for (int rb = 0; rb < (nb > 0 ? na : 0); rb += FT) {
        const int i = rb + tid;
        const int j = i < na ? (int)matchOf[i] : 0xFFFF;
        const bool ok = j != 0xFFFF;
        const unsigned long long m = __ballot(ok);
        const uint32_t before = (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
        if (lane == 0) wsum[wave] = (uint32_t)__popcll(m);
        __syncthreads();
        uint32_t woff = 0, total = 0;
        for (int w = 0; w < FW; w++) {
            if (w < wave) woff += wsum[w];
            total += wsum[w];
        }
        if (ok) {
            const uint32_t pos = base + woff + before;
            if (pos < p.out_cap) {
                mage_dmatch mm;
                mm.query_idx = i;
                mm.train_idx = j;
                mm.img_idx = -1;  // cv::DMatch(query, train, distance) (FeatureMatcher.cpp:159-162)
                mm.distance = (float)rowd[i];
                o[pos] = mm;
            }
        }
        base += total;
        __syncthreads();
    }
    if (tid == 0) n_out[pair] = base;
}

template <bool PADMASK>
__global__ __launch_bounds__(MT) void match_kernel(const uint8_t* __restrict__ A,
                                                   const uint32_t* __restrict__ nA,
                                                   const uint8_t* __restrict__ B,
                                                   const uint32_t* __restrict__ nB, MatchParams p,
                                                   mage_dmatch* __restrict__ out,
                                                   uint32_t* __restrict__ n_out,
                                                   uint32_t* __restrict__ status)
{
    __shared__ v4i stage[NBUF][SC / 32][8][kWave];  // [buffer][tile][k-step][lane] operands
    // resident path: packed B (8 words per descriptor) then the column states; streaming path:
    // the column states only
    __shared__ __attribute__((aligned(16))) uint32_t pool[NRES * 10];
    __shared__ uint32_t wsum[MW];
    static_assert(NRES * 10 >= 2 * NMAX, "column states of the streaming path fit the pool");

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
    const uint32_t* Aw = reinterpret_cast<const uint32_t*>(A + pair * p.a_pitch);
    const uint32_t* Bw = reinterpret_cast<const uint32_t*>(B + pair * p.b_pitch);
    int2* rows = p.rows + (long long)pair * NMAX;
    const bool res = nb <= NRES;
    int* colM1 = reinterpret_cast<int*>(pool) + (res ? 8 * nb : 0);
    int* colM2 = colM1 + nb;
    for (int j = tid; j < nb; j += MT) {
        colM1[j] = NONE;
        colM2[j] = NONE;
    }
    if (na > 0 && nb > 0) {
        if (res) {
            const uint4* src = reinterpret_cast<const uint4*>(Bw);
            for (int k = tid; k < 2 * nb; k += MT) reinterpret_cast<uint4*>(pool)[k] = src[k];
            __syncthreads();
            if (!PADMASK && nb <= 64 * 32)
                row_passes<Keys16, true>(Aw, Bw, pool, na, nb, stage, colM1, colM2, rows);
            else
                row_passes<Keys32<PADMASK>, true>(Aw, Bw, pool, na, nb, stage, colM1, colM2, rows);
        } else {
            row_passes<Keys32<PADMASK>, false>(Aw, Bw, pool, na, nb, stage, colM1, colM2, rows);
        }
    }
    __syncthreads();

    // cross-check + ordered compaction (ascending A index, FeatureMatcher.cpp:142-167)
    uint32_t base = 0;
    mage_dmatch* o = out + (long long)pair * p.out_cap;
    for (int rb = 0; rb < (nb > 0 ? na : 0); rb += MT) {
        const int i = rb + tid;
        bool ok = false;
        int j = 0, d = 0;
        if (i < na) {
            const int2 r = rows[i];
            if (accept(r.x, r.y, maxDist, p.min_diff)) {
                j = key_index(r.x);
                d = key_dist(r.x);
                ok = accept(colM1[j], colM2[j], maxDist, p.min_diff) && key_index(colM1[j]) == i;
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
                mm.train_idx = j;
                mm.img_idx = -1;  // cv::DMatch(query, train, distance) (FeatureMatcher.cpp:159-162)
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
                        uint32_t* dStatus, hipStream_t st, long long nbMax)
{
    MatchParams mp{};
    mp.max_dist = maxDist;
    mp.min_diff = minDiff;
    mp.out_cap = cap;
    mp.a_pitch = aPitch;
    mp.b_pitch = bPitch;
    // the fp4 kernel when every pair's B side provably fits it (nbMax: the pair pitch's capacity,
    // or the host-known count)
    if (maxDist < 128 && minDiff >= 1 && nbMax > 0 && nbMax <= FNB) {
        launch("match.two_way", match_fp4_kernel, dim3(pairs), dim3(FT), 0, st, dA, dnA, dB, dnB, mp, dOut, dN, dStatus);
        MAGE_HIP(hipGetLastError());
        return MAGE_OK;
    }
    void* rows = stream_scratch(st, STREAM_MATCH_ROWS, (size_t)pairs * NMAX * sizeof(int2));
    if (!rows) return MAGE_ENOMEM;
    mp.rows = static_cast<int2*>(rows);
    {
        launch("match.two_way", maxDist < 128 ? match_kernel<false> : match_kernel<true>, dim3(pairs), dim3(MT), 0, st,
               dA, dnA, dB, dnB, mp, dOut, dN, dStatus);
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
    void* status = mage::stream_scratch((hipStream_t)stream, mage::STREAM_MATCH_STATUS, 4);
    if (!status) return MAGE_ENOMEM;
    return mage::match_batch(d_desc_a, a_pitch, d_n_a, d_desc_b, b_pitch, d_n_b, pairs, max_distance,
                             min_difference, d_out, cap, d_n, static_cast<uint32_t*>(status), (hipStream_t)stream,
                             b_pitch > 0 ? b_pitch / 32 : -1);
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
    mage::HostScratch* sp = mage::host_scratch(dev, mage::SCRATCH_MATCH);
    if (!sp) return MAGE_EDEVICE;
    mage::HostScratch& S = *sp;
    // device layout [a][b][counts: nA, nB, total, status][out]: inputs packed at their device
    // offsets in pinned memory, one copy each way
    const size_t na = ia.size(), nb = ib.size(), ocap = na;
    auto al = [](size_t v) { return (v + 255) & ~(size_t)255; };
    const size_t oa = 0, ob = al(32 * na), oc = al(ob + 32 * nb), oo = al(oc + 16), total_bytes = oo + sizeof(mage_dmatch) * ocap;
    if ((r = S.buf.reserve(total_bytes)) != MAGE_OK || (r = S.host.reserve(total_bytes)) != MAGE_OK) return r;
    char* h = S.host.as<char>();
    char* d = S.buf.as<char>();
    for (size_t k = 0; k < na; k++) std::memcpy(h + oa + 32 * k, desc_a + 32 * (size_t)ia[k], 32);
    for (size_t k = 0; k < nb; k++) std::memcpy(h + ob + 32 * k, desc_b + 32 * (size_t)ib[k], 32);
    const uint32_t counts[4] = {(uint32_t)na, (uint32_t)nb, 0, 0};
    std::memcpy(h + oc, counts, 16);
    MAGE_HIP(hipMemcpyAsync(d, h, oo, hipMemcpyHostToDevice, S.st));
    uint32_t* dn = reinterpret_cast<uint32_t*>(d + oc);
    r = mage::match_batch(reinterpret_cast<const uint8_t*>(d + oa), 0, dn, reinterpret_cast<const uint8_t*>(d + ob), 0,
                          dn + 1, 1, max_distance, min_difference, reinterpret_cast<mage_dmatch*>(d + oo),
                          (uint32_t)ocap, dn + 2, dn + 3, S.st, (long long)nb);
    if (r != MAGE_OK) return r;
    MAGE_HIP(hipMemcpyAsync(h + oc, d + oc, total_bytes - oc, hipMemcpyDeviceToHost, S.st));
    MAGE_HIP(hipStreamSynchronize(S.st));
    const uint32_t total = reinterpret_cast<const uint32_t*>(h + oc)[2];
    const mage_dmatch* tmp = reinterpret_cast<const mage_dmatch*>(h + oo);
    const uint32_t nw = std::min<uint32_t>(std::min<uint32_t>(total, (uint32_t)ocap), cap);
    for (uint32_t k = 0; k < nw; k++) {
        out[k] = tmp[k];
        out[k].query_idx = (int32_t)ia[tmp[k].query_idx];
        out[k].train_idx = (int32_t)ib[tmp[k].train_idx];
    }
    *n = nw;
    return total > cap ? MAGE_ECAPACITY : MAGE_OK;
}

}  // extern "C"
