// orb.hip — ORB extraction on MI355X (gfx950): FAST-9/16 + NMS, retain + grid ANMS, fused
// Gaussian blur + pre-rotated BRIEF.  Replaces OrbDetector::DetectAndCompute
// (Core/MAGESLAM/Source/Image/OpenCVModified.cpp:771-886).
//
// Pipeline for a batch of B frames (all device resident), three launches:
//   1. fast_nms_kernel  grid (W/120, H/30, B): tile + halo staged in LDS; each thread scores a
//      4-px x 8-row strip from a register window with packed-f16 min3/max3 ladders (two pixels
//      per instruction), then a dword-vectorised strict 3x3 NMS, border filter, per-tile LDS
//      compaction, one global atomic per tile.  Candidates are packed u32 (y<<20 | x<<8 | score).
//   2. select_kernel    grid (B), 1024 threads: 256-bin histogram -> RetainBestFeatures cut,
//      bbox, 32x32 cell counting sort, per-item ANMS ring search, 64-bit key bitonic sort
//      (registers / wave shuffles / LDS by stride),
//      emits keypoints in canonical order (ANMS rank r desc, strength desc, raster asc).
//   3. describe_kernel  grid (cap/4, B), one wave per keypoint: raw window -> separable 8U
//      Gaussian (OpenCV Q8 taps) in LDS -> 256 tests -> four 64-bit ballots = the descriptor.
// The whole-frame blur of the reference (OpenCVModified.cpp:853-865) is replaced by blurring
// only the windows the descriptors sample: same values, no full-frame write/read.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <type_traits>
#include <vector>

#include "common.hpp"
#include "lds_sort.hpp"
#include "orb_tables.hpp"

namespace mage {
namespace {

// ------------------------------------------------------------------------------------------
// 1. FAST-9/16 + NMS
// ------------------------------------------------------------------------------------------
// Output tile TW x TH.  Scores are computed for the (TW + 8) x (TH + 2) region starting at
// (tx0 - 4, ty0 - 1): whole 4-pixel groups plus the 1-pixel NMS ring.  The image region staged
// in LDS starts at (tx0 - 8, ty0 - 4) so every group's 12-byte window row is three aligned dwords.
constexpr int TW = 120, TH = 30;
constexpr int GX = (TW + 8) / 4;       // 32 score groups per row
constexpr int SR = 8;                  // score rows per thread strip
constexpr int SROWS = TH + 2;          // 32 score rows
constexpr int LW = TW + 16;            // 136 image bytes per LDS row (34 dwords)
constexpr int LH = TH + 8;             // 38 image rows
constexpr int FAST_THREADS = GX * (SROWS / SR);  // 128
constexpr int TCAP = (TW / 2) * (TH / 2);        // candidates per tile: strict 3x3 maxima are never 8-adjacent
static_assert(SROWS % SR == 0, "strips tile the score rows");
static_assert(TW % 8 == 0, "tile origin stays qword aligned");

struct FastParams {
    int w, h, stride;
    long long pitch;
    int threshold;
    int xlo, xhi, ylo, yhi;  // emission window (FAST range ∩ RunByImageBorder)
    unsigned cand_cap;  // per frame: tiles x TCAP
    int tiles;          // tiles per frame (per-tile candidate counts)
    int tiles_x;        // tile columns per frame
    int dword_ok;  // frames 4-byte aligned with width, stride and pitch multiples of 4
    int qword_ok;  // frames 8-byte aligned, stride and pitch multiples of 8 (interior tiles)
    // fused 7-tap Gaussian (8U fixed point) of the tile into `blur` (null: no blur)
    uint8_t* blur;
    int blur_stride;           // multiple of 4, >= w: columns written
    long long blur_pitch;      // bytes between blurred frames
    int blur_bcols;            // brick columns per brick row (BLUR_BRICK layout)
    const uint4* blur_ops;     // per lane: the MFMA band operands of the taps (blur_operands)
    // candidate gate (see gate_strip): the batch's gate G is *gate; the launch re-arms the next
    // batch's gate word (*gate_next = 255, lowered by select_kernel) and the redo list (redo[0])
    const int* gate;
    int* gate_next;
    uint32_t* redo;  // [count, frame...]: frames select_kernel sends back through the exact path
};

struct Tile {
    int x, y;  // tile column / row in the frame
};

// Orders one wave's LDS writes before its other lanes' reads (when the waves of a workgroup
// work on disjoint data no workgroup barrier is needed).
__device__ __forceinline__ void wave_lds_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

typedef _Float16 h2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ h2 as_h2(uint32_t u) { return __builtin_bit_cast(h2, u); }
__device__ __forceinline__ uint32_t as_u32(h2 h) { return __builtin_bit_cast(uint32_t, h); }
// v_pk_minimum3_f16 / v_pk_maximum3_f16 (gfx950)
__device__ __forceinline__ h2 min3h(h2 a, h2 b, h2 c)
{
    return __builtin_elementwise_minimum(__builtin_elementwise_minimum(a, b), c);
}
__device__ __forceinline__ h2 max3h(h2 a, h2 b, h2 c)
{
    return __builtin_elementwise_maximum(__builtin_elementwise_maximum(a, b), c);
}

// Bytes (k, k+1) of dword d as two f16 lanes holding 1024 + byte: [b_k, 0x64, b_k+1, 0x64].
// The 1024 offset is exact in f16 and cancels in every difference.
__device__ __forceinline__ h2 pair_in(uint32_t d, int k)
{
    return as_h2(__builtin_amdgcn_perm(d, 0x64646464u, (uint32_t)((4 + k) | ((5 + k) << 16))));
}
__device__ __forceinline__ h2 pair_cross(uint32_t lo, uint32_t hi)  // (lo.b3, hi.b0)
{
    return as_h2(__builtin_amdgcn_perm(hi, lo, 0x0C040C03u) | 0x64006400u);
}

// The 9 adjacent byte pairs (i, i+1), i = 1..9, of a 12-byte window row; q[i - 1].
__device__ __forceinline__ void window_row(uint32_t d0, uint32_t d1, uint32_t d2, h2 (&q)[9])
{
    q[0] = pair_in(d0, 1);
    q[1] = pair_in(d0, 2);
    q[2] = pair_cross(d0, d1);
    q[3] = pair_in(d1, 0);
    q[4] = pair_in(d1, 1);
    q[5] = pair_in(d1, 2);
    q[6] = pair_cross(d1, d2);
    q[7] = pair_in(d2, 0);
    q[8] = pair_in(d2, 1);
}

// Ring of FAST_t<16> (makeOffsets, OpenCVModified.cpp:890-921) as (dx, dy).
__host__ __device__ constexpr int ring_dx(int k)
{
    constexpr int v[16] = {0, 1, 2, 3, 3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1};
    return v[k];
}
__host__ __device__ constexpr int ring_dy(int k)
{
    constexpr int v[16] = {3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1, 0, 1, 2, 3};
    return v[k];
}

// FAST-9/16 raw score for two horizontally adjacent pixels (group pixels 2p, 2p + 1) from the
// 7 window rows w[dy + 3], branch-free.  With d_k = v - x_k over the 16-pixel ring, let
// A = max over the 16 cyclic 9-arcs of min(d) and B = min over the arcs of max(d).  "Some 9
// contiguous ring pixels are all darker than v - t" (the segment test of FAST_t<16>,
// OpenCVModified.cpp:1415-1479) is exactly A > t, "all brighter than v + t" is -B > t, and
// cornerScore<16> (:927-1071; its scalar and SSE2 branches agree on corners) is max(A, -B) - 1.
// Since min over an arc of (v - x) = v - max over the arc of x, A = v - min_k X9[k] and
// B = v - max_k N9[k] with X9 / N9 the 9-arc max / min of the ring values themselves: 9-arc
// extrema are min3/max3 of three 3-arc extrema.  Every value is an integer (offset 1024), exact
// in f16, so the packed f16 min3/max3 give the integer result.
// min_k X9[k]: the dark ladder (A = v - lo)
__device__ __forceinline__ h2 fast_dark_lo(const h2 (&x)[16])
{
    h2 t3[16];
#pragma unroll
    for (int k = 0; k < 16; k++) t3[k] = max3h(x[k], x[(k + 1) & 15], x[(k + 2) & 15]);
    h2 lo = min3h(max3h(t3[0], t3[3], t3[6]), max3h(t3[1], t3[4], t3[7]), max3h(t3[2], t3[5], t3[8]));
#pragma unroll
    for (int k = 3; k < 15; k += 2)
        lo = min3h(lo, max3h(t3[k], t3[(k + 3) & 15], t3[(k + 6) & 15]), max3h(t3[k + 1], t3[(k + 4) & 15], t3[(k + 7) & 15]));
    return __builtin_elementwise_minimum(lo, max3h(t3[15], t3[2], t3[5]));
}
// max_k N9[k]: the bright ladder (-B = hi - v)
__device__ __forceinline__ h2 fast_bright_hi(const h2 (&x)[16])
{
    h2 t3[16];
#pragma unroll
    for (int k = 0; k < 16; k++) t3[k] = min3h(x[k], x[(k + 1) & 15], x[(k + 2) & 15]);
    h2 hi = max3h(min3h(t3[0], t3[3], t3[6]), min3h(t3[1], t3[4], t3[7]), min3h(t3[2], t3[5], t3[8]));
#pragma unroll
    for (int k = 3; k < 15; k += 2)
        hi = max3h(hi, min3h(t3[k], t3[(k + 3) & 15], t3[(k + 6) & 15]), min3h(t3[k + 1], t3[(k + 4) & 15], t3[(k + 7) & 15]));
    return __builtin_elementwise_maximum(hi, min3h(t3[15], t3[2], t3[5]));
}
__device__ __forceinline__ h2 fast_raw_ring(h2 v, const h2 (&x)[16])
{
    // the two ladders one after the other (16 3-arc extrema live at a time, not 32)
    const h2 lo = fast_dark_lo(x);
    const h2 hi = fast_bright_hi(x);
    return __builtin_elementwise_maximum(v - lo, hi - v);
}

template <int P>
__device__ __forceinline__ h2 fast_raw2(const h2 (&w)[7][9])
{
    h2 x[16];
#pragma unroll
    for (int k = 0; k < 16; k++) x[k] = w[ring_dy(k) + 3][4 + 2 * P + ring_dx(k) - 1];
    return fast_raw_ring(w[3][4 + 2 * P - 1], x);
}

// Score bytes of two pixels from their raw scores: raw > t ? raw - 1 : 0, as 1024 + score.
__device__ __forceinline__ uint32_t score2(h2 raw, h2 tf)
{
    const h2 zero = {(_Float16)0.0f, (_Float16)0.0f}, one = {(_Float16)1.0f, (_Float16)1.0f};
    const h2 step = __builtin_elementwise_minimum(__builtin_elementwise_maximum(raw - tf, zero), one);
    const h2 k1024 = {(_Float16)1024.0f, (_Float16)1024.0f};
    return as_u32(raw * step - step + k1024);
}
// The same with the clamp output modifier: step = clamp(raw - t, 0, 1) is 0 or 1 (integers), and
// (raw - 1) step + 1024 is exact; 3 instructions instead of 6 (the gated pass only: in the
// exact strips the asm block costs the register allocator its freedom and the kernel spills).
__device__ __forceinline__ uint32_t score2_clamp(h2 raw, h2 tf)
{
    const h2 one = {(_Float16)1.0f, (_Float16)1.0f}, k1024 = {(_Float16)1024.0f, (_Float16)1024.0f};
    uint32_t step;
    asm("v_pk_add_f16 %0, %1, %2 neg_lo:[0,1] neg_hi:[0,1] clamp" : "=v"(step) : "v"(as_u32(raw)), "v"(as_u32(tf)));
    return as_u32(__builtin_elementwise_fma(raw - one, as_h2(step), k1024));
}

__device__ __forceinline__ int reflect101(int i, int n)
{
    if (n == 1) return 0;
    while ((unsigned)i >= (unsigned)n) i = i < 0 ? -i : 2 * n - 2 - i;
    return i;
}

// Stage the LW x LH image window into LDS, reflect-101 outside the frame (BORDER_DEFAULT of the
// reference's GaussianBlur; FAST never reads outside the frame, its range is [3, w-4]).  When
// the row pitch and the width are multiples of 4, dwords wholly inside the frame are moved with
// 4-byte loads.
__device__ __forceinline__ void load_tile(const uint8_t* __restrict__ src, const FastParams& p,
                                          uint8_t (*img)[LW], Tile T)
{
    const int gx0 = T.x * TW - 8, gy0 = T.y * TH - 4;
    if (p.qword_ok && gx0 >= 0 && gx0 + LW <= p.w && gy0 >= 0 && gy0 + LH <= p.h) {
        // interior tile (most of them): no reflection, addresses by increment.  A row is 8
        // sixteen-byte loads + one 8-byte tail (9 threads per row, 14 rows per pass; 16-byte global
        // loads need only dword alignment), stored as 8-byte LDS writes (rows are 8-byte aligned)
        static_assert(LW == 8 * 16 + 8, "row = 8 x 16 + 8 bytes");
        constexpr int RSTEP = FAST_THREADS / 9, NPASS = (LH + RSTEP - 1) / RSTEP;  // 14 rows per pass, 3 passes
        const int c = threadIdx.x % 9, r0 = threadIdx.x / 9;
        if (r0 < RSTEP) {
            // chunk 8 (the row's last 8 bytes) loads bytes 120..135 and keeps the upper half, so
            // every load is 16 bytes and stays inside the tile row; all loads issue before the writes
            const uint8_t* g = src + (long long)(gy0 + r0) * p.stride + gx0 + (c < 8 ? 16 * c : 120);
            const long long gstep = (long long)RSTEP * p.stride;
            typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
            u32x4 v[NPASS];
#pragma unroll
            for (int k = 0; k < NPASS; k++)
                if (r0 + k * RSTEP < LH) __builtin_memcpy(&v[k], g + k * gstep, 16);
#pragma unroll
            for (int k = 0; k < NPASS; k++) {
                const int r = r0 + k * RSTEP;
                if (r >= LH) break;
                if (c < 8) {
                    uint2* d = reinterpret_cast<uint2*>(&img[r][16 * c]);
                    d[0] = make_uint2(v[k][0], v[k][1]);
                    d[1] = make_uint2(v[k][2], v[k][3]);
                } else {
                    *reinterpret_cast<uint2*>(&img[r][128]) = make_uint2(v[k][2], v[k][3]);
                }
            }
        }
        return;
    }
    constexpr int DW = LW / 4;
    for (int i = threadIdx.x; i < LH * DW; i += FAST_THREADS) {
        const int r = i / DW, c = i - r * DW;
        const int gx = gx0 + 4 * c, gy = reflect101(gy0 + r, p.h);
        const uint8_t* row = src + (long long)gy * p.stride;
        uint32_t v;
        if (p.dword_ok && gx >= 0 && gx + 3 < p.w) {
            v = *reinterpret_cast<const uint32_t*>(row + gx);
        } else {
            v = 0;
#pragma unroll
            for (int q = 0; q < 4; q++) v |= (uint32_t)row[reflect101(gx + q, p.w)] << (8 * q);
        }
        *reinterpret_cast<uint32_t*>(&img[r][4 * c]) = v;
    }
}

// Scores of the thread's strip: group gx (4 columns), score rows [SR * chunk, SR * chunk + SR),
// written as one dword per row into sc.  Pixels outside the FAST range [3, w-4] x [3, h-4]
// score 0.
__device__ __forceinline__ void score_strip(const uint8_t (*img)[LW], uint32_t (*sc)[GX], const FastParams& p, Tile T)
{
    const int gx = threadIdx.x % GX, chunk = threadIdx.x / GX;
    const int X0 = T.x * TW - 4 + 4 * gx;     // image column of the group's first pixel
    const int Y0 = T.y * TH - 1 + SR * chunk;  // image row of the strip's first score row
    uint32_t colmask = 0;
#pragma unroll
    for (int q = 0; q < 4; q++)
        if (X0 + q >= 3 && X0 + q <= p.w - 4) colmask |= 0xFFu << (8 * q);
    const _Float16 t = (_Float16)(float)p.threshold;
    const h2 tf = {t, t};
    // window rows: LDS row (score row) + dy + 3; the strip needs LDS rows SR*chunk .. +SR+5.
    // A rolling 7-row window of f16 pairs; row r + 7's dwords are fetched one row ahead, and a
    // scheduling barrier per row keeps the compiler from hoisting every row's LDS reads (and
    // their registers) to the top: the strip fits 96 VGPRs, 5 waves per SIMD.
    const uint32_t* base = reinterpret_cast<const uint32_t*>(&img[SR * chunk][0]) + gx;
    h2 win[7][9];
#pragma unroll
    for (int r = 0; r < 6; r++) {
        const uint32_t* rp = base + r * (LW / 4);
        window_row(rp[0], rp[1], rp[2], win[r + 1]);
    }
    uint32_t nx0 = base[6 * (LW / 4)], nx1 = base[6 * (LW / 4) + 1], nx2 = base[6 * (LW / 4) + 2];
#pragma unroll
    for (int r = 0; r < SR; r++) {
#pragma unroll
        for (int k = 0; k < 6; k++)
#pragma unroll
            for (int i = 0; i < 9; i++) win[k][i] = win[k + 1][i];
        window_row(nx0, nx1, nx2, win[6]);
        if (r + 1 < SR) {
            const uint32_t* rp = base + (r + 7) * (LW / 4);
            nx0 = rp[0];
            nx1 = rp[1];
            nx2 = rp[2];
        }
        const uint32_t s0 = score2(fast_raw2<0>(win), tf);
        const uint32_t s1 = score2(fast_raw2<1>(win), tf);
        uint32_t bytes = __builtin_amdgcn_perm(s1, s0, 0x06040200u);  // low bytes of the 4 lanes
        const int Y = Y0 + r;
        if (Y < 3 || Y > p.h - 4) bytes = 0;
        sc[SR * chunk + r][gx] = bytes & colmask;
    }
}

// Candidate gate.  Only keypoints with a score of at least the retain cut survive
// RetainBestFeatures (OpenCVModified.cpp:571-617), and the cut of a frame is never below
// `lower` = max((int)(minNumThreshold * FeatureStrength), FastThreshold).  Given a gate G that
// is at most the frame's `lower`, the kept set only depends on the scores >= G and on the strict
// 3x3 maxima among them, so pixels that cannot reach G need no exact score:
//   * score >= G needs 9 contiguous ring pixels all darker than v - G (or all brighter than
//     v + G), and every 9-arc of the 16-ring holds at least two of the compass pixels 0, 4, 8,
//     12; so the second largest of (v - x_c), or of (x_c - v), over the compass exceeds G;
//   * a pixel failing that test scores < G; its stored score 0 is still below every score >= G,
//     so the strict 3x3 maxima with scores >= G are exactly those of the full score map;
//   * the passing 4-pixel groups are scored exactly with the threshold raised to G (scores < G
//     become 0, so only maxima >= G are emitted).
// select_kernel checks that G <= lower for the frame (the histogram above G is exact) and sends
// every frame that fails the check through the exact path again (fast_redo_kernel +
// select_redo_kernel); the output never depends on G.  G comes from the previous batch of the
// same detector: 15/16 of the smallest `lower` over its frames (frames of a stream change slowly).
//
// gate_strip: the compass test of the thread's 4-px x 8-row strip; zeroes the strip's score
// dwords and returns bit 8 q + r set when pixel q of score row SR * chunk + r passes.
// MAGE_GATE_ANTIPODAL: the tighter form of the same necessary condition — a 9-arc of the 16-ring
// holds at least one of the antipodal pixels 0 / 8 and one of 4 / 12, so "all darker" needs
// max(min(x0, x8), min(x4, x12)) < v - G (and "all brighter" min(max(x0, x8), max(x4, x12)) > v + G):
// two packed ops fewer per pixel pair, and never more pixels listed.
__device__ __forceinline__ uint32_t gate_strip(const uint8_t (*img)[LW], uint32_t (*sc)[GX], int G,
                                               const FastParams& p, Tile T)
{
    const int gx = threadIdx.x % GX, chunk = threadIdx.x / GX;
    // pixels outside the FAST range [3, w-4] x [3, h-4] are never listed (their score is 0), so
    // the scoring pass has no range test; only strips at the frame border build the mask
    uint32_t keep = ~0u;
    const int X0 = T.x * TW - 4 + 4 * gx, Y0 = T.y * TH - 1 + SR * chunk;
    if (X0 < 3 || X0 + 3 > p.w - 4 || Y0 < 3 || Y0 + SR - 1 > p.h - 4) {
        uint32_t rows = 0;
#pragma unroll
        for (int r = 0; r < SR; r++)
            if (Y0 + r >= 3 && Y0 + r <= p.h - 4) rows |= 1u << r;
        keep = 0;
#pragma unroll
        for (int q = 0; q < 4; q++)
            if (X0 + q >= 3 && X0 + q <= p.w - 4) keep |= rows << (8 * q);
    }
    constexpr int RP = LW / 4;
    const uint32_t* w32 = reinterpret_cast<const uint32_t*>(&img[SR * chunk][0]) + gx;
    // Pixels as f16 denormals (byte b -> pattern 0x00bb = b * 2^-24; f16 denormals are preserved,
    // .amdhsa_float_denorm_mode_16_64 3): every difference and comparison is exact as with the
    // 1024 + b form, and the zero high byte is v_perm's constant selector 0x0C, so any two bytes of
    // two dwords become a pair in one v_perm (no v_alignbyte for the x +- 3 pixels).
    auto pr = [](uint32_t s0, uint32_t s1, uint32_t sel) { return as_h2(__builtin_amdgcn_perm(s0, s1, sel)); };
    const uint32_t g1 = (uint32_t)(G + 1);
    const h2 gp1 = as_h2(g1 | (g1 << 16));
    // the centre dwords of LDS rows SR*chunk .. +SR+5 as f16 pairs, once: a row is the centre of
    // one score row and the up / down compass pixels of the rows 3 below / above
    h2 cp[SR + 6][2];
#pragma unroll
    for (int k = 0; k < SR + 6; k++) {
        const uint32_t c = w32[k * RP + 1];
        cp[k][0] = pr(c, c, 0x0C010C00u);  // pixels x, x + 1
        cp[k][1] = pr(c, c, 0x0C030C02u);  // x + 2, x + 3
    }
    uint32_t neg = 0;  // bit 8 q + r: pixel q of score row SR*chunk + r fails
#pragma unroll
    for (int r = 0; r < SR; r++) {
        const uint32_t* rp = w32 + (r + 3) * RP;  // LDS row of score row SR*chunk + r
        const uint32_t l = rp[0], c = rp[1], n = rp[2];  // bytes x - 4 .., x .., x + 4 ..
        // x - 3 and x + 3 of pixel pairs (x, x + 1) and (x + 2, x + 3)
        const h2 ep[2] = {pr(l, l, 0x0C020C01u), pr(c, l, 0x0C040C03u)};
        const h2 dp[2] = {pr(n, c, 0x0C040C03u), pr(n, n, 0x0C020C01u)};
        uint32_t t2[2];
#pragma unroll
        for (int P = 0; P < 2; P++) {
            const h2 v = cp[r + 3][P], a = cp[r][P], b = cp[r + 6][P];
            const h2 e = ep[P], d = dp[P];
            // every 9-arc holds one of the antipodal pixels 0 / 8 (a, b) and one of 4 / 12 (d, e)
            const h2 hi = __builtin_elementwise_minimum(__builtin_elementwise_maximum(a, b), __builtin_elementwise_maximum(d, e));
            const h2 lo = __builtin_elementwise_maximum(__builtin_elementwise_minimum(a, b), __builtin_elementwise_minimum(d, e));
            t2[P] = as_u32(__builtin_elementwise_maximum(hi - v, v - lo) - gp1);  // >= 0: may reach G
        }
        sc[SR * chunk + r][gx] = 0u;
        // the signs of pixels 0..3 as 0xFF / 0x00 bytes (v_perm sign-extension selectors 8-11:
        // bits 15 / 31 of each source), kept at bits 8 q + r (one v_bitop3)
        const uint32_t sb = __builtin_amdgcn_perm(t2[1], t2[0], 0x0B0A0908u);
        neg |= sb & (0x01010101u << r);
    }
    return ~neg & keep;
}

// LDS byte offsets of the 16 ring pixels (and the centre, entry 16) from (centre - 3 LW - 3):
// (dy + 3) LW + dx + 3 — every offset non-negative, as the DS offset field requires.
static_assert(LW == 136, "ring_d16's immediate offsets assume LW = 136");
#define MAGE_RING_D16(i, j, o)                                                  \
    "ds_read_u8 %" #i ", %34 offset:" #o "\n\t"                                 \
    "ds_read_u8_d16_hi %" #j ", %35 offset:" #o "\n\t"
// The 16 ring bytes and the centre of two pixels (LDS byte addresses aa / ab of their
// centre - 3 LW - 3): ra[k] = byte_a, rb[k] = byte_b << 16 (a d16_hi load zero-fills the low
// half on SRAM-ECC parts such as MI355X).  One asm block with its own lgkmcnt(0): the compiler's
// wait insertion does not see asm loads.
__device__ __forceinline__ void ring_d16(uint32_t aa, uint32_t ab, uint32_t (&ra)[17], uint32_t (&rb)[17])
{
    asm volatile(MAGE_RING_D16(0, 17, 819) MAGE_RING_D16(1, 18, 820) MAGE_RING_D16(2, 19, 685)
                 MAGE_RING_D16(3, 20, 550) MAGE_RING_D16(4, 21, 414) MAGE_RING_D16(5, 22, 278)
                 MAGE_RING_D16(6, 23, 141) MAGE_RING_D16(7, 24, 4) MAGE_RING_D16(8, 25, 3)
                 MAGE_RING_D16(9, 26, 2) MAGE_RING_D16(10, 27, 137) MAGE_RING_D16(11, 28, 272)
                 MAGE_RING_D16(12, 29, 408) MAGE_RING_D16(13, 30, 544) MAGE_RING_D16(14, 31, 681)
                 MAGE_RING_D16(15, 32, 818) MAGE_RING_D16(16, 33, 411)
                 "s_waitcnt lgkmcnt(0)"
                 : "=&v"(ra[0]), "=&v"(ra[1]), "=&v"(ra[2]), "=&v"(ra[3]), "=&v"(ra[4]), "=&v"(ra[5]),
                   "=&v"(ra[6]), "=&v"(ra[7]), "=&v"(ra[8]), "=&v"(ra[9]), "=&v"(ra[10]), "=&v"(ra[11]),
                   "=&v"(ra[12]), "=&v"(ra[13]), "=&v"(ra[14]), "=&v"(ra[15]), "=&v"(ra[16]),
                   "=&v"(rb[0]), "=&v"(rb[1]), "=&v"(rb[2]), "=&v"(rb[3]), "=&v"(rb[4]), "=&v"(rb[5]),
                   "=&v"(rb[6]), "=&v"(rb[7]), "=&v"(rb[8]), "=&v"(rb[9]), "=&v"(rb[10]), "=&v"(rb[11]),
                   "=&v"(rb[12]), "=&v"(rb[13]), "=&v"(rb[14]), "=&v"(rb[15]), "=&v"(rb[16])
                 : "v"(aa), "v"(ab)
                 : "memory");
}
#undef MAGE_RING_D16
__host__ __device__ constexpr int ring_off(int k) { return (ring_dy(k) + 3) * LW + ring_dx(k) + 3; }
static_assert(ring_off(0) == 819 && ring_off(1) == 820 && ring_off(2) == 685 && ring_off(3) == 550 &&
              ring_off(4) == 414 && ring_off(5) == 278 && ring_off(6) == 141 && ring_off(7) == 4 &&
              ring_off(8) == 3 && ring_off(9) == 2 && ring_off(10) == 137 && ring_off(11) == 272 &&
              ring_off(12) == 408 && ring_off(13) == 544 && ring_off(14) == 681 && ring_off(15) == 818 &&
              3 * LW + 3 == 411, "ring_d16 offsets");

__device__ __forceinline__ uint32_t lds_addr(const void* p)
{
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}

// Listed pixel of the gated pass: item = (thread << 5) | bit, bit 8 q + r of the thread's
// gate_strip mask (GX = 32 groups per strip row, SR = 8 rows), so the listing loop writes
// `base | bit`.  Score row SR * chunk + r and score column 4 gx + q:
static_assert(GX == 32 && SR == 8, "item layout");
__device__ __forceinline__ uint32_t item_row(uint32_t it) { return ((it >> 7) & ~7u) | (it & 7u); }  // it < 4096
__device__ __forceinline__ uint32_t item_col(uint32_t it) { return __builtin_amdgcn_ubfe(it, 3, 7); }

// Exact scores of two listed pixels (score row << 7 | score column) at once, one per f16 lane,
// with threshold tf (listed pixels lie inside the FAST range, gate_strip).  Returns the two
// score bytes (a in bits 0-7, b in bits 16-23).
__device__ __forceinline__ uint32_t score_pixels(const uint8_t (*img)[LW], uint8_t* scb, uint32_t ia, uint32_t ib,
                                             h2 tf, h2 gp1)
{
    // LDS centre of score pixel (sr, x): image row sr + 3, column x + 4
    const uint32_t ra_ = item_row(ia), ca_ = item_col(ia), rb_ = item_row(ib), cb_ = item_col(ib);
    const uint8_t* ca = &img[ra_ + 3][ca_ + 4];
    const uint8_t* cb = &img[rb_ + 3][cb_ + 4];
    h2 x[16];
    uint32_t ra[17], rb[17];
    ring_d16(lds_addr(ca - 3 * LW - 3), lds_addr(cb - 3 * LW - 3), ra, rb);
    // One ladder per pixel.  A listed pixel passed gate_strip's dark or bright bound (antipodal
    // compass pixels 0 / 8 and 4 / 12, the same f16 arithmetic), and a side whose bound fails
    // scores <= G, i.e. 0 after the threshold G: so only the passing side needs its 9-arc
    // ladder.  Pixels whose dark bound fails are mirrored (byte ^ 0xFF: the bright segment test
    // on x is the dark one on 255 - x), so every lane runs the dark ladder; a pixel passing
    // both bounds (none on the C2 stream) makes the wave also run the other ladder.
    const uint32_t K = 0x64006400u;
    const h2 c0 = as_h2(ra[0] | rb[0] | K), c4 = as_h2(ra[4] | rb[4] | K);
    const h2 c8 = as_h2(ra[8] | rb[8] | K), c12 = as_h2(ra[12] | rb[12] | K);
    const h2 v0 = as_h2(ra[16] | rb[16] | K);
    const h2 hic = __builtin_elementwise_minimum(__builtin_elementwise_maximum(c0, c8), __builtin_elementwise_maximum(c4, c12));
    const h2 loc = __builtin_elementwise_maximum(__builtin_elementwise_minimum(c0, c8), __builtin_elementwise_minimum(c4, c12));
    const uint32_t dk = as_u32((v0 - loc) - gp1), br = as_u32((hic - v0) - gp1);  // sign set: that bound fails
    // [m_a, 0x64, m_b, 0x64]: m = 0xFF where the dark bound fails (v_perm sign-byte selectors 8 / 9)
    const uint32_t M = __builtin_amdgcn_perm(0x64646464u, dk, 0x04090408u);
#pragma unroll
    for (int k = 0; k < 16; k++) x[k] = as_h2((ra[k] | rb[k]) ^ M);
    const h2 v = as_h2((ra[16] | rb[16]) ^ M);
    h2 raw = v - fast_dark_lo(x);
    if (__builtin_amdgcn_ballot_w64(((dk | br) & 0x80008000u) != 0x80008000u))
        raw = __builtin_elementwise_maximum(raw, fast_bright_hi(x) - v);
    const uint32_t sv = score2_clamp(raw, tf);
    // (listed pixels lie inside the FAST range: gate_strip)
    const uint32_t sa = sv & 0xFFu, sb = (sv >> 16) & 0xFFu;
    scb[ra_ * (4 * GX) + ca_] = (uint8_t)sa;
    scb[rb_ * (4 * GX) + cb_] = (uint8_t)sb;
    return sa | (sb << 16);
}

// Fused Gaussian 7x7 on the matrix cores (v_mfma_i32_16x16x64_i8, integer-exact).  Both separable
// passes are GEMMs with a constant banded (Toeplitz) operand of the taps; per 16-column strip:
//   row pass  H = I · T: A = 16 image rows x a 64-byte window (only its first 32 bytes reach the
//             band; bytes enter as b - 128 = b ^ 0x80, the bias returns through C = 128 * 257),
//             B[k][n] = tap[k - n - 5]; one MFMA per 16 H rows, H <= 257 * 255 exactly in i32.
//   col pass  Y = Tc · H straight from the row pass accumulators: register r of lane l holds H
//             row 4 (l >> 4) + r of column l & 15, so the lane's 12 values of the three H blocks
//             are its 12 K elements (order free: A and B share the lane-local K order).  H is split
//             into bytes (hi, lo), two MFMAs per 16 output rows; Y + 2^15 = 256 hi-sum + lo-sum
//             (C = 128 * 257 for each, + 2^15 for lo); out = min(255, (Y + 2^15) >> 16).
//             The column pass is computed transposed (Y^T = H^T Tc^T: the H bytes as the A
//             operand, the band as B; A and B share the lane layout), so a lane holds 4
//             consecutive columns of one output row: one dword, stored straight to the frame
//             (no LDS tile, no barrier, no copy loop).
constexpr int BLUR_STRIPS = (TW + 15) / 16;  // 8 (the last is half used)

// BLUR_BRICK layout of the blurred frames (written here, read only by describe_blurred_kernel):
// 128-byte bricks of 4 rows x 32 bytes, row-major over bricks.  A keypoint's 15-row window then
// touches ~8 cache lines instead of ~20 (one per row), and describe was bound by the L1 / TA
// line traffic of its window loads.
__device__ __forceinline__ long long brick_offset(int y, int x, int bcols)
{
    return ((long long)(y >> 2) * bcols + (x >> 5)) * 128 + (y & 3) * 32 + (x & 31);
}

__device__ __forceinline__ void blur_mfma(const uint8_t (*img)[LW], const FastParams& p, int f, Tile T)
{
    typedef int v4i __attribute__((ext_vector_type(4)));
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int n = lane & 15, g = lane >> 4;
    // the lane's band operands (host-built, blur_operands): row-pass B and col-pass A of both
    // output blocks
    const uint4 o0 = p.blur_ops[3 * lane], o1 = p.blur_ops[3 * lane + 1], o2 = p.blur_ops[3 * lane + 2];
    const v4i tb = {(int)o0.x, (int)o0.y, (int)o0.z, (int)o0.w};
    const v4i ta[2] = {{(int)o1.x, (int)o1.y, (int)o1.z, (int)o1.w}, {(int)o2.x, (int)o2.y, (int)o2.z, (int)o2.w}};
    // row pass: H' = sum tap (b - 128) + 128 = H - 32768 in [-32768, 32767] (the operands hold
    // b ^ 0x80), so the high byte of H' is its signed i8 digit and only the low byte needs the
    // 0x80 bias.  Column pass with C = 0: the constants ride in each lane's spare K slots 12..15
    // (A dword 3 x B dword 3 = {-128, a1} . {-64, 1}, four K groups): hi 4 (8192 + 64) = 33024,
    // lo 4 (8192 + 32) = 32896, so that 256 Yh + Yl = sum tc H' + 257 * 2^15 + 2^15 = Y + 2^15.
    const v4i c_row = {128, 128, 128, 128};
    const v4i c_zero = {0, 0, 0, 0};
    // lane: output row 16 o + n, tile columns 16 s + 4 g .. + 3 (rows >= TH, columns >= TW
    // and columns past the blurred frame's stride are not stored); the BLUR_BRICK offset of
    // (Y, X) advances by one brick (128 B) per two strips and by 4 brick rows per output block
    const int ylim = min(TH, p.h - T.y * TH);
    uint8_t* fb = p.blur + (long long)f * p.blur_pitch;
    const int Y0 = T.y * TH + n, X0 = T.x * TW + 16 * wave + 4 * g;
    uint32_t off = (uint32_t)((((Y0 >> 2) * p.blur_bcols + (X0 >> 5)) << 7) + ((Y0 & 3) << 5) + (X0 & 31));
    const uint32_t ostep = (uint32_t)p.blur_bcols << 9;
    const bool yok[2] = {n < ylim, 16 + n < ylim};
    for (int s = wave; s < BLUR_STRIPS; s += FAST_THREADS / kWave, off += 128u) {
        // H block b: H rows 16 b - 3 + m (tile coordinates) = LDS rows 16 b + 1 + m; the window
        // is LDS columns 16 s .. + 63 (tile columns 16 s - 8 ..), of which lanes g < 2 load the
        // 32 bytes the band reaches; clamped reads only feed discarded outputs
        v4i H[3];
#pragma unroll
        for (int b = 0; b < 3; b++) {
            // lanes g >= 2 meet zero band bytes: whatever they load (clamped in the row) adds 0
            const int row = min(16 * b + 1 + n, LH - 1);
            const int c0 = min(16 * s + 16 * g, LW - 8), c1 = min(16 * s + 16 * g + 8, LW - 8);
            const uint2 d0 = *reinterpret_cast<const uint2*>(&img[row][c0]);
            const uint2 d1 = *reinterpret_cast<const uint2*>(&img[row][c1]);
            // bytes b enter as the signed i8 b - 128 = b ^ 0x80 (full-rate v_xor_b32 here instead of
            // a biasing pass over the LDS tile and a barrier)
            const v4i a = {(int)(d0.x ^ 0x80808080u), (int)(d0.y ^ 0x80808080u), (int)(d1.x ^ 0x80808080u),
                           (int)(d1.y ^ 0x80808080u)};
            H[b] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, tb, c_row, 0, 0, 0);
        }
        // bytes of H': per block one dword of lo bytes (^ 0x80) and one of signed hi bytes
        v4i lo = {0, 0, 0, 0x00002080}, hi = {0, 0, 0, 0x00004080};
#pragma unroll
        for (int b = 0; b < 3; b++) {
            const uint32_t p01 = __builtin_amdgcn_perm((uint32_t)H[b][1], (uint32_t)H[b][0], 0x05010400u);  // lo0 lo1 hi0 hi1
            const uint32_t p23 = __builtin_amdgcn_perm((uint32_t)H[b][3], (uint32_t)H[b][2], 0x05010400u);
            lo[b] = (int)(__builtin_amdgcn_perm(p23, p01, 0x05040100u) ^ 0x80808080u);
            hi[b] = (int)__builtin_amdgcn_perm(p23, p01, 0x07060302u);
        }
        const int x = 16 * s + 4 * g, X = T.x * TW + x;
        const bool xok = x < TW && X < p.blur_stride;
#pragma unroll
        for (int o = 0; o < 2; o++) {
            const v4i yh = __builtin_amdgcn_mfma_i32_16x16x64_i8(hi, ta[o], c_zero, 0, 0, 0);
            const v4i yl = __builtin_amdgcn_mfma_i32_16x16x64_i8(lo, ta[o], c_zero, 0, 0, 0);
            // out_r = min(255, t_r >> 16), t_r = (yh << 8) + yl: the high halves of two t's as u16
            // lanes (one v_perm), saturated two at a time (v_pk_min_u16), then their low bytes
            typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
            uint32_t t[4];
#pragma unroll
            for (int r = 0; r < 4; r++) t[r] = ((uint32_t)yh[r] << 8) + (uint32_t)yl[r];
            const u16x2 cap = {255, 255};
            const uint32_t h01 = __builtin_bit_cast(uint32_t, __builtin_elementwise_min(
                __builtin_bit_cast(u16x2, __builtin_amdgcn_perm(t[1], t[0], 0x07060302u)), cap));
            const uint32_t h23 = __builtin_bit_cast(uint32_t, __builtin_elementwise_min(
                __builtin_bit_cast(u16x2, __builtin_amdgcn_perm(t[3], t[2], 0x07060302u)), cap));
            const uint32_t w = __builtin_amdgcn_perm(h23, h01, 0x06040200u);
            if (yok[o] && xok) *reinterpret_cast<uint32_t*>(fb + (off + (o ? ostep : 0u))) = w;
        }
    }
}

#ifndef MAGE_FAST_WAVES_PER_EU
#define MAGE_FAST_WAVES_PER_EU 6  // 80 VGPRs, a few spilled setup values; with the candidates written straight
                                  // to global memory (11.3 KB LDS) 12 workgroups per CU: C2 fast_nms 0.362 ->
                                  // 0.350 ms (5 waves: 86 VGPRs, no spills; 7: 72 VGPRs, 76 B spilled, 0.353)
#endif
#ifndef MAGE_FAST_STAMPS
#define MAGE_FAST_STAMPS 0  // tools/fast_stamps.py: per-phase s_memtime of each wave of frames 0..14
#endif
#if MAGE_FAST_STAMPS
__device__ unsigned long long g_fast_stamps[4096][2][16];
#define FAST_STAMP(k)                                                                                   \
    if ((threadIdx.x & 63) == 0 && f < 15) {                                                           \
        const int t_ = f * p.tiles + T.y * p.tiles_x + T.x;              \
        if (t_ < 4096) g_fast_stamps[t_][threadIdx.x >> 6][k] = __builtin_amdgcn_s_memtime();           \
    }
#else
#define FAST_STAMP(k)
#endif
// One tile of frame f: load, score (gated when G > threshold, see gate_strip), NMS, emission,
// and the fused blur when `blur`.
template <bool kMayGate>
__device__ __forceinline__ void fast_tile(const uint8_t* __restrict__ frames, const FastParams& p, int f, int G,
                                          bool blur, uint32_t* __restrict__ cand, uint32_t* __restrict__ counts,
                                          Tile T)
{
    __shared__ __attribute__((aligned(16))) uint8_t img[LH][LW];
    __shared__ uint32_t sc[SROWS][GX];  // scores; then the blurred tile
    // the tile's candidates (strict 3x3 maxima are never 8-adjacent: <= TCAP): written straight
    // into the tile's slot of the frame's candidate buffer (MAGE_FAST_DIRECT_OUT; no LDS list and
    // copy loop: 3.6 KB less LDS per workgroup), or staged in LDS
    const int tix = T.y * p.tiles_x + T.x;
    uint32_t* const tile_out = cand + (long long)f * p.cand_cap + (long long)tix * TCAP;
    uint32_t* const list = tile_out;
    // gated pass: per wave, the pixels (score row << 7 | score column) that may reach the gate;
    // a wave with more than ICAP of them sends its tile through the exact strips (s_dense)
    constexpr uint32_t ICAP = 512;
    __shared__ __attribute__((aligned(4))) uint16_t items[FAST_THREADS / kWave][ICAP];
    __shared__ uint32_t s_cnt, s_dense;
    FAST_STAMP(0);
    load_tile(frames + (long long)f * p.pitch, p, img, T);
    if (threadIdx.x == 0) s_cnt = s_dense = 0;
    __syncthreads();
    FAST_STAMP(1);
    const bool gated = kMayGate && G > p.threshold;
    uint32_t total = 0;  // gated: the wave's listed pixels
    if (gated) {
        // gated: compass test per strip, then the wave's passing groups scored exactly,
        // compacted over the wave's lanes
        const uint32_t pix = gate_strip(img, sc, G, p, T);
        FAST_STAMP(2);
        const uint32_t cnt = __builtin_popcount(pix);
        uint32_t pre = 0;
#pragma unroll
        for (int j = 0; j < 6; j++) {
            const uint64_t b = __ballot((cnt >> j) & 1u);
            pre += __builtin_amdgcn_mbcnt_hi((uint32_t)(b >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)b, 0u)) << j;
            total += (uint32_t)__builtin_popcountll(b) << j;
        }
        if (total > ICAP) {
            if (__lane_id() == 0) s_dense = 1u;  // this tile goes through the exact strips
        } else {
            uint16_t* wl = items[threadIdx.x / kWave];
            const uint32_t ibase = threadIdx.x << 5;  // item layout: item_row / item_col
            uint32_t rb = pix;
            while (rb) {
                const int b = __builtin_ctz(rb);
                rb &= rb - 1u;
                wl[pre++] = (uint16_t)(ibase | (uint32_t)b);
            }
        }
        FAST_STAMP(3);
        __syncthreads();  // s_dense is final
        FAST_STAMP(4);
        if (s_dense) {
            score_strip(img, sc, p, T);
        } else {
            // the wave's listed pixels, two per lane; the ones that reach G (the only
            // possible maxima) are compacted in place to the front of the list for the NMS
            uint16_t* wl = items[threadIdx.x / kWave];
            const _Float16 gt = (_Float16)(float)G, gt1 = (_Float16)(float)(G + 1);
            const h2 tg = {gt, gt}, tg1 = {gt1, gt1};
            uint8_t* scb = reinterpret_cast<uint8_t*>(&sc[0][0]);
            uint32_t nz = 0;
            for (uint32_t i0 = 0; i0 < total; i0 += 2 * kWave) {
                const uint32_t i = i0 + 2 * __lane_id();
                uint32_t ia = 0, ib = 0;
                bool fa = false, fb = false;
                if (i < total) {
                    const uint32_t pr = *reinterpret_cast<const uint32_t*>(&wl[i]);  // i even: one dword
                    ia = pr & 0xFFFFu;
                    ib = i + 1 < total ? pr >> 16 : ia;
                    const uint32_t ss = score_pixels(img, scb, ia, ib, tg, tg1);
                    fa = (ss & 0xFFu) != 0;
                    fb = i + 1 < total && (ss >> 16) != 0;
                }
                // every lane read its items before any lane writes (writes land below i0 + 128)
                const uint64_t ba = __ballot(fa), bb = __ballot(fb);
                const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(ba >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)ba, 0u)) +
                                       __builtin_amdgcn_mbcnt_hi((uint32_t)(bb >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bb, 0u));
                const uint32_t pa = nz + below;
                if (fa) wl[pa] = (uint16_t)ia;
                if (fb) wl[pa + (fa ? 1u : 0u)] = (uint16_t)ib;
                nz += (uint32_t)(__builtin_popcountll(ba) + __builtin_popcountll(bb));
            }
            total = nz;
            FAST_STAMP(5);
        }
    } else {
        score_strip(img, sc, p, T);
    }
    // the blur only reads the image tile (biased for the i8 MFMA operands in registers) and writes
    // the frame directly: a wave runs it as soon as its own scoring is done, ahead of the barrier
    FAST_STAMP(6);
    if (blur) blur_mfma(img, p, f, T);
    FAST_STAMP(7);
    __syncthreads();
    // strict 3x3 non-maximum suppression (OpenCVModified.cpp:1499-1509) + border filter, four
    // pixels per dword: output group og (score dword og + 1), tile rows [8 * chunk, +8).  Scores
    // are split into even / odd pixels as f16 lanes (1024 + s); per score row the left / right
    // neighbour-aligned copies and the 3-wide maximum are formed once and rolled down, so a
    // pixel's 8-neighbour maximum is max(H3(up), H3(down), left, right).
    if (gated && !s_dense) {
        // gated: every score outside the listed pixels is 0, so the strict 3x3 maxima are among
        // them; per listed output pixel (score rows 1..TH, columns 4..TW+3) the 8 neighbours
        const uint16_t* wl = items[threadIdx.x / kWave];
        const uint8_t* scb = reinterpret_cast<const uint8_t*>(&sc[0][0]);
        constexpr int RB = 4 * GX;  // score row bytes
        for (uint32_t i0 = 0; i0 < total; i0 += kWave) {
            const uint32_t i = i0 + __lane_id();
            bool m = false;
            uint32_t c = 0;
            if (i < total) {
                const uint32_t it = wl[i];
                const int sr = (int)item_row(it), x = (int)item_col(it);
                const int X = T.x * TW + x - 4, Y = T.y * TH + sr - 1;
                if (sr >= 1 && sr <= TH && x >= 4 && x < TW + 4 && X >= p.xlo && X <= p.xhi && Y >= p.ylo &&
                    Y <= p.yhi) {
                    const uint8_t* q = scb + sr * RB + x;
                    const uint32_t v = q[0];
                    const uint32_t nb = max(max(max(q[-RB - 1], q[-RB]), max(q[-RB + 1], q[-1])),
                                            max(max(q[1], q[RB - 1]), max(q[RB], q[RB + 1])));
                    m = v > nb;  // v = 0 never is: its neighbours are >= 0
                    c = ((uint32_t)Y << 20) | ((uint32_t)X << 8) | v;
                }
            }
            const uint64_t b = __ballot(m);
            if (b) {
                uint32_t base = 0;
                if (__lane_id() == 0) base = atomicAdd(&s_cnt, (uint32_t)__builtin_popcountll(b));
                base = __builtin_amdgcn_readfirstlane(base);  // all lanes active here: lane 0's value
                const uint32_t pre = __builtin_amdgcn_mbcnt_hi((uint32_t)(b >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)b, 0u));
                if (m) list[base + pre] = c;
            }
        }
    } else {
        constexpr int OG = TW / 4;  // 30 output groups per row
        const int og = threadIdx.x % 32, chunk = threadIdx.x / 32;
        const int X0 = T.x * TW + 4 * og;
        const int oy0 = 8 * chunk, oy1 = min(oy0 + 8, TH);
        // strict maxima of the lane's 4 x 8 strip as a bit mask: bit 4 r + q = pixel (X0 + q, row oy0 + r)
        uint32_t bits = 0;
        if (og < OG) {
            uint32_t colbits = 0;  // emission window columns (FAST range ∩ RunByImageBorder)
#pragma unroll
            for (int q = 0; q < 4; q++)
                if (X0 + q >= p.xlo && X0 + q <= p.xhi) colbits |= 1u << q;
            auto even = [](uint32_t d) { return as_h2(__builtin_amdgcn_perm(d, 0x64646464u, 0x00060004u)); };
            auto odd = [](uint32_t d) { return as_h2(__builtin_amdgcn_perm(d, 0x64646464u, 0x00070005u)); };
            struct RowV {
                h2 ce, co, le, lo, re, ro, he, ho;  // centre, left, right, 3-wide max (even, odd)
            };
            auto load_row = [&](int srow) {
                RowV v;
                const uint32_t l = sc[srow][og], c = sc[srow][og + 1], r = sc[srow][og + 2];
                const uint32_t L = __builtin_amdgcn_alignbyte(c, l, 3), R = __builtin_amdgcn_alignbyte(r, c, 1);
                v.ce = even(c);
                v.co = odd(c);
                v.le = even(L);
                v.lo = odd(L);
                v.re = even(R);
                v.ro = odd(R);
                v.he = max3h(v.le, v.ce, v.re);
                v.ho = max3h(v.lo, v.co, v.ro);
                return v;
            };
            RowV U = load_row(oy0), M = load_row(oy0 + 1);
            const h2 one = {(_Float16)1.0f, (_Float16)1.0f};
            for (int oy = oy0; oy < oy1; oy++) {
                const RowV D = load_row(oy + 2);
                // ge / go >= 1: strict maximum (scores are integers; a zero score never is one, its
                // neighbours are >= 0); the sign bits of g - 1 are the complement
                const h2 te = M.ce - __builtin_elementwise_maximum(max3h(U.he, D.he, M.le), M.re) - one;
                const h2 to = M.co - __builtin_elementwise_maximum(max3h(U.ho, D.ho, M.lo), M.ro) - one;
                const uint32_t sgn = ((as_u32(te) & 0x80008000u) >> 1) | (as_u32(to) & 0x80008000u);
                const uint32_t nib = ~(((sgn >> 14) & 3u) | ((sgn >> 28) & 0xCu)) & colbits;
                const int Y = T.y * TH + oy;
                if (Y >= p.ylo && Y <= p.yhi) bits |= nib << (4 * (oy - oy0));
                U = M;
                M = D;
            }
        }
        // one LDS atomic per wave: exclusive prefix of the lanes' counts (<= 32) from the
        // ballots of their bit planes, then each lane writes its maxima at base + prefix
        const uint32_t cnt = __builtin_popcount(bits);
        uint32_t pre = 0, total = 0;
#pragma unroll
        for (int j = 0; j < 6; j++) {
            const uint64_t b = __ballot((cnt >> j) & 1u);
            pre += __builtin_amdgcn_mbcnt_hi((uint32_t)(b >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)b, 0u)) << j;
            total += (uint32_t)__builtin_popcountll(b) << j;
        }
        if (total) {
            uint32_t base = 0;
            if (__lane_id() == 0) base = atomicAdd(&s_cnt, total);
            uint32_t idx = __builtin_amdgcn_readfirstlane(base) + pre;
            const uint8_t* scb = reinterpret_cast<const uint8_t*>(&sc[0][0]);
            while (bits) {
                const int b = __builtin_ctz(bits);
                bits &= bits - 1u;
                const int oy = oy0 + (b >> 2), q = b & 3;
                const uint32_t sv = scb[(oy + 1) * (4 * GX) + 4 * (og + 1) + q];
                list[idx++] = ((uint32_t)(T.y * TH + oy) << 20) | ((uint32_t)(X0 + q) << 8) | sv;
            }
        }
    }
    FAST_STAMP(8);
    __syncthreads();  // s_cnt and the tile's list are final
    FAST_STAMP(11);
    // the tile's own slot of the frame's candidate buffer (TCAP entries) and count: no global
    // atomics (the 264 tiles of a 720p frame run at once, and one counter per frame serialised
    // them at the L2)
    const uint32_t n = s_cnt;
    if (threadIdx.x == 0) counts[(long long)f * p.tiles + tix] = n;
    FAST_STAMP(12);
}

__global__ __launch_bounds__(FAST_THREADS, MAGE_FAST_WAVES_PER_EU) void fast_nms_kernel(const uint8_t* __restrict__ frames,
                                                                FastParams p,
                                                                uint32_t* __restrict__ cand,
                                                                uint32_t* __restrict__ counts)
{
    // one workgroup per tile (a persistent loop over tiles was measured 25 % slower: the loop's
    // live state spilled 29 VGPRs / 10 SGPRs at 5 waves per SIMD)
    const int G = p.gate ? *p.gate : 0;
    if (p.gate_next && (blockIdx.x | blockIdx.y | blockIdx.z | threadIdx.x) == 0) {
        *p.gate_next = 255;  // lowered by this batch's select_kernel
        p.redo[0] = 0;
    }
    fast_tile<true>(frames, p, blockIdx.z, G, p.blur != nullptr, cand, counts, Tile{(int)blockIdx.x, (int)blockIdx.y});
}

// The exact (ungated) pass over the frames select_kernel listed in p.redo; no blur (the gated
// pass wrote it).  A small 1-D grid strides over (listed frame, tile): the list is almost always
// empty, and a grid of the frame's 264 tiles x 2 cost 4 us per batch just to dispatch.
constexpr int REDO_BLOCKS = 64;
__global__ __launch_bounds__(FAST_THREADS, 4) void fast_redo_kernel(const uint8_t* __restrict__ frames,
                                                                 FastParams p,
                                                                 uint32_t* __restrict__ cand,
                                                                 uint32_t* __restrict__ counts)
{
    const uint32_t n = p.redo[0], tiles = (uint32_t)p.tiles;
    for (uint32_t w = blockIdx.x; w < n * tiles; w += gridDim.x) {
        const uint32_t z = w / tiles, t = w - z * tiles;
        const int ty = (int)(t / (uint32_t)p.tiles_x), tx = (int)t - ty * p.tiles_x;
        fast_tile<false>(frames, p, (int)p.redo[1 + z], 0, false, cand, counts, Tile{tx, ty});
        __syncthreads();
    }
}

__global__ __launch_bounds__(FAST_THREADS) void fast_score_map_kernel(const uint8_t* __restrict__ src,
                                                                      FastParams p,
                                                                      uint8_t* __restrict__ score)
{
    __shared__ __attribute__((aligned(16))) uint8_t img[LH][LW];
    __shared__ uint32_t sc[SROWS][GX];
    const Tile T{(int)blockIdx.x, (int)blockIdx.y};
    load_tile(src, p, img, T);
    __syncthreads();
    score_strip(img, sc, p, T);
    __syncthreads();
    const uint8_t* scb = reinterpret_cast<const uint8_t*>(&sc[0][0]);
    for (int i = threadIdx.x; i < TW * TH; i += FAST_THREADS) {
        const int oy = i / TW, ox = i - oy * TW;
        const int X = blockIdx.x * TW + ox, Y = blockIdx.y * TH + oy;
        if (X >= p.w || Y >= p.h) continue;
        score[(long long)Y * p.w + X] = scb[(oy + 1) * (4 * GX) + ox + 4];
    }
}

// ------------------------------------------------------------------------------------------
// 2. Retain + ANMS + canonical ordering
// ------------------------------------------------------------------------------------------
constexpr int SEL_THREADS = 1024;
constexpr int KMAX = 8192;     // retained items handled in LDS
constexpr int CELLMAX = 4096;  // grid cells (NumCellsX * NumCellsY)

struct SelectParams {
    int w, h;
    unsigned cand_cap;
    int tiles;  // FAST tiles per frame (per-tile candidate slots of TCAP entries)
    int nfeatures;
    int max_num;  // (int)(nfeatures * FeatureFactor)  (ComputeKeyPoints :723)
    unsigned out_cap;
    int fast_threshold;
    float feature_strength;
    int strong;
    float min_r, max_r;
    int cells_x, cells_y;
    float kp_size;   // PatchSize * layerScale (:716)
    int level;       // octave
    float scale;     // layerScale: pt *= scale (:756-760)
    int accumulate;  // append after the n_out[f] keypoints of the previous levels (Insert)
    uint16_t* lvl;   // per keypoint (level << 8 | rotation); rotation filled by orient_kernel
    const int* gate;  // the gate of this batch's FAST pass (FastParams::gate)
    int* gate_next;   // atomicMin of 15/16 of each frame's `lower` (0: no retain, no gate)
    uint32_t* redo;   // frames to run through the exact path again
};

enum : uint32_t { ST_KMAX = 1u, ST_CELLS = 2u };

__device__ __forceinline__ int cand_x(uint32_t c) { return (int)((c >> 8) & 0xFFFu); }
__device__ __forceinline__ int cand_y(uint32_t c) { return (int)(c >> 20); }
__device__ __forceinline__ int cand_s(uint32_t c) { return (int)(c & 0xFFu); }

static_assert(SEL_THREADS == SORT_THREADS, "select_kernel sorts with the shared LDS sort");

#ifndef MAGE_SELECT_STAMPS
#define MAGE_SELECT_STAMPS 0  // tools/select_stamps.py: per-phase s_memtime of each frame's workgroup
#endif
#if MAGE_SELECT_STAMPS
__device__ unsigned long long g_sel_stamps[1024][16];
#define SEL_STAMP(k) \
    if (threadIdx.x == 0 && f < 1024) g_sel_stamps[f][k] = __builtin_amdgcn_s_memtime()
#else
#define SEL_STAMP(k)
#endif

// Frame f; G is the candidate gate its FAST pass ran with (no gate when G <= fast_threshold).
#ifndef MAGE_GATE_SHIFT
#define MAGE_GATE_SHIFT 4  // next gate = lower - lower / 2^MAGE_GATE_SHIFT (15/16: tools/gate_probe.py)
#endif
__device__ __forceinline__ void select_frame(int f, int G, const uint32_t* __restrict__ cand,
                                             const uint32_t* __restrict__ counts, const SelectParams& p,
                                             mage_keypoint* __restrict__ kp_out, uint32_t* __restrict__ xy_out,
                                             uint32_t* __restrict__ n_out, uint32_t* __restrict__ status)
{
    __shared__ uint32_t hist[256];
    __shared__ uint32_t items[KMAX];
    __shared__ uint32_t sorted[KMAX];
    __shared__ uint32_t cellStart[CELLMAX + 1];
    __shared__ unsigned long long keys[KMAX];
    __shared__ int s_cut, s_K, s_minX, s_maxX, s_minY, s_maxY, s_minS, s_gmax, s_mcd2, s_mode;
    __shared__ float s_rob, s_robInv;

    const int tid = threadIdx.x;
    SEL_STAMP(0);
    // per-tile candidate slots (fast_tile): tile t holds CNT[t] entries at C + t * TCAP
    const uint32_t* C = cand + (long long)f * p.cand_cap;
    const uint32_t* CNT = counts + (long long)f * p.tiles;
    const int base = p.accumulate ? (int)n_out[f] : 0;  // read before any barrier; updated at the end
    for (int i = tid; i < 256; i += SEL_THREADS) hist[i] = 0;
    if (tid == 0) {
        s_K = 0;
        s_minX = s_minY = s_minS = 0x7FFFFFFF;
        s_maxX = s_maxY = -1;
    }
    // tile offsets: all counts fetched at once, exclusive scan by one wave (in `sorted`, free
    // until the cell sort): the candidate count n0 and each tile's count
    const int T = p.tiles;
    uint32_t* tstart = sorted;
    for (int t = tid; t < T; t += SEL_THREADS) tstart[t] = min(CNT[t], (uint32_t)TCAP);
    __syncthreads();
    if (tid < kWave) {
        const int per = (T + kWave) / kWave;
        const int b0 = tid * per, b1 = min(b0 + per, T + 1);
        uint32_t sum = 0;
        for (int i = b0; i < b1; i++) sum += i < T ? tstart[i] : 0u;
        uint32_t incl = sum;
        for (int off = 1; off < kWave; off <<= 1) {
            const uint32_t o = __shfl_up(incl, off);
            if (tid >= off) incl += o;
        }
        uint32_t run = incl - sum;
        for (int i = b0; i < b1; i++) {
            const uint32_t c = i < T ? tstart[i] : 0u;
            tstart[i] = run;
            run += c;
        }
    }
    __syncthreads();
    SEL_STAMP(1);
    const int n0 = (int)tstart[T];
    // the candidates tile by tile (4 threads per tile slot: no binary search per candidate)
    // the thread's first SEL_CR entries of its tile slot are loaded once, all in flight together,
    // and kept in registers for both passes below
    constexpr int SEL_CR = 4;
    uint32_t creg[SEL_CR];
    const int tt0 = tid >> 2;
    const int e0 = tid < 4 * T ? (int)(tstart[tt0 + 1] - tstart[tt0]) : 0;
    const uint32_t* ct0 = C + (long long)tt0 * TCAP;
#pragma unroll
    for (int j = 0; j < SEL_CR; j++) {
        const int jj = (tid & 3) + 4 * j;
        creg[j] = jj < e0 ? ct0[jj] : 0u;
    }
    auto for_each_cand = [&](auto&& fn) {
#pragma unroll
        for (int j = 0; j < SEL_CR; j++)
            if ((tid & 3) + 4 * j < e0) fn(creg[j]);
        for (int j = (tid & 3) + 4 * SEL_CR; j < e0; j += 4) fn(ct0[j]);
        for (int w = tid + SEL_THREADS; w < 4 * T; w += SEL_THREADS) {
            const int t = w >> 2;
            const int e = (int)(tstart[t + 1] - tstart[t]);
            const uint32_t* ct = C + (long long)t * TCAP;
            for (int j = w & 3; j < e; j += 4) fn(ct[j]);
        }
    };
    for_each_cand([&](uint32_t c) { atomicAdd(&hist[cand_s(c)], 1u); });
    __syncthreads();
    SEL_STAMP(2);

    const int N = p.nfeatures;
    if (tid < kWave) {
        // RetainBestFeatures (OpenCVModified.cpp:571-617) by one wave: suffix sums of the
        // histogram (lane l holds bins 4l..4l+3), then the two downward scans as the largest bins
        // whose suffix reaches N and max_num (the reference's loops stop at the first such bin)
        const int minThreshold = p.fast_threshold;
        int sfx[4];
        int run = 0;
#pragma unroll
        for (int j = 3; j >= 0; j--) {
            run += (int)hist[4 * tid + j];
            sfx[j] = run;
        }
        int above = run;  // inclusive suffix over lanes >= tid, then exclusive
#pragma unroll
        for (int off = 1; off < kWave; off <<= 1) {
            const int o = __shfl_down(above, off);
            if (tid + off < kWave) above += o;
        }
        above -= run;
        int hiN = -1, hiM = -1;  // largest bin with suffix >= N / >= max_num
#pragma unroll
        for (int j = 0; j < 4; j++) {
            if (sfx[j] + above >= N) hiN = 4 * tid + j;
            if (sfx[j] + above >= p.max_num) hiM = 4 * tid + j;
        }
#pragma unroll
        for (int m = 32; m >= 1; m >>= 1) {
            hiN = max(hiN, __shfl_xor(hiN, m));
            hiM = max(hiM, __shfl_xor(hiM, m));
        }
        if (tid == 0) {
            int lower = 0;
            if (n0 <= N) {
                s_mode = 0;  // no retain / ANMS: keep all, raster order
                s_cut = 0;
            } else {
                const int minNumThreshold = hiN >= minThreshold ? hiN : minThreshold;
                lower = max((int)__fmul_rn((float)minNumThreshold, p.feature_strength), minThreshold);
                s_cut = max(hiM, lower);
                s_mode = 1;
            }
            // gated FAST pass (gate_strip): only the candidates >= G are here, so the decision
            // above is the reference's only when more than N of them exist and lower >= G;
            // otherwise the frame goes through the exact path again
            if (G > p.fast_threshold && (s_mode == 0 || lower < G)) {
                s_mode = 2;
                const uint32_t k = atomicAdd(&p.redo[0], 1u);
                p.redo[1 + k] = (uint32_t)f;  // fast_redo_kernel rewrites the frame's tile slots
            } else if (p.gate_next) {
                atomicMin(p.gate_next, s_mode == 1 ? lower - (lower >> MAGE_GATE_SHIFT) : 0);
            }
        }
    }
    __syncthreads();
    SEL_STAMP(3);
    if (s_mode == 2) return;
    const int cut = s_cut;
    for_each_cand([&](uint32_t c) {
        if (cand_s(c) >= cut) {
            const int pos = atomicAdd(&s_K, 1);
            if (pos < KMAX) items[pos] = c;
        }
    });
    __syncthreads();
    SEL_STAMP(4);
    int K = s_K;
    if (K > KMAX) {
        if (tid == 0) atomicOr(status, ST_KMAX);
        K = KMAX;
    }
    int P = 1;
    while (P < K) P <<= 1;
    const bool anms = s_mode == 1 && N <= K;  // AdaptiveNonMaximalSuppresion early return :177-180

    if (!anms) {
        for (int i = tid; i < P; i += SEL_THREADS) {
            unsigned long long key = 0;
            if (i < K) {
                uint32_t c = items[i];
                uint32_t raster = (uint32_t)cand_y(c) * (uint32_t)p.w + (uint32_t)cand_x(c);
                key = ((unsigned long long)(0xFFFFFFFFu - raster) << 8) | (unsigned long long)cand_s(c);
            }
            keys[i] = key;
        }
        __syncthreads();
        sort_desc(keys, P);
    } else {
        const int numX = p.cells_x, numY = p.cells_y, ncell = numX * numY;
        if (ncell > CELLMAX) {
            if (tid == 0) {
                atomicOr(status, ST_CELLS);
                n_out[f] = (uint32_t)base;
            }
            return;
        }
        {
            // bounding box and weakest response: per thread, then per wave (butterfly), then one
            // LDS atomic per wave and quantity (1024 threads on 5 words serialised the LDS)
            int mnX = 0x7FFFFFFF, mxX = -1, mnY = 0x7FFFFFFF, mxY = -1, mnS = 0x7FFFFFFF;
            for (int i = tid; i < K; i += SEL_THREADS) {
                const uint32_t c = items[i];
                mnX = min(mnX, cand_x(c));
                mxX = max(mxX, cand_x(c));
                mnY = min(mnY, cand_y(c));
                mxY = max(mxY, cand_y(c));
                mnS = min(mnS, cand_s(c));
            }
#pragma unroll
            for (int m = 32; m >= 1; m >>= 1) {
                mnX = min(mnX, __shfl_xor(mnX, m));
                mxX = max(mxX, __shfl_xor(mxX, m));
                mnY = min(mnY, __shfl_xor(mnY, m));
                mxY = max(mxY, __shfl_xor(mxY, m));
                mnS = min(mnS, __shfl_xor(mnS, m));
            }
            if ((tid & (kWave - 1)) == 0 && mxX >= 0) {
                atomicMin(&s_minX, mnX);
                atomicMax(&s_maxX, mxX);
                atomicMin(&s_minY, mnY);
                atomicMax(&s_maxY, mxY);
                atomicMin(&s_minS, mnS);
            }
        }
        for (int i = tid; i <= ncell; i += SEL_THREADS) cellStart[i] = 0;
        __syncthreads();
        SEL_STAMP(5);
        const int minX = s_minX, maxX = s_maxX, minY = s_minY, maxY = s_maxY;
        if (tid == 0) {
            // robustness factor (OpenCVModified.cpp:205-214), float arithmetic as written
            const int t = p.fast_threshold;
            float hi = __fsub_rn((float)p.strong, (float)t);
            float val = fminf(hi, fmaxf(0.0f, __fsub_rn((float)s_minS, (float)t)));
            float range = fmaxf(0.0f, __fsub_rn(p.max_r, p.min_r));
            float rob = __fsub_rn(p.max_r, __fmul_rn(__fdiv_rn(val, (float)(p.strong - t)), range));
            s_rob = rob;
            s_robInv = __fdiv_rn(1.0f, rob);
            s_gmax = (int)(((double)(maxX - minX)) * ((double)(maxY - minY)) / (double)N);
            int dx = max((maxX - minX) / numX, 1), dy = max((maxY - minY) / numY, 1);
            s_mcd2 = min(dx, dy) * min(dx, dy);
        }
        // counting sort by cell
        for (int i = tid; i < K; i += SEL_THREADS) {
            uint32_t c = items[i];
            int cx = (cand_x(c) - minX) * numX / (maxX + 1 - minX);
            int cy = (cand_y(c) - minY) * numY / (maxY + 1 - minY);
            atomicAdd(&cellStart[cy * numX + cx + 1], 1u);
        }
        __syncthreads();
        if (tid < kWave) {  // exclusive scan of ncell+1 entries by one wave
            const int per = (ncell + 1 + kWave - 1) / kWave;
            const int b0 = tid * per, b1 = min(b0 + per, ncell + 1);
            uint32_t s = 0;
            for (int i = b0; i < b1; i++) s += cellStart[i];
            uint32_t incl = s;
            for (int off = 1; off < kWave; off <<= 1) {
                uint32_t o = __shfl_up(incl, off);
                if (tid >= off) incl += o;
            }
            uint32_t run = incl - s;
            for (int i = b0; i < b1; i++) {
                run += cellStart[i];
                cellStart[i] = run;
            }
        }
        __syncthreads();
        SEL_STAMP(6);
        uint32_t* fill = reinterpret_cast<uint32_t*>(keys);  // cell fill cursors (keys unused yet)
        for (int i = tid; i < ncell; i += SEL_THREADS) fill[i] = cellStart[i];
        __syncthreads();
        for (int i = tid; i < K; i += SEL_THREADS) {
            uint32_t c = items[i];
            int cx = (cand_x(c) - minX) * numX / (maxX + 1 - minX);
            int cy = (cand_y(c) - minY) * numY / (maxY + 1 - minY);
            uint32_t pos = atomicAdd(&fill[cy * numX + cx], 1u);
            sorted[pos] = c;
        }
        __syncthreads();
        SEL_STAMP(7);
        const float rob = s_rob, robInv = s_robInv;
        const int gmax = s_gmax, mcd2 = s_mcd2;
        // Ring search (OpenCVModified.cpp:266-326).  Its result is min(gmax, d^2 to the nearest
        // stronger item): an item in ring d is at least (d - 1) cells of side >= sqrt(mcd2) away,
        // so the rings it stops before cannot lower minR2.  Every ring it can visit lies within
        // D - 1 of the item's cell, D the first ring with max(0, D - 1)^2 mcd2 >= gmax; for small D
        // the (2D - 1)^2 square is searched row by row (a row's cells are one contiguous run of
        // the cell-sorted items) without the ring loop's per-cell bookkeeping, and items are taken
        // in cell order so neighbouring lanes read the same runs.
        int D = 0;
        while (max(0, D - 1) * max(0, D - 1) * mcd2 < gmax && D < 5) D++;
        const bool square = max(0, D - 1) * max(0, D - 1) * mcd2 >= gmax;
        unsigned long long mykeys[KMAX / SEL_THREADS];
#pragma unroll
        for (int q = 0; q < KMAX / SEL_THREADS; q++) {
            int i = tid + q * SEL_THREADS;
            unsigned long long key = 0;
            if (i < K) {
                uint32_t c = sorted[i];
                const int x = cand_x(c), y = cand_y(c), s = cand_s(c);
                const int cx = (x - minX) * numX / (maxX + 1 - minX);
                const int cy = (y - minY) * numY / (maxY + 1 - minY);
                const float strength = (float)s;
                const float sth = strength >= 0 ? __fadd_rn(__fmul_rn(strength, rob), 0.002f)
                                                 : __fadd_rn(__fmul_rn(strength, robInv), 0.002f);
                int minR2 = gmax;
                if (square) {
                    const int x0 = max(cx - (D - 1), 0), x1 = min(cx + (D - 1), numX - 1);
                    const int y0 = max(cy - (D - 1), 0), y1 = min(cy + (D - 1), numY - 1);
                    // (float)s > sth for an integer s in [0, 255]: s >= floor(sth) + 1 (no conversion
                    // per visited item; a branch-free select and one LDS atomic per wave for the
                    // item / key appends measured 1-2 % slower)
                    const int sthi = (int)fminf(floorf(sth), 256.0f) + 1;
                    auto visit = [&](uint32_t o) {
                        const int ddx = x - cand_x(o), ddy = y - cand_y(o);
                        const int d2 = __mul24(ddx, ddx) + __mul24(ddy, ddy);
                        if (cand_s(o) >= sthi) minR2 = min(minR2, d2);
                    };
                    for (int cYY = y0; cYY <= y1; cYY++) {
                        const uint32_t e = cellStart[cYY * numX + x1 + 1];
                        uint32_t qq = cellStart[cYY * numX + x0];
                        // four items of the row's run per step: their LDS reads in flight together
                        for (; qq + 4 <= e; qq += 4) {
                            const uint32_t o0 = sorted[qq], o1 = sorted[qq + 1], o2 = sorted[qq + 2], o3 = sorted[qq + 3];
                            visit(o0);
                            visit(o1);
                            visit(o2);
                            visit(o3);
                        }
                        for (; qq < e; qq++) visit(sorted[qq]);
                    }
                } else {
                    for (int d = 0; max(0, d - 1) * max(0, d - 1) * mcd2 < minR2; d++) {
                        for (int yy = -d; yy <= d; yy++) {
                            const int cYY = cy + yy;
                            if (cYY < 0 || cYY >= numY) continue;
                            const bool edgeRow = (yy == -d || yy == d);
                            const int step = edgeRow ? 1 : max(2 * d, 1);
                            for (int xx = -d; xx <= d; xx += step) {
                                const int cXX = cx + xx;
                                if (cXX < 0 || cXX >= numX) continue;
                                const int cell = cYY * numX + cXX;
                                const uint32_t e = cellStart[cell + 1];
                                for (uint32_t qq = cellStart[cell]; qq < e; qq++) {
                                    uint32_t o = sorted[qq];
                                    if ((float)cand_s(o) > sth) {
                                        int ddx = x - cand_x(o), ddy = y - cand_y(o);
                                        minR2 = min(minR2, ddx * ddx + ddy * ddy);
                                    }
                                }
                            }
                        }
                    }
                }
                uint32_t raster = (uint32_t)y * (uint32_t)p.w + (uint32_t)x;
                key = ((unsigned long long)(uint32_t)minR2 << 40) | ((unsigned long long)s << 32) |
                      (unsigned long long)(0xFFFFFFFFu - raster);
            }
            mykeys[q] = key;
        }
        __syncthreads();  // fill cursors (aliasing keys) are dead now
        SEL_STAMP(8);
        // Top-N preselection: keys order by minR2 first, so with t the largest minR2 such that at
        // least N items have minR2 >= t, the N largest keys are among those items.  When they fit
        // a smaller power of two, only they are sorted (C2: ~2035 of ~2625 -> 2048 keys instead
        // of 4096); the histogram's last bin collects minR2 >= SEL_HB - 1, where the cut is then
        // too coarse and the full sort runs.
        int Psort = P;
        {
            constexpr int SEL_HB = 1024;
            uint32_t* mhist = items;  // dead after the ring search
            __shared__ int s_thr, s_sel, s_fill;
            for (int i = tid; i < SEL_HB; i += SEL_THREADS) mhist[i] = 0;
            if (tid == 0) s_fill = 0;
            __syncthreads();
#pragma unroll
            for (int q = 0; q < KMAX / SEL_THREADS; q++) {
                const int i = tid + q * SEL_THREADS;
                if (i < K) atomicAdd(&mhist[min((int)(mykeys[q] >> 40), SEL_HB - 1)], 1u);
            }
            __syncthreads();
            SEL_STAMP(11);
            if (tid < kWave) {  // lane l: bins 16 l .. 16 l + 15; suffix sums, largest bin reaching N
                constexpr int BPL = SEL_HB / kWave;
                int sfx[BPL];
                int run = 0;
#pragma unroll
                for (int j = BPL - 1; j >= 0; j--) {
                    run += (int)mhist[BPL * tid + j];
                    sfx[j] = run;
                }
                int above = run;
#pragma unroll
                for (int off = 1; off < kWave; off <<= 1) {
                    const int o = __shfl_down(above, off);
                    if (tid + off < kWave) above += o;
                }
                above -= run;
                int tb = -1, cnt = 0;
#pragma unroll
                for (int j = 0; j < BPL; j++)
                    if (sfx[j] + above >= N) {
                        tb = BPL * tid + j;
                        cnt = sfx[j] + above;
                    }
#pragma unroll
                for (int m = 32; m >= 1; m >>= 1) {
                    const int otb = __shfl_xor(tb, m), ocnt = __shfl_xor(cnt, m);
                    if (otb > tb) {
                        tb = otb;
                        cnt = ocnt;
                    }
                }
                if (tid == 0) {
                    s_thr = tb;
                    s_sel = cnt;
                }
            }
            __syncthreads();
            SEL_STAMP(12);
            const int tb = s_thr, csel = s_sel;
            int Pp = SORT_THREADS;
            while (Pp < csel) Pp <<= 1;
            if (tb >= 0 && tb < SEL_HB - 1 && Pp < P) {
#pragma unroll
                for (int q = 0; q < KMAX / SEL_THREADS; q++) {
                    const int i = tid + q * SEL_THREADS;
                    if (i < K && (int)(mykeys[q] >> 40) >= tb) keys[atomicAdd(&s_fill, 1)] = mykeys[q];
                }
                for (int i = csel + tid; i < Pp; i += SEL_THREADS) keys[i] = 0ull;
                Psort = Pp;
            } else {
#pragma unroll
                for (int q = 0; q < KMAX / SEL_THREADS; q++) {
                    int i = tid + q * SEL_THREADS;
                    if (i < P) keys[i] = mykeys[q];
                }
            }
        }
        __syncthreads();
        SEL_STAMP(13);
        sort_desc(keys, Psort);
        SEL_STAMP(9);
    }

    int nout = anms ? min(N, K) : K;
    // ImageData::Insert copies what still fits after the previous levels (ImageData.h:65-70)
    nout = max(min(nout, (int)p.out_cap - base), 0);
    mage_keypoint* kp = kp_out + (long long)f * p.out_cap + base;
    uint32_t* xy = xy_out + (long long)f * p.out_cap + base;
    uint16_t* lv = p.lvl ? p.lvl + (long long)f * p.out_cap + base : nullptr;
    for (int i = tid; i < nout; i += SEL_THREADS) {
        unsigned long long key = keys[i];
        uint32_t raster, s;
        if (anms) {
            raster = 0xFFFFFFFFu - (uint32_t)(key & 0xFFFFFFFFull);
            s = (uint32_t)((key >> 32) & 0xFFu);
        } else {
            raster = 0xFFFFFFFFu - (uint32_t)(key >> 8);
            s = (uint32_t)(key & 0xFFu);
        }
        uint32_t y = raster / (uint32_t)p.w, x = raster - y * (uint32_t)p.w;
        mage_keypoint k;
        k.x = __fmul_rn((float)x, p.scale);
        k.y = __fmul_rn((float)y, p.scale);
        k.size = p.kp_size;
        k.angle = 0.0f;
        k.response = (float)s;
        k.octave = p.level;
        k.class_id = -1;
        kp[i] = k;
        xy[i] = (y << 16) | x;  // level coordinates = the descriptor centre cvRound(pt / layerScale)
        if (lv) lv[i] = (uint16_t)(p.level << 8);
    }
    if (tid == 0) n_out[f] = (uint32_t)(base + nout);
    SEL_STAMP(10);
}

__global__ __launch_bounds__(SEL_THREADS) void select_kernel(const uint32_t* __restrict__ cand,
                                                             const uint32_t* __restrict__ counts, SelectParams p,
                                                             mage_keypoint* __restrict__ kp_out,
                                                             uint32_t* __restrict__ xy_out,
                                                             uint32_t* __restrict__ n_out,
                                                             uint32_t* __restrict__ status)
{
    select_frame(blockIdx.x, p.gate ? *p.gate : 0, cand, counts, p, kp_out, xy_out, n_out, status);
}

// The frames of p.redo after fast_redo_kernel; blockIdx.x strides over the list.
__global__ __launch_bounds__(SEL_THREADS) void select_redo_kernel(const uint32_t* __restrict__ cand,
                                                                  const uint32_t* __restrict__ counts, SelectParams p,
                                                                  mage_keypoint* __restrict__ kp_out,
                                                                  uint32_t* __restrict__ xy_out,
                                                                  uint32_t* __restrict__ n_out,
                                                                  uint32_t* __restrict__ status)
{
    const uint32_t n = p.redo[0];
    for (uint32_t z = blockIdx.x; z < n; z += gridDim.x) {
        select_frame((int)p.redo[1 + z], 0, cand, counts, p, kp_out, xy_out, n_out, status);
        __syncthreads();
    }
}

// ------------------------------------------------------------------------------------------
// 3. Blur-in-window + pre-rotated BRIEF
// ------------------------------------------------------------------------------------------
constexpr int DESC_WAVES = 4;
constexpr int RMAX = 18;  // max |pattern offset| over both tables and all rotations
constexpr int KHMAX = 7;  // max Gaussian half-size (ksize <= 15)

struct LevelImages {
    const uint8_t* base[MAGE_MAX_LEVELS];
    long long pitch[MAGE_MAX_LEVELS];
    int stride[MAGE_MAX_LEVELS];
};

struct DescParams {
    LevelImages lev;  // per level: blurred images (describe_blurred_kernel) or raw (describe_kernel)
    int lw[MAGE_MAX_LEVELS], lh[MAGE_MAX_LEVELS];
    const uint16_t* lvl;  // per keypoint (level << 8 | rotation), null: level 0, rotation 0
    unsigned out_cap;
    int R;      // sampling radius of the pattern rotations in use
    int ksize;  // Gaussian taps (<= 1: no blur)
    int taps[2 * KHMAX + 1];
    int dword_ok;
    int chunks, frames;  // describe_blurred_kernel grid decomposition
    // random pattern (patch sizes other than 15 / 31): rotation-0 table rotated per keypoint by
    // its angle (ComputeOrbDescriptors); kp_angle[7 * index] is the keypoint's angle field
    int random;
    const float* kp_angle;
    const uint4* blur_ops;  // describe_win_kernel: the fused blur's MFMA band operands (blur_operands)
};

// GetComputeOrbDescriptorsValue (OpenCVModified.cpp:442-448): the pattern point rotated in f32
// (x a - y b, x b + y a; no contraction) and rounded half-to-even like cvRound.
__device__ __forceinline__ char4 rotate_test(char4 e, float a, float b)
{
    const float x0 = __fsub_rn(__fmul_rn((float)e.x, a), __fmul_rn((float)e.y, b));
    const float y0 = __fadd_rn(__fmul_rn((float)e.x, b), __fmul_rn((float)e.y, a));
    const float x1 = __fsub_rn(__fmul_rn((float)e.z, a), __fmul_rn((float)e.w, b));
    const float y1 = __fadd_rn(__fmul_rn((float)e.z, b), __fmul_rn((float)e.w, a));
    return make_char4((signed char)__float2int_rn(x0), (signed char)__float2int_rn(y0),
                      (signed char)__float2int_rn(x1), (signed char)__float2int_rn(y1));
}

// (a, b) = ((float)cos, (float)sin) of the angle in radians, angle *= (float)(CV_PI / 180) in
// f32 (ComputeOrbDescriptors :466-467); the f64 cos / sin rounded to f32.
__device__ __forceinline__ void pattern_rotation(float angle_deg, float& a, float& b)
{
    const float ang = __fmul_rn(angle_deg, (float)(3.1415926535897932384626433832795 / 180.0f));
    a = (float)cos((double)ang);
    b = (float)sin((double)ang);
}

// One wave per keypoint.  RB bounds the pattern radius (7: patch 15, 13: patch 31, rotation 0;
// 18: any rotation) and sizes the per-wave LDS, so the default configuration keeps 8 waves per
// SIMD resident.  Interior windows are fetched with aligned dword loads (row segments kept at
// their byte phase `s`); windows touching the border use reflect-101 byte loads.
template <int RB>
__global__ __launch_bounds__(DESC_WAVES * kWave) void describe_kernel(
    DescParams p, const uint32_t* __restrict__ xy_in,
    const uint32_t* __restrict__ n_in, const int8_t* __restrict__ pattern,
    uint8_t* __restrict__ desc_out)
{
    constexpr int RAWMAX = 2 * (RB + KHMAX) + 1;    // raw window side
    constexpr int RAWP = ((RAWMAX + 3 + 3) / 4) * 4;  // row pitch: covers any byte phase
    constexpr int BDMAX = 2 * RB + 1;
    __shared__ __attribute__((aligned(16))) uint8_t raw[DESC_WAVES][RAWMAX * RAWP];
    __shared__ int rowp[DESC_WAVES][RAWMAX * BDMAX];
    __shared__ uint8_t blur[DESC_WAVES][BDMAX * BDMAX];

    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;  // wave: scalar
    const int f = blockIdx.y;
    const int k = blockIdx.x * DESC_WAVES + wave;
    if (k >= (int)n_in[f]) return;
    const int kh = p.ksize > 1 ? p.ksize / 2 : 0;
    const int R = p.R, Rr = R + kh, rawDim = 2 * Rr + 1, bd = 2 * R + 1;
    const uint32_t v = xy_in[(long long)f * p.out_cap + k];
    const int cx = (int)(v & 0xFFFFu), cy = (int)(v >> 16);
    const int lr = p.lvl ? p.lvl[(long long)f * p.out_cap + k] : 0, l = lr >> 8, rot = lr & 0xFF;
    const uint8_t* src = p.lev.base[l] + (long long)f * p.lev.pitch[l];
    const int W = p.lw[l], H = p.lh[l], stride = p.lev.stride[l];
    uint8_t* rw = raw[wave];
    const int x0 = cx - Rr, y0 = cy - Rr;
    const int xa = x0 & ~3, s = x0 - xa;
    const int nd = (s + rawDim + 3) >> 2;  // dwords per row
    if (p.dword_ok && x0 >= 0 && y0 >= 0 && y0 + rawDim <= H && xa + 4 * nd <= W) {
        for (int i = lane; i < rawDim * nd; i += kWave) {
            const int r = i / nd, c = i - r * nd;
            *reinterpret_cast<uint32_t*>(rw + r * RAWP + 4 * c) =
                *reinterpret_cast<const uint32_t*>(src + (long long)(y0 + r) * stride + xa + 4 * c);
        }
    } else {
        for (int i = lane; i < rawDim * rawDim; i += kWave) {
            const int r = i / rawDim, c = i - r * rawDim;
            const int gy = reflect101(y0 + r, H), gx = reflect101(x0 + c, W);
            rw[r * RAWP + s + c] = src[(long long)gy * stride + gx];
        }
    }
    wave_lds_sync();
    const uint8_t* rb = rw + s;  // raw(r, c) = rb[r * RAWP + c]
    if (kh > 0) {
        for (int i = lane; i < rawDim * bd; i += kWave) {
            const int r = i / bd, c = i - r * bd;
            const uint8_t* q = rb + r * RAWP + c;
            int acc = 0;
            for (int t = 0; t < p.ksize; t++) acc += p.taps[t] * q[t];
            rowp[wave][i] = acc;
        }
        wave_lds_sync();
    }
    for (int i = lane; i < bd * bd; i += kWave) {
        const int r = i / bd, c = i - r * bd;
        int o;
        if (kh > 0) {
            int acc = 0;
            for (int t = 0; t < p.ksize; t++) acc += p.taps[t] * rowp[wave][(r + t) * bd + c];
            o = (acc + (1 << 15)) >> 16;
            o = o < 0 ? 0 : (o > 255 ? 255 : o);
        } else {
            o = rb[r * RAWP + c];
        }
        blur[wave][i] = (uint8_t)o;
    }
    wave_lds_sync();
    // rotation: cvRound(angle / 12) % 30 (0 without orientation, OpenCVModified.cpp:748-754, :526)
    // or, for the random pattern, the keypoint angle itself
    const char4* pat = reinterpret_cast<const char4*>(pattern) + (p.random ? 0 : rot * 256);
    float ra = 1.f, rb_ = 0.f;
    if (p.random) pattern_rotation(p.kp_angle[7 * ((long long)f * p.out_cap + k)], ra, rb_);
    unsigned long long* dst = reinterpret_cast<unsigned long long*>(desc_out + ((long long)f * p.out_cap + k) * 32);
#pragma unroll
    for (int chunk = 0; chunk < 4; chunk++) {
        char4 e = pat[chunk * kWave + lane];  // (x0, y0, x1, y1) of bit 64*chunk + lane
        if (p.random) e = rotate_test(e, ra, rb_);
        const int t0 = blur[wave][(R + e.y) * bd + R + e.x];
        const int t1 = blur[wave][(R + e.w) * bd + R + e.z];
        const unsigned long long m = __ballot(t0 < t1);
        if (lane == 0) dst[chunk] = m;
    }
}

// Descriptors from the frame blurred by fast_nms_kernel: each wave handles KPW keypoints; it
// issues the window loads of all of them (aligned dwords, rows kept at byte phase s) before
// the first LDS write, so the L2 round trips overlap, then runs the 256 tests per keypoint.
#ifndef MAGE_DESC_KPW
#define MAGE_DESC_KPW 4
#endif
constexpr int KPW = MAGE_DESC_KPW;
#ifndef MAGE_DESC_KPW7
#define MAGE_DESC_KPW7 8  // one level, radius <= 7 (C2): describe 0.074 ms at 4, 0.069-0.071 at 8, 0.091 at 12 or 16,
                          // 0.095 at 2 (tools/abl.py): more window loads in flight per wave
#endif
constexpr int KPW7 = MAGE_DESC_KPW7;
#ifndef MAGE_DESC_KP_WIDE
#define MAGE_DESC_KP_WIDE 2  // keypoints per wave for the rotated (radius 18) windows: rBRIEF-31 describe 0.205 ms at 1, 0.192 at 2, 0.230 at 3 (pattern rows hoisted; before that 0.254 at 1, 0.306 at 2)
#endif

// f(std::integral_constant<int, j>) for j = 0 .. N-1, unrolled at compile time
template <int N, int J = 0, class F>
__device__ __forceinline__ void static_for(F&& f)
{
    if constexpr (J < N) {
        f(std::integral_constant<int, J>{});
        static_for<N, J + 1>(f);
    }
}
// Compact windows (MAGE_DESC_COMPACT, the default): a keypoint's window is staged as its own
// BDMAX rows x the 16-byte parts that hold its columns (from x0 & ~15), not as whole bricks:
// C2 (patch 15): 15 rows x 2 parts = 30 16-byte loads (480 B) per keypoint instead of 5 x 2
// bricks (80 loads, 1280 B), so two keypoints share one load instruction (lane halves); the
// lines touched drop from 10 to 5 for the ~55 % of windows inside one 32-byte brick column.
// LDS rows have an odd number of 16-byte parts, so the 4-5 dwords a row's tests read start 4
// banks apart for 8 consecutive rows (tests bank as (a / 4) mod 32).
template <int RB, bool MULTI, int KP>
__global__ __launch_bounds__(DESC_WAVES * kWave) void describe_blurred_kernel(
    DescParams p, const uint32_t* __restrict__ xy_in, const uint32_t* __restrict__ n_in,
    const int8_t* __restrict__ pattern, uint8_t* __restrict__ desc_out)
{
    constexpr int BDMAX = 2 * RB + 1;
    constexpr int NP = (BDMAX + 30) / 16;  // 16-byte parts per window row (any column phase)
    constexpr int NI = BDMAX * NP;         // 16-byte items per keypoint
    constexpr int WPC = 16 * (NP | 1);     // LDS row pitch
    constexpr bool PAIR = !MULTI && NI <= 32 && KP % 2 == 0;  // lanes 0-31 / 32-63: two keypoints
    constexpr int NLDC = (NI + kWave - 1) / kWave;
    constexpr int NSLOT = PAIR ? KP / 2 : KP * NLDC;
    __shared__ __attribute__((aligned(16))) uint8_t win[DESC_WAVES][KP][BDMAX * WPC];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;  // wave: scalar
    // XCD-aware 1-D grid (the whole-brick variant below explains it)
    const int xcd = blockIdx.x & 7, slot = blockIdx.x >> 3;
    const int chunk = slot % p.chunks, f = (slot / p.chunks) * 8 + xcd;
    if (f >= p.frames) return;
    const int k0 = (chunk * DESC_WAVES + wave) * KP;
    const int n = (int)n_in[f];
    if (k0 >= n) return;
    const int R = p.R;
    // the tests' pattern rows, issued ahead of the window loads so both round trips overlap
    // (without orientation the wave's keypoints share one set; the per-keypoint loads of the
    // loop below had left each of its 4 chunks waiting on an L2 round trip of its own)
    constexpr int NE = MULTI ? KP : 1;
    const char4* pat = reinterpret_cast<const char4*>(pattern);
    char4 e[NE][4];
    float ang[KP];
#pragma unroll
    for (int q = 0; q < NE; q++) {
        const long long ki = (long long)f * p.out_cap + min(k0 + q, n - 1);
        const int rot = MULTI ? (p.lvl[ki] & 0xFF) : 0;
        const char4* pr = pat + (p.random ? 0 : rot * 256);  // cvRound(angle / 12) % 30 (:526)
#pragma unroll
        for (int c = 0; c < 4; c++) e[q][c] = pr[c * kWave + lane];  // (x0, y0, x1, y1) of bit 64*c + lane
    }
    if (p.random)
#pragma unroll
        for (int q = 0; q < KP; q++) ang[q] = p.kp_angle[7 * ((long long)f * p.out_cap + min(k0 + q, n - 1))];
    // load slot j: keypoint q, item i = row i / NP, part i % NP; keypoints keep the pattern
    // radius from the border (RunByImageBorder), so the clamps only keep reads inside the level
    // (a native vector type: HIP's uint4 struct copies stayed memcpys through a private array,
    // which PromoteAlloca then placed in LDS — 8 KB per workgroup of loads bounced through LDS)
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    u32x4 v[NSLOT];
    static_for<NSLOT>([&](auto jc) {
        constexpr int j = decltype(jc)::value;
        const int q = PAIR ? 2 * j + (lane >> 5) : j / NLDC;
        const int i = PAIR ? (lane & 31) : lane + kWave * (j % NLDC);
        const long long ki = (long long)f * p.out_cap + min(k0 + q, n - 1);
        const int l = MULTI ? (__builtin_amdgcn_readfirstlane(p.lvl[ki]) >> 8) : 0;  // wave-uniform (no PAIR)
        const uint32_t xy = xy_in[ki];
        const uint8_t* src = p.lev.base[l] + (long long)f * p.lev.pitch[l];
        const int bcols = p.lev.stride[l], brows = (p.lh[MULTI ? l : 0] + 3) >> 2;
        const int x0 = (int)(xy & 0xFFFFu) - R, y0 = (int)(xy >> 16) - R;
        const int r = i / NP, pt = i - r * NP;
        const int gy = min(max(y0 + r, 0), 4 * brows - 1);
        const int gx = min(max((x0 & ~15) + 16 * pt, 0), 32 * bcols - 16);
        if (i < NI)
            v[j] = *reinterpret_cast<const u32x4*>(src + ((long long)(gy >> 2) * bcols + (gx >> 5)) * 128 +
                                                   (gy & 3) * 32 + (gx & 31));
    });
    static_for<NSLOT>([&](auto jc) {
        constexpr int j = decltype(jc)::value;
        const int q = PAIR ? 2 * j + (lane >> 5) : j / NLDC;
        const int i = PAIR ? (lane & 31) : lane + kWave * (j % NLDC);
        const int r = i / NP, pt = i - r * NP;
        if (i < NI) *reinterpret_cast<u32x4*>(&win[wave][q][r * WPC + 16 * pt]) = v[j];
    });
    wave_lds_sync();
#pragma unroll
    for (int q = 0; q < KP; q++) {
        const int k = k0 + q;
        if (k >= n) break;
        const long long ki = (long long)f * p.out_cap + k;
        const uint32_t xy = xy_in[ki];
        const uint8_t* wb = &win[wave][q][((int)(xy & 0xFFFFu) - R) & 15];  // (x0 & 15): the window's column phase
        char4 eq[4];
#pragma unroll
        for (int c = 0; c < 4; c++) eq[c] = e[MULTI ? q : 0][c];
        if (p.random) {  // random pattern: rotation by the keypoint angle
            float ra, rb_;
            pattern_rotation(ang[q], ra, rb_);
#pragma unroll
            for (int c = 0; c < 4; c++) eq[c] = rotate_test(eq[c], ra, rb_);
        }
        int t0[4], t1[4];
#pragma unroll
        for (int c = 0; c < 4; c++) {
            t0[c] = wb[(R + eq[c].y) * WPC + R + eq[c].x];
            t1[c] = wb[(R + eq[c].w) * WPC + R + eq[c].z];
        }
        // lane c stores the descriptor's 64-bit word c
        unsigned long long mw = 0;
#pragma unroll
        for (int c = 0; c < 4; c++) {
            const unsigned long long m = __ballot(t0[c] < t1[c]);
            mw = lane == c ? m : mw;
        }
        if (lane < 4) reinterpret_cast<unsigned long long*>(desc_out + ki * 32)[lane] = mw;
    }
}
// Whole-brick windows (MAGE_DESC_COMPACT=0): MULTI = false (one level, no orientation: the
// default configuration): level 0 and rotation 0 without the per-keypoint level lookups.


// Descriptors with the 7-tap Gaussian computed per keypoint window on the matrix cores instead of
// over the whole frame (the default configuration: one level, rotation 0, pattern radius <= 7).
// The 2000 windows of a 720p frame cover about half of its pixels, and the full-frame blur was
// ~30 % of the FAST pass (and its 1 byte / pixel write).  Per keypoint: a 32-row x 48-byte raw
// window (16-byte loads, any 16-byte phase) staged in LDS; the H blocks of the row pass and the
// transposed column pass exactly as blur_mfma (same band operands, same integer arithmetic:
// H = sum tap * b, out = min(255, (sum tap * H + 2^15) >> 16)), giving the 16 x 16 blurred block
// at (cx - R, cy - R); then the 256 tests.  Windows whose 7x7 support leaves the image take the
// reflect-101 gather path.
__global__ __launch_bounds__(DESC_WAVES * kWave) void describe_win_kernel(
    DescParams p, const uint32_t* __restrict__ xy_in, const uint32_t* __restrict__ n_in,
    const int8_t* __restrict__ pattern, uint8_t* __restrict__ desc_out)
{
    typedef int v4i __attribute__((ext_vector_type(4)));
    constexpr int WR = 32, WB = 48;  // window rows (two H blocks), bytes per row (16-byte phase)
    __shared__ __attribute__((aligned(16))) uint8_t raw[DESC_WAVES][KPW][WR * WB];
    __shared__ __attribute__((aligned(16))) uint8_t bw[DESC_WAVES][KPW][256];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int xcd = blockIdx.x & 7, slot = blockIdx.x >> 3;  // XCD-aware, as describe_blurred_kernel
    const int chunk = slot % p.chunks, f = (slot / p.chunks) * 8 + xcd;
    if (f >= p.frames) return;
    const int k0 = (chunk * DESC_WAVES + wave) * KPW;
    const int n = (int)n_in[f];
    if (k0 >= n) return;
    const int R = p.R;
    const uint8_t* src = p.lev.base[0] + (long long)f * p.lev.pitch[0];
    const int stride = p.lev.stride[0], W = p.lw[0], H = p.lh[0];
    // staging items: the 2R + 7 <= 21 window rows the kept outputs read x 3 segments of 16 bytes,
    // one per lane (rows 21..31 of the H blocks feed only output rows >= 15, never read)
    uint4 v[KPW];
    int cx[KPW], cy[KPW], sh[KPW];
#pragma unroll
    for (int q = 0; q < KPW; q++) {
        const uint32_t xy = xy_in[(long long)f * p.out_cap + min(k0 + q, n - 1)];
        cx[q] = (int)(xy & 0xFFFFu);
        cy[q] = (int)(xy >> 16);
        const int wx = cx[q] - R - 8, wy = cy[q] - R - 3;  // band byte 0, H row 0
        const int xa = wx & ~15;
        sh[q] = wx - xa;
        const int i = min(lane, 62), r = i / 3, c = i - 3 * r;
        const int gy = min(max(wy + r, 0), H - 1), gx = min(max(xa + 16 * c, 0), stride - 16);
        v[q] = *reinterpret_cast<const uint4*>(src + (long long)gy * stride + gx);
    }
#pragma unroll
    for (int q = 0; q < KPW; q++)
        if (lane < 63) *reinterpret_cast<uint4*>(&raw[wave][q][(lane / 3) * WB + 16 * (lane % 3)]) = v[q];
    wave_lds_sync();
    const int n16 = lane & 15, g = lane >> 4;
    const uint4 o0 = p.blur_ops[3 * lane], o1 = p.blur_ops[3 * lane + 1];
    const v4i tb = {(int)o0.x, (int)o0.y, (int)o0.z, (int)o0.w};
    const v4i ta = {(int)o1.x, (int)o1.y, (int)o1.z, (int)o1.w};  // output block 0
    const v4i c_row = {32896, 32896, 32896, 32896};                // 128 * 257
    const v4i c_hi = c_row, c_lo = {65664, 65664, 65664, 65664};   // + 2^15
#pragma unroll
    for (int q = 0; q < KPW; q++) {
        const bool inside = cx[q] - R - 3 >= 0 && cx[q] + R + 3 < W && cy[q] - R - 3 >= 0 && cy[q] + R + 3 < H;
        if (inside) {
            // row pass: lane (row n16 of block b, K group g) takes window bytes 16 (g & 1) ..
            // + 15 of row 16 b + n16 (groups 2, 3 meet zero band bytes)
            const int bo = sh[q] + 16 * (g & 1);
            v4i Hb[2];
#pragma unroll
            for (int b = 0; b < 2; b++) {
                const uint32_t* rw = reinterpret_cast<const uint32_t*>(&raw[wave][q][(16 * b + n16) * WB + (bo & ~3)]);
                uint32_t d[5];
#pragma unroll
                for (int i = 0; i < 5; i++) d[i] = rw[i];
                v4i a;
#pragma unroll
                for (int i = 0; i < 4; i++) a[i] = (int)(__builtin_amdgcn_alignbyte(d[i + 1], d[i], bo & 3) ^ 0x80808080u);
                Hb[b] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, tb, c_row, 0, 0, 0);
            }
            v4i lo = {0, 0, 0, 0}, hi = {0, 0, 0, 0};
#pragma unroll
            for (int b = 0; b < 2; b++) {
                const uint32_t p01 = __builtin_amdgcn_perm((uint32_t)Hb[b][1], (uint32_t)Hb[b][0], 0x05010400u);
                const uint32_t p23 = __builtin_amdgcn_perm((uint32_t)Hb[b][3], (uint32_t)Hb[b][2], 0x05010400u);
                lo[b] = (int)(__builtin_amdgcn_perm(p23, p01, 0x05040100u) ^ 0x80808080u);
                hi[b] = (int)(__builtin_amdgcn_perm(p23, p01, 0x07060302u) ^ 0x80808080u);
            }
            // column pass, transposed: lane (output row n16, group g) gets columns 4g .. 4g + 3
            const v4i yh = __builtin_amdgcn_mfma_i32_16x16x64_i8(hi, ta, c_hi, 0, 0, 0);
            const v4i yl = __builtin_amdgcn_mfma_i32_16x16x64_i8(lo, ta, c_lo, 0, 0, 0);
            uint32_t w = 0;
#pragma unroll
            for (int r = 0; r < 4; r++) w |= min(255u, (((uint32_t)yh[r] << 8) + (uint32_t)yl[r]) >> 16) << (8 * r);
            *reinterpret_cast<uint32_t*>(&bw[wave][q][16 * n16 + 4 * g]) = w;
        } else {
            // reflect-101 at the image border (BORDER_REFLECT_101 of the full-frame blur)
            const int bd = 2 * R + 1;
            for (int i = lane; i < bd * bd; i += kWave) {
                const int oy = i / bd, ox = i - oy * bd;
                const int y = cy[q] - R + oy, x = cx[q] - R + ox;
                int acc = 0;
                for (int ty = 0; ty < 7; ty++) {
                    const uint8_t* row = src + (long long)reflect101(y + ty - 3, H) * stride;
                    int hs = 0;
                    for (int tx = 0; tx < 7; tx++) hs += p.taps[tx] * row[reflect101(x + tx - 3, W)];
                    acc += p.taps[ty] * hs;
                }
                bw[wave][q][16 * oy + ox] = (uint8_t)min(255, (acc + (1 << 15)) >> 16);
            }
        }
    }
    wave_lds_sync();
    const char4* pat = reinterpret_cast<const char4*>(pattern);
#pragma unroll
    for (int q = 0; q < KPW; q++) {
        const int k = k0 + q;
        if (k >= n) break;
        const uint8_t* wb = bw[wave][q];
        unsigned long long* dst = reinterpret_cast<unsigned long long*>(desc_out + ((long long)f * p.out_cap + k) * 32);
#pragma unroll
        for (int c = 0; c < 4; c++) {
            const char4 e = pat[c * kWave + lane];  // (x0, y0, x1, y1) of bit 64*c + lane, rotation 0
            const int t0 = wb[(R + e.y) * 16 + R + e.x];
            const int t1 = wb[(R + e.w) * 16 + R + e.z];
            const unsigned long long m = __ballot(t0 < t1);
            if (lane == 0) dst[c] = m;
        }
    }
}

// ------------------------------------------------------------------------------------------
// 4. Pyramid levels > 0: resize(INTER_LINEAR) of the previous level (OpenCVModified.cpp:833)
// ------------------------------------------------------------------------------------------
// OpenCV 3.4.0 8U linear resize (imgproc/src/resize.cpp, non-IPP build): per output column
// xofs / (a0, a1) and per output row yofs / (b0, b1) are the host-computed fixed-point tables
// (saturate_cast<short>(w * 2048)); the horizontal pass is exact in int32; the vertical pass is
// the SSE2 VResizeLinearVec_32s8u formula below the last 16/4-wide block boundary `xv`, the
// scalar FixedPtCast<int, uchar, 22> after it.
struct ResizeParams {
    int sw, sh, sstride;
    long long spitch;
    int dw, dh, dstride;
    long long dpitch;
    int xmax, xv;
    int area2;  // both scales exactly 2: cv::resize takes resizeAreaFast_ instead (xv = its SIMD bound)
    const int* xofs;
    const uint32_t* alpha;  // a0 | a1 << 16
    const int* yofs;
    const uint32_t* beta;   // b0 | b1 << 16
};

__global__ __launch_bounds__(256) void resize_linear_kernel(const uint8_t* __restrict__ src,
                                                           uint8_t* __restrict__ dst, ResizeParams p)
{
    const int f = blockIdx.z, dy = blockIdx.y;
    const int dx = blockIdx.x * blockDim.x + threadIdx.x;
    if (dx >= p.dw) return;
    const uint8_t* S = src + (long long)f * p.spitch;
    if (p.area2) {
        // is_area_fast && iscale_x == iscale_y == 2: INTER_LINEAR becomes INTER_AREA; the SSE2
        // 8-wide blocks round (sum + 2) >> 2, the scalar tail cvRound(sum * 0.25f)
        const uint8_t* s0 = S + (long long)(2 * dy) * p.sstride + 2 * dx;
        const int sum = s0[0] + s0[1] + s0[p.sstride] + s0[p.sstride + 1];
        dst[(long long)f * p.dpitch + (long long)dy * p.dstride + dx] =
            (uint8_t)(dx < p.xv ? (sum + 2) >> 2 : __float2int_rn((float)sum * 0.25f));
        return;
    }
    const int sy = p.yofs[dy];
    const uint8_t* r0 = S + (long long)min(max(sy, 0), p.sh - 1) * p.sstride;
    const uint8_t* r1 = S + (long long)min(max(sy + 1, 0), p.sh - 1) * p.sstride;
    const int sx = p.xofs[dx];
    const uint32_t a = p.alpha[dx], b = p.beta[dy];
    const int a0 = (short)(a & 0xFFFFu), a1 = (short)(a >> 16), b0 = (short)(b & 0xFFFFu), b1 = (short)(b >> 16);
    int h0, h1;
    if (dx < p.xmax) {
        h0 = r0[sx] * a0 + r0[sx + 1] * a1;
        h1 = r1[sx] * a0 + r1[sx + 1] * a1;
    } else {
        h0 = r0[sx] * 2048;
        h1 = r1[sx] * 2048;
    }
    int v;
    if (dx < p.xv)
        v = (((((int)(short)(h0 >> 4)) * b0) >> 16) + ((((int)(short)(h1 >> 4)) * b1) >> 16) + 2) >> 2;
    else
        v = (h0 * b0 + h1 * b1 + (1 << 21)) >> 22;
    dst[(long long)f * p.dpitch + (long long)dy * p.dstride + dx] = (uint8_t)min(max(v, 0), 255);
}

// The same resize with a workgroup per band of RZ_BAND output rows (and frame): the source rows
// the band reads are staged in LDS (dynamic size: rows x source width, from the host's row tables)
// with dword loads, then each thread forms four consecutive output pixels from LDS bytes (exactly
// resize_linear_kernel's arithmetic) and stores them as one dword.  One small workgroup per output
// row left the launch dispatch-bound (0.67 ms for the 3 levels of 256 frames).
constexpr int RZ_MAXW = 4096;  // source rows up to this width (resize_linear_kernel beyond)
constexpr int RZ_BAND = 8;     // output rows per workgroup
constexpr size_t RZ_MAX_LDS = 60 * 1024;

// Source rows of band `band` (first, count) from the host copy of the row table.
inline void rz_band_rows(const int* yofs, int dh, int sh, int area2, int band, int& r0, int& n)
{
    const int d0 = band * RZ_BAND, d1 = std::min(d0 + RZ_BAND, dh) - 1;
    if (area2) {
        r0 = 2 * d0;
        n = 2 * (d1 - d0 + 1);
        return;
    }
    r0 = std::min(std::max(yofs[d0], 0), sh - 1);
    const int r1 = std::min(std::max(yofs[d1] + 1, 0), sh - 1);
    n = r1 - r0 + 1;
}

// LDS bytes per workgroup for a resize (rows of the widest band x padded source width)
inline size_t rz_lds_bytes(const int* yofs, int sw, int sh, int dh, int area2)
{
    int maxn = 0;
    for (int b = 0; b * RZ_BAND < dh; b++) {
        int r0, n;
        rz_band_rows(yofs, dh, sh, area2, b, r0, n);
        maxn = std::max(maxn, n);
    }
    return (size_t)maxn * (size_t)((sw + 15) & ~15);
}

__global__ __launch_bounds__(256) void resize_band_kernel(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                          ResizeParams p)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t rz_rows[];
    const int f = blockIdx.z, tid = threadIdx.x;
    const int d0 = blockIdx.x * RZ_BAND, nd = min(RZ_BAND, p.dh - d0);
    const int swp = (p.sw + 15) & ~15;
    const uint8_t* S = src + (long long)f * p.spitch;
    int r0, r1;
    if (p.area2) {
        r0 = 2 * d0;
        r1 = 2 * (d0 + nd) - 1;
    } else {
        r0 = min(max(p.yofs[d0], 0), p.sh - 1);
        r1 = min(max(p.yofs[d0 + nd - 1] + 1, 0), p.sh - 1);
    }
    const int nr = r1 - r0 + 1;
    const bool aligned = (reinterpret_cast<uintptr_t>(S) & 3) == 0 && (p.sstride & 3) == 0 && (p.sw & 3) == 0;
    if (aligned) {
        const int wq = p.sw >> 2;
        for (int i = tid; i < nr * wq; i += 256) {
            const int r = i / wq, q = i - r * wq;
            reinterpret_cast<uint32_t*>(rz_rows + (size_t)r * swp)[q] =
                reinterpret_cast<const uint32_t*>(S + (long long)(r0 + r) * p.sstride)[q];
        }
    } else {
        for (int i = tid; i < nr * p.sw; i += 256) {
            const int r = i / p.sw, x = i - r * p.sw;
            rz_rows[(size_t)r * swp + x] = S[(long long)(r0 + r) * p.sstride + x];
        }
    }
    __syncthreads();
    const int nq = (p.dw + 3) >> 2;
    if (!p.area2 && nq <= 256) {
        // a thread keeps one 4-pixel column group for the band's rows: its horizontal taps
        // (source column, the two weights, which formula) are read once, not per output pixel
        const int rgn = 256 / nq, x4 = tid % nq, rs = tid / nq;
        if (rs >= rgn) return;
        int sx[4], a0[4], a1[4];
        bool in[4], lin[4], vec[4];
#pragma unroll
        for (int e = 0; e < 4; e++) {
            const int dx = 4 * x4 + e;
            in[e] = dx < p.dw;
            sx[e] = in[e] ? p.xofs[dx] : 0;
            const uint32_t a = in[e] ? p.alpha[dx] : 0u;
            a0[e] = (short)(a & 0xFFFFu);
            a1[e] = (short)(a >> 16);
            lin[e] = dx < p.xmax;
            vec[e] = dx < p.xv;
        }
        for (int dr = rs; dr < nd; dr += rgn) {
            const int dy = d0 + dr;
            const int sy = p.yofs[dy];
            const uint8_t* R0 = rz_rows + (size_t)(min(max(sy, 0), p.sh - 1) - r0) * swp;
            const uint8_t* R1 = rz_rows + (size_t)(min(max(sy + 1, 0), p.sh - 1) - r0) * swp;
            const uint32_t bb = p.beta[dy];
            const int b0 = (short)(bb & 0xFFFFu), b1 = (short)(bb >> 16);
            uint32_t out = 0;
#pragma unroll
            for (int e = 0; e < 4; e++) {
                int h0, h1;
                if (lin[e]) {
                    h0 = R0[sx[e]] * a0[e] + R0[sx[e] + 1] * a1[e];
                    h1 = R1[sx[e]] * a0[e] + R1[sx[e] + 1] * a1[e];
                } else {
                    h0 = R0[sx[e]] * 2048;
                    h1 = R1[sx[e]] * 2048;
                }
                int v;
                if (vec[e])
                    v = (((((int)(short)(h0 >> 4)) * b0) >> 16) + ((((int)(short)(h1 >> 4)) * b1) >> 16) + 2) >> 2;
                else
                    v = (h0 * b0 + h1 * b1 + (1 << 21)) >> 22;
                v = min(max(v, 0), 255);
                out |= in[e] ? (uint32_t)v << (8 * e) : 0u;
            }
            uint8_t* D = dst + (long long)f * p.dpitch + (long long)dy * p.dstride;
            if ((reinterpret_cast<uintptr_t>(D) & 3) == 0 && 4 * x4 + 3 < p.dw) {
                *reinterpret_cast<uint32_t*>(D + 4 * x4) = out;
            } else {
                for (int e = 0; e < 4 && 4 * x4 + e < p.dw; e++) D[4 * x4 + e] = (uint8_t)(out >> (8 * e));
            }
        }
        return;
    }
    for (int it = tid; it < nd * nq; it += 256) {
        const int dr = it / nq, x4 = it - dr * nq, dy = d0 + dr;
        const uint8_t *R0, *R1;
        int b0 = 0, b1 = 0;
        if (p.area2) {
            R0 = rz_rows + (size_t)(2 * dy - r0) * swp;
            R1 = R0 + swp;
        } else {
            const int sy = p.yofs[dy];
            R0 = rz_rows + (size_t)(min(max(sy, 0), p.sh - 1) - r0) * swp;
            R1 = rz_rows + (size_t)(min(max(sy + 1, 0), p.sh - 1) - r0) * swp;
            const uint32_t b = p.beta[dy];
            b0 = (short)(b & 0xFFFFu);
            b1 = (short)(b >> 16);
        }
        uint32_t out = 0;
#pragma unroll
        for (int e = 0; e < 4; e++) {
            const int dx = 4 * x4 + e;
            if (dx >= p.dw) break;
            int v;
            if (p.area2) {
                const int sum = R0[2 * dx] + R0[2 * dx + 1] + R1[2 * dx] + R1[2 * dx + 1];
                v = dx < p.xv ? (sum + 2) >> 2 : __float2int_rn((float)sum * 0.25f);
            } else {
                const int sx = p.xofs[dx];
                const uint32_t a = p.alpha[dx];
                const int a0 = (short)(a & 0xFFFFu), a1 = (short)(a >> 16);
                int h0, h1;
                if (dx < p.xmax) {
                    h0 = R0[sx] * a0 + R0[sx + 1] * a1;
                    h1 = R1[sx] * a0 + R1[sx + 1] * a1;
                } else {
                    h0 = R0[sx] * 2048;
                    h1 = R1[sx] * 2048;
                }
                if (dx < p.xv)
                    v = (((((int)(short)(h0 >> 4)) * b0) >> 16) + ((((int)(short)(h1 >> 4)) * b1) >> 16) + 2) >> 2;
                else
                    v = (h0 * b0 + h1 * b1 + (1 << 21)) >> 22;
                v = min(max(v, 0), 255);
            }
            out |= (uint32_t)v << (8 * e);
        }
        uint8_t* D = dst + (long long)f * p.dpitch + (long long)dy * p.dstride;
        if ((reinterpret_cast<uintptr_t>(D) & 3) == 0 && 4 * x4 + 3 < p.dw) {
            *reinterpret_cast<uint32_t*>(D + 4 * x4) = out;
        } else {
            for (int e = 0; e < 4 && 4 * x4 + e < p.dw; e++) D[4 * x4 + e] = (uint8_t)(out >> (8 * e));
        }
    }
}

// ------------------------------------------------------------------------------------------
// 5. ICAngles (UseOrientation, OpenCVModified.cpp:399-437) + rotation index (:526)
// ------------------------------------------------------------------------------------------
struct OrientParams {
    LevelImages lev;  // unblurred levels
    unsigned out_cap;
    int half_k;
    int umax[32];
    int chunks, frames;  // orient_rows_kernel's XCD-aware 1-D grid
};

// cv::fastAtan2 (OpenCV 3.4.0 core mathfuncs_core, polynomial atan in degrees), each float
// operation rounded as the scalar host code does.
__device__ __forceinline__ float fast_atan2_deg(float y, float x)
{
    const float k = (float)(180 / 3.141592653589793);
    const float p1 = 0.9997878412794807f * k, p3 = -0.3258083974640975f * k;
    const float p5 = 0.1555786518463281f * k, p7 = -0.04432655554792128f * k;
    const float eps = (float)2.2204460492503131e-16;
    const float ax = fabsf(x), ay = fabsf(y);
    float a, c, c2;
    if (ax >= ay) {
        c = __fdiv_rn(ay, __fadd_rn(ax, eps));
        c2 = __fmul_rn(c, c);
        a = __fmul_rn(__fadd_rn(__fmul_rn(__fadd_rn(__fmul_rn(__fadd_rn(__fmul_rn(p7, c2), p5), c2), p3), c2), p1), c);
    } else {
        c = __fdiv_rn(ax, __fadd_rn(ay, eps));
        c2 = __fmul_rn(c, c);
        a = __fsub_rn(90.f, __fmul_rn(__fadd_rn(__fmul_rn(__fadd_rn(__fmul_rn(__fadd_rn(__fmul_rn(p7, c2), p5), c2), p3), c2), p1), c));
    }
    if (x < 0) a = __fsub_rn(180.f, a);
    if (y < 0) a = __fsub_rn(360.f, a);
    return a;
}

// One wave per keypoint: lane u + half_k sums column u of the circular patch (|u| <= umax[|v|])
// of the unblurred level around the keypoint; integer moments m_10 = sum u I, m_01 = sum v I
// are order independent, so the wave reduction equals the reference's loops.
__global__ __launch_bounds__(256) void orient_kernel(mage_keypoint* __restrict__ kp, const uint32_t* __restrict__ xy,
                                                    uint16_t* __restrict__ lvl, const uint32_t* __restrict__ n_in,
                                                    OrientParams p)
{
    const int f = blockIdx.y;
    const int k = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (k >= (int)n_in[f]) return;
    const long long i = (long long)f * p.out_cap + k;
    const int l = lvl[i] >> 8;
    const uint32_t c = xy[i];
    const int cx = (int)(c & 0xFFFFu), cy = (int)(c >> 16);
    const int u = lane - p.half_k;
    int m10 = 0, m01 = 0;
    if (lane <= 2 * p.half_k) {
        const uint8_t* col = p.lev.base[l] + (long long)f * p.lev.pitch[l] + cx + u;
        const int au = abs(u);
        for (int v = -p.half_k; v <= p.half_k; v++) {
            if (au <= p.umax[abs(v)]) {
                const int val = col[(long long)(cy + v) * p.lev.stride[l]];
                m10 += u * val;
                m01 += v * val;
            }
        }
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        m10 += __shfl_xor(m10, off);
        m01 += __shfl_xor(m01, off);
    }
    if (lane == 0) {
        const float angle = fast_atan2_deg((float)m01, (float)m10);
        kp[i].angle = angle;
        // rot = cvRound(angle / ROTATION_INCREMENT_DEGREES) % ROTATION_INCREMENT_COUNT (:526)
        const int rot = ((int)rintf(__fdiv_rn(angle, 12.0f))) % 30;
        lvl[i] = (uint16_t)((l << 8) | rot);
    }
}

// The same moments with a row per lane (5 <= half_k <= 15: lanes 32 s + j hold row v = j - half_k of
// half-wave s's keypoints, OR_KPL of them per half-wave): the row's 2 half_k + 1 bytes come from 9 aligned dword loads
// issued together, are realigned to the window start (v_alignbyte), and two v_dot4_u32_u8 per
// dword against the row's disc mask give sum_u (u + half_k) I and sum_u I; then
// m_10 = sum (u + half_k) I - half_k sum I and m_01 = v sum I, summed over the rows by shuffles.
// Integer sums: identical to orient_kernel's per-pixel loop.
constexpr int OR_ROWS = 32;  // lanes per keypoint
#ifndef MAGE_OR_KPL
#define MAGE_OR_KPL 2  // rBRIEF-31 orient 0.188 ms at 1, 0.183 at 2, 0.187 at 4
#endif
constexpr int OR_KPL = MAGE_OR_KPL;          // keypoints per half-wave
constexpr int ORIENT_PER_BLOCK = 8 * OR_KPL;  // keypoints per 256-thread workgroup
__global__ __launch_bounds__(256) void orient_rows_kernel(mage_keypoint* __restrict__ kp,
                                                          const uint32_t* __restrict__ xy, uint16_t* __restrict__ lvl,
                                                          const uint32_t* __restrict__ n_in, OrientParams p)
{
    __shared__ uint32_t wmask[16][8];  // per |v|: the byte mask of the disc row (0x01 bytes in range)
    const int h = p.half_k;
    if (threadIdx.x < 16 * 8) {
        const int av = threadIdx.x >> 3, d = threadIdx.x & 7;
        const int um = av <= h ? p.umax[av] : -1;  // bytes j in [h - um, h + um]
        uint32_t m = 0;
#pragma unroll
        for (int b = 0; b < 4; b++) {
            const int j = 4 * d + b;
            if (um >= 0 && j >= h - um && j <= h + um) m |= 1u << (8 * b);
        }
        wmask[av][d] = m;
    }
    __syncthreads();
    // XCD-aware 1-D grid (as describe_blurred_kernel): block b runs on XCD b % 8 and every keypoint
    // chunk of frame f gets a block on XCD f % 8, so a frame's level images are fetched into one L2
    // (a 2-D grid spread each frame's chunks over all eight and fetched every level 8 times)
    const int xcd = blockIdx.x & 7, slot = blockIdx.x >> 3;
    const int chunk = slot % p.chunks, f = (slot / p.chunks) * 8 + xcd;
    if (f >= p.frames) return;  // the whole workgroup
    const int lane = threadIdx.x & 63, j = lane & (OR_ROWS - 1);
    const int n = (int)n_in[f];
    if (n == 0 || chunk * ORIENT_PER_BLOCK >= n) return;  // the whole workgroup (no barrier follows)
    const int v = j - h;
    const uint32_t* mrow = wmask[v < 0 ? -v : v];
    // OR_KPL keypoints per half-wave (ORIENT_PER_BLOCK per workgroup): every load of all of them
    // is issued before the first one is used
    int kk[OR_KPL], ll[OR_KPL];
    long long ii[OR_KPL];
    uint32_t cc[OR_KPL];
#pragma unroll
    for (int t = 0; t < OR_KPL; t++) {
        kk[t] = chunk * ORIENT_PER_BLOCK + t * 8 + (threadIdx.x >> 6) * 2 + (lane >> 5);
        ii[t] = (long long)f * p.out_cap + min(kk[t], max(n - 1, 0));
        ll[t] = lvl[ii[t]] >> 8;
        cc[t] = xy[ii[t]];
    }
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    uint32_t d[OR_KPL][9], shv[OR_KPL];
#pragma unroll
    for (int t = 0; t < OR_KPL; t++) {
        const int cx = (int)(cc[t] & 0xFFFFu), cy = (int)(cc[t] >> 16);
        const int l = ll[t];
        // rows past the window (j > 2h) read the window's last row; their sums are discarded
        const int vv = min(v, h);
        const uint8_t* row = p.lev.base[l] + (long long)f * p.lev.pitch[l] + (long long)(cy + vv) * p.lev.stride[l] + cx - h;
        const uintptr_t a = reinterpret_cast<uintptr_t>(row);
        const uint32_t* al = reinterpret_cast<const uint32_t*>(a & ~(uintptr_t)3);
        const uint32_t sh = (uint32_t)(a & 3u);
        shv[t] = sh;
        // only the dwords holding window bytes: the last read byte is x + h + 3 at most, inside the
        // level for every keypoint (the oriented border ceil(h sqrt 2) >= h + 3 for h >= 5)
        const int qlast = (int)(sh + 2 * h) >> 2;
        if (qlast >= 7) {
            // dwords 0..7 all hold window bytes: two 16-byte loads (dword aligned) instead of eight
            // dword loads, a third of the address instructions through the TA
            u32x4 a0, a1;
            __builtin_memcpy(&a0, al, 16);
            __builtin_memcpy(&a1, al + 4, 16);
            d[t][0] = a0[0], d[t][1] = a0[1], d[t][2] = a0[2], d[t][3] = a0[3];
            d[t][4] = a1[0], d[t][5] = a1[1], d[t][6] = a1[2], d[t][7] = a1[3];
            d[t][8] = qlast >= 8 ? al[8] : 0u;
        } else {
#pragma unroll
            for (int q = 0; q < 9; q++) d[t][q] = q <= qlast ? al[q] : 0u;
        }
    }
#pragma unroll
    for (int t = 0; t < OR_KPL; t++) {
        uint32_t s1 = 0, sw = 0;  // sum I, sum (u + h) I over the row
#pragma unroll
        for (int q = 0; q < 8; q++) {
            const uint32_t w = __builtin_amdgcn_alignbyte(d[t][q + 1], d[t][q], shv[t]);  // bytes 4q .. 4q+3 of the row
            const uint32_t m = mrow[q];
            const uint32_t pos = 0x03020100u + 0x04040404u * (uint32_t)q;  // byte j = u + h
            s1 = __builtin_amdgcn_udot4(w, m, s1, false);
            sw = __builtin_amdgcn_udot4(w, pos & (m * 0xFFu), sw, false);
        }
        if (j > 2 * h) s1 = sw = 0;
        int m10 = (int)sw - h * (int)s1, m01 = v * (int)s1;
#pragma unroll
        for (int off = OR_ROWS / 2; off >= 1; off >>= 1) {
            m10 += __shfl_xor(m10, off);
            m01 += __shfl_xor(m01, off);
        }
        if (j == 0 && kk[t] < n) {
            const float angle = fast_atan2_deg((float)m01, (float)m10);
            kp[ii[t]].angle = angle;
            const int rot = ((int)rintf(__fdiv_rn(angle, 12.0f))) % 30;  // (:526)
            lvl[ii[t]] = (uint16_t)((ll[t] << 8) | rot);
        }
    }
}

__global__ void synth_frames_kernel(uint8_t* __restrict__ out, int w, int h, long long pitch,
                                    unsigned t0, unsigned long long seed)
{
    const int f = blockIdx.z;
    const int x = blockIdx.x * blockDim.x + threadIdx.x;
    const int y = blockIdx.y;
    if (x >= w) return;
    const unsigned long long t = (unsigned long long)(t0 + f);
    const unsigned long long u = (unsigned long long)x + 3ull * t, v = (unsigned long long)y + 2ull * t;
    auto mix = [](unsigned long long z) {
        z += 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        return z ^ (z >> 31);
    };
    const unsigned long long K1 = 0x9E3779B97F4A7C15ull, K2 = 0xC2B2AE3D27D4EB4Full;
    unsigned long long base = mix(seed ^ ((u >> 3) * K1) ^ ((v >> 3) * K2));
    unsigned long long fine = mix(seed ^ 0xA5A5A5A5ull ^ ((u / 3) * K1) ^ ((v / 3) * K2));
    int g = (int)(base >> 56) + (int)((fine >> 56) % 49ull) - 24;
    out[(long long)f * pitch + (long long)y * w + x] = (uint8_t)(g < 0 ? 0 : (g > 255 ? 255 : g));
}

}  // namespace

// ------------------------------------------------------------------------------------------
// Host side
// ------------------------------------------------------------------------------------------

struct LevelGeom {
    int w = 0, h = 0, stride = 0;
    long long pitch = 0;
    int bcols = 0;           // blurred level: 32-byte brick columns per brick row (4 image rows)
    long long bpitch = 0;    // blurred level: bytes per frame (bcols x 128 x brick rows)
    float scale = 1.f;
    int nfeatures = 0;
    size_t off = 0, boff = 0, coff = 0;  // pyramid / blurred / candidate offsets (per frame)
    unsigned cand_cap = 0;
    int tiles = 0;    // FAST tiles of the level
    size_t toff = 0;  // per-tile count offset (per frame)
    int xmax = 0, xv = 0;                 // resize tables (levels > 0)
    int area2 = 0;                        // exact 2x: INTER_AREA fast path
    size_t xofs = 0, yofs = 0, alpha = 0, beta = 0;
};

struct Geometry {
    int w = -1, h = -1, L = 0;
    LevelGeom lv[MAGE_MAX_LEVELS];
    size_t pyr_bytes = 0, blur_bytes = 0, cand_total = 0, tile_total = 0;
    std::vector<int> tab_ints;
    std::vector<uint32_t> tab_words;
    bool tab_valid = false;
};

struct OrbDetector {
    mage_orb_settings s{};
    int device = 0;
    int taps[2 * KHMAX + 1] = {0};
    int R = 7;
    bool random_pattern = false;  // PatchSize not 15 / 31: MakeRandomPattern + per-keypoint rotation
    Geometry geo;
    DeviceBuffer pattern, cand, counts, xy, status, img, kp, desc, n, blurred, pyr, rtab, lvl, blur_ops;
    // candidate gates (gate_strip): int[2][MAGE_MAX_LEVELS], slot gate_par is read by the next
    // batch, the other slot is re-armed and lowered by it; redo lists per level
    DeviceBuffer gates, redo;
    int gate_par = 0;
    uint32_t last_batch = 0;  // redo list stride of the last batch
};

// cv::resize(INTER_LINEAR) 8UC1 tables from a sw x sh source to dw x dh (OpenCV 3.4.0
// resize.cpp resizeGeneric_ setup, see resize_linear_kernel): per output column xofs and the
// fixed-point (a0, a1), per output row yofs and (b0, b1), appended to ints / words; the offsets,
// xmax (first column that reads the last source column), the SIMD bound xv and the exact-2x
// INTER_AREA switch go to v.
void resize_tables(int sw, int sh, int dw, int dh, std::vector<int>& ints, std::vector<uint32_t>& words, LevelGeom& v)
{
    struct Dim { int w, h; };
    const Dim src{sw, sh}, dst{dw, dh};
    const double scale_x = 1. / ((double)dst.w / src.w), scale_y = 1. / ((double)dst.h / src.h);
    v.xmax = dst.w;
    v.xofs = ints.size();
    v.alpha = words.size();
    for (int dx = 0; dx < dst.w; dx++) {
        float fx = (float)((dx + 0.5) * scale_x - 0.5);
        int sx = (int)std::floor(fx);
        fx -= sx;
        if (sx < 0) fx = 0, sx = 0;
        if (sx + 1 >= src.w) {
            v.xmax = std::min(v.xmax, dx);
            if (sx >= src.w - 1) fx = 0, sx = src.w - 1;
        }
        ints.push_back(sx);
        const int a0 = (int)std::lrint((1.f - fx) * 2048), a1 = (int)std::lrint(fx * 2048);
        words.push_back((uint32_t)(uint16_t)a0 | ((uint32_t)(uint16_t)a1 << 16));
    }
    v.yofs = ints.size();
    v.beta = words.size();
    for (int dy = 0; dy < dst.h; dy++) {
        float fy = (float)((dy + 0.5) * scale_y - 0.5);
        int sy = (int)std::floor(fy);
        fy -= sy;
        ints.push_back(sy);
        const int b0 = (int)std::lrint((1.f - fy) * 2048), b1 = (int)std::lrint(fy * 2048);
        words.push_back((uint32_t)(uint16_t)b0 | ((uint32_t)(uint16_t)b1 << 16));
    }
    int xv = 0;
    while (xv <= dst.w - 16) xv += 16;
    while (xv < dst.w - 4) xv += 4;
    v.xv = xv;
    v.area2 = scale_x == 2.0 && scale_y == 2.0;
    if (v.area2) v.xv = dst.w / 8 * 8;
}

mage_status resize_linear_device(const uint8_t* src, int sw, int sh, int sstride, uint8_t* dst, int dw, int dh,
                                 int dstride, hipStream_t st)
{
    MAGE_REQUIRE(src && dst && sw > 0 && sh > 0 && dw > 0 && dh > 0 && sstride >= sw && dstride >= dw, MAGE_EINVAL,
                 "resize: invalid image geometry");
    // the tables of the last geometry stay in this thread's stream scratch; a new geometry is
    // uploaded (and waited for: the source vectors are pageable) before the launch
    struct Key {
        int dev, sw, sh, dw, dh;
        hipStream_t st;
        const void* tab;
    };
    thread_local std::vector<Key> cache;
    int dev = 0;
    MAGE_HIP(hipGetDevice(&dev));
    Key* k = nullptr;
    for (auto& c : cache)  // one entry per (device, stream): the scratch holds one table set
        if (c.dev == dev && c.st == st) k = &c;
    if (k && !(k->sw == sw && k->sh == sh && k->dw == dw && k->dh == dh)) k->sw = -1;
    std::vector<int> ints;
    std::vector<uint32_t> words;
    LevelGeom v;
    resize_tables(sw, sh, dw, dh, ints, words, v);
    const size_t ib = ints.size() * 4, wb = words.size() * 4;
    uint8_t* tab = static_cast<uint8_t*>(stream_scratch(st, STREAM_RESIZE_TABLES, ib + wb));
    if (!tab) return MAGE_ENOMEM;
    if (!k || k->tab != tab || k->sw < 0) {
        MAGE_HIP(hipMemcpyAsync(tab, ints.data(), ib, hipMemcpyHostToDevice, st));
        MAGE_HIP(hipMemcpyAsync(tab + ib, words.data(), wb, hipMemcpyHostToDevice, st));
        MAGE_HIP(hipStreamSynchronize(st));
        if (k) *k = Key{dev, sw, sh, dw, dh, st, tab};
        else cache.push_back(Key{dev, sw, sh, dw, dh, st, tab});
    }
    const int* it = reinterpret_cast<const int*>(tab);
    const uint32_t* wt = reinterpret_cast<const uint32_t*>(tab + ib);
    ResizeParams rp{};
    rp.sw = sw;
    rp.sh = sh;
    rp.sstride = sstride;
    rp.dw = dw;
    rp.dh = dh;
    rp.dstride = dstride;
    rp.xmax = v.xmax;
    rp.xv = v.xv;
    rp.area2 = v.area2;
    rp.xofs = it + v.xofs;
    rp.yofs = it + v.yofs;
    rp.alpha = wt + v.alpha;
    rp.beta = wt + v.beta;
    const size_t lds = rz_lds_bytes(ints.data() + v.yofs, sw, sh, dh, v.area2);
    if (rp.sw <= RZ_MAXW && lds <= RZ_MAX_LDS)
        launch("image.resize", resize_band_kernel, dim3((dh + RZ_BAND - 1) / RZ_BAND, 1, 1), dim3(256), lds, st, src, dst,
               rp);
    else
        launch("image.resize", resize_linear_kernel, dim3((dw + 255) / 256, dh, 1), dim3(256), 0, st, src, dst, rp);
    MAGE_HIP(hipGetLastError());
    return MAGE_OK;
}

namespace {

// MakeRandomPattern (OpenCVModified.cpp:551-560) with OpenCV 3.4.0's cv::RNG (multiply-with-carry:
// state = (unsigned)state * 4164903690 + (state >> 32); uniform(a, b) = a + next() % (b - a)),
// seed 0x34985739; stored as (x0, y0, x1, y1) per test like the pre-rotated tables.
void make_random_pattern(int patch, int8_t out[1024])
{
    uint64_t st = 0x34985739u;
    auto uniform = [&](int a, int b) {
        st = (uint64_t)(uint32_t)st * 4164903690ull + (st >> 32);
        return a == b ? a : (int)((uint32_t)st % (uint32_t)(b - a) + (uint32_t)a);
    };
    for (int i = 0; i < 512; i++) {
        out[2 * i] = (int8_t)uniform(-patch / 2, patch / 2 + 1);
        out[2 * i + 1] = (int8_t)uniform(-patch / 2, patch / 2 + 1);
    }
}

// cv::getGaussianKernel(ksize, 2, CV_32F) -> convertTo(CV_32S, 1<<8) (OpenCV 3.4.0
// createSeparableLinearFilter, 8U smoothing path; see DESIGN.md §Blur for why this path).
// Lane operands of blur_mfma for the 7 taps, 3 x uint4 per lane (i8 bytes):
//   [0] row-pass B: B[k = 16 g + j][n] = tap[k - n - 5]
//   [1], [2] col-pass A of output block o = 0, 1: A[m = n][K element 4 b + r] = tap of H row
//            16 b - 3 + 4 g + r for output row 16 o + m = tap[16 (b - o) + 4 g + r - n] (b < 3)
// with n = lane & 15, g = lane >> 4, out-of-band taps 0.
void blur_operands(const int* taps, uint32_t out[64 * 12])
{
    auto tap = [&](int t) -> uint32_t { return (t >= 0 && t <= 6) ? (uint32_t)taps[t] & 0xFFu : 0u; };
    for (int lane = 0; lane < 64; lane++) {
        const int n = lane & 15, g = lane >> 4;
        uint32_t* o = out + 12 * lane;
        for (int d = 0; d < 4; d++) {
            uint32_t w = 0;
            for (int e = 0; e < 4; e++) w |= tap(16 * g + 4 * d + e - n - 5) << (8 * e);
            o[d] = w;
        }
        // dword 3 (K slots 12..15 of the lane's group): {-64, 1, 0, 0}, the partner of the
        // bias bytes blur_mfma keeps in the A operands' dword 3 (an A dword 3 of 0 adds nothing)
        for (int ob = 0; ob < 2; ob++)
            for (int b = 0; b < 4; b++) {
                uint32_t w = 0;
                if (b < 3)
                    for (int r = 0; r < 4; r++) w |= tap(16 * (b - ob) + 4 * g + r - n) << (8 * r);
                else
                    w = 0x000001C0u;
                o[4 + 4 * ob + b] = w;
            }
    }
}

void gaussian_taps(int ksize, double sigma, int* taps)
{
    std::vector<float> cf(ksize);
    double sum = 0;
    double sg = sigma > 0 ? sigma : ((ksize - 1) * 0.5 - 1) * 0.3 + 0.8;
    double scale2 = -0.5 / (sg * sg);
    for (int i = 0; i < ksize; i++) {
        double x = i - (ksize - 1) * 0.5;
        cf[i] = (float)std::exp(scale2 * x * x);
        sum += cf[i];
    }
    sum = 1. / sum;
    for (int i = 0; i < ksize; i++) {
        cf[i] = (float)(cf[i] * sum);
        taps[i] = (int)std::lrint((double)cf[i] * 256.0);
    }
}

mage_status validate(const OrbDetector* o, int w, int h, int stride)
{
    MAGE_REQUIRE(o != nullptr, MAGE_EINVAL, "null detector");
    MAGE_REQUIRE(w > 0 && h > 0 && stride >= w, MAGE_EINVAL, "bad image geometry");
    MAGE_REQUIRE(w <= 4095 && h <= 4095, MAGE_EUNSUPPORTED, "frames up to 4095x4095 supported");
    return MAGE_OK;
}

// Pyramid geometry (DetectAndCompute :785-804): layerScale = (float)pow(f, l) (getScale :564-567),
// level size (cvRound(cols / scale), cvRound(rows / scale)); per-level budget (ComputeKeyPoints
// :659-669) in float as written.  Levels > 0 live in one device buffer, rows padded to 4 bytes.
void level_geometry(OrbDetector* o, int w, int h)
{
    const mage_orb_settings& s = o->s;
    Geometry& g = o->geo;
    g.w = w;
    g.h = h;
    g.L = (int)s.nlevels;
    const float factor = 1.0f / s.scale_factor;
    float nd = (int)s.nfeatures * (1 - factor) / (1 - (float)std::pow((double)factor, (double)g.L));
    int sum = 0;
    size_t off = 0, boff = 0, coff = 0, toff = 0;
    for (int l = 0; l < g.L; l++) {
        LevelGeom& v = g.lv[l];
        v.scale = (float)std::pow((double)s.scale_factor, (double)l);
        v.w = l == 0 ? w : (int)std::lrint((float)w / v.scale);
        v.h = l == 0 ? h : (int)std::lrint((float)h / v.scale);
        v.stride = (v.w + 3) & ~3;
        v.pitch = (long long)v.stride * v.h;
        v.off = l == 0 ? 0 : off;
        if (l > 0) off += (size_t)v.pitch;
        v.bcols = (v.stride + 31) / 32;
        v.bpitch = (long long)v.bcols * 128 * ((v.h + 3) / 4);
        v.boff = boff;
        boff += (size_t)v.bpitch;
        v.tiles = ((v.w + TW - 1) / TW) * ((v.h + TH - 1) / TH);
        v.cand_cap = (unsigned)v.tiles * TCAP;
        v.coff = coff;
        coff += v.cand_cap;
        v.toff = toff;
        toff += v.tiles;
        if (l < g.L - 1) {
            v.nfeatures = (int)std::lrint(nd);
            sum += v.nfeatures;
            nd *= factor;
        } else {
            v.nfeatures = std::max((int)s.nfeatures - sum, 0);
        }
    }
    g.pyr_bytes = off;
    g.blur_bytes = boff;
    g.cand_total = coff;
    g.tile_total = toff;
    // resize(INTER_LINEAR) tables of levels > 0 (OpenCV 3.4.0 resize.cpp, see resize_linear_kernel)
    std::vector<int> ints;
    std::vector<uint32_t> words;
    for (int l = 1; l < g.L; l++) {
        resize_tables(g.lv[l - 1].w, g.lv[l - 1].h, g.lv[l].w, g.lv[l].h, ints, words, g.lv[l]);
    }
    g.tab_ints = ints;
    g.tab_words = words;
    g.tab_valid = false;
}

mage_status run_batch(OrbDetector* o, const uint8_t* d_frames, uint32_t batch, int w, int h,
                      int stride, long long pitch, mage_keypoint* d_kp, uint8_t* d_desc,
                      uint32_t cap, uint32_t* d_n, hipStream_t st)
{
    const mage_orb_settings& s = o->s;
    Geometry& g = o->geo;
    if (g.w != w || g.h != h || g.L != (int)s.nlevels) level_geometry(o, w, h);
    const int L = g.L;
    // select_kernel's tile offsets live in its KMAX-entry LDS array (frames up to ~29 MP)
    MAGE_REQUIRE(g.lv[0].tiles < KMAX, MAGE_EUNSUPPORTED, "frame too large for the candidate tile table");
    const bool multi = L > 1 || s.use_orientation;
    mage_status r;
    if ((r = o->cand.reserve((size_t)batch * g.cand_total * 4)) != MAGE_OK) return r;
    if ((r = o->counts.reserve((size_t)batch * g.tile_total * 4)) != MAGE_OK) return r;
    if ((r = o->xy.reserve((size_t)batch * std::max(cap, 1u) * 4)) != MAGE_OK) return r;
    // the sticky status word starts at zero (a fresh allocation may hold stale bytes)
    const bool fresh_status = o->status.ptr == nullptr;
    if ((r = o->status.reserve(4)) != MAGE_OK) return r;
    if (fresh_status) MAGE_HIP(hipMemsetAsync(o->status.ptr, 0, 4, st));
    // gates start at 0 (no gate: the first batch runs the exact path and sets the next gate)
    const bool fresh_gates = o->gates.ptr == nullptr;
    if ((r = o->gates.reserve(2 * MAGE_MAX_LEVELS * sizeof(int))) != MAGE_OK) return r;
    if (fresh_gates) MAGE_HIP(hipMemsetAsync(o->gates.ptr, 0, 2 * MAGE_MAX_LEVELS * sizeof(int), st));
    if ((r = o->redo.reserve((size_t)L * (1 + batch) * 4)) != MAGE_OK) return r;
    o->last_batch = batch;
    int* gate_cur = o->gates.as<int>() + o->gate_par * MAGE_MAX_LEVELS;
    int* gate_nxt = o->gates.as<int>() + (1 - o->gate_par) * MAGE_MAX_LEVELS;
    o->gate_par ^= 1;
    if (multi && (r = o->lvl.reserve((size_t)batch * std::max(cap, 1u) * 2)) != MAGE_OK) return r;
    if (L > 1 && (r = o->pyr.reserve((size_t)batch * g.pyr_bytes)) != MAGE_OK) return r;
    if (!g.tab_valid && L > 1) {
        const size_t ib = g.tab_ints.size() * 4, wb = g.tab_words.size() * 4;
        if ((r = o->rtab.reserve(ib + wb)) != MAGE_OK) return r;
        MAGE_HIP(hipMemcpy(o->rtab.ptr, g.tab_ints.data(), ib, hipMemcpyHostToDevice));
        MAGE_HIP(hipMemcpy(o->rtab.as<uint8_t>() + ib, g.tab_words.data(), wb, hipMemcpyHostToDevice));
        g.tab_valid = true;
    }

    // level images: 0 = the caller's frames, > 0 = the pyramid buffer (batch-major per level)
    LevelImages raw{};
    for (int l = 0; l < L; l++) {
        if (l == 0) {
            raw.base[0] = d_frames;
            raw.pitch[0] = pitch;
            raw.stride[0] = stride;
        } else {
            raw.base[l] = o->pyr.as<uint8_t>() + (size_t)batch * g.lv[l].off;
            raw.pitch[l] = g.lv[l].pitch;
            raw.stride[l] = g.lv[l].stride;
        }
    }
    if (L > 1) {
        const int* ints = o->rtab.as<int>();
        const uint32_t* words = reinterpret_cast<const uint32_t*>(o->rtab.as<uint8_t>() + g.tab_ints.size() * 4);
        KernelTimer _kt("orb.pyramid", st);
        for (int l = 1; l < L; l++) {
            const LevelGeom &src = g.lv[l - 1], &dst = g.lv[l];
            ResizeParams rp{};
            rp.sw = src.w;
            rp.sh = src.h;
            rp.sstride = raw.stride[l - 1];
            rp.spitch = raw.pitch[l - 1];
            rp.dw = dst.w;
            rp.dh = dst.h;
            rp.dstride = dst.stride;
            rp.dpitch = dst.pitch;
            rp.xmax = dst.xmax;
            rp.xv = dst.xv;
            rp.area2 = dst.area2;
            rp.xofs = ints + dst.xofs;
            rp.yofs = ints + dst.yofs;
            rp.alpha = words + dst.alpha;
            rp.beta = words + dst.beta;
            const size_t lds = rz_lds_bytes(g.tab_ints.data() + dst.yofs, src.w, src.h, dst.h, dst.area2);
            if (src.w <= RZ_MAXW && lds <= RZ_MAX_LDS)
                hipLaunchKernelGGL(resize_band_kernel, dim3((dst.h + RZ_BAND - 1) / RZ_BAND, 1, batch), dim3(256), lds, st,
                                   raw.base[l - 1], const_cast<uint8_t*>(raw.base[l]), rp);
            else
                hipLaunchKernelGGL(resize_linear_kernel, dim3((dst.w + 255) / 256, dst.h, batch), dim3(256), 0, st,
                                   raw.base[l - 1], const_cast<uint8_t*>(raw.base[l]), rp);
        }
    }
    MAGE_HIP(hipGetLastError());

    // the default 7-tap Gaussian is fused into the FAST pass (the tile is already in LDS);
    // other kernel sizes blur inside the descriptor windows instead
    // MAGE_WIN_BLUR=1 (experiment, off by default): in the default configuration (one level,
    // rotation 0, radius <= 7, 16-byte aligned frames) blur per keypoint window inside
    // describe_win_kernel instead of over the frame.  Bit-exact, but at C2 it moved 0.16 ms into
    // describe for 0.09 ms out of FAST, so the fused frame blur stays the default.
    static const bool win_blur_opt = getenv("MAGE_WIN_BLUR") && getenv("MAGE_WIN_BLUR")[0] == '1';
    const bool win_blur = win_blur_opt && cap > 0 && s.gaussian_kernel_size == 7 && L == 1 && !s.use_orientation &&
                          !o->random_pattern && o->R <= 7 && stride % 16 == 0 && pitch % 16 == 0 &&
                          (uintptr_t)d_frames % 16 == 0;
    const bool fused_blur = cap > 0 && s.gaussian_kernel_size == 7 && !win_blur;
    if (fused_blur && (r = o->blurred.reserve((size_t)batch * g.blur_bytes)) != MAGE_OK) return r;
    LevelImages blurred{};
    const int half = (int)s.patch_size / 2;
    // RunByImageBorder(halfPatchSize), or cvCeil(halfPatchSize * sqrt(2.f)) when orienting (:711-712)
    const int border = s.use_orientation ? (int)std::ceil(half * std::sqrt(2.0f)) : half;
    for (int l = 0; l < L; l++) {
        const LevelGeom& v = g.lv[l];
        const int W = v.w, H = v.h;
        FastParams fp{};
        fp.w = W;
        fp.h = H;
        fp.stride = raw.stride[l];
        fp.pitch = raw.pitch[l];
        fp.threshold = std::min(std::max((int)s.fast_threshold, 0), 255);
        fp.xlo = std::max(3, border);
        fp.xhi = std::min(W - 4, W - border - 1);
        fp.ylo = std::max(3, border);
        fp.yhi = std::min(H - 4, H - border - 1);
        if (H <= 2 * border || W <= 2 * border) fp.xhi = -1;  // RunByImageBorder clears all
        fp.cand_cap = v.cand_cap;
        fp.tiles = v.tiles;
        fp.tiles_x = (W + TW - 1) / TW;
        fp.dword_ok = (fp.stride % 4 == 0) && (fp.pitch % 4 == 0) && ((uintptr_t)raw.base[l] % 4 == 0);
        fp.qword_ok = (fp.stride % 8 == 0) && (fp.pitch % 8 == 0) && ((uintptr_t)raw.base[l] % 8 == 0);
        if (fused_blur) {
            blurred.base[l] = o->blurred.as<uint8_t>() + (size_t)batch * v.boff;
            blurred.pitch[l] = v.bpitch;
            blurred.stride[l] = v.bcols;  // brick layout (BLUR_BRICK): brick columns, not bytes
            fp.blur = const_cast<uint8_t*>(blurred.base[l]);
            fp.blur_stride = v.stride;
            fp.blur_pitch = v.bpitch;
            fp.blur_bcols = v.bcols;
            fp.blur_ops = o->blur_ops.as<uint4>();
        }
        uint32_t* cand = o->cand.as<uint32_t>() + (size_t)batch * v.coff;
        uint32_t* counts = o->counts.as<uint32_t>() + (size_t)batch * v.toff;  // every tile writes its count
        uint32_t* redo = o->redo.as<uint32_t>() + (size_t)l * (1 + batch);
        fp.gate = gate_cur + l;
        fp.gate_next = gate_nxt + l;
        fp.redo = redo;
        const dim3 fgrid((W + TW - 1) / TW, (H + TH - 1) / TH, batch);
        launch("orb.fast_nms", fast_nms_kernel, fgrid, dim3(FAST_THREADS), 0, st, raw.base[l], fp, cand, counts);
        MAGE_HIP(hipGetLastError());

        SelectParams sp{};
        sp.w = W;
        sp.h = H;
        sp.cand_cap = v.cand_cap;
        sp.tiles = v.tiles;
        sp.nfeatures = v.nfeatures;  // nfeaturesPerLevel[level] (:659-669)
        sp.max_num = (int)((float)v.nfeatures * s.feature_factor);
        sp.out_cap = cap;
        sp.fast_threshold = (int)s.fast_threshold;
        sp.feature_strength = s.feature_strength;
        sp.strong = s.strong_response;
        sp.min_r = s.min_robust_factor;
        sp.max_r = s.max_robust_factor;
        sp.cells_x = s.num_cells_x;
        sp.cells_y = s.num_cells_y;
        sp.kp_size = (float)s.patch_size * v.scale;
        sp.level = l;
        sp.scale = v.scale;
        sp.accumulate = l > 0;
        sp.lvl = multi ? o->lvl.as<uint16_t>() : nullptr;
        sp.gate = gate_cur + l;
        sp.gate_next = gate_nxt + l;
        sp.redo = redo;
        launch("orb.select", select_kernel, dim3(batch), dim3(SEL_THREADS), 0, st, cand, counts, sp, d_kp,
               o->xy.as<uint32_t>(), d_n, o->status.as<uint32_t>());
        MAGE_HIP(hipGetLastError());
        // frames whose gate was above their retain bound: the exact path (no-ops when none)
        // (small grids: a frame rarely takes this path, and an empty list should cost little)
        launch("orb.fast_redo", fast_redo_kernel, dim3(REDO_BLOCKS), dim3(FAST_THREADS), 0,
               st, raw.base[l], fp, cand, counts);
        launch("orb.select_redo", select_redo_kernel, dim3(std::min(batch, 8u)), dim3(SEL_THREADS), 0, st, cand,
               counts, sp, d_kp, o->xy.as<uint32_t>(), d_n, o->status.as<uint32_t>());
        MAGE_HIP(hipGetLastError());
    }

    if (cap > 0 && s.use_orientation) {
        OrientParams op{};
        op.lev = raw;
        op.out_cap = cap;
        op.half_k = half;
        // u_max (ComputeKeyPoints :671-686)
        int vmax = (int)std::floor(half * std::sqrt(2.f) / 2 + 1), vmin = (int)std::ceil(half * std::sqrt(2.f) / 2);
        for (int v = 0; v <= vmax; ++v) op.umax[v] = (int)std::lrint(std::sqrt((double)half * half - v * v));
        for (int v = half, v0 = 0; v >= vmin; --v) {
            while (op.umax[v0] == op.umax[v0 + 1]) ++v0;
            op.umax[v] = v0;
            ++v0;
        }
        if (half >= 5 && half <= 15)  // a disc row per lane, 2 x OR_KPL keypoints per wave
        {
            op.chunks = (int)((cap + ORIENT_PER_BLOCK - 1) / ORIENT_PER_BLOCK);
            op.frames = (int)batch;
            launch("orb.orient", orient_rows_kernel, dim3((unsigned)(op.chunks * ((batch + 7) / 8) * 8)), dim3(256), 0, st,
                   d_kp, o->xy.as<uint32_t>(), o->lvl.as<uint16_t>(), d_n, op);
        }
        else
            launch("orb.orient", orient_kernel, dim3((cap + 3) / 4, batch), dim3(256), 0, st, d_kp, o->xy.as<uint32_t>(),
                   o->lvl.as<uint16_t>(), d_n, op);
        MAGE_HIP(hipGetLastError());
    }

    if (cap > 0) {
        DescParams dp{};
        dp.lev = fused_blur ? blurred : raw;
        for (int l = 0; l < L; l++) {
            dp.lw[l] = g.lv[l].w;
            dp.lh[l] = g.lv[l].h;
        }
        dp.lvl = multi ? o->lvl.as<uint16_t>() : nullptr;
        dp.out_cap = cap;
        dp.R = o->R;
        dp.ksize = (int)s.gaussian_kernel_size;
        for (int i = 0; i < 2 * KHMAX + 1; i++) dp.taps[i] = o->taps[i];
        dp.dword_ok = (stride % 4 == 0) && (pitch % 4 == 0) && ((uintptr_t)d_frames % 4 == 0);
        dp.random = o->random_pattern;
        dp.kp_angle = reinterpret_cast<const float*>(d_kp) + 3;  // mage_keypoint.angle
        {
            if (win_blur) {
                dp.chunks = (int)((cap + DESC_WAVES * KPW - 1) / (DESC_WAVES * KPW));
                dp.frames = (int)batch;
                dp.blur_ops = o->blur_ops.as<uint4>();
                const dim3 g3((unsigned)(dp.chunks * ((batch + 7) / 8) * 8), 1, 1);
                launch("orb.describe", describe_win_kernel, g3, dim3(DESC_WAVES * kWave), 0, st, dp,
                       (const uint32_t*)o->xy.as<uint32_t>(), d_n, (const int8_t*)o->pattern.as<int8_t>(), d_desc);
            } else if (fused_blur) {
                // keypoints per wave: 8 for one level at radius <= 7, 4 up to radius 13, and
                // MAGE_DESC_KP_WIDE for the wide (rotated, radius > 13) windows, whose LDS (37 rows
                // x 96 bytes each) otherwise left two workgroups per CU
                const int kp = !multi && dp.R <= 7 ? KPW7 : (dp.R <= 13 ? KPW : MAGE_DESC_KP_WIDE);
                dp.chunks = (int)((cap + DESC_WAVES * kp - 1) / (DESC_WAVES * kp));
                dp.frames = (int)batch;
                const dim3 g3((unsigned)(dp.chunks * ((batch + 7) / 8) * 8), 1, 1);
                auto kern = multi ? (dp.R <= 7 ? describe_blurred_kernel<7, true, KPW>
                                               : (dp.R <= 13 ? describe_blurred_kernel<13, true, KPW> : describe_blurred_kernel<RMAX, true, MAGE_DESC_KP_WIDE>))
                                  : (dp.R <= 7 ? describe_blurred_kernel<7, false, KPW7>
                                               : (dp.R <= 13 ? describe_blurred_kernel<13, false, KPW> : describe_blurred_kernel<RMAX, false, MAGE_DESC_KP_WIDE>));
                launch("orb.describe", kern, g3, dim3(DESC_WAVES * kWave), 0, st, dp, (const uint32_t*)o->xy.as<uint32_t>(),
                       d_n, (const int8_t*)o->pattern.as<int8_t>(), d_desc);
            } else {
                const dim3 g3((cap + DESC_WAVES - 1) / DESC_WAVES, batch);
                auto kern = dp.R <= 7 ? describe_kernel<7> : (dp.R <= 13 ? describe_kernel<13> : describe_kernel<RMAX>);
                launch("orb.describe", kern, g3, dim3(DESC_WAVES * kWave), 0, st, dp, (const uint32_t*)o->xy.as<uint32_t>(),
                       d_n, (const int8_t*)o->pattern.as<int8_t>(), d_desc);
            }
        }
        MAGE_HIP(hipGetLastError());
    }
    return MAGE_OK;
}

mage_status check_status(OrbDetector* o, hipStream_t st)
{
    uint32_t flags = 0;
    MAGE_HIP(hipMemcpyAsync(&flags, o->status.ptr, 4, hipMemcpyDeviceToHost, st));
    MAGE_HIP(hipStreamSynchronize(st));
    MAGE_REQUIRE(!(flags & ST_KMAX), MAGE_ECAPACITY, "retained keypoints exceed the LDS capacity (8192)");
    MAGE_REQUIRE(!(flags & ST_CELLS), MAGE_EUNSUPPORTED, "NumCellsX*NumCellsY > 4096");
    return MAGE_OK;
}

// ------------------------------------------------------------------------------------------
// 6. UndistortKeypoints (OrbFeatureDetector.cpp:30-62): cv::undistortPoints of OpenCV 3.4.0
//    (imgproc/undistort.cpp, cvUndistortPoints) with R = noArray(), P = the undistorted camera
//    matrix, in f64: normalise, 5 fixed-point iterations x = (x0 - delta(x)) * icdist(x) (the
//    tilt compensation is the identity for zero tilt terms), then RR = P * I applied in
//    homogeneous form, stored as float.  Same expressions, same order as the C source.
// ------------------------------------------------------------------------------------------
struct UndistortParams {
    double cx, cy, ifx, ify;
    double k[12];
    int iters;
    double RR[3][3];
};

__device__ __forceinline__ void undistort_point(const UndistortParams& u, float& px, float& py)
{
    const double* k = u.k;
    double x = px, y = py;
    x = (x - u.cx) * u.ifx;
    y = (y - u.cy) * u.ify;
    const double x0 = x, y0 = y;
    for (int j = 0; j < u.iters; j++) {
        const double r2 = x * x + y * y;
        const double icdist = (1 + ((k[7] * r2 + k[6]) * r2 + k[5]) * r2) / (1 + ((k[4] * r2 + k[1]) * r2 + k[0]) * r2);
        const double deltaX = 2 * k[2] * x * y + k[3] * (r2 + 2 * x * x) + k[8] * r2 + k[9] * r2 * r2;
        const double deltaY = k[2] * (r2 + 2 * y * y) + 2 * k[3] * x * y + k[10] * r2 + k[11] * r2 * r2;
        x = (x0 - deltaX) * icdist;
        y = (y0 - deltaY) * icdist;
    }
    const double xx = u.RR[0][0] * x + u.RR[0][1] * y + u.RR[0][2];
    const double yy = u.RR[1][0] * x + u.RR[1][1] * y + u.RR[1][2];
    const double ww = 1. / (u.RR[2][0] * x + u.RR[2][1] * y + u.RR[2][2]);
    px = (float)(xx * ww);
    py = (float)(yy * ww);
}

__global__ __launch_bounds__(256) void undistort_kernel(UndistortParams u, mage_keypoint* __restrict__ kp,
                                                        long long pitch, const uint32_t* __restrict__ n)
{
    const int i = blockIdx.x * 256 + threadIdx.x, f = blockIdx.y;
    if (i >= (int)n[f]) return;
    mage_keypoint& k = kp[(long long)f * pitch + i];
    float x = k.x, y = k.y;
    undistort_point(u, x, y);
    k.x = x;
    k.y = y;
}

UndistortParams undistort_params(const mage_calibration& d, const mage_calibration& p)
{
    UndistortParams u{};
    const double fx = d.fx, fy = d.fy;
    u.cx = d.cx;
    u.cy = d.cy;
    u.ifx = 1. / fx;
    u.ify = 1. / fy;
    for (int i = 0; i < d.ndist && i < 8; i++) u.k[i] = d.dist[i];
    u.iters = d.ndist > 0 ? 5 : 0;
    const double P[3][3] = {{p.fx, 0, p.cx}, {0, p.fy, p.cy}, {0, 0, 1}};
    for (int r = 0; r < 3; r++)
        for (int c = 0; c < 3; c++) u.RR[r][c] = P[r][c];  // P * R with R = I
    return u;
}

mage_status check_calibration(const mage_calibration* c)
{
    MAGE_REQUIRE(c, MAGE_EINVAL, "null calibration");
    MAGE_REQUIRE(c->ndist == 0 || c->ndist == 5 || c->ndist == 8, MAGE_EINVAL,
                 "ndist must be 0 (None), 5 (Poly3k) or 8 (Rational6k)");
    MAGE_REQUIRE(c->fx != 0.f && c->fy != 0.f, MAGE_EINVAL, "zero focal length");
    return MAGE_OK;
}

}  // namespace
}  // namespace mage

using mage::OrbDetector;

struct mage_orb : OrbDetector {};

extern "C" {

mage_status mage_undistort_keypoints_batch_device(const mage_calibration* distorted,
                                                  const mage_calibration* undistorted, mage_keypoint* d_kp,
                                                  int64_t pitch, const uint32_t* d_n, uint32_t batch,
                                                  mage_stream stream)
{
    using namespace mage;
    mage_status r;
    if ((r = check_calibration(distorted)) != MAGE_OK || (r = check_calibration(undistorted)) != MAGE_OK) return r;
    if (batch == 0 || pitch <= 0) return MAGE_OK;
    MAGE_REQUIRE(d_kp && d_n, MAGE_EINVAL, "null buffer");
    const UndistortParams u = undistort_params(*distorted, *undistorted);
    launch("orb.undistort", undistort_kernel, dim3((unsigned)((pitch + 255) / 256), batch), dim3(256), 0,
           (hipStream_t)stream, u, d_kp, (long long)pitch, d_n);
    MAGE_HIP(hipGetLastError());
    return MAGE_OK;
}

mage_status mage_undistort_keypoints(const mage_calibration* distorted, const mage_calibration* undistorted,
                                     mage_keypoint* kp, uint32_t n, int device)
{
    using namespace mage;
    mage_status r;
    if ((r = check_calibration(distorted)) != MAGE_OK || (r = check_calibration(undistorted)) != MAGE_OK) return r;
    if (n == 0) return MAGE_OK;
    MAGE_REQUIRE(kp, MAGE_EINVAL, "null keypoints");
    if ((r = bind_device(device)) != MAGE_OK) return r;
    HostScratch* sp = host_scratch(device, SCRATCH_UNDISTORT);
    if (!sp) return MAGE_EDEVICE;
    HostScratch& S = *sp;
    if ((r = S.buf.reserve(sizeof(mage_keypoint) * (size_t)n)) != MAGE_OK || (r = S.aux.reserve(4)) != MAGE_OK) return r;
    MAGE_HIP(hipMemcpyAsync(S.buf.ptr, kp, sizeof(mage_keypoint) * (size_t)n, hipMemcpyHostToDevice, S.st));
    MAGE_HIP(hipMemcpyAsync(S.aux.ptr, &n, 4, hipMemcpyHostToDevice, S.st));
    if ((r = mage_undistort_keypoints_batch_device(distorted, undistorted, S.buf.as<mage_keypoint>(), n,
                                                   S.aux.as<uint32_t>(), 1, (mage_stream)S.st)) != MAGE_OK)
        return r;
    MAGE_HIP(hipMemcpyAsync(kp, S.buf.ptr, sizeof(mage_keypoint) * (size_t)n, hipMemcpyDeviceToHost, S.st));
    MAGE_HIP(hipStreamSynchronize(S.st));
    return MAGE_OK;
}

mage_status mage_orb_create(const mage_orb_settings* settings, int device, mage_orb** out)
{
    MAGE_REQUIRE(settings && out, MAGE_EINVAL, "null argument");
    *out = nullptr;
    const mage_orb_settings& s = *settings;
    // CV_Assert(m_patchSize >= 2) (OpenCVModified.cpp:776)
    MAGE_REQUIRE(s.patch_size >= 2, MAGE_EINVAL, "patchSize must be >= 2");
    MAGE_REQUIRE(s.gaussian_kernel_size <= 1 || (s.gaussian_kernel_size % 2 == 1 && s.gaussian_kernel_size <= 15),
                 MAGE_EINVAL, "GaussianKernelSize must be odd and <= 15");
    MAGE_REQUIRE(s.num_cells_x >= 1 && s.num_cells_y >= 1, MAGE_EINVAL, "NumCells must be >= 1");
    MAGE_REQUIRE(s.nlevels >= 1 && s.nlevels <= MAGE_MAX_LEVELS, MAGE_EUNSUPPORTED, "NumLevels must be 1..8");
    MAGE_REQUIRE(s.nlevels == 1 || (s.scale_factor > 1.0f && std::isfinite(s.scale_factor)), MAGE_EINVAL,
                 "ScaleFactor must be > 1");
    mage_status r = mage::bind_device(device);
    if (r != MAGE_OK) return r;
    auto* o = new mage_orb();
    o->s = s;
    o->device = device;
    if (s.gaussian_kernel_size > 1) mage::gaussian_taps((int)s.gaussian_kernel_size, 2.0, o->taps);
    // patch 15 / 31: the pre-rotated tables (30 rotations); any other size: MakeRandomPattern
    // (OpenCVModified.cpp:877-884) in the rotation-0 slot, rotated per keypoint in the kernel
    o->random_pattern = !(s.patch_size == 15 || s.patch_size == 31);
    int8_t random_table[1024];
    if (o->random_pattern) mage::make_random_pattern((int)s.patch_size, random_table);
    const int8_t* table = o->random_pattern ? random_table
                                            : (s.patch_size == 31 ? mage_bit_pattern_31_rotated : mage_bit_pattern_15_rotated);
    // sampling radius: rotation 0 only, all 30 rotations when orienting, or for the random
    // pattern rotated by any angle: ceil(|p|) bounds |cvRound| of the rotated point
    int R = 0;
    if (o->random_pattern) {
        for (int i = 0; i < 512; i++) {
            const int x = table[2 * i], y = table[2 * i + 1];
            R = std::max(R, s.use_orientation ? (int)std::ceil(std::sqrt((double)(x * x + y * y))) : std::max(std::abs(x), std::abs(y)));
        }
    } else {
        for (int i = 0; i < (s.use_orientation ? 30 : 1) * 1024; i++) R = std::max(R, std::abs((int)table[i]));
    }
    if (R > mage::RMAX) {
        delete o;
        mage::set_error("pattern radius exceeds 18 (PatchSize too large for this build)");
        return MAGE_EUNSUPPORTED;
    }
    o->R = R;
    if ((r = o->pattern.reserve(30 * 1024)) != MAGE_OK) {
        delete o;
        return r;
    }
    if (hipMemcpy(o->pattern.ptr, table, (o->random_pattern ? 1 : 30) * 1024, hipMemcpyHostToDevice) != hipSuccess) {
        delete o;
        mage::set_error("pattern upload failed");
        return MAGE_EDEVICE;
    }
    if (s.gaussian_kernel_size == 7) {  // the fused MFMA blur's band operands
        uint32_t ops[64 * 12];
        mage::blur_operands(o->taps, ops);
        if ((r = o->blur_ops.reserve(sizeof(ops))) != MAGE_OK) {
            delete o;
            return r;
        }
        if (hipMemcpy(o->blur_ops.ptr, ops, sizeof(ops), hipMemcpyHostToDevice) != hipSuccess) {
            delete o;
            mage::set_error("blur operand upload failed");
            return MAGE_EDEVICE;
        }
    }
    *out = o;
    return MAGE_OK;
}

mage_status mage_orb_destroy(mage_orb* orb)
{
    if (!orb) return MAGE_OK;
    for (auto* b : {&orb->pattern, &orb->cand, &orb->counts, &orb->xy, &orb->status, &orb->img, &orb->kp,
                    &orb->desc, &orb->n, &orb->blurred, &orb->pyr, &orb->rtab, &orb->lvl, &orb->blur_ops,
                    &orb->gates, &orb->redo})
        b->release();
    delete orb;
    return MAGE_OK;
}

mage_status mage_orb_detect_and_compute_batch_device(mage_orb* orb, const uint8_t* d_frames,
                                                     uint32_t batch, int32_t width,
                                                     int32_t height, int32_t stride,
                                                     int64_t frame_pitch, mage_keypoint* d_kp,
                                                     uint8_t* d_desc, uint32_t cap,
                                                     uint32_t* d_n, mage_stream stream)
{
    mage_status r = mage::validate(orb, width, height, stride);
    if (r != MAGE_OK) return r;
    if (batch == 0) return MAGE_OK;
    MAGE_REQUIRE(d_frames && d_kp && d_n && (d_desc || cap == 0), MAGE_EINVAL, "null buffer");
    MAGE_HIP(hipSetDevice(orb->device));
    return mage::run_batch(orb, d_frames, batch, width, height, stride, frame_pitch, d_kp, d_desc,
                           cap, d_n, (hipStream_t)stream);
}

mage_status mage_orb_detect_and_compute(mage_orb* orb, const uint8_t* img, int32_t width,
                                        int32_t height, int32_t stride, mage_keypoint* kp,
                                        uint8_t* desc, uint32_t cap, uint32_t* n)
{
    mage_status r = mage::validate(orb, width, height, stride);
    if (r != MAGE_OK) return r;
    MAGE_REQUIRE(img && n && (cap == 0 || (kp && desc)), MAGE_EINVAL, "null buffer");
    MAGE_HIP(hipSetDevice(orb->device));
    *n = 0;
    const size_t bytes = (size_t)stride * height;
    if ((r = orb->img.reserve(bytes)) != MAGE_OK) return r;
    if ((r = orb->kp.reserve(sizeof(mage_keypoint) * std::max(cap, 1u))) != MAGE_OK) return r;
    if ((r = orb->desc.reserve(32 * (size_t)std::max(cap, 1u))) != MAGE_OK) return r;
    if ((r = orb->n.reserve(4)) != MAGE_OK) return r;
    if ((r = orb->status.reserve(4)) != MAGE_OK) return r;
    hipStream_t st = nullptr;
    MAGE_HIP(hipMemsetAsync(orb->status.ptr, 0, 4, st));
    MAGE_HIP(hipMemcpyAsync(orb->img.ptr, img, bytes, hipMemcpyHostToDevice, st));
    r = mage::run_batch(orb, orb->img.as<uint8_t>(), 1, width, height, stride, (long long)bytes,
                        orb->kp.as<mage_keypoint>(), orb->desc.as<uint8_t>(), cap,
                        orb->n.as<uint32_t>(), st);
    if (r != MAGE_OK) return r;
    if ((r = mage::check_status(orb, st)) != MAGE_OK) return r;
    uint32_t count = 0;
    MAGE_HIP(hipMemcpy(&count, orb->n.ptr, 4, hipMemcpyDeviceToHost));
    if (count) {
        MAGE_HIP(hipMemcpy(kp, orb->kp.ptr, sizeof(mage_keypoint) * count, hipMemcpyDeviceToHost));
        MAGE_HIP(hipMemcpy(desc, orb->desc.ptr, 32 * (size_t)count, hipMemcpyDeviceToHost));
    }
    *n = count;
    return MAGE_OK;
}

mage_status mage_orb_status(mage_orb* orb, mage_stream stream)
{
    MAGE_REQUIRE(orb, MAGE_EINVAL, "null detector");
    MAGE_HIP(hipSetDevice(orb->device));
    if (!orb->status.ptr) return MAGE_OK;
    return mage::check_status(orb, (hipStream_t)stream);
}

mage_status mage_orb_reset_status(mage_orb* orb, mage_stream stream)
{
    MAGE_REQUIRE(orb, MAGE_EINVAL, "null detector");
    MAGE_HIP(hipSetDevice(orb->device));
    mage_status r = orb->status.reserve(4);
    if (r != MAGE_OK) return r;
    MAGE_HIP(hipMemsetAsync(orb->status.ptr, 0, 4, (hipStream_t)stream));
    return MAGE_OK;
}

mage_status mage_orb_set_fast_gate(mage_orb* orb, uint32_t level, int32_t gate, mage_stream stream)
{
    MAGE_REQUIRE(orb && level < MAGE_MAX_LEVELS && gate >= 0 && gate <= 255, MAGE_EINVAL, "bad arguments");
    MAGE_HIP(hipSetDevice(orb->device));
    const bool fresh = orb->gates.ptr == nullptr;
    mage_status r = orb->gates.reserve(2 * MAGE_MAX_LEVELS * sizeof(int));
    if (r != MAGE_OK) return r;
    hipStream_t st = (hipStream_t)stream;
    if (fresh) MAGE_HIP(hipMemsetAsync(orb->gates.ptr, 0, 2 * MAGE_MAX_LEVELS * sizeof(int), st));
    int* slot = orb->gates.as<int>() + orb->gate_par * MAGE_MAX_LEVELS + level;
    MAGE_HIP(hipMemcpyAsync(slot, &gate, sizeof(int), hipMemcpyHostToDevice, st));
    MAGE_HIP(hipStreamSynchronize(st));
    return MAGE_OK;
}

mage_status mage_orb_fast_gate_stats(mage_orb* orb, uint32_t level, int32_t* last_gate, int32_t* next_gate,
                                     uint32_t* last_redo, mage_stream stream)
{
    MAGE_REQUIRE(orb && level < MAGE_MAX_LEVELS && last_gate && next_gate && last_redo, MAGE_EINVAL, "bad arguments");
    MAGE_HIP(hipSetDevice(orb->device));
    *last_gate = *next_gate = 0;
    *last_redo = 0;
    if (!orb->gates.ptr) return MAGE_OK;
    hipStream_t st = (hipStream_t)stream;
    const int* g = orb->gates.as<int>();
    MAGE_HIP(hipMemcpyAsync(last_gate, g + (1 - orb->gate_par) * MAGE_MAX_LEVELS + level, sizeof(int),
                            hipMemcpyDeviceToHost, st));
    MAGE_HIP(hipMemcpyAsync(next_gate, g + orb->gate_par * MAGE_MAX_LEVELS + level, sizeof(int),
                            hipMemcpyDeviceToHost, st));
    const int L = orb->geo.L;
    if (orb->redo.ptr && (int)level < L)
        MAGE_HIP(hipMemcpyAsync(last_redo, orb->redo.as<uint32_t>() + (size_t)level * (1 + orb->last_batch), 4,
                                hipMemcpyDeviceToHost, st));
    MAGE_HIP(hipStreamSynchronize(st));
    return MAGE_OK;
}

#if MAGE_FAST_STAMPS
// development build only (tools/fast_stamps.py): the per-wave phase stamps of the last FAST pass
mage_status mage_debug_fast_stamps(unsigned long long* out)
{
    MAGE_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(mage::g_fast_stamps), sizeof(mage::g_fast_stamps)));
    return MAGE_OK;
}
#endif
#if MAGE_SELECT_STAMPS
// development build only (tools/select_stamps.py): the per-frame phase stamps of the last select
mage_status mage_debug_select_stamps(unsigned long long* out)
{
    MAGE_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(mage::g_sel_stamps), sizeof(mage::g_sel_stamps)));
    return MAGE_OK;
}
#endif

mage_status mage_orb_fast_score_map(const uint8_t* img, int32_t width, int32_t height,
                                    int32_t stride, int32_t threshold, uint8_t* score_map,
                                    int device)
{
    MAGE_REQUIRE(img && score_map && width > 0 && height > 0 && stride >= width, MAGE_EINVAL, "bad arguments");
    mage_status r = mage::bind_device(device);
    if (r != MAGE_OK) return r;
    mage::DeviceBuffer dimg, dscore;
    if ((r = dimg.reserve((size_t)stride * height)) != MAGE_OK) return r;
    if ((r = dscore.reserve((size_t)width * height)) != MAGE_OK) {
        dimg.release();
        return r;
    }
    mage::FastParams fp{};
    fp.w = width;
    fp.h = height;
    fp.stride = stride;
    fp.threshold = std::min(std::max((int)threshold, 0), 255);
    fp.dword_ok = (width % 4 == 0) && (stride % 4 == 0);
    fp.qword_ok = (stride % 8 == 0);
    hipError_t e = hipMemcpy(dimg.ptr, img, (size_t)stride * height, hipMemcpyHostToDevice);
    if (e == hipSuccess) {
        dim3 g((width + mage::TW - 1) / mage::TW, (height + mage::TH - 1) / mage::TH);
        hipLaunchKernelGGL(mage::fast_score_map_kernel, g, dim3(mage::FAST_THREADS), 0, nullptr,
                           dimg.as<uint8_t>(), fp, dscore.as<uint8_t>());
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpy(score_map, dscore.ptr, (size_t)width * height, hipMemcpyDeviceToHost);
    dimg.release();
    dscore.release();
    if (e != hipSuccess) {
        mage::set_error(std::string("fast score map: ") + hipGetErrorString(e));
        return MAGE_EDEVICE;
    }
    return MAGE_OK;
}

mage_status mage_synth_frames_device(uint8_t* d_out, uint32_t count, int32_t width,
                                     int32_t height, int64_t frame_pitch, uint32_t t0,
                                     uint64_t seed, mage_stream stream)
{
    MAGE_REQUIRE(d_out && width > 0 && height > 0 && frame_pitch >= (int64_t)width * height,
                 MAGE_EINVAL, "bad arguments");
    if (count == 0) return MAGE_OK;
    dim3 g((width + 255) / 256, height, count);
    hipLaunchKernelGGL(mage::synth_frames_kernel, g, dim3(256), 0, (hipStream_t)stream, d_out,
                       width, height, (long long)frame_pitch, t0, (unsigned long long)seed);
    MAGE_HIP(hipGetLastError());
    return MAGE_OK;
}

mage_status mage_resize_linear_device(const uint8_t* d_src, int32_t sw, int32_t sh, int32_t src_stride, uint8_t* d_dst,
                                      int32_t dw, int32_t dh, int32_t dst_stride, mage_stream stream)
{
    return mage::resize_linear_device(d_src, sw, sh, src_stride, d_dst, dw, dh, dst_stride, (hipStream_t)stream);
}

}  // extern "C"
