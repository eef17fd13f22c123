/*
 * orb_oracle.c — CPU restatement of MAGE-SLAM's ORB extractor (TEST INFRASTRUCTURE ONLY).
 *
 * This file is the parity oracle and the timed CPU baseline for the ORB hot path.  It is
 * linked only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, never by
 * the product library under mageslam_amd/.
 *
 * PARITY UNPINNED: the reference cannot be built here (OpenCV 3.4.0 / g2o / Eigen absent,
 * MSVC-only sources) and ships no fixtures, golden vectors or tests for this
 * path.  This restatement follows the reference line by line as cited below;
 * the only data taken from the reference are the pre-rotated BRIEF tables
 * (OpenCVModified.cpp:74-138, extracted by tools/extract_patterns.py).  Third-party steps are
 * restated from their published algorithms:
 *   - OpenCV 3.4.0 GaussianBlur 8U (separable, kernel quantised to Q8, (s+2^15)>>16),
 *   - OpenCV 3.4.0 resize INTER_LINEAR 8U (fixed-point coefficients, SSE2 vertical pass; non-IPP
 *     build) and fastAtan2 (polynomial atan in degrees), for NumLevels > 1 / UseOrientation,
 *   - each pyramid level blurred as an isolated image (reflect-101 at its own borders; the
 *     reference blurs ROIs of one packed buffer, so pixels within 3 px of an inner level edge
 *     there depend on neighbouring levels or unwritten memory — never sampled when the border
 *     exceeds the pattern radius by 4, as in the oriented rBRIEF-31 configuration), and
 *   - the canonical keypoint order (the reference's order depends on MSVC std::nth_element).
 * Build with -ffp-contract=off: the ANMS comparisons are float-exact.
 *
 * Reference paths: Core/MAGESLAM/Source/Image/OpenCVModified.cpp unless noted.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/mage_hot.h"

/* Ring offsets of FAST 9/16, makeOffsets (OpenCVModified.cpp:890-921). */
static const int kRing16[16][2] = {{0, 3},  {1, 3},   {2, 2},   {3, 1},   {3, 0},  {3, -1},
                                   {2, -2}, {1, -3},  {0, -3},  {-1, -3}, {-2, -2}, {-3, -1},
                                   {-3, 0}, {-3, 1},  {-2, 2},  {-1, 3}};

static int imin(int a, int b) { return a < b ? a : b; }
static int imax(int a, int b) { return a > b ? a : b; }

/* cornerScore<16>, scalar branch (OpenCVModified.cpp:1030-1064).  The x64 reference runs the
 * SSE2 branches (:935-972, :1278-1338); oracle/fast_sse2.c restates them and
 * tests/test_oracle.py::test_verify_simd_sse2_build_equals_scalar_oracle checks that the SSE2
 * build's score map equals this scalar one (the reference's VERIFY_SIMD property, :1265-1271). */
static int corner_score16(const uint8_t* p, const int pixel[25], int threshold)
{
    int d[25];
    int v = p[0];
    for (int k = 0; k < 25; k++) d[k] = (short)(v - p[pixel[k]]);
    int a0 = threshold;
    for (int k = 0; k < 16; k += 2) {
        int a = imin(d[k + 1], d[k + 2]);
        a = imin(a, d[k + 3]);
        if (a <= a0) continue;
        a = imin(a, d[k + 4]);
        a = imin(a, d[k + 5]);
        a = imin(a, d[k + 6]);
        a = imin(a, d[k + 7]);
        a = imin(a, d[k + 8]);
        a0 = imax(a0, imin(a, d[k]));
        a0 = imax(a0, imin(a, d[k + 9]));
    }
    int b0 = -a0;
    for (int k = 0; k < 16; k += 2) {
        int b = imax(d[k + 1], d[k + 2]);
        b = imax(b, d[k + 3]);
        b = imax(b, d[k + 4]);
        b = imax(b, d[k + 5]);
        if (b >= b0) continue;
        b = imax(b, d[k + 6]);
        b = imax(b, d[k + 7]);
        b = imax(b, d[k + 8]);
        b0 = imin(b0, imax(b, d[k]));
        b0 = imin(b0, imax(b, d[k + 9]));
    }
    return -b0 - 1;
}

/* Segment test of FAST_t<16>, scalar path (OpenCVModified.cpp:1415-1479): some cyclic run of
 * more than K=8 ring pixels all darker than v-t or all brighter than v+t. */
static int is_corner16(const uint8_t* p, const int pixel[25], int t)
{
    int v = p[0];
    int vt = v - t, count = 0;
    for (int k = 0; k < 25; k++) {
        if (p[pixel[k]] < vt) {
            if (++count > 8) return 1;
        } else
            count = 0;
    }
    vt = v + t;
    count = 0;
    for (int k = 0; k < 25; k++) {
        if (p[pixel[k]] > vt) {
            if (++count > 8) return 1;
        } else
            count = 0;
    }
    return 0;
}

static void make_offsets(int pixel[25], int stride)
{
    for (int k = 0; k < 16; k++) pixel[k] = kRing16[k][0] + kRing16[k][1] * stride;
    for (int k = 16; k < 25; k++) pixel[k] = pixel[k - 16];
}

/* Score map: rows 3..H-4, cols 3..W-4 are tested (FAST_t loop bounds :1248, :1269, :1415);
 * everything else is 0. */
void oracle_fast_score_map(const uint8_t* img, int w, int h, int stride, int threshold,
                           uint8_t* score)
{
    int pixel[25];
    make_offsets(pixel, stride);
    threshold = imin(imax(threshold, 0), 255);
    memset(score, 0, (size_t)w * h);
    for (int y = 3; y < h - 3; y++) {
        for (int x = 3; x < w - 3; x++) {
            const uint8_t* p = img + (size_t)y * stride + x;
            if (is_corner16(p, pixel, threshold))
                score[(size_t)y * w + x] = (uint8_t)corner_score16(p, pixel, threshold);
        }
    }
}

typedef struct {
    int x, y;
    int score;
} cand_t;

/* FAST with strict 3x3 NMS, emission in raster order (OpenCVModified.cpp:1489-1509).
 * Returns the candidate count; `out` must hold w*h/4+w+h entries. */
/* The score map of the reference's x64 build (SSE2 cornerScore + row loop, fast_sse2.c; equal
 * to the scalar one, tests/test_oracle.py) when set: bench.py's CPU baseline times that build. */
static int g_fast_sse2 = 0;
void oracle_fast_score_map_sse2(const uint8_t* img, int w, int h, int stride, int threshold, uint8_t* score,
                                int* simd_cols);
void oracle_set_fast_sse2(int on) { g_fast_sse2 = on != 0; }

static int fast_nms(const uint8_t* img, int w, int h, int stride, int t, uint8_t* score,
                    cand_t* out)
{
    if (g_fast_sse2)
        oracle_fast_score_map_sse2(img, w, h, stride, t, score, NULL);
    else
        oracle_fast_score_map(img, w, h, stride, t, score);
    int n = 0;
    for (int y = 3; y < h - 3; y++) {
        for (int x = 3; x < w - 3; x++) {
            int s = score[(size_t)y * w + x];
            if (!s) continue;
            const uint8_t* c = score + (size_t)y * w + x;
            if (s > c[-1] && s > c[1] && s > c[-w - 1] && s > c[-w] && s > c[-w + 1] &&
                s > c[w - 1] && s > c[w] && s > c[w + 1]) {
                out[n].x = x;
                out[n].y = y;
                out[n].score = s;
                n++;
            }
        }
    }
    return n;
}

/* OpenCV cvRound: round half to even (used by cvRound(double) on x64). */
static int cv_round(double v) { return (int)lrint(v); }

/* Gaussian taps of cv::getGaussianKernel(ksize, sigma, CV_32F) quantised by convertTo(CV_32S,
 * 256) in createSeparableLinearFilter (OpenCV 3.4.0 filter.cpp, the 8U smoothing path). */
void oracle_gaussian_taps(int ksize, double sigma, int* taps)
{
    float cf[64];
    double sum = 0;
    double s = sigma > 0 ? sigma : ((ksize - 1) * 0.5 - 1) * 0.3 + 0.8;
    double scale2 = -0.5 / (s * s);
    for (int i = 0; i < ksize; i++) {
        double x = i - (ksize - 1) * 0.5;
        cf[i] = (float)exp(scale2 * x * x);
        sum += cf[i];
    }
    sum = 1. / sum;
    for (int i = 0; i < ksize; i++) {
        cf[i] = (float)(cf[i] * sum);
        taps[i] = cv_round((double)cf[i] * 256.0);
    }
}

static int reflect101(int i, int n)
{
    if (n == 1) return 0;
    while (i < 0 || i >= n) {
        if (i < 0) i = -i;
        if (i >= n) i = 2 * n - 2 - i;
    }
    return i;
}

/* GaussianBlur(ksize, sigma=2, BORDER_REFLECT_101) on an 8-bit image (OpenCVModified.cpp:853-865):
 * int32 row pass, int32 column pass, (sum + 2^15) >> 16, saturate to u8. */
void oracle_gaussian_blur(const uint8_t* src, int w, int h, int stride, int ksize, uint8_t* dst)
{
    int taps[64];
    oracle_gaussian_taps(ksize, 2.0, taps);
    int r = ksize / 2;
    int32_t* rows = (int32_t*)malloc(sizeof(int32_t) * (size_t)w * h);
    for (int y = 0; y < h; y++)
        for (int x = 0; x < w; x++) {
            int32_t s = 0;
            for (int k = -r; k <= r; k++) s += taps[k + r] * src[(size_t)y * stride + reflect101(x + k, w)];
            rows[(size_t)y * w + x] = s;
        }
    for (int y = 0; y < h; y++)
        for (int x = 0; x < w; x++) {
            int32_t s = 0;
            for (int k = -r; k <= r; k++) s += taps[k + r] * rows[(size_t)reflect101(y + k, h) * w + x];
            int v = (s + (1 << 15)) >> 16;
            dst[(size_t)y * w + x] = (uint8_t)(v < 0 ? 0 : v > 255 ? 255 : v);
        }
    free(rows);
}

typedef struct {
    int x, y;
    float strength;
    int r;
    int idx; /* canonical: raster rank within the retained set */
} anms_item;

static int cmp_item_rank(const void* pa, const void* pb)
{
    const anms_item* a = (const anms_item*)pa;
    const anms_item* b = (const anms_item*)pb;
    if (a->r != b->r) return a->r > b->r ? -1 : 1;
    if (a->strength != b->strength) return a->strength > b->strength ? -1 : 1;
    return a->idx < b->idx ? -1 : (a->idx > b->idx ? 1 : 0);
}

/* RetainBestFeatures (OpenCVModified.cpp:571-617).  Returns the lowest response kept; the
 * kept set {response >= cut} is exactly what nth_element keeps because the count stops on a
 * histogram-bin boundary. */
static int retain_cut(const cand_t* c, int n, int minThreshold, int maxNum, int minNum,
                      float responseFactor)
{
    unsigned hist[256];
    memset(hist, 0, sizeof(hist));
    for (int i = 0; i < n; i++) hist[imin(imax(c[i].score, 0), 255)]++;
    size_t minNumThreshold = (size_t)minThreshold;
    int num = 0;
    for (int i = 255; i >= minThreshold; i--) {
        num += (int)hist[i];
        if (num >= minNum) {
            minNumThreshold = (size_t)i;
            break;
        }
    }
    int lower = imax((int)((float)minNumThreshold * responseFactor), minThreshold);
    num = 0;
    int i;
    for (i = 255; i >= lower; i--) {
        num += (int)hist[i];
        if (num >= maxNum) break;
    }
    return i < lower ? lower : i;
}

/* AdaptiveNonMaximalSuppresion (OpenCVModified.cpp:144-360) on items[0..n) (raster order);
 * writes the kept items to `kept` in canonical order (r desc, strength desc, idx asc) and
 * returns their count. */
static int anms(anms_item* items, int n, int numToKeep, int threshold, const mage_orb_settings* s,
                anms_item* kept)
{
    const int numX = s->num_cells_x, numY = s->num_cells_y;
    const float ROBUST_EPS = 0.002f;
    if (n == 0) return 0;
    if ((unsigned)numToKeep > (unsigned)n) {
        memcpy(kept, items, sizeof(anms_item) * n);
        return n;
    }
    int minX = items[0].x, maxX = items[0].x, minY = items[0].y, maxY = items[0].y;
    float minStrength = items[0].strength;
    for (int i = 0; i < n; i++) {
        minX = imin(minX, items[i].x);
        minY = imin(minY, items[i].y);
        maxX = imax(maxX, items[i].x);
        maxY = imax(maxY, items[i].y);
        if (items[i].strength < minStrength) minStrength = items[i].strength;
    }
    float robust;
    {
        /* mira::clamp<float> = fmin(hi, fmax(lo, v)) (arcana/math.h:57-67) */
        float hi = (float)s->strong_response - (float)threshold;
        float val = fminf(hi, fmaxf(0.0f, minStrength - (float)threshold));
        float range = fmaxf(0.0f, s->max_robust_factor - s->min_robust_factor);
        robust = s->max_robust_factor - (val / (float)(s->strong_response - threshold)) * range;
    }
    float robustInv = 1.0f / robust;

    /* bucket: cell lists (order inside a cell does not change r: every item stronger than s
     * is visited, OpenCVModified.cpp:268-326) */
    int ncell = numX * numY;
    int* cellStart = (int*)calloc((size_t)ncell + 1, sizeof(int));
    int* cellOf = (int*)malloc(sizeof(int) * n);
    int* order = (int*)malloc(sizeof(int) * n);
    for (int i = 0; i < n; i++) {
        int cx = (items[i].x - minX) * numX / (maxX + 1 - minX);
        int cy = (items[i].y - minY) * numY / (maxY + 1 - minY);
        cellOf[i] = cy * numX + cx;
        cellStart[cellOf[i] + 1]++;
    }
    for (int c = 0; c < ncell; c++) cellStart[c + 1] += cellStart[c];
    {
        int* fill = (int*)malloc(sizeof(int) * ncell);
        memcpy(fill, cellStart, sizeof(int) * ncell);
        for (int i = 0; i < n; i++) order[fill[cellOf[i]]++] = i;
        free(fill);
    }
    int globalMaxR2 = (int)(((double)(maxX - minX)) * ((double)(maxY - minY)) / (double)numToKeep);
    int minCellDelta2;
    {
        int dx = imax((maxX - minX) / numX, 1);
        int dy = imax((maxY - minY) / numY, 1);
        minCellDelta2 = imin(dx, dy) * imin(dx, dy);
    }
    for (int i = 0; i < n; i++) {
        anms_item* it = &items[i];
        int cx = cellOf[i] % numX, cy = cellOf[i] / numX;
        int minR2 = globalMaxR2;
        float sth = (it->strength >= 0) ? (it->strength * robust + ROBUST_EPS)
                                        : (it->strength * robustInv + ROBUST_EPS);
        for (int d = 0; imax(0, d - 1) * imax(0, d - 1) * minCellDelta2 < minR2; d++) {
            for (int yy = -d; yy <= d; yy++) {
                int cYY = yy + cy;
                if (cYY < 0 || cYY >= numY) continue;
                for (int xx = -d; xx <= d; xx++) {
                    int cXX = xx + cx;
                    if (cXX < 0 || cXX >= numX || imax(abs(xx), abs(yy)) != d) continue;
                    int cell = cYY * numX + cXX;
                    for (int q = cellStart[cell]; q < cellStart[cell + 1]; q++) {
                        const anms_item* o = &items[order[q]];
                        if (o->strength > sth) {
                            int ddx = it->x - o->x, ddy = it->y - o->y;
                            int rr = ddx * ddx + ddy * ddy;
                            if (rr < minR2) minR2 = rr;
                        }
                    }
                }
            }
        }
        it->r = minR2;
    }
    free(cellStart);
    free(cellOf);
    free(order);
    memcpy(kept, items, sizeof(anms_item) * n);
    qsort(kept, n, sizeof(anms_item), cmp_item_rank);
    return numToKeep;
}

/* ComputeOrbDescriptorsPrerotated (OpenCVModified.cpp:502-549) on the blurred level. */
static void describe(const uint8_t* blurred, int stride, const signed char* pattern_table,
                     int cx, int cy, int rot, uint8_t* desc)
{
    const uint8_t* center = blurred + (ptrdiff_t)cy * stride + cx;
    const signed char* pattern = pattern_table + rot * 1024;
    for (int i = 0; i < 32; i++, pattern += 32) {
        int val = 0;
        for (int bit = 0; bit < 8; bit++) {
            const signed char* q = pattern + 4 * bit;
            int t0 = center[q[1] * stride + q[0]];
            int t1 = center[q[3] * stride + q[2]];
            val |= (t0 < t1) << bit;
        }
        desc[i] = (uint8_t)val;
    }
}

static int cv_roundf(float v) { return (int)lrintf(v); }

/* cv::RNG (OpenCV 3.4.0 core/operations.hpp): multiply-with-carry, state = (unsigned)state *
 * 4164903690 + (state >> 32); uniform(a, b) = a == b ? a : (int)(next() % (b - a) + a). */
static uint32_t cv_rng_next(uint64_t* st)
{
    *st = (uint64_t)(uint32_t)*st * 4164903690ULL + (*st >> 32);
    return (uint32_t)*st;
}

static int cv_rng_uniform(uint64_t* st, int a, int b)
{
    return a == b ? a : (int)(cv_rng_next(st) % (uint32_t)(b - a) + (uint32_t)a);
}

/* MakeRandomPattern (OpenCVModified.cpp:551-560): 512 points from RNG(0x34985739), x then y in
 * [-patch/2, patch/2]; out holds them as (x0, y0, x1, y1) per test, the layout of the
 * pre-rotated tables (test t compares points 2t and 2t+1, ComputeOrbDescriptors :475-486). */
void oracle_random_pattern(int patch_size, signed char out[1024])
{
    uint64_t st = 0x34985739u;
    for (int i = 0; i < 512; i++) {
        out[2 * i] = (signed char)cv_rng_uniform(&st, -patch_size / 2, patch_size / 2 + 1);
        out[2 * i + 1] = (signed char)cv_rng_uniform(&st, -patch_size / 2, patch_size / 2 + 1);
    }
}

/* ComputeOrbDescriptors (OpenCVModified.cpp:452-492) for the random pattern: the keypoint angle
 * (degrees) times (float)(CV_PI / 180) in f32, a = (float)cos, b = (float)sin, every point
 * rotated in f32 (x a - y b, x b + y a) and rounded with cvRound (GetComputeOrbDescriptorsValue
 * :442-448). */
static void describe_random(const uint8_t* blurred, int stride, const signed char* pts, int cx, int cy,
                            float angle_deg, uint8_t* desc)
{
    const uint8_t* center = blurred + (ptrdiff_t)cy * stride + cx;
    const float angle = angle_deg * (float)(3.1415926535897932384626433832795 / 180.0f);  /* CV_PI */
    const float a = (float)cos(angle), b = (float)sin(angle);
    for (int i = 0; i < 32; i++) {
        int val = 0;
        for (int bit = 0; bit < 8; bit++) {
            const signed char* q = pts + 4 * (8 * i + bit);
            const float x0 = (float)q[0] * a - (float)q[1] * b, y0 = (float)q[0] * b + (float)q[1] * a;
            const float x1 = (float)q[2] * a - (float)q[3] * b, y1 = (float)q[2] * b + (float)q[3] * a;
            const int t0 = center[cv_roundf(y0) * stride + cv_roundf(x0)];
            const int t1 = center[cv_roundf(y1) * stride + cv_roundf(x1)];
            val |= (t0 < t1) << bit;
        }
        desc[i] = (uint8_t)val;
    }
}
static int cv_floorf(float v) { int i = (int)v; return i - (i > v); }
static int cv_ceilf(float v) { int i = (int)v; return i + (i < v); }

/* cv::resize(src, dst, dsize, 0, 0, INTER_LINEAR) for CV_8UC1, OpenCV 3.4.0 resizeGeneric_ with
 * HResizeLinear<uchar,int,short,2048> and VResizeLinear<uchar,int,short,FixedPtCast<..,22>> plus
 * the SSE2 VResizeLinearVec_32s8u (imgproc/src/resize.cpp): coefficients are
 * saturate_cast<short>(w * 2048); the horizontal pass is exact in int; the vector part of the
 * vertical pass computes ((((S0>>4)*b0)>>16) + (((S1>>4)*b1)>>16) + 2) >> 2 for x below the
 * last 16-wide / 4-wide block boundary, the scalar tail (S0*b0 + S1*b1 + 2^21) >> 22. */
void oracle_resize_linear(const uint8_t* src, int sw, int sh, int sstride, uint8_t* dst, int dw, int dh,
                          int dstride)
{
    const double scale_x = 1. / ((double)dw / sw), scale_y = 1. / ((double)dh / sh);
    if (scale_x == 2.0 && scale_y == 2.0) {
        /* cv::resize turns INTER_LINEAR into INTER_AREA when both scales are exactly 2
         * (is_area_fast && iscale_x == iscale_y == 2); resizeAreaFast_: SSE2 8-wide blocks while
         * dx <= w - 8 give (sum + 2) >> 2, the scalar tail saturate_cast<uchar>(sum * 0.25f)
         * (cvRound: half to even) */
        const int xv8 = dw / 8 * 8;
        for (int dy = 0; dy < dh; dy++) {
            const uint8_t* S0 = src + (size_t)(2 * dy) * sstride;
            const uint8_t* S1 = S0 + sstride;
            for (int dx = 0; dx < dw; dx++) {
                const int sum = S0[2 * dx] + S0[2 * dx + 1] + S1[2 * dx] + S1[2 * dx + 1];
                dst[(size_t)dy * dstride + dx] = (uint8_t)(dx < xv8 ? (sum + 2) >> 2 : cv_roundf((float)sum * 0.25f));
            }
        }
        return;
    }
    int* xofs = (int*)malloc(sizeof(int) * dw);
    short* ialpha = (short*)malloc(sizeof(short) * 2 * dw);
    int xmax = dw;
    for (int dx = 0; dx < dw; dx++) {
        float fx = (float)((dx + 0.5) * scale_x - 0.5);
        int sx = cv_floorf(fx);
        fx -= sx;
        if (sx < 0) fx = 0, sx = 0;
        if (sx + 1 >= sw) {
            xmax = imin(xmax, dx);
            if (sx >= sw - 1) fx = 0, sx = sw - 1;
        }
        xofs[dx] = sx;
        ialpha[2 * dx] = (short)cv_roundf((1.f - fx) * 2048);
        ialpha[2 * dx + 1] = (short)cv_roundf(fx * 2048);
    }
    int xv = 0;
    while (xv <= dw - 16) xv += 16;
    while (xv < dw - 4) xv += 4;
    int* rows = (int*)malloc(sizeof(int) * 2 * dw);
    for (int dy = 0; dy < dh; dy++) {
        float fy = (float)((dy + 0.5) * scale_y - 0.5);
        int sy = cv_floorf(fy);
        fy -= sy;
        const int b0 = (short)cv_roundf((1.f - fy) * 2048), b1 = (short)cv_roundf(fy * 2048);
        for (int k = 0; k < 2; k++) {
            const uint8_t* S = src + (size_t)imin(imax(sy + k, 0), sh - 1) * sstride;
            int* D = rows + k * dw;
            for (int dx = 0; dx < dw; dx++) {
                const int sx = xofs[dx];
                D[dx] = dx < xmax ? S[sx] * ialpha[2 * dx] + S[sx + 1] * ialpha[2 * dx + 1] : S[sx] * 2048;
            }
        }
        uint8_t* out = dst + (size_t)dy * dstride;
        for (int x = 0; x < dw; x++) {
            int v;
            if (x < xv) {
                const int s0 = (int)(short)(rows[x] >> 4), s1 = (int)(short)(rows[dw + x] >> 4);
                v = (((s0 * b0) >> 16) + ((s1 * b1) >> 16) + 2) >> 2;
            } else {
                v = (rows[x] * b0 + rows[dw + x] * b1 + (1 << 21)) >> 22;
            }
            out[x] = (uint8_t)(v < 0 ? 0 : v > 255 ? 255 : v);
        }
    }
    free(xofs);
    free(ialpha);
    free(rows);
}

/* cv::fastAtan2 (OpenCV 3.4.0 core/src/mathfuncs_core: polynomial atan in degrees). */
float oracle_fast_atan2(float y, float x)
{
    const float k = (float)(180 / 3.141592653589793);
    const float p1 = 0.9997878412794807f * k, p3 = -0.3258083974640975f * k;
    const float p5 = 0.1555786518463281f * k, p7 = -0.04432655554792128f * k;
    const float eps = (float)2.2204460492503131e-16;
    float ax = fabsf(x), ay = fabsf(y), a, c, c2;
    if (ax >= ay) {
        c = ay / (ax + eps);
        c2 = c * c;
        a = (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    } else {
        c = ax / (ay + eps);
        c2 = c * c;
        a = 90.f - (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    }
    if (x < 0) a = 180.f - a;
    if (y < 0) a = 360.f - a;
    return a;
}

/* u_max of ComputeKeyPoints (OpenCVModified.cpp:671-686); umax must hold halfPatch + 2. */
void oracle_umax(int halfPatchSize, int* umax)
{
    int v, v0, vmax = cv_floorf(halfPatchSize * sqrtf(2.f) / 2 + 1);
    int vmin = cv_ceilf(halfPatchSize * sqrtf(2.f) / 2);
    for (v = 0; v <= vmax; ++v) umax[v] = cv_round(sqrt((double)halfPatchSize * halfPatchSize - v * v));
    for (v = halfPatchSize, v0 = 0; v >= vmin; --v) {
        while (umax[v0] == umax[v0 + 1]) ++v0;
        umax[v] = v0;
        ++v0;
    }
}

/* ICAngles (OpenCVModified.cpp:399-437) for one keypoint at integer level coordinates. */
float oracle_ic_angle(const uint8_t* img, int stride, int x, int y, const int* umax, int half_k)
{
    const uint8_t* center = img + (ptrdiff_t)y * stride + x;
    int m_01 = 0, m_10 = 0;
    for (int u = -half_k; u <= half_k; ++u) m_10 += u * center[u];
    for (int v = 1; v <= half_k; ++v) {
        int v_sum = 0;
        int d = umax[v];
        for (int u = -d; u <= d; ++u) {
            int val_plus = center[u + v * stride], val_minus = center[u - v * stride];
            v_sum += (val_plus - val_minus);
            m_10 += u * (val_plus + val_minus);
        }
        m_01 += v * v_sum;
    }
    return oracle_fast_atan2((float)m_01, (float)m_10);
}

/* Pyramid geometry of DetectAndCompute (:785-804): layerScale = (float)pow(f, l) (getScale
 * :564-567), level size (cvRound(cols/scale), cvRound(rows/scale)). */
void oracle_level_geometry(int w, int h, int nlevels, float scale_factor, float* layer_scale, int* lw, int* lh)
{
    for (int l = 0; l < nlevels; l++) {
        layer_scale[l] = (float)pow((double)scale_factor, (double)l);
        lw[l] = cv_roundf((float)w / layer_scale[l]);
        lh[l] = cv_roundf((float)h / layer_scale[l]);
    }
}

/* nfeaturesPerLevel (ComputeKeyPoints :659-669), float arithmetic as written. */
void oracle_features_per_level(int nfeatures, float scale_factor, int nlevels, int* per_level)
{
    float factor = 1.0f / scale_factor;
    float nd = nfeatures * (1 - factor) / (1 - (float)pow((double)factor, (double)nlevels));
    int sum = 0;
    for (int l = 0; l < nlevels - 1; l++) {
        per_level[l] = cv_roundf(nd);
        sum += per_level[l];
        nd *= factor;
    }
    per_level[nlevels - 1] = imax(nfeatures - sum, 0);
}

typedef struct {
    int x, y, level;
    float strength;
} level_kp;

/* OrbDetector::DetectAndCompute (OpenCVModified.cpp:771-886): pyramid
 * (resize INTER_LINEAR), per-level FAST + border + Retain + ANMS with the per-level budget,
 * Insert truncation, ICAngles (UseOrientation), pt *= layerScale, per-level blur and the
 * descriptors: pre-rotated tables for patch 15 / 31, the random pattern (MakeRandomPattern +
 * ComputeOrbDescriptors, :877-884) otherwise.  Returns MAGE_OK and the count in *n_out. */
int oracle_orb_detect(const mage_orb_settings* s, const signed char* pattern_table,
                      const uint8_t* img, int w, int h, int stride, mage_keypoint* kp,
                      uint8_t* desc, uint32_t cap, uint32_t* n_out)
{
    *n_out = 0;
    if (s->patch_size < 2) return MAGE_EINVAL;
    if (s->nlevels < 1 || s->nlevels > MAGE_MAX_LEVELS) return MAGE_EUNSUPPORTED;
    const int prerotated = s->patch_size == 15 || s->patch_size == 31;
    signed char random_pts[1024];
    if (!prerotated) oracle_random_pattern((int)s->patch_size, random_pts);
    if (s->gaussian_kernel_size > 1 && (s->gaussian_kernel_size % 2) == 0) return MAGE_EINVAL;

    const int L = (int)s->nlevels;
    const int nfeatures = (int)s->nfeatures;
    const int fastThreshold = (int)s->fast_threshold;
    const int halfPatch = (int)s->patch_size / 2;
    /* RunByImageBorder(halfPatchSize), or the hypotenuse when orienting (:711-712) */
    const int border = s->use_orientation ? cv_ceilf(halfPatch * sqrtf(2.0f)) : halfPatch;

    float layerScale[MAGE_MAX_LEVELS];
    int lw[MAGE_MAX_LEVELS], lh[MAGE_MAX_LEVELS], perLevel[MAGE_MAX_LEVELS];
    uint8_t* lev[MAGE_MAX_LEVELS];
    oracle_level_geometry(w, h, L, s->scale_factor, layerScale, lw, lh);
    oracle_features_per_level(nfeatures, s->scale_factor, L, perLevel);
    for (int l = 0; l < L; l++) {
        lev[l] = (uint8_t*)malloc((size_t)lw[l] * lh[l] + 1);
        if (l == 0)
            for (int y = 0; y < h; y++) memcpy(lev[0] + (size_t)y * w, img + (size_t)y * stride, w);
        else
            oracle_resize_linear(lev[l - 1], lw[l - 1], lh[l - 1], lw[l - 1], lev[l], lw[l], lh[l], lw[l]);
    }

    level_kp* all = (level_kp*)malloc(sizeof(level_kp) * (cap + 1));
    uint32_t nall = 0;
    for (int l = 0; l < L && nall < cap; l++) {
        const int W = lw[l], H = lh[l], N = perLevel[l];
        uint8_t* score = (uint8_t*)malloc((size_t)W * H + 1);
        int capc = (W / 2 + 2) * (H / 2 + 2);
        cand_t* cand = (cand_t*)malloc(sizeof(cand_t) * capc);
        int nc = fast_nms(lev[l], W, H, W, fastThreshold, score, cand);
        /* RunByImageBorder (:619-639): keep b <= x < W-b, b <= y < H-b */
        int m = 0;
        if (H > border * 2 && W > border * 2) {
            for (int i = 0; i < nc; i++)
                if (cand[i].x >= border && cand[i].x < W - border && cand[i].y >= border && cand[i].y < H - border)
                    cand[m++] = cand[i];
        }
        nc = m;
        anms_item* items = (anms_item*)malloc(sizeof(anms_item) * (nc + 1));
        anms_item* kept = (anms_item*)malloc(sizeof(anms_item) * (nc + 1));
        int nk;
        if (nc > N) {
            int maxNum = (int)((float)N * s->feature_factor);
            int cut = retain_cut(cand, nc, fastThreshold, maxNum, N, s->feature_strength);
            int ni = 0;
            for (int i = 0; i < nc; i++)
                if (cand[i].score >= cut) {
                    items[ni].x = cand[i].x;
                    items[ni].y = cand[i].y;
                    items[ni].strength = (float)cand[i].score;
                    items[ni].r = 0;
                    items[ni].idx = ni;
                    ni++;
                }
            nk = anms(items, ni, N, fastThreshold, s, kept);
        } else {
            for (int i = 0; i < nc; i++) {
                kept[i].x = cand[i].x;
                kept[i].y = cand[i].y;
                kept[i].strength = (float)cand[i].score;
                kept[i].r = 0;
                kept[i].idx = i;
            }
            nk = nc;
        }
        /* ImageData::Insert copies what still fits (ImageData.h:65-70) */
        for (int i = 0; i < nk && nall < cap; i++, nall++) {
            all[nall].x = kept[i].x;
            all[nall].y = kept[i].y;
            all[nall].level = l;
            all[nall].strength = kept[i].strength;
        }
        free(score);
        free(cand);
        free(items);
        free(kept);
    }

    /* keypoint fields: FAST emits KeyPoint(x, y, 7, -1, score) (:1508); octave / size
     * (:713-717); angle by ICAngles on the unblurred level or 0 (:748-754); pt *= layerScale
     * (:756-760). */
    int umax[64];
    if (s->use_orientation) oracle_umax(halfPatch, umax);
    for (uint32_t i = 0; i < nall; i++) {
        const level_kp* q = &all[i];
        const float sc = layerScale[q->level];
        kp[i].x = (float)q->x * sc;
        kp[i].y = (float)q->y * sc;
        kp[i].size = (float)s->patch_size * sc;
        kp[i].angle = s->use_orientation ? oracle_ic_angle(lev[q->level], lw[q->level], q->x, q->y, umax, halfPatch) : 0.0f;
        kp[i].response = q->strength;
        kp[i].octave = q->level;
        kp[i].class_id = -1;
    }
    *n_out = nall;

    if (nall > 0) {
        uint8_t* blurred[MAGE_MAX_LEVELS];
        for (int l = 0; l < L; l++) {
            blurred[l] = (uint8_t*)malloc((size_t)lw[l] * lh[l] + 1);
            if (s->gaussian_kernel_size > 1)
                oracle_gaussian_blur(lev[l], lw[l], lh[l], lw[l], (int)s->gaussian_kernel_size, blurred[l]);
            else
                memcpy(blurred[l], lev[l], (size_t)lw[l] * lh[l]);
        }
        for (uint32_t i = 0; i < nall; i++) {
            /* ComputeOrbDescriptorsPrerotated (:516-530): centre = cvRound(pt * (1.f/layerScale)),
             * rot = cvRound(angle / 12) % 30 */
            const int l = all[i].level;
            const float sc = 1.f / layerScale[l];
            const int cx = cv_roundf(kp[i].x * sc), cy = cv_roundf(kp[i].y * sc);
            if (prerotated) {
                const int rot = cv_roundf(kp[i].angle / 12.0f) % 30;
                describe(blurred[l], lw[l], pattern_table, cx, cy, rot, desc + 32 * (size_t)i);
            } else {
                describe_random(blurred[l], lw[l], random_pts, cx, cy, kp[i].angle, desc + 32 * (size_t)i);
            }
        }
        for (int l = 0; l < L; l++) free(blurred[l]);
    }
    for (int l = 0; l < L; l++) free(lev[l]);
    free(all);
    return MAGE_OK;
}

/* ------------------------------------------------------------------------------------------ */
/* Matching (Core/MAGESLAM/Source/Tracking/FeatureMatcher.cpp)                                  */
/* ------------------------------------------------------------------------------------------ */

/* GetDescriptorDistance, SWAR branch (FeatureMatcher.cpp:488-500). */
int oracle_hamming(const uint8_t* a, const uint8_t* b)
{
    int result = 0;
    for (int k = 0; k < 8; k++) {
        uint32_t x, y;
        memcpy(&x, a + 4 * k, 4);
        memcpy(&y, b + 4 * k, 4);
        uint32_t bits = x ^ y;
        bits = bits - ((bits >> 1) & 0x55555555u);
        bits = (bits & 0x33333333u) + ((bits >> 2) & 0x33333333u);
        result += (int)((((bits + (bits >> 4)) & 0x0F0F0F0Fu) * 0x01010101u) >> 24);
    }
    return result;
}

/* One direction of BFMatcher::radiusMatch (OpenCV 3.4.0, inclusive radius) reduced to what
 * Match reads: the best candidate (lowest distance, lowest index on ties) and whether the
 * row passes the delta test (FeatureMatcher.cpp:125-137, 144-156).  best[i] = -1 if rejected. */
static void best_rows(const uint8_t* q, const int* qi, int nq, const uint8_t* t, const int* ti,
                      int nt, int maxDist, int minDiff, int* best, int* bestDist)
{
    for (int i = 0; i < nq; i++) {
        int d0 = 1 << 30, d1 = 1 << 30, j0 = -1, cnt = 0;
        for (int j = 0; j < nt; j++) {
            int d = oracle_hamming(q + 32 * (size_t)qi[i], t + 32 * (size_t)ti[j]);
            if (d > maxDist) continue;
            cnt++;
            if (d < d0) {
                d1 = d0;
                d0 = d;
                j0 = j;
            } else if (d < d1)
                d1 = d;
        }
        best[i] = -1;
        bestDist[i] = d0;
        if (cnt == 0) continue;
        if (cnt > 1 && (float)(d1 - d0) < (float)minDiff) continue;
        best[i] = j0;
    }
}

/* UndistortKeypoints (OrbFeatureDetector.cpp:30-62): OpenCV 3.4.0 cvUndistortPoints with
 * R = noArray() and P = the undistorted camera matrix — f64 normalisation, 5 fixed-point
 * iterations (tilt compensation is the identity for zero tilt terms), RR = P * I in homogeneous
 * form, float output.  kd / kp: fx, fy, cx, cy; dist: ndist (0, 5 or 8) coefficients K1 K2 P1 P2
 * K3 [K4 K5 K6]; pts: n (x, y) pairs, in place. */
void oracle_undistort_points(const float* kd, const float* dist, int ndist, const float* kp, float* pts, int n)
{
    double k[14] = {0};
    for (int i = 0; i < ndist && i < 8; i++) k[i] = dist[i];
    const int iters = ndist > 0 ? 5 : 0;
    const double fx = kd[0], fy = kd[1], cx = kd[2], cy = kd[3];
    const double ifx = 1. / fx, ify = 1. / fy;
    const double RR[3][3] = {{kp[0], 0, kp[2]}, {0, kp[1], kp[3]}, {0, 0, 1}};
    for (int i = 0; i < n; i++) {
        double x = pts[2 * i], y = pts[2 * i + 1];
        x = (x - cx) * ifx;
        y = (y - cy) * ify;
        const double x0 = x, y0 = y;
        for (int j = 0; j < iters; j++) {
            double r2 = x * x + y * y;
            double icdist = (1 + ((k[7] * r2 + k[6]) * r2 + k[5]) * r2) / (1 + ((k[4] * r2 + k[1]) * r2 + k[0]) * r2);
            double deltaX = 2 * k[2] * x * y + k[3] * (r2 + 2 * x * x) + k[8] * r2 + k[9] * r2 * r2;
            double deltaY = k[2] * (r2 + 2 * y * y) + 2 * k[3] * x * y + k[10] * r2 + k[11] * r2 * r2;
            x = (x0 - deltaX) * icdist;
            y = (y0 - deltaY) * icdist;
        }
        double xx = RR[0][0] * x + RR[0][1] * y + RR[0][2];
        double yy = RR[1][0] * x + RR[1][1] * y + RR[1][2];
        double ww = 1. / (RR[2][0] * x + RR[2][1] * y + RR[2][2]);
        pts[2 * i] = (float)(xx * ww);
        pts[2 * i + 1] = (float)(yy * ww);
    }
}

/* RadiusMatch (FeatureMatcher.cpp:294-378 batch, :386-446 per query) with the target
 * KeypointSpatialIndex (KeypointSpatialIndex.cpp:46-106): the R-tree box query keeps targets with
 * |x - qx| <= radius, |y - qy| <= radius (boundary inclusive) and the query's octave (octave
 * coordinate 100 * octave, query range +-1).  Candidates are visited in ascending target index
 * (the R-tree's visiting order is unspecified; SURVEY.md §8(f) 1 fixes this order).  Per query:
 * best starts at maxDist + 1, second at INT_MAX; a strictly smaller distance moves best into
 * second (:425-437); accepted when (second - best) > minDiff (:441).  Batch: when more than one
 * query matched, a match survives only if its distance is the strict minimum among the matches
 * to its target (:342-371).  Output in query order; returns the number of matches. */
uint32_t oracle_radius_match(const mage_keypoint* qkp, const float* qpos, const uint8_t* qmask,
                             const uint8_t* qdesc, uint32_t nq, const mage_keypoint* tkp,
                             const uint8_t* tmask, const uint8_t* tdesc, uint32_t nt, float radius,
                             int maxDist, int minDiff, mage_dmatch* out, uint32_t cap)
{
    mage_dmatch* almost = (mage_dmatch*)malloc(sizeof(mage_dmatch) * (nq + 1));
    uint32_t na = 0;
    for (uint32_t q = 0; q < nq; q++) {
        if (qmask && !qmask[q]) continue;
        const float px = qpos ? qpos[2 * q] : qkp[q].x, py = qpos ? qpos[2 * q + 1] : qkp[q].y;
        const float oq = (float)qkp[q].octave * 100.0f;
        int best = maxDist + 1, second = 2147483647, train = -1;
        for (uint32_t t = 0; t < nt; t++) {
            const float ot = (float)tkp[t].octave * 100.0f;
            if (!(tkp[t].x >= px - radius && tkp[t].x <= px + radius && tkp[t].y >= py - radius &&
                  tkp[t].y <= py + radius && ot >= oq - 1.0f && ot <= oq + 1.0f))
                continue;
            if (tmask && !tmask[t]) continue;
            const int d = oracle_hamming(qdesc + 32 * (size_t)q, tdesc + 32 * (size_t)t);
            if (d < best) {
                train = (int)t;
                second = best;
                best = d;
            }
        }
        if (train != -1 && (second - best) > minDiff) {
            almost[na].query_idx = (int)q;
            almost[na].train_idx = train;
            almost[na].img_idx = 0;
            almost[na].distance = (float)best;
            na++;
        }
    }
    uint32_t n = 0;
    if (na > 1) {
        float* bd = (float*)malloc(sizeof(float) * (nt + 1));
        float* sd = (float*)malloc(sizeof(float) * (nt + 1));
        for (uint32_t t = 0; t < nt; t++) bd[t] = sd[t] = 3.402823466e+38f;
        for (uint32_t i = 0; i < na; i++) {
            const int t = almost[i].train_idx;
            if (almost[i].distance < bd[t]) {
                sd[t] = bd[t];
                bd[t] = almost[i].distance;
            } else if (almost[i].distance < sd[t]) {
                sd[t] = almost[i].distance;
            }
        }
        for (uint32_t i = 0; i < na; i++) {
            const int t = almost[i].train_idx;
            if (almost[i].distance == bd[t] && bd[t] < sd[t]) {
                if (n < cap) out[n] = almost[i];
                n++;
            }
        }
        free(bd);
        free(sd);
    } else {
        for (uint32_t i = 0; i < na; i++) {
            if (n < cap) out[n] = almost[i];
            n++;
        }
    }
    free(almost);
    return n;
}

/* Match (FeatureMatcher.cpp:61-190).  Returns the number of matches written. */
uint32_t oracle_match(const uint8_t* da, uint32_t na, const uint8_t* ma, const uint8_t* db,
                      uint32_t nb, const uint8_t* mb, int maxDist, int minDiff, mage_dmatch* out,
                      uint32_t cap)
{
    int* ia = (int*)malloc(sizeof(int) * (na + 1));
    int* ib = (int*)malloc(sizeof(int) * (nb + 1));
    int ca = 0, cb = 0;
    for (uint32_t i = 0; i < na; i++)
        if (!ma || ma[i]) ia[ca++] = (int)i;
    for (uint32_t i = 0; i < nb; i++)
        if (!mb || mb[i]) ib[cb++] = (int)i;
    uint32_t n = 0;
    if (ca && cb) {
        int* fwd = (int*)malloc(sizeof(int) * ca);
        int* fwdD = (int*)malloc(sizeof(int) * ca);
        int* bwd = (int*)malloc(sizeof(int) * cb);
        int* bwdD = (int*)malloc(sizeof(int) * cb);
        best_rows(da, ia, ca, db, ib, cb, maxDist, minDiff, fwd, fwdD);
        best_rows(db, ib, cb, da, ia, ca, maxDist, minDiff, bwd, bwdD);
        for (int i = 0; i < ca; i++) {
            int j = fwd[i];
            if (j < 0 || bwd[j] != i) continue;
            if (n < cap) {
                out[n].query_idx = ia[i];
                out[n].train_idx = ib[j];
                out[n].img_idx = -1; /* cv::DMatch(int, int, float): imgIdx = -1 */
                out[n].distance = (float)fwdD[i];
            }
            n++;
        }
        free(fwd);
        free(fwdD);
        free(bwd);
        free(bwdD);
    }
    free(ia);
    free(ib);
    return n;
}

/* TrackLocalMap's per-map-point loop (TrackLocalMap.cpp:175-256) reduced to its matching: for each
 * projected map point in order — hide the keypoint a pose-estimation outlier point was matched to
 * when it is currently unassociated (:192-203), MatchMapPointToCurrentFrame = the single-query
 * RadiusMatch (FeatureMatcher.cpp:386-446) against the unassociated keypoints (box |x - qx| <= r,
 * |y - qy| <= r, the query's octave; ascending keypoint order as above), unhide (:224-229), and on a
 * match associate the keypoint: unassociatedMask[t] = false (:249-255).  mask: 1 = unassociated,
 * updated in place; hide[i] = -1 for none; result[i] = keypoint or -1. */
void oracle_local_map_match(const float* qpos, const int32_t* qoct, const uint8_t* qdesc, const int32_t* hide,
                            uint32_t nq, const mage_keypoint* tkp, const uint8_t* tdesc, uint32_t nt, uint8_t* mask,
                            float radius, int maxDist, int minDiff, int32_t* result)
{
    for (uint32_t q = 0; q < nq; q++) {
        const int h = hide ? hide[q] : -1;
        int hidden = 0;
        if (h >= 0 && mask[h]) {
            mask[h] = 0;
            hidden = 1;
        }
        const float px = qpos[2 * q], py = qpos[2 * q + 1];
        const float oq = (float)qoct[q] * 100.0f;
        int best = maxDist + 1, second = 2147483647, train = -1;
        for (uint32_t t = 0; t < nt; t++) {
            const float ot = (float)tkp[t].octave * 100.0f;
            if (!(tkp[t].x >= px - radius && tkp[t].x <= px + radius && tkp[t].y >= py - radius &&
                  tkp[t].y <= py + radius && ot >= oq - 1.0f && ot <= oq + 1.0f))
                continue;
            if (!mask[t]) continue;
            const int d = oracle_hamming(qdesc + 32 * (size_t)q, tdesc + 32 * (size_t)t);
            if (d < best) {
                train = (int)t;
                second = best;
                best = d;
            }
        }
        if (hidden) mask[h] = 1;
        if (train != -1 && (second - best) > minDiff) {
            result[q] = train;
            mask[train] = 0;
        } else {
            result[q] = -1;
        }
    }
}
