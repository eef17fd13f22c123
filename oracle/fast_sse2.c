/*
 * fast_sse2.c — the x64 (SSE2) build of MAGE-SLAM's FAST_t<16>, restated (TEST INFRASTRUCTURE ONLY).
 *
 * The reference is built for x64 with CV_SSE2, so the branches it actually runs are the SSE2
 * ones: the 16-pixel FAST row loop (OpenCVModified.cpp:1278-1338) with the scalar loop for the
 * row tail (:1415-1479), and the SSE2 cornerScore<16> (:935-972) for every corner (the scalar
 * cornerScore branch :1030-1064 is not compiled in that build).  The oracle (orb_oracle.c) and the
 * GPU kernel follow the scalar branches.  The reference's own self-check VERIFY_SIMD (:1265-1271,
 * :1408-1486) asserts that its SIMD row loop and scalar row loop write the same score row; this
 * file lets tests/test_oracle.py check the stronger statement the parity path relies on — the
 * SSE2 build's whole score map equals the scalar oracle's — on random, saturated and synthetic
 * frames, so it is checked rather than cited.
 *
 * Restated with <emmintrin.h> intrinsics, the same operations in the same order as the
 * reference; linked only into the oracle library, never into the product.
 */
#include <emmintrin.h>
#include <stdint.h>
#include <string.h>

static const int kRing16s[16][2] = {{0, 3},  {1, 3},   {2, 2},   {3, 1},   {3, 0},  {3, -1},
                                    {2, -2}, {1, -3},  {0, -3},  {-1, -3}, {-2, -2}, {-3, -1},
                                    {-3, 0}, {-3, 1},  {-2, 2},  {-1, 3}};

/* cornerScore<16>, CV_SSE2 branch (OpenCVModified.cpp:927-972): the threshold argument is not
 * read (q0 starts at -1000). */
static int corner_score16_sse2(const uint8_t* ptr, const int pixel[25])
{
    const int N = 25;
    short d[25];
    const int v = ptr[0];
    for (int k = 0; k < N; k++) d[k] = (short)(v - ptr[pixel[k]]);
    __m128i q0 = _mm_set1_epi16(-1000), q1 = _mm_set1_epi16(1000);
    for (int k = 0; k < 16; k += 8) {
        __m128i v0 = _mm_loadu_si128((const __m128i*)(d + k + 1));
        __m128i v1 = _mm_loadu_si128((const __m128i*)(d + k + 2));
        __m128i a = _mm_min_epi16(v0, v1);
        __m128i b = _mm_max_epi16(v0, v1);
        for (int o = 3; o <= 8; o++) {
            v0 = _mm_loadu_si128((const __m128i*)(d + k + o));
            a = _mm_min_epi16(a, v0);
            b = _mm_max_epi16(b, v0);
        }
        v0 = _mm_loadu_si128((const __m128i*)(d + k));
        q0 = _mm_max_epi16(q0, _mm_min_epi16(a, v0));
        q1 = _mm_min_epi16(q1, _mm_max_epi16(b, v0));
        v0 = _mm_loadu_si128((const __m128i*)(d + k + 9));
        q0 = _mm_max_epi16(q0, _mm_min_epi16(a, v0));
        q1 = _mm_min_epi16(q1, _mm_max_epi16(b, v0));
    }
    q0 = _mm_max_epi16(q0, _mm_sub_epi16(_mm_setzero_si128(), q1));
    q0 = _mm_max_epi16(q0, _mm_unpackhi_epi64(q0, q0));
    q0 = _mm_max_epi16(q0, _mm_srli_si128(q0, 4));
    q0 = _mm_max_epi16(q0, _mm_srli_si128(q0, 2));
    return (short)_mm_cvtsi128_si32(q0) - 1;
}

/* FAST_t<16> of the SSE2 build, score rows only (the `curr` rows NMS reads, :1258-1487): rows
 * 3..h-4; the SIMD loop while j < w-19 (with its 8-pixel step back when only the upper half of a
 * block can hold corners), then the scalar loop with threshold_tab (:694-698) up to w-4.  `score`
 * (w x h) is 0 outside corners, as curr is memset per row.  `simd_cols` (h entries, may be NULL)
 * receives, per row, the column where the SIMD loop stopped (VERIFY_SIMD's simdEntriesWritten). */
void oracle_fast_score_map_sse2(const uint8_t* img, int w, int h, int stride, int threshold, uint8_t* score,
                                int* simd_cols)
{
    const int K = 8, N = 25, quarter = 4;
    int pixel[25];
    for (int k = 0; k < 16; k++) pixel[k] = kRing16s[k][0] + kRing16s[k][1] * stride;
    for (int k = 16; k < 25; k++) pixel[k] = pixel[k - 16];
    const int fast_threshold = threshold;
    threshold = threshold < 0 ? 0 : threshold > 255 ? 255 : threshold;
    uint8_t threshold_tab[512];
    for (int t = -255; t <= 255; t++)
        threshold_tab[t + 255] = (uint8_t)(t < -fast_threshold ? 1 : t > fast_threshold ? 2 : 0);
    const __m128i delta = _mm_set1_epi8(-128), t = _mm_set1_epi8((char)threshold), K16 = _mm_set1_epi8((char)K);
    memset(score, 0, (size_t)w * h);
    for (int i = 3; i < h - 3; i++) {
        const uint8_t* ptr = img + (size_t)i * stride + 3;
        uint8_t* curr = score + (size_t)i * w;
        int j = 3;
        for (; j < w - 16 - 3; j += 16, ptr += 16) {
            __m128i m0, m1;
            __m128i v0 = _mm_loadu_si128((const __m128i*)ptr);
            __m128i v1 = _mm_xor_si128(_mm_subs_epu8(v0, t), delta);
            v0 = _mm_xor_si128(_mm_adds_epu8(v0, t), delta);
            __m128i x0 = _mm_sub_epi8(_mm_loadu_si128((const __m128i*)(ptr + pixel[0])), delta);
            __m128i x1 = _mm_sub_epi8(_mm_loadu_si128((const __m128i*)(ptr + pixel[quarter])), delta);
            __m128i x2 = _mm_sub_epi8(_mm_loadu_si128((const __m128i*)(ptr + pixel[2 * quarter])), delta);
            __m128i x3 = _mm_sub_epi8(_mm_loadu_si128((const __m128i*)(ptr + pixel[3 * quarter])), delta);
            m0 = _mm_and_si128(_mm_cmpgt_epi8(x0, v0), _mm_cmpgt_epi8(x1, v0));
            m1 = _mm_and_si128(_mm_cmpgt_epi8(v1, x0), _mm_cmpgt_epi8(v1, x1));
            m0 = _mm_or_si128(m0, _mm_and_si128(_mm_cmpgt_epi8(x1, v0), _mm_cmpgt_epi8(x2, v0)));
            m1 = _mm_or_si128(m1, _mm_and_si128(_mm_cmpgt_epi8(v1, x1), _mm_cmpgt_epi8(v1, x2)));
            m0 = _mm_or_si128(m0, _mm_and_si128(_mm_cmpgt_epi8(x2, v0), _mm_cmpgt_epi8(x3, v0)));
            m1 = _mm_or_si128(m1, _mm_and_si128(_mm_cmpgt_epi8(v1, x2), _mm_cmpgt_epi8(v1, x3)));
            m0 = _mm_or_si128(m0, _mm_and_si128(_mm_cmpgt_epi8(x3, v0), _mm_cmpgt_epi8(x0, v0)));
            m1 = _mm_or_si128(m1, _mm_and_si128(_mm_cmpgt_epi8(v1, x3), _mm_cmpgt_epi8(v1, x0)));
            m0 = _mm_or_si128(m0, m1);
            const int mask = _mm_movemask_epi8(m0);
            if (mask == 0) continue;
            if ((mask & 255) == 0) {
                j -= 8;
                ptr -= 8;
                continue;
            }
            __m128i c0 = _mm_setzero_si128(), c1 = c0, max0 = c0, max1 = c0;
            for (int k = 0; k < N; k++) {
                __m128i x = _mm_xor_si128(_mm_loadu_si128((const __m128i*)(ptr + pixel[k])), delta);
                m0 = _mm_cmpgt_epi8(x, v0);
                m1 = _mm_cmpgt_epi8(v1, x);
                c0 = _mm_and_si128(_mm_sub_epi8(c0, m0), m0);
                c1 = _mm_and_si128(_mm_sub_epi8(c1, m1), m1);
                max0 = _mm_max_epu8(max0, c0);
                max1 = _mm_max_epu8(max1, c1);
            }
            max0 = _mm_max_epu8(max0, max1);
            int m = _mm_movemask_epi8(_mm_cmpgt_epi8(max0, K16));
            for (int k = 0; m > 0 && k < 16; k++, m >>= 1)
                if (m & 1) curr[j + k] = (uint8_t)corner_score16_sse2(ptr + k, pixel);
        }
        if (simd_cols) simd_cols[i] = j;
        for (; j < w - 3; j++, ptr++) {
            const int v = ptr[0];
            const uint8_t* tab = &threshold_tab[0] - v + 255;
            int d = tab[ptr[pixel[0]]] | tab[ptr[pixel[8]]];
            if (d == 0) continue;
            d &= tab[ptr[pixel[2]]] | tab[ptr[pixel[10]]];
            d &= tab[ptr[pixel[4]]] | tab[ptr[pixel[12]]];
            d &= tab[ptr[pixel[6]]] | tab[ptr[pixel[14]]];
            if (d == 0) continue;
            d &= tab[ptr[pixel[1]]] | tab[ptr[pixel[9]]];
            d &= tab[ptr[pixel[3]]] | tab[ptr[pixel[11]]];
            d &= tab[ptr[pixel[5]]] | tab[ptr[pixel[13]]];
            d &= tab[ptr[pixel[7]]] | tab[ptr[pixel[15]]];
            if (d & 1) {
                int vt = v - threshold, count = 0;
                for (int k = 0; k < N; k++) {
                    const int x = ptr[pixel[k]];
                    if (x < vt) {
                        if (++count > K) {
                            curr[j] = (uint8_t)corner_score16_sse2(ptr, pixel);
                            break;
                        }
                    } else
                        count = 0;
                }
            }
            if (d & 2) {
                int vt = v + threshold, count = 0;
                for (int k = 0; k < N; k++) {
                    const int x = ptr[pixel[k]];
                    if (x > vt) {
                        if (++count > K) {
                            curr[j] = (uint8_t)corner_score16_sse2(ptr, pixel);
                            break;
                        }
                    } else
                        count = 0;
                }
            }
        }
    }
}
