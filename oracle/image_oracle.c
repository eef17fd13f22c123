/*
 * image_oracle.c — CPU restatement of the frame-ingest / undistortion path (TEST INFRASTRUCTURE
 * ONLY: used by tests/, never by the product).
 *
 * Follows Core/MAGESLAM/Source/Image/ImagePreprocessor.cpp:71-120 (CalculateUndistortedCalibration,
 * UndistortImage) and restates the OpenCV 3.4.0 calls it makes (README.md:21; parity unpinned, no
 * OpenCV here):
 *   cv::initUndistortRectifyMap(K, dist, noArray(), K', size, CV_32FC1, map1, map2)
 *     iR = inv(K' * I) by cv::invert's 3x3 closed form (det3 + cofactors, CV_64F), row-sequential
 *     accumulation _x += ir[0] ..., rational + tangential model, identity tilt, maps as (float)u/v;
 *   cv::remap(src, dst, map1, map2, INTER_LINEAR) with BORDER_CONSTANT 0: per pixel X = cvRound(u*32),
 *     Y = cvRound(v*32) (float products), integer part X >> 5 / Y >> 5 as short, fraction index
 *     (Y & 31) * 32 + (X & 31); initInterTab2D's fixed-point bilinear table (coefficients *32768,
 *     saturate_cast<short>: the (0, 0) entry saturates to 32767 and the table's sum fix-up adds the
 *     missing 1 to its fourth weight); (sum + 2^14) >> 15; inliers (0 <= sx < W-1, 0 <= sy < H-1) read
 *     the 2x2 block, outliers read each in-range tap and 0 for the others, or 0 outright when the
 *     block is entirely outside.
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

/* CalculateUndistortedCalibration: fx, fy kept, principal point at the image centre (float). */
void oracle_undistorted_intrinsics(const float* kd, int w, int h, float* kn)
{
    kn[0] = kd[0];
    kn[1] = kd[1];
    kn[2] = (float)w * 0.5f;
    kn[3] = (float)h * 0.5f;
}

/* kd, kn: {fx, fy, cx, cy}; dist: OpenCV order k1 k2 p1 p2 [k3 [k4 k5 k6]] (ndist 0, 4, 5 or 8). */
void oracle_undistort_map(const float* kd, const float* dist, int ndist, const float* kn, int w, int h, float* mapx,
                          float* mapy)
{
    double k[14] = {0};
    for (int i = 0; i < ndist && i < 14; i++) k[i] = (double)dist[i];
    const double k1 = k[0], k2 = k[1], p1 = k[2], p2 = k[3];
    const double k3 = ndist >= 5 ? k[4] : 0., k4 = ndist >= 8 ? k[5] : 0., k5 = ndist >= 8 ? k[6] : 0.,
                 k6 = ndist >= 8 ? k[7] : 0.;
    const double s1 = 0, s2 = 0, s3 = 0, s4 = 0;
    /* Ar = K' (double), R = I: Ar * R is exact */
    double S[9] = {kn[0], 0, kn[2], 0, kn[1], kn[3], 0, 0, 1};
#define Sd(r, c) S[(r)*3 + (c)]
    double d = Sd(0, 0) * (Sd(1, 1) * Sd(2, 2) - Sd(1, 2) * Sd(2, 1)) - Sd(0, 1) * (Sd(1, 0) * Sd(2, 2) - Sd(1, 2) * Sd(2, 0)) +
               Sd(0, 2) * (Sd(1, 0) * Sd(2, 1) - Sd(1, 1) * Sd(2, 0));
    double ir[9] = {0};
    if (d != 0.) {
        d = 1. / d;
        ir[0] = (Sd(1, 1) * Sd(2, 2) - Sd(1, 2) * Sd(2, 1)) * d;
        ir[1] = (Sd(0, 2) * Sd(2, 1) - Sd(0, 1) * Sd(2, 2)) * d;
        ir[2] = (Sd(0, 1) * Sd(1, 2) - Sd(0, 2) * Sd(1, 1)) * d;
        ir[3] = (Sd(1, 2) * Sd(2, 0) - Sd(1, 0) * Sd(2, 2)) * d;
        ir[4] = (Sd(0, 0) * Sd(2, 2) - Sd(0, 2) * Sd(2, 0)) * d;
        ir[5] = (Sd(0, 2) * Sd(1, 0) - Sd(0, 0) * Sd(1, 2)) * d;
        ir[6] = (Sd(1, 0) * Sd(2, 1) - Sd(1, 1) * Sd(2, 0)) * d;
        ir[7] = (Sd(0, 1) * Sd(2, 0) - Sd(0, 0) * Sd(2, 1)) * d;
        ir[8] = (Sd(0, 0) * Sd(1, 1) - Sd(0, 1) * Sd(1, 0)) * d;
    }
#undef Sd
    const double u0 = kd[2], v0 = kd[3], fx = kd[0], fy = kd[1];
    for (int i = 0; i < h; i++) {
        double _x = i * ir[1] + ir[2], _y = i * ir[4] + ir[5], _w = i * ir[7] + ir[8];
        for (int j = 0; j < w; j++, _x += ir[0], _y += ir[3], _w += ir[6]) {
            double ww = 1. / _w, x = _x * ww, y = _y * ww;
            double x2 = x * x, y2 = y * y;
            double r2 = x2 + y2, _2xy = 2 * x * y;
            double kr = (1 + ((k3 * r2 + k2) * r2 + k1) * r2) / (1 + ((k6 * r2 + k5) * r2 + k4) * r2);
            double xd = (x * kr + p1 * _2xy + p2 * (r2 + 2 * x2) + s1 * r2 + s2 * r2 * r2);
            double yd = (y * kr + p1 * (r2 + 2 * y2) + p2 * _2xy + s3 * r2 + s4 * r2 * r2);
            /* identity tilt: vecTilt = (xd, yd, 1), invProj = 1 */
            double invProj = 1.;
            double u = fx * invProj * xd + u0;
            double v = fy * invProj * yd + v0;
            mapx[(size_t)i * w + j] = (float)u;
            mapy[(size_t)i * w + j] = (float)v;
        }
    }
}

static void bilinear_weights(int a, int wts[4])
{
    const int tx = a & 31, ty = a >> 5;
    wts[0] = (32 - ty) * (32 - tx) * 32;
    wts[1] = (32 - ty) * tx * 32;
    wts[2] = ty * (32 - tx) * 32;
    wts[3] = ty * tx * 32;
    if (a == 0) { /* saturate_cast<short>(32768.f) = 32767, fix-up adds 1 to entry 3 */
        wts[0] = 32767;
        wts[3] = 1;
    }
}

static int iround_f(float v) { return (int)lrintf(v); }

void oracle_remap_linear(const uint8_t* src, int sw, int sh, int sstride, const float* mapx, const float* mapy, int dw,
                         int dh, uint8_t* dst, int dstride)
{
    const unsigned width1 = (unsigned)(sw > 1 ? sw - 1 : 0), height1 = (unsigned)(sh > 1 ? sh - 1 : 0);
    for (int y = 0; y < dh; y++)
        for (int x = 0; x < dw; x++) {
            const float fu = mapx[(size_t)y * dw + x], fv = mapy[(size_t)y * dw + x];
            const int X = iround_f(fu * 32.0f), Y = iround_f(fv * 32.0f);
            int sx = X >> 5, sy = Y >> 5;
            if (sx > 32767) sx = 32767;
            if (sx < -32768) sx = -32768;
            if (sy > 32767) sy = 32767;
            if (sy < -32768) sy = -32768;
            const int a = (Y & 31) * 32 + (X & 31);
            int w[4];
            bilinear_weights(a, w);
            int v0, v1, v2, v3;
            if ((unsigned)sx < width1 && (unsigned)sy < height1) {
                const uint8_t* S = src + (size_t)sy * sstride + sx;
                v0 = S[0];
                v1 = S[1];
                v2 = S[sstride];
                v3 = S[sstride + 1];
            } else if (sx >= sw || sx + 1 < 0 || sy >= sh || sy + 1 < 0) {
                dst[(size_t)y * dstride + x] = 0;
                continue;
            } else {
                const int x0ok = sx >= 0 && sx < sw, x1ok = sx + 1 >= 0 && sx + 1 < sw;
                const int y0ok = sy >= 0 && sy < sh, y1ok = sy + 1 >= 0 && sy + 1 < sh;
                v0 = x0ok && y0ok ? src[(size_t)sy * sstride + sx] : 0;
                v1 = x1ok && y0ok ? src[(size_t)sy * sstride + sx + 1] : 0;
                v2 = x0ok && y1ok ? src[(size_t)(sy + 1) * sstride + sx] : 0;
                v3 = x1ok && y1ok ? src[(size_t)(sy + 1) * sstride + sx + 1] : 0;
            }
            int r = (v0 * w[0] + v1 * w[1] + v2 * w[2] + v3 * w[3] + (1 << 14)) >> 15;
            dst[(size_t)y * dstride + x] = (uint8_t)(r < 0 ? 0 : r > 255 ? 255 : r);
        }
}

/* ---- ImagePreprocessor::ScaleImageForCameraConfiguration (ImagePreprocessor.cpp:18-65) ------
 * Restated geometry (the image step is oracle_resize_linear, orb_oracle.c):
 *   targetToSource = ToCVMat4x4(source.Extrinsics) * ToCVMat4x4(target.Extrinsics).inv()   (:34)
 *     cv::Matx44f: products with the sum started at 0 and taken left to right; inv() = LU with
 *     partial pivoting (OpenCV 3.4.0 Matx_FastInvOp -> hal::LU32f / LUImpl, eps 10*FLT_EPSILON,
 *     all zeros if singular);
 *   CalculateOverlapCropSourceInTarget (MageUtil.cpp:13-58): the 4 source corners (0,0), (W-1,0),
 *     (0,H-1), (W-1,H-1) UnProject'ed (Utils/cv.h:270-278: inv(K_src) (3x3 adjugate over the float
 *     determinant, Matx_FastInvOp<_Tp,3>) x pixel, * depth, then Invert(targetToSource) (cv.h:226-262:
 *     transposed rotation x negated translation) x (p, 1)), ProjectUndistorted with the identity view
 *     (Reprojection.cpp:26-42); min initialised to FLT_MAX, max to FLT_MIN (the smallest positive
 *     float, as the reference does); width = max - min + 1; Rect{(int)min.x, (int)min.y,
 *     (size_t)width, (size_t)height} -> cv::Rect (ToCVRect, cv.h:429-432);
 *   IsEntirelyOffscreen (cv.h:405-418) -> not ok;
 *   scale = max(crop.width / (float)W, crop.height / (float)H); size (int)(W * scale);
 *   GetScaledIntrinsics (CameraCalibration.cpp:150-157) when scale != 1.
 * cfg layout (float[22] view of mage_camera_config): extrinsics[16] (M11..M44), fx, fy, cx, cy, then
 * width / height as uint32 (read through w_h). */
#include <float.h>

static void o_mul(const float* a, const float* b, float* c, int m, int l, int n)
{
    for (int i = 0; i < m; i++)
        for (int j = 0; j < n; j++) {
            float s = 0.f;
            for (int k = 0; k < l; k++) s += a[i * l + k] * b[k * n + j];
            c[i * n + j] = s;
        }
}

static void o_inv4(const float* src, float* inv)
{
    float a[4][4], b[4][4];
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++) {
            a[i][j] = src[4 * i + j];
            b[i][j] = i == j ? 1.f : 0.f;
        }
    for (int i = 0; i < 4; i++) {
        int p = i;
        for (int j = i + 1; j < 4; j++)
            if (fabsf(a[j][i]) > fabsf(a[p][i])) p = j;
        if (fabsf(a[p][i]) < FLT_EPSILON * 10) {
            memset(inv, 0, 16 * sizeof(float));
            return;
        }
        if (p != i) {
            for (int j = i; j < 4; j++) {
                float t = a[i][j];
                a[i][j] = a[p][j];
                a[p][j] = t;
            }
            for (int j = 0; j < 4; j++) {
                float t = b[i][j];
                b[i][j] = b[p][j];
                b[p][j] = t;
            }
        }
        float d = -1.f / a[i][i];
        for (int j = i + 1; j < 4; j++) {
            float alpha = a[j][i] * d;
            for (int k = i + 1; k < 4; k++) a[j][k] += alpha * a[i][k];
            for (int k = 0; k < 4; k++) b[j][k] += alpha * b[i][k];
        }
    }
    for (int i = 3; i >= 0; i--)
        for (int j = 0; j < 4; j++) {
            float s = b[i][j];
            for (int k = i + 1; k < 4; k++) s -= a[i][k] * b[k][j];
            b[i][j] = s / a[i][i];
        }
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++) inv[4 * i + j] = b[i][j];
}

static void o_inv3(const float* m, float* r)
{
    float d = m[0] * (m[4] * m[8] - m[7] * m[5]) - m[1] * (m[3] * m[8] - m[6] * m[5]) +
              m[2] * (m[3] * m[7] - m[6] * m[4]);
    if (d == 0) {
        memset(r, 0, 9 * sizeof(float));
        return;
    }
    d = 1 / d;
    r[0] = (m[4] * m[8] - m[5] * m[7]) * d;
    r[1] = (m[2] * m[7] - m[1] * m[8]) * d;
    r[2] = (m[1] * m[5] - m[2] * m[4]) * d;
    r[3] = (m[5] * m[6] - m[3] * m[8]) * d;
    r[4] = (m[0] * m[8] - m[2] * m[6]) * d;
    r[5] = (m[2] * m[3] - m[0] * m[5]) * d;
    r[6] = (m[3] * m[7] - m[4] * m[6]) * d;
    r[7] = (m[1] * m[6] - m[0] * m[7]) * d;
    r[8] = (m[0] * m[4] - m[1] * m[3]) * d;
}

/* returns ok; crop[4], scale, out_wh[2], out_k[4] = {fx, fy, cx, cy} of the prepared camera */
int oracle_scale_geometry(const float* src_ext, const float* src_k, const uint32_t* src_wh, const float* tgt_ext,
                          const float* tgt_k, const uint32_t* tgt_wh, float depth, int* crop, float* scale,
                          uint32_t* out_wh, float* out_k)
{
    float ti[16], t2s[16];
    o_inv4(tgt_ext, ti);
    o_mul(src_ext, ti, t2s, 4, 4, 4);
    const float Ks[9] = {src_k[0], 0, src_k[2], 0, src_k[1], src_k[3], 0, 0, 1};
    float Ki[9];
    o_inv3(Ks, Ki);
    const float rot[16] = {t2s[0], t2s[4], t2s[8], 0, t2s[1], t2s[5], t2s[9], 0, t2s[2], t2s[6], t2s[10], 0, 0, 0, 0, 1};
    const float tr[16] = {1, 0, 0, -t2s[3], 0, 1, 0, -t2s[7], 0, 0, 1, -t2s[11], 0, 0, 0, 1};
    float vinv[16];
    o_mul(rot, tr, vinv, 4, 4, 4);
    const float mc = (float)src_wh[0] - 1, mr = (float)(src_wh[1] - 1);
    const float cx[4] = {0, mc, 0, mc}, cy[4] = {0, 0, mr, mr};
    float lox = FLT_MAX, loy = FLT_MAX, hix = FLT_MIN, hiy = FLT_MIN;
    for (int c = 0; c < 4; c++) {
        const float pix[3] = {(float)(int)cx[c], (float)(int)cy[c], 1.f};
        float cam[3];
        o_mul(Ki, pix, cam, 3, 3, 1);
        for (int k = 0; k < 3; k++) cam[k] *= depth;
        const float h4[4] = {cam[0], cam[1], cam[2], 1};
        float w[4];
        o_mul(vinv, h4, w, 4, 4, 1);
        const float eye[12] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0};
        const float w4[4] = {w[0], w[1], w[2], 1};
        float v[3];
        o_mul(eye, w4, v, 3, 4, 1);
        const float z = v[2] != 0 ? v[2] : 1;
        const float px = (v[0] / z) * tgt_k[0] + tgt_k[2];
        const float py = (v[1] / z) * tgt_k[1] + tgt_k[3];
        if (px < lox) lox = px;
        if (py < loy) loy = py;
        if (px > hix) hix = px;
        if (py > hiy) hiy = py;
    }
    const float wd = hix - lox + 1, ht = hiy - loy + 1;
    crop[0] = (int)lox;
    crop[1] = (int)loy;
    crop[2] = (int)(size_t)wd;
    crop[3] = (int)(size_t)ht;
    out_wh[0] = src_wh[0];
    out_wh[1] = src_wh[1];
    for (int k = 0; k < 4; k++) out_k[k] = src_k[k];
    const int mxh = crop[2] + crop[0] - 1, mxv = crop[3] + crop[1] - 1;
    if (mxh < 0 || crop[0] > (int)(tgt_wh[0] - 1) || mxv < 0 || crop[1] > (int)(tgt_wh[1] - 1)) {
        *scale = 0.f;
        return 0;
    }
    const float sx = crop[2] / (float)src_wh[0], sy = crop[3] / (float)src_wh[1];
    const float s = sx > sy ? sx : sy;
    *scale = s;
    if (s != 1.0f) {
        out_wh[0] = (uint32_t)(int)((float)src_wh[0] * s);
        out_wh[1] = (uint32_t)(int)((float)src_wh[1] * s);
        for (int k = 0; k < 4; k++) out_k[k] = src_k[k] * s;
    }
    return 1;
}
