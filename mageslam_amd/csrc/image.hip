// image.hip — frame undistortion on MI355X (gfx950): ImagePreprocessor::UndistortImage
// (Core/MAGESLAM/Source/Image/ImagePreprocessor.cpp:71-120).
//
// The reference caches cv::initUndistortRectifyMap(K, dist, noArray(), K', size, CV_32FC1) once per
// calibration and runs cv::remap(INTER_LINEAR, BORDER_CONSTANT 0) on every distorted frame.  Same
// split here:
//   undistort_map_kernel  once per calibration: thread per row, the row-sequential accumulation
//                         _x += ir[0] ... of OpenCV 3.4.0 in fp64 (built with -ffp-contract=off:
//                         bit-exact maps), written as the two CV_32FC1 planes
//   remap_boxes_kernel    once per calibration: per 64x16 output tile, the bounding box of its
//                         in-range source taps
//   remap_linear_kernel   per batch of frames: workgroup per 64x16 tile x 64 frames, thread per 4
//                         output pixels.  The maps are read once as float4 (coalesced) and kept as
//                         register coefficients: X = rint(u * 32) -> the short integer part and the
//                         5+5-bit fraction index of remap's fixed-point path, initInterTab2D's
//                         bilinear weights (x 32768, the saturated (0,0) entry included).  Per frame
//                         the tile's source box is staged in LDS with dword loads and the 4 taps of
//                         each pixel are LDS byte reads; (sum + 2^14) >> 15, one dword store;
//                         constant-0 border as remapBilinear treats outliers.  HBM-bound: ~2 B per
//                         pixel and frame (box in, pixel out) + the map / 64.  The box of frame f + 1
//                         is loaded into registers while frame f is computed (LDS double buffer).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <climits>
#include <limits>
#include <utility>
#include <cmath>

#include "common.hpp"

struct mage_undistorter {
    int device = 0;
    int width = 0, height = 0;
    mage_calibration undistorted{};
    mage::DeviceBuffer maps;     // [mapx (W*H floats)][mapy (W*H floats)]
    mage::DeviceBuffer boxes;    // per 64x16 output tile: the source box staged in LDS (int4)
    mage::DeviceBuffer scratch;  // host-path frames
    hipStream_t st = nullptr;
};

namespace mage {
namespace {

struct MapParams {
    double ir[9];
    double fx, fy, u0, v0;
    double k1, k2, p1, p2, k3, k4, k5, k6;
    int w, h;
    float* mapx;
    float* mapy;
};

__global__ __launch_bounds__(64) void undistort_map_kernel(MapParams p)
{
    const int i = blockIdx.x * 64 + threadIdx.x;
    if (i >= p.h) return;
    const double* ir = p.ir;
    double _x = i * ir[1] + ir[2], _y = i * ir[4] + ir[5], _w = i * ir[7] + ir[8];
    float* mx = p.mapx + (long long)i * p.w;
    float* my = p.mapy + (long long)i * p.w;
    for (int j = 0; j < p.w; j++, _x += ir[0], _y += ir[3], _w += ir[6]) {
        const double ww = 1. / _w, x = _x * ww, y = _y * ww;
        const double x2 = x * x, y2 = y * y;
        const double r2 = x2 + y2, _2xy = 2 * x * y;
        const double kr = (1 + ((p.k3 * r2 + p.k2) * r2 + p.k1) * r2) / (1 + ((p.k6 * r2 + p.k5) * r2 + p.k4) * r2);
        // s1..s4 = 0 (at most 8 coefficients): the terms s*r2 add exact zeros
        const double xd = (x * kr + p.p1 * _2xy + p.p2 * (r2 + 2 * x2) + 0.0 * r2 + 0.0 * r2 * r2);
        const double yd = (y * kr + p.p1 * (r2 + 2 * y2) + p.p2 * _2xy + 0.0 * r2 + 0.0 * r2 * r2);
        const double invProj = 1.;  // identity tilt (tauX = tauY = 0)
        mx[j] = (float)(p.fx * invProj * xd + p.u0);
        my[j] = (float)(p.fy * invProj * yd + p.v0);
    }
}

struct RemapParams {
    const uint8_t* src;
    int sw, sh, sstride;
    long long spitch;
    const float* mapx;
    const float* mapy;
    uint8_t* dst;
    int dw, dh, dstride;
    long long dpitch;
};

// One output pixel's remap coefficients: the map-dependent part, shared by every frame.
struct RemapTap {
    int sx, sy;  // integer source position (short range)
    int w0, w1, w2, w3;
    int mode;  // 0: inlier 2x2 block, 1: outlier with some taps inside, 2: entirely outside
};

__device__ __forceinline__ RemapTap remap_tap(int sw, int sh, float fu, float fv)
{
    RemapTap t;
    const int X = __float2int_rn(fu * 32.0f), Y = __float2int_rn(fv * 32.0f);
    t.sx = min(max(X >> 5, -32768), 32767);
    t.sy = min(max(Y >> 5, -32768), 32767);
    const int tx = X & 31, ty = Y & 31;
    t.w0 = (32 - ty) * (32 - tx) * 32;
    t.w1 = (32 - ty) * tx * 32;
    t.w2 = ty * (32 - tx) * 32;
    t.w3 = ty * tx * 32;
    if ((tx | ty) == 0) {  // initInterTab2D: saturate_cast<short>(32768.f) = 32767, fix-up +1 on entry 3
        t.w0 = 32767;
        t.w3 = 1;
    }
    if ((unsigned)t.sx < (unsigned)max(sw - 1, 0) && (unsigned)t.sy < (unsigned)max(sh - 1, 0)) t.mode = 0;
    else if (t.sx >= sw || t.sx + 1 < 0 || t.sy >= sh || t.sy + 1 < 0) t.mode = 2;
    else t.mode = 1;
    return t;
}

__device__ __forceinline__ unsigned remap_apply(const RemapTap& t, const uint8_t* __restrict__ S0, int sw, int sh,
                                                int sstride)
{
    int v0, v1, v2, v3;
    if (t.mode == 0) {
        const uint8_t* S = S0 + (long long)t.sy * sstride + t.sx;
        v0 = S[0];
        v1 = S[1];
        v2 = S[sstride];
        v3 = S[sstride + 1];
    } else if (t.mode == 2) {
        return 0;
    } else {
        const bool x0 = t.sx >= 0 && t.sx < sw, x1 = t.sx + 1 >= 0 && t.sx + 1 < sw;
        const bool y0 = t.sy >= 0 && t.sy < sh, y1 = t.sy + 1 >= 0 && t.sy + 1 < sh;
        v0 = x0 && y0 ? S0[(long long)t.sy * sstride + t.sx] : 0;
        v1 = x1 && y0 ? S0[(long long)t.sy * sstride + t.sx + 1] : 0;
        v2 = x0 && y1 ? S0[(long long)(t.sy + 1) * sstride + t.sx] : 0;
        v3 = x1 && y1 ? S0[(long long)(t.sy + 1) * sstride + t.sx + 1] : 0;
    }
    const int r = (v0 * t.w0 + v1 * t.w1 + v2 * t.w2 + v3 * t.w3 + (1 << 14)) >> 15;
    return (unsigned)min(max(r, 0), 255);
}

// Output tiles of 64 x 16 pixels: 256 threads x 4 consecutive pixels.  Each tile's source taps
// fall in a small box (the map is smooth); the box is computed once per calibration and, per frame,
// staged into LDS with dword loads, so the 4 taps per pixel are LDS byte reads instead of four
// scattered global byte loads.  Tiles whose box exceeds RM_BOX_BYTES read taps from global memory.
constexpr int RM_TW = 64, RM_TH = 16;
constexpr int RM_BOX_BYTES = 8192;
// Frames per workgroup: the map (8 B per pixel) is read once per RM_FRAMES frames and its
// coefficients stay in registers.
constexpr int RM_FRAMES = 64;

// Per tile: (x0 aligned down to 4, y0, padded width (multiple of 4), height) of the box holding every
// in-range tap; width -1 = global fallback, 0 = no in-range tap.
__global__ __launch_bounds__(256) void remap_boxes_kernel(const float* __restrict__ mapx, const float* __restrict__ mapy,
                                                          int w, int h, int4* __restrict__ boxes)
{
    __shared__ int bx0, bx1, by0, by1;
    if (threadIdx.x == 0) {
        bx0 = by0 = INT_MAX;
        bx1 = by1 = INT_MIN;
    }
    __syncthreads();
    const int x = blockIdx.x * RM_TW + (threadIdx.x % (RM_TW / 4)) * 4, y = blockIdx.y * RM_TH + threadIdx.x / (RM_TW / 4);
    int lx0 = INT_MAX, lx1 = INT_MIN, ly0 = INT_MAX, ly1 = INT_MIN;
    if (y < h)
        for (int k = 0; k < 4 && x + k < w; k++) {
            const RemapTap t = remap_tap(w, h, mapx[(long long)y * w + x + k], mapy[(long long)y * w + x + k]);
            if (t.mode == 2) continue;
            for (int dy = 0; dy < 2; dy++)
                for (int dx = 0; dx < 2; dx++) {
                    const int sx = t.sx + dx, sy = t.sy + dy;
                    if (sx < 0 || sx >= w || sy < 0 || sy >= h) continue;
                    lx0 = min(lx0, sx);
                    lx1 = max(lx1, sx);
                    ly0 = min(ly0, sy);
                    ly1 = max(ly1, sy);
                }
        }
    atomicMin(&bx0, lx0);
    atomicMax(&bx1, lx1);
    atomicMin(&by0, ly0);
    atomicMax(&by1, ly1);
    __syncthreads();
    if (threadIdx.x != 0) return;
    int4 b = make_int4(0, 0, 0, 0);
    if (bx1 >= bx0) {
        const int xa = bx0 & ~3, wp = ((bx1 + 1 - xa) + 3) & ~3, hh = by1 - by0 + 1;
        b = make_int4(xa, by0, wp * hh <= RM_BOX_BYTES ? wp : -1, hh);
    }
    boxes[blockIdx.y * gridDim.x + blockIdx.x] = b;
}

__global__ __launch_bounds__(256) void remap_linear_kernel(RemapParams p, const int4* __restrict__ boxes, int batch,
                                                           int aligned)
{
    __shared__ __attribute__((aligned(16))) uint8_t box[2 * RM_BOX_BYTES];  // double buffered
    const int tid = threadIdx.x;
    const int x0 = blockIdx.x * RM_TW + (tid % (RM_TW / 4)) * 4, y = blockIdx.y * RM_TH + tid / (RM_TW / 4);
    const int f0 = blockIdx.z * RM_FRAMES, nf = min(RM_FRAMES, batch - f0);
    const int4 bb = boxes[blockIdx.y * gridDim.x + blockIdx.x];
    const bool live = x0 < p.dw && y < p.dh;
    const int npx = live ? min(4, p.dw - x0) : 0;
    const long long m = (long long)y * p.dw + x0;
    RemapTap t[4];
    if (npx == 4 && (m & 3) == 0) {
        const float4 u = *reinterpret_cast<const float4*>(p.mapx + m);
        const float4 v = *reinterpret_cast<const float4*>(p.mapy + m);
        t[0] = remap_tap(p.sw, p.sh, u.x, v.x);
        t[1] = remap_tap(p.sw, p.sh, u.y, v.y);
        t[2] = remap_tap(p.sw, p.sh, u.z, v.z);
        t[3] = remap_tap(p.sw, p.sh, u.w, v.w);
    } else {
        for (int k = 0; k < 4; k++)
            t[k] = remap_tap(p.sw, p.sh, k < npx ? p.mapx[m + k] : 0.f, k < npx ? p.mapy[m + k] : 0.f);
    }
    const bool staged = bb.z > 0;
    // Staged tiles run branch-free per pixel: the 4 taps' LDS offsets (clamped into the box) and
    // their weights packed as u16 pairs, with the weight of every out-of-range tap set to 0 —
    // remapBilinear's constant-0 border, since a 0 weight removes that tap's value from the sum.
    int off[4][4];
    uint32_t w01[4], w23[4];
    if (staged) {
        const int last = bb.z * bb.w - 1;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const RemapTap& q = t[k];
#pragma unroll
            for (int d = 0; d < 4; d++) {
                const int sx = q.sx + (d & 1), sy = q.sy + (d >> 1);
                const bool in = q.mode != 2 && sx >= 0 && sx < p.sw && sy >= 0 && sy < p.sh;
                off[k][d] = in ? min(max((sy - bb.y) * bb.z + (sx - bb.x), 0), last) : 0;
            }
            const bool i0 = q.mode != 2 && q.sx >= 0 && q.sx < p.sw && q.sy >= 0 && q.sy < p.sh;
            const bool i1 = q.mode != 2 && q.sx + 1 >= 0 && q.sx + 1 < p.sw && q.sy >= 0 && q.sy < p.sh;
            const bool i2 = q.mode != 2 && q.sx >= 0 && q.sx < p.sw && q.sy + 1 >= 0 && q.sy + 1 < p.sh;
            const bool i3 = q.mode != 2 && q.sx + 1 >= 0 && q.sx + 1 < p.sw && q.sy + 1 >= 0 && q.sy + 1 < p.sh;
            w01[k] = (uint32_t)(i0 ? q.w0 : 0) | (uint32_t)(i1 ? q.w1 : 0) << 16;
            w23[k] = (uint32_t)(i2 ? q.w2 : 0) | (uint32_t)(i3 ? q.w3 : 0) << 16;
        }
    }
    typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
    // box staging, software-pipelined: frame f + 1's dwords are loaded into registers while frame f
    // is computed from the other LDS buffer (one barrier per frame)
    const int wd = staged ? bb.z >> 2 : 1, nd = staged ? wd * bb.w : 0;
    uint32_t stage[RM_BOX_BYTES / 4 / 256];
    auto fetch = [&](int f) {
        const uint8_t* S0 = p.src + f * p.spitch;
#pragma unroll
        for (int j = 0; j < RM_BOX_BYTES / 4 / 256; j++) {
            const int i = tid + 256 * j;
            if (i >= nd) break;
            const int rr = i / wd, c = (i - rr * wd) * 4;
            const uint8_t* s = S0 + (long long)(bb.y + rr) * p.sstride + bb.x + c;
            uint32_t v;
            if (aligned && bb.x + c + 3 < p.sw) {
                v = *reinterpret_cast<const uint32_t*>(s);
            } else {  // row end: bytes inside the frame only
                v = 0;
                for (int k = 0; k < 4; k++)
                    if (bb.x + c + k < p.sw) v |= (uint32_t)s[k] << (8 * k);
            }
            stage[j] = v;
        }
    };
    if (staged) fetch(f0);
    for (int f = f0; f < f0 + nf; f++) {
        const uint8_t* S0 = p.src + f * p.spitch;
        unsigned r = 0;
        if (staged) {
            uint8_t* buf = box + (f & 1) * RM_BOX_BYTES;
#pragma unroll
            for (int j = 0; j < RM_BOX_BYTES / 4 / 256; j++) {
                const int i = tid + 256 * j;
                if (i >= nd) break;
                const int rr = i / wd, c = (i - rr * wd) * 4;
                *reinterpret_cast<uint32_t*>(buf + rr * bb.z + c) = stage[j];
            }
            if (f + 1 < f0 + nf) fetch(f + 1);
            __syncthreads();  // buf complete; the other buffer's readers (frame f - 1) are done
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const uint32_t v01 = (uint32_t)buf[off[k][0]] | (uint32_t)buf[off[k][1]] << 16;
                const uint32_t v23 = (uint32_t)buf[off[k][2]] | (uint32_t)buf[off[k][3]] << 16;
                const uint32_t s = __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, v23), __builtin_bit_cast(u16x2, w23[k]),
                                                          __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, v01),
                                                                                 __builtin_bit_cast(u16x2, w01[k]),
                                                                                 1u << 14, false),
                                                          false);
                r |= (s >> 15) << (8 * k);  // weights sum to <= 2^15: the result is <= 255
            }
        } else {
            for (int k = 0; k < npx; k++) r |= remap_apply(t[k], S0, p.sw, p.sh, p.sstride) << (8 * k);
        }
        if (!live) continue;
        uint8_t* D = p.dst + f * p.dpitch + (long long)y * p.dstride + x0;
        if (npx == 4 && (reinterpret_cast<uintptr_t>(D) & 3) == 0) {
            *reinterpret_cast<unsigned*>(D) = r;
        } else {
            for (int k = 0; k < npx; k++) D[k] = (uint8_t)(r >> (8 * k));
        }
    }
}

mage_status remap_launch(const mage_undistorter* u, const uint8_t* d_src, int src_stride, long long src_pitch,
                         uint8_t* d_dst, int dst_stride, long long dst_pitch, uint32_t batch, hipStream_t st)
{
    if (batch == 0) return MAGE_OK;
    RemapParams p{};
    p.src = d_src;
    p.sw = u->width;
    p.sh = u->height;
    p.sstride = src_stride;
    p.spitch = src_pitch;
    p.mapx = u->maps.as<const float>();
    p.mapy = u->maps.as<const float>() + (size_t)u->width * u->height;
    p.dst = d_dst;
    p.dw = u->width;
    p.dh = u->height;
    p.dstride = dst_stride;
    p.dpitch = dst_pitch;
    // dword staging loads need 4-byte aligned rows in every frame
    const int aligned = ((reinterpret_cast<uintptr_t>(d_src) | (uintptr_t)src_stride | (uintptr_t)src_pitch) & 3) == 0;
    launch("image.remap", remap_linear_kernel,
           dim3((u->width + RM_TW - 1) / RM_TW, (u->height + RM_TH - 1) / RM_TH, (batch + RM_FRAMES - 1) / RM_FRAMES),
           dim3(256), 0, st, p, (const int4*)u->boxes.as<int4>(), (int)batch, aligned);
    MAGE_HIP(hipGetLastError());
    return MAGE_OK;
}

// Benchmark / test input (BASELINE.json C4): a textured plane Z = plane_z seen by a moving pinhole
// camera.  Pixel (x, y) casts the ray R^T K^-1 (x, y, 1) from the camera centre C; the hit (X, Y)
// picks texel (floor(X s) + off, floor(Y s) + off) of the same seeded texture as the panning
// sequence.  fp64 in a fixed operation order (no contraction): synth.scene_frames reproduces it
// byte for byte.
struct SceneParams {
    int w, h;
    long long pitch;
    double fx, fy, cx, cy, plane_z, scale;
    long long off;
    unsigned long long seed;
    const double* cams;  // per frame: R row-major (9), C (3)
};

__global__ __launch_bounds__(256) void synth_scene_kernel(uint8_t* __restrict__ out, SceneParams p)
{
    const int x = blockIdx.x * 256 + threadIdx.x, y = blockIdx.y, f = blockIdx.z;
    if (x >= p.w) return;
    const double* c = p.cams + 12 * f;
    const double dx = ((double)x - p.cx) / p.fx, dy = ((double)y - p.cy) / p.fy;
    const double dwx = (c[0] * dx + c[3] * dy) + c[6];
    const double dwy = (c[1] * dx + c[4] * dy) + c[7];
    const double dwz = (c[2] * dx + c[5] * dy) + c[8];
    const double lam = (p.plane_z - c[11]) / dwz;
    const double X = c[9] + lam * dwx, Y = c[10] + lam * dwy;
    const unsigned long long u = (unsigned long long)((long long)floor(X * p.scale) + p.off);
    const unsigned long long v = (unsigned long long)((long long)floor(Y * p.scale) + p.off);
    auto mix = [](unsigned long long z) {
        z += 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        return z ^ (z >> 31);
    };
    const unsigned long long K1 = 0x9E3779B97F4A7C15ull, K2 = 0xC2B2AE3D27D4EB4Full;
    const unsigned long long base = mix(p.seed ^ ((u >> 3) * K1) ^ ((v >> 3) * K2));
    const unsigned long long fine = mix(p.seed ^ 0xA5A5A5A5ull ^ ((u / 3) * K1) ^ ((v / 3) * K2));
    const int g = (int)(base >> 56) + (int)((fine >> 56) % 49ull) - 24;
    out[f * p.pitch + (long long)y * p.w + x] = (uint8_t)(g < 0 ? 0 : (g > 255 ? 255 : g));
}

// ---- ScaleImageForCameraConfiguration geometry (ImagePreprocessor.cpp:18-65) ----------------
// cv::Matx44f arithmetic as OpenCV 3.4.0 evaluates it in float: products element by element with
// the sum started at 0 and taken left to right (Matx_MatMulOp), inverse() by LU with partial
// pivoting (Matx_FastInvOp -> hal::LU32f, eps = 10 FLT_EPSILON; zeros if singular), the 3x3
// inverse by the adjugate over a float determinant (Matx_FastInvOp<_Tp, 3>).
void matx_mul(const float* a, const float* b, float* out, int m, int l, int n)
{
    for (int i = 0; i < m; i++)
        for (int j = 0; j < n; j++) {
            float s = 0.f;
            for (int k = 0; k < l; k++) s += a[i * l + k] * b[k * n + j];
            out[i * n + j] = s;
        }
}

void matx44_inv_lu(const float* a, float* b)
{
    float A[16];
    for (int i = 0; i < 16; i++) A[i] = a[i], b[i] = (i % 5 == 0) ? 1.f : 0.f;
    const int m = 4;
    for (int i = 0; i < m; i++) {
        int k = i;
        for (int j = i + 1; j < m; j++)
            if (std::fabs(A[j * m + i]) > std::fabs(A[k * m + i])) k = j;
        if (std::fabs(A[k * m + i]) < FLT_EPSILON * 10) {
            for (int t = 0; t < 16; t++) b[t] = 0.f;
            return;
        }
        if (k != i) {
            for (int j = i; j < m; j++) std::swap(A[i * m + j], A[k * m + j]);
            for (int j = 0; j < m; j++) std::swap(b[i * m + j], b[k * m + j]);
        }
        const float d = -1.f / A[i * m + i];
        for (int j = i + 1; j < m; j++) {
            const float alpha = A[j * m + i] * d;
            for (int t = i + 1; t < m; t++) A[j * m + t] += alpha * A[i * m + t];
            for (int t = 0; t < m; t++) b[j * m + t] += alpha * b[i * m + t];
        }
    }
    for (int i = m - 1; i >= 0; i--)
        for (int j = 0; j < m; j++) {
            float s = b[i * m + j];
            for (int t = i + 1; t < m; t++) s -= A[i * m + t] * b[t * m + j];
            b[i * m + j] = s / A[i * m + i];
        }
}

void matx33_inv(const float* a, float* b)
{
#define A_(i, j) a[(i) * 3 + (j)]
    float d = (float)(double)(A_(0, 0) * (A_(1, 1) * A_(2, 2) - A_(2, 1) * A_(1, 2)) -
                              A_(0, 1) * (A_(1, 0) * A_(2, 2) - A_(2, 0) * A_(1, 2)) +
                              A_(0, 2) * (A_(1, 0) * A_(2, 1) - A_(2, 0) * A_(1, 1)));
    if (d == 0) {
        for (int t = 0; t < 9; t++) b[t] = 0.f;
        return;
    }
    d = 1 / d;
    b[0] = (A_(1, 1) * A_(2, 2) - A_(1, 2) * A_(2, 1)) * d;
    b[1] = (A_(0, 2) * A_(2, 1) - A_(0, 1) * A_(2, 2)) * d;
    b[2] = (A_(0, 1) * A_(1, 2) - A_(0, 2) * A_(1, 1)) * d;
    b[3] = (A_(1, 2) * A_(2, 0) - A_(1, 0) * A_(2, 2)) * d;
    b[4] = (A_(0, 0) * A_(2, 2) - A_(0, 2) * A_(2, 0)) * d;
    b[5] = (A_(0, 2) * A_(1, 0) - A_(0, 0) * A_(1, 2)) * d;
    b[6] = (A_(1, 0) * A_(2, 1) - A_(1, 1) * A_(2, 0)) * d;
    b[7] = (A_(0, 1) * A_(2, 0) - A_(0, 0) * A_(2, 1)) * d;
    b[8] = (A_(0, 0) * A_(1, 1) - A_(0, 1) * A_(1, 0)) * d;
#undef A_
}

// Utils/cv.h:226-262 Invert: the rigid inverse (transposed rotation) x (negated translation)
void rigid_invert(const float* T, float* out)
{
    const float R[16] = {T[0], T[4], T[8], 0, T[1], T[5], T[9], 0, T[2], T[6], T[10], 0, 0, 0, 0, 1};
    const float Tr[16] = {1, 0, 0, -T[3], 0, 1, 0, -T[7], 0, 0, 1, -T[11], 0, 0, 0, 1};
    matx_mul(R, Tr, out, 4, 4, 4);
}

void camera_matrix(const mage_camera_config& c, float K[9])
{
    const float k[9] = {c.fx, 0, c.cx, 0, c.fy, c.cy, 0, 0, 1};
    for (int i = 0; i < 9; i++) K[i] = k[i];
}

}  // namespace

// ScaleImageForCameraConfiguration's geometry (ImagePreprocessor.cpp:32-57 with
// CalculateOverlapCropSourceInTarget, MageUtil.cpp:13-58, UnProject / ProjectUndistorted,
// Utils/cv.h:270-278 and Reprojection.cpp:26-42, IsEntirelyOffscreen, Utils/cv.h:405-418).
mage_status scale_geometry(const mage_camera_config& src, const mage_camera_config& tgt, float depth, int crop[4],
                           float* scale, mage_camera_config* prepared, int* ok)
{
    MAGE_REQUIRE(src.width > 0 && src.height > 0 && tgt.width > 0 && tgt.height > 0, MAGE_EINVAL,
                 "camera configurations need a nonzero size");
    float tinv[16], t2s[16];
    matx44_inv_lu(tgt.extrinsics, tinv);
    matx_mul(src.extrinsics, tinv, t2s, 4, 4, 4);  // targetToSource
    float Ks[9], Ksi[9], Kt[9], view_inv[16];
    camera_matrix(src, Ks);
    matx33_inv(Ks, Ksi);
    camera_matrix(tgt, Kt);
    rigid_invert(t2s, view_inv);
    const float maxc = (float)src.width - 1, maxr = (float)(src.height - 1);
    const float corners[4][2] = {{0, 0}, {maxc, 0}, {0, maxr}, {maxc, maxr}};
    float mnx = std::numeric_limits<float>::max(), mny = std::numeric_limits<float>::max();
    float mxx = std::numeric_limits<float>::min(), mxy = std::numeric_limits<float>::min();
    for (auto& pt : corners) {
        const float pix[3] = {(float)(int)pt[0], (float)(int)pt[1], 1.f};
        float cs[3];
        matx_mul(Ksi, pix, cs, 3, 3, 1);
        for (float& v : cs) v *= depth;
        const float c4[4] = {cs[0], cs[1], cs[2], 1};
        float w[4];
        matx_mul(view_inv, c4, w, 4, 4, 1);
        // ProjectUndistorted with the identity 3x4 view matrix
        const float eye[12] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0};
        const float w4[4] = {w[0], w[1], w[2], 1};
        float cam[3];
        matx_mul(eye, w4, cam, 3, 4, 1);
        const float div = cam[2] != 0 ? cam[2] : 1;
        const float px = (cam[0] / div) * Kt[0] + Kt[2], py = (cam[1] / div) * Kt[4] + Kt[5];
        mnx = std::min(mnx, px);
        mny = std::min(mny, py);
        mxx = std::max(mxx, px);
        mxy = std::max(mxy, py);
    }
    const float width = mxx - mnx + 1, height = mxy - mny + 1;
    MAGE_REQUIRE(width >= 0 && height >= 0, MAGE_EINVAL, "overlap crop with a negative extent (camera behind)");
    // mage::Rect {int, int, size_t, size_t} -> cv::Rect (ToCVRect, Utils/cv.h:429-432)
    crop[0] = (int)mnx;
    crop[1] = (int)mny;
    crop[2] = (int)(size_t)width;
    crop[3] = (int)(size_t)height;
    const int maxh = crop[2] + crop[0] - 1, maxv = crop[3] + crop[1] - 1;
    const bool offx = maxh < 0 || crop[0] > (int)(tgt.width - 1);
    const bool offy = maxv < 0 || crop[1] > (int)(tgt.height - 1);
    *prepared = src;
    if (offx || offy) {
        *ok = 0;
        *scale = 0.f;
        return MAGE_OK;
    }
    *ok = 1;
    const float s = std::max(crop[2] / (float)src.width, crop[3] / (float)src.height);
    *scale = s;
    if (s != 1.0f) {
        // cv::Size{(int)(Width * scale), ...}; GetScaledIntrinsics for the calibration
        prepared->width = (uint32_t)(int)((float)src.width * s);
        prepared->height = (uint32_t)(int)((float)src.height * s);
        prepared->cx = src.cx * s;
        prepared->cy = src.cy * s;
        prepared->fx = src.fx * s;
        prepared->fy = src.fy * s;
    }
    return MAGE_OK;
}

namespace {
}  // namespace
}  // namespace mage

extern "C" {

mage_status mage_scale_for_camera_configuration(const mage_camera_config* source, const mage_camera_config* target,
                                                float max_depth_meters, int32_t crop_xywh[4], float* scale,
                                                mage_camera_config* prepared, int32_t* ok)
{
    MAGE_REQUIRE(source && target && crop_xywh && scale && prepared && ok, MAGE_EINVAL, "null argument");
    int crop[4], k = 0;
    mage_status r = mage::scale_geometry(*source, *target, max_depth_meters, crop, scale, prepared, &k);
    for (int i = 0; i < 4; i++) crop_xywh[i] = crop[i];
    *ok = k;
    return r;
}

mage_status mage_scale_image_for_camera_configuration_device(const mage_camera_config* source,
                                                             const mage_camera_config* target, float max_depth_meters,
                                                             const uint8_t* d_src, int32_t src_stride, uint8_t* d_dst,
                                                             int32_t dst_stride, int64_t dst_capacity,
                                                             mage_camera_config* prepared, float* scale, int32_t* ok,
                                                             mage_stream stream)
{
    MAGE_REQUIRE(source && target && prepared && scale && ok && d_src && d_dst, MAGE_EINVAL, "null argument");
    int crop[4], k = 0;
    mage_status r = mage::scale_geometry(*source, *target, max_depth_meters, crop, scale, prepared, &k);
    *ok = k;
    if (r != MAGE_OK || !k) return r;
    const int sw = (int)source->width, sh = (int)source->height, dw = (int)prepared->width, dh = (int)prepared->height;
    MAGE_REQUIRE(src_stride >= sw && dst_stride >= dw && dw > 0 && dh > 0, MAGE_EINVAL, "invalid image strides");
    MAGE_REQUIRE((int64_t)dst_stride * (dh - 1) + dw <= dst_capacity, MAGE_ECAPACITY,
                 "destination too small for the prepared image");
    hipStream_t st = (hipStream_t)stream;
    if (*scale != 1.0f) return mage::resize_linear_device(d_src, sw, sh, src_stride, d_dst, dw, dh, dst_stride, st);
    // preparedImage = rawSourceImage.clone()
    MAGE_HIP(hipMemcpy2DAsync(d_dst, dst_stride, d_src, src_stride, sw, sh, hipMemcpyDeviceToDevice, st));
    return MAGE_OK;
}

mage_status mage_undistorter_create(const mage_calibration* distorted, int32_t width, int32_t height, int device,
                                    mage_undistorter** out, mage_calibration* undistorted)
{
    using namespace mage;
    MAGE_REQUIRE(out && distorted, MAGE_EINVAL, "null argument");
    *out = nullptr;
    MAGE_REQUIRE(width > 0 && height > 0 && width <= 32767 && height <= 32767, MAGE_EINVAL, "bad image size");
    MAGE_REQUIRE(distorted->ndist == 0 || distorted->ndist == 4 || distorted->ndist == 5 || distorted->ndist == 8,
                 MAGE_EINVAL, "distortion: 0, 4, 5 or 8 coefficients");
    mage_status r = bind_device(device);
    if (r != MAGE_OK) return r;
    auto* u = new mage_undistorter();
    u->device = device;
    u->width = width;
    u->height = height;
    // CalculateUndistortedCalibration (ImagePreprocessor.cpp:71-104): fx, fy kept, principal point
    // at the image centre, no distortion
    mage_calibration un{};
    un.fx = distorted->fx;
    un.fy = distorted->fy;
    un.cx = (float)width * 0.5f;
    un.cy = (float)height * 0.5f;
    un.ndist = 0;
    u->undistorted = un;
    if (undistorted) *undistorted = un;
    MapParams p{};
    // iR = (K' * I).inv(DECOMP_LU): cv::invert's 3x3 closed form in double
    const double S[9] = {un.fx, 0, un.cx, 0, un.fy, un.cy, 0, 0, 1};
    auto Sd = [&](int rr, int c) { return S[rr * 3 + c]; };
    double d = Sd(0, 0) * (Sd(1, 1) * Sd(2, 2) - Sd(1, 2) * Sd(2, 1)) - Sd(0, 1) * (Sd(1, 0) * Sd(2, 2) - Sd(1, 2) * Sd(2, 0)) +
               Sd(0, 2) * (Sd(1, 0) * Sd(2, 1) - Sd(1, 1) * Sd(2, 0));
    if (d != 0.) {
        d = 1. / d;
        p.ir[0] = (Sd(1, 1) * Sd(2, 2) - Sd(1, 2) * Sd(2, 1)) * d;
        p.ir[1] = (Sd(0, 2) * Sd(2, 1) - Sd(0, 1) * Sd(2, 2)) * d;
        p.ir[2] = (Sd(0, 1) * Sd(1, 2) - Sd(0, 2) * Sd(1, 1)) * d;
        p.ir[3] = (Sd(1, 2) * Sd(2, 0) - Sd(1, 0) * Sd(2, 2)) * d;
        p.ir[4] = (Sd(0, 0) * Sd(2, 2) - Sd(0, 2) * Sd(2, 0)) * d;
        p.ir[5] = (Sd(0, 2) * Sd(1, 0) - Sd(0, 0) * Sd(1, 2)) * d;
        p.ir[6] = (Sd(1, 0) * Sd(2, 1) - Sd(1, 1) * Sd(2, 0)) * d;
        p.ir[7] = (Sd(0, 1) * Sd(2, 0) - Sd(0, 0) * Sd(2, 1)) * d;
        p.ir[8] = (Sd(0, 0) * Sd(1, 1) - Sd(0, 1) * Sd(1, 0)) * d;
    }
    p.fx = distorted->fx;
    p.fy = distorted->fy;
    p.u0 = distorted->cx;
    p.v0 = distorted->cy;
    const int nd = distorted->ndist;
    const float* k = distorted->dist;
    p.k1 = nd >= 4 ? k[0] : 0.;
    p.k2 = nd >= 4 ? k[1] : 0.;
    p.p1 = nd >= 4 ? k[2] : 0.;
    p.p2 = nd >= 4 ? k[3] : 0.;
    p.k3 = nd >= 5 ? k[4] : 0.;
    p.k4 = nd >= 8 ? k[5] : 0.;
    p.k5 = nd >= 8 ? k[6] : 0.;
    p.k6 = nd >= 8 ? k[7] : 0.;
    p.w = width;
    p.h = height;
    const size_t npx = (size_t)width * height;
    if ((r = u->maps.reserve(8 * npx)) != MAGE_OK) {
        delete u;
        return r;
    }
    p.mapx = u->maps.as<float>();
    p.mapy = u->maps.as<float>() + npx;
    if (hipStreamCreateWithFlags(&u->st, hipStreamNonBlocking) != hipSuccess) {
        u->maps.release();
        delete u;
        set_error("hipStreamCreate failed");
        return MAGE_EDEVICE;
    }
    launch("image.undistort_map", undistort_map_kernel, dim3((height + 63) / 64), dim3(64), 0, u->st, p);
    const dim3 tiles((width + RM_TW - 1) / RM_TW, (height + RM_TH - 1) / RM_TH);
    if (u->boxes.reserve(16ull * tiles.x * tiles.y) == MAGE_OK)
        launch("image.remap_boxes", remap_boxes_kernel, tiles, dim3(256), 0, u->st, (const float*)p.mapx,
               (const float*)p.mapy, width, height, u->boxes.as<int4>());
    if (!u->boxes.ptr || hipGetLastError() != hipSuccess || hipStreamSynchronize(u->st) != hipSuccess) {
        u->maps.release();
        u->boxes.release();
        (void)hipStreamDestroy(u->st);
        delete u;
        set_error("undistortion map kernel failed");
        return MAGE_EDEVICE;
    }
    *out = u;
    return MAGE_OK;
}

mage_status mage_undistorter_destroy(mage_undistorter* u)
{
    if (!u) return MAGE_OK;
    (void)hipSetDevice(u->device);
    u->maps.release();
    u->boxes.release();
    u->scratch.release();
    if (u->st) (void)hipStreamDestroy(u->st);
    delete u;
    return MAGE_OK;
}

mage_status mage_undistorter_get_maps(mage_undistorter* u, float* mapx, float* mapy)
{
    using namespace mage;
    MAGE_REQUIRE(u && mapx && mapy, MAGE_EINVAL, "null argument");
    MAGE_HIP(hipSetDevice(u->device));
    const size_t npx = (size_t)u->width * u->height;
    MAGE_HIP(hipMemcpy(mapx, u->maps.ptr, 4 * npx, hipMemcpyDeviceToHost));
    MAGE_HIP(hipMemcpy(mapy, u->maps.as<float>() + npx, 4 * npx, hipMemcpyDeviceToHost));
    return MAGE_OK;
}

mage_status mage_undistort_image(mage_undistorter* u, const uint8_t* src, int32_t src_stride, uint8_t* dst,
                                 int32_t dst_stride)
{
    using namespace mage;
    MAGE_REQUIRE(u && src && dst, MAGE_EINVAL, "null argument");
    MAGE_REQUIRE(src_stride >= u->width && dst_stride >= u->width, MAGE_EINVAL, "stride smaller than the width");
    MAGE_HIP(hipSetDevice(u->device));
    const size_t n = (size_t)u->width * u->height;
    mage_status r = u->scratch.reserve(2 * n);
    if (r != MAGE_OK) return r;
    uint8_t* ds = u->scratch.as<uint8_t>();
    MAGE_HIP(hipMemcpy2DAsync(ds, u->width, src, src_stride, u->width, u->height, hipMemcpyHostToDevice, u->st));
    if ((r = remap_launch(u, ds, u->width, (long long)n, ds + n, u->width, (long long)n, 1, u->st)) != MAGE_OK) return r;
    MAGE_HIP(hipMemcpy2DAsync(dst, dst_stride, ds + n, u->width, u->width, u->height, hipMemcpyDeviceToHost, u->st));
    MAGE_HIP(hipStreamSynchronize(u->st));
    return MAGE_OK;
}

mage_status mage_undistort_image_batch_device(mage_undistorter* u, const uint8_t* d_src, int32_t src_stride,
                                              int64_t src_pitch, uint8_t* d_dst, int32_t dst_stride, int64_t dst_pitch,
                                              uint32_t batch, mage_stream stream)
{
    using namespace mage;
    MAGE_REQUIRE(u && (batch == 0 || (d_src && d_dst)), MAGE_EINVAL, "null argument");
    MAGE_REQUIRE(src_stride >= u->width && dst_stride >= u->width, MAGE_EINVAL, "stride smaller than the width");
    MAGE_REQUIRE(batch <= 1 || (src_pitch >= (int64_t)src_stride * u->height && dst_pitch >= (int64_t)dst_stride * u->height),
                 MAGE_EINVAL, "frame pitch smaller than one frame");
    return remap_launch(u, d_src, src_stride, src_pitch, d_dst, dst_stride, dst_pitch, batch, (hipStream_t)stream);
}

}  // extern "C"

extern "C" mage_status mage_synth_scene_device(uint8_t* d_out, uint32_t count, int32_t width, int32_t height,
                                              int64_t frame_pitch, const double* d_cams, double fx, double fy,
                                              double cx, double cy, double plane_z, double texel_scale,
                                              int64_t texel_offset, uint64_t seed, mage_stream stream)
{
    using namespace mage;
    MAGE_REQUIRE(d_out && d_cams && width > 0 && height > 0 && frame_pitch >= (int64_t)width * height, MAGE_EINVAL,
                 "bad arguments");
    if (count == 0) return MAGE_OK;
    SceneParams p{width, height, (long long)frame_pitch, fx, fy, cx, cy, plane_z, texel_scale,
                  (long long)texel_offset, (unsigned long long)seed, d_cams};
    launch("synth.scene", synth_scene_kernel, dim3((width + 255) / 256, height, count), dim3(256), 0,
           (hipStream_t)stream, d_out, p);
    MAGE_HIP(hipGetLastError());
    return MAGE_OK;
}
