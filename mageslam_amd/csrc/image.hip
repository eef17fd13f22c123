// image.hip — frame undistortion on MI355X (gfx950): ImagePreprocessor::UndistortImage
// (Core/MAGESLAM/Source/Image/ImagePreprocessor.cpp:71-120).
//
// The reference caches cv::initUndistortRectifyMap(K, dist, noArray(), K', size, CV_32FC1) once per
// calibration and runs cv::remap(INTER_LINEAR, BORDER_CONSTANT 0) on every distorted frame.  Same
// split here:
//   undistort_map_kernel  once per calibration: thread per row, the row-sequential accumulation
//                         _x += ir[0] ... of OpenCV 3.4.0 in fp64 (built with -ffp-contract=off:
//                         bit-exact maps), written as the two CV_32FC1 planes
//   remap_linear_kernel   per batch of frames: thread per 4 output pixels (one dword store), the
//                         maps read as float4 (coalesced, 32 B per thread), X = rint(u * 32): the
//                         short integer part and the 5+5-bit fraction index of remap's fixed-point
//                         path, initInterTab2D's bilinear weights (x 32768, the saturated (0,0) entry
//                         included), (sum + 2^14) >> 15; constant-0 border as remapBilinear treats
//                         outliers.  HBM-bound: 8 B of map + 1 B out per pixel, the source taps hit
//                         L2 (the map is shared by every frame of the batch).
#include <hip/hip_runtime.h>

#include <cmath>

#include "common.hpp"

struct mage_undistorter {
    int device = 0;
    int width = 0, height = 0;
    mage_calibration undistorted{};
    mage::DeviceBuffer maps;     // [mapx (W*H floats)][mapy (W*H floats)]
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

__device__ __forceinline__ unsigned remap_px(const uint8_t* __restrict__ S0, int sw, int sh, int sstride, float fu,
                                             float fv)
{
    const int X = __float2int_rn(fu * 32.0f), Y = __float2int_rn(fv * 32.0f);
    const int sx = min(max(X >> 5, -32768), 32767), sy = min(max(Y >> 5, -32768), 32767);
    const int tx = X & 31, ty = Y & 31;
    int w0 = (32 - ty) * (32 - tx) * 32, w1 = (32 - ty) * tx * 32, w2 = ty * (32 - tx) * 32, w3 = ty * tx * 32;
    if ((tx | ty) == 0) {  // initInterTab2D: saturate_cast<short>(32768.f) = 32767, fix-up +1 on entry 3
        w0 = 32767;
        w3 = 1;
    }
    int v0, v1, v2, v3;
    if ((unsigned)sx < (unsigned)max(sw - 1, 0) && (unsigned)sy < (unsigned)max(sh - 1, 0)) {
        const uint8_t* S = S0 + (long long)sy * sstride + sx;
        v0 = S[0];
        v1 = S[1];
        v2 = S[sstride];
        v3 = S[sstride + 1];
    } else if (sx >= sw || sx + 1 < 0 || sy >= sh || sy + 1 < 0) {
        return 0;
    } else {
        const bool x0 = sx >= 0 && sx < sw, x1 = sx + 1 >= 0 && sx + 1 < sw;
        const bool y0 = sy >= 0 && sy < sh, y1 = sy + 1 >= 0 && sy + 1 < sh;
        v0 = x0 && y0 ? S0[(long long)sy * sstride + sx] : 0;
        v1 = x1 && y0 ? S0[(long long)sy * sstride + sx + 1] : 0;
        v2 = x0 && y1 ? S0[(long long)(sy + 1) * sstride + sx] : 0;
        v3 = x1 && y1 ? S0[(long long)(sy + 1) * sstride + sx + 1] : 0;
    }
    const int r = (v0 * w0 + v1 * w1 + v2 * w2 + v3 * w3 + (1 << 14)) >> 15;
    return (unsigned)min(max(r, 0), 255);
}

__global__ __launch_bounds__(256) void remap_linear_kernel(RemapParams p)
{
    const int qx = blockIdx.x * 256 + threadIdx.x;  // group of 4 output pixels
    const int y = blockIdx.y, f = blockIdx.z;
    const int x0 = qx * 4;
    if (x0 >= p.dw) return;
    const uint8_t* S0 = p.src + f * p.spitch;
    uint8_t* D = p.dst + f * p.dpitch + (long long)y * p.dstride;
    const long long m = (long long)y * p.dw + x0;
    if (x0 + 4 <= p.dw && (m & 3) == 0) {
        const float4 u = *reinterpret_cast<const float4*>(p.mapx + m);
        const float4 v = *reinterpret_cast<const float4*>(p.mapy + m);
        const unsigned r = remap_px(S0, p.sw, p.sh, p.sstride, u.x, v.x) |
                           remap_px(S0, p.sw, p.sh, p.sstride, u.y, v.y) << 8 |
                           remap_px(S0, p.sw, p.sh, p.sstride, u.z, v.z) << 16 |
                           remap_px(S0, p.sw, p.sh, p.sstride, u.w, v.w) << 24;
        if ((reinterpret_cast<uintptr_t>(D + x0) & 3) == 0) {
            *reinterpret_cast<unsigned*>(D + x0) = r;
            return;
        }
        for (int k = 0; k < 4; k++) D[x0 + k] = (uint8_t)(r >> (8 * k));
        return;
    }
    for (int k = 0; k < 4 && x0 + k < p.dw; k++)
        D[x0 + k] = (uint8_t)remap_px(S0, p.sw, p.sh, p.sstride, p.mapx[m + k], p.mapy[m + k]);
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
    const int quads = (u->width + 3) / 4;
    launch("image.remap", remap_linear_kernel, dim3((quads + 255) / 256, u->height, batch), dim3(256), 0, st, p);
    MAGE_HIP(hipGetLastError());
    return MAGE_OK;
}

}  // namespace
}  // namespace mage

extern "C" {

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
    if (hipGetLastError() != hipSuccess || hipStreamSynchronize(u->st) != hipSuccess) {
        u->maps.release();
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
