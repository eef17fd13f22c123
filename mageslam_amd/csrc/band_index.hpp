// band_index.hpp — the LDS / global band index that replaces KeypointSpatialIndex's R*-tree
// (Image/KeypointSpatialIndex.cpp:46-106): 64-bit keys (octave, orderable f32 y, index) sorted
// ascending, so the box query |y - qy| <= r of one octave is a contiguous run found by two binary
// searches, followed by the exact f32 box test on each run entry.  Shared by RadiusMatch
// (radius.hip) and TrackLocalMap's per-point matching (localmap.hip).
#pragma once

#include <hip/hip_runtime.h>

namespace mage {

__device__ __forceinline__ unsigned orderable(float v)
{
    const unsigned u = __float_as_uint(v);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

__device__ __forceinline__ unsigned long long band_key(int octave, float y, unsigned idx)
{
    return ((unsigned long long)(octave & 0xFF) << 56) | ((unsigned long long)orderable(y) << 24) | idx;
}

// first position in keys[0, n) (ascending) with keys[pos] >= k
__device__ __forceinline__ int lower_bound_keys(const unsigned long long* keys, int n, unsigned long long k)
{
    int lo = 0, hi = n;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (keys[mid] < k) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

}  // namespace mage
