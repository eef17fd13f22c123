// depth_noise.hpp — the seeded depth error of new map points (mage_track_settings::
// map_point_depth_noise), shared by the host loop (track.cpp) and the device loop (track.hip);
// tracking.py depth_noise_factor is the same arithmetic in numpy.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace mage {

// 1 + sigma g for keypoint i of the keyframe made at frame fid: g = (a + b + c + d - 131070) / sd,
// a..d the 16-bit fields of splitmix64(seed ^ fid K1 ^ i K2), sd = 65536 sqrt(1/3) (a sum of four
// uniform 16-bit draws: unit variance, nearly normal).  Double arithmetic in this order.
__host__ __device__ inline double depth_noise_factor(uint64_t fid, uint64_t i, float sigma)
{
    uint64_t z = 0xDE9785EEDull ^ (fid * 0x9E3779B97F4A7C15ull) ^ (i * 0xC2B2AE3D27D4EB4Full);
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    const uint64_t q = (z & 0xFFFFu) + ((z >> 16) & 0xFFFFu) + ((z >> 32) & 0xFFFFu) + (z >> 48);
    const double inv_sd = 2.642899791822628e-05;   // 1 / (65536 sqrt(1/3)), tracking.py _DEPTH_INV_SD
    const double g = ((double)q - 131070.0) * inv_sd;
    return 1.0 + (double)sigma * g;
}

}  // namespace mage
