// shs_lightbin_internal.hpp -- launch interface of shs_lightbin.hip (the software library's CPU light
// binning, build_light_bin_culling, on the GPU).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace shs_dev {

// A frustum-visible light: the Jolt bounding sphere of its world AABB and the AABB itself, and its
// local index (lights stay in ascending local order).
struct alignas(16) BinLight {
    float cx, cy, cz, r;
    float mnx, mny, mnz, index_f;   // index_f: the local index as float bits
    float mxx, mxy, mxz, pad;
};

struct LightBinParams {
    int32_t W, H;
    uint32_t ts, bx, by, slices, cap, n_vis;
    float inv_vp[16];               // glm::inverse(view_proj)
    const float2 *ndc_range;        // near / far NDC z: per tile (mode 2), per slice (mode 3), or null (-1, 1)
    int32_t ndc_per_tile;
    const BinLight *lights;         // n_vis frustum-visible lights
    uint32_t *counts;               // bins
    uint32_t *indices;              // bins * cap
};

}  // namespace shs_dev

namespace shs_internal {
hipError_t launch_light_bin(const shs_dev::LightBinParams &p, hipStream_t s);
}  // namespace shs_internal
