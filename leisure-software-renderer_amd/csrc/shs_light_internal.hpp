// shs_light_internal.hpp -- launch wrapper of the light-list binning kernels (shs_light.hip).
#pragma once
#include <hip/hip_runtime.h>

#include "shs_lib_device.hpp"

namespace shs_internal {
// k_light_project, (mode 2) k_depth_reduce over `depth`, k_light_cull; proj: 2 float4 per light,
// ranges: one float2 per tile, counts: p.n_lists, indices: p.n_lists * p.max_per_tile.
hipError_t launch_light_cull(const shs_dev::LightCullParams &p, const shs_dev::CullLight *lights, float4 *proj,
                             const float *depth, float2 *ranges, uint32_t *counts, uint32_t *indices, hipStream_t s);
}  // namespace shs_internal
