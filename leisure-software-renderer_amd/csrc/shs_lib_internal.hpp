// shs_lib_internal.hpp -- launch wrappers of the library-path kernels (shs_lib.hip) for shs_abi.cpp.
#pragma once
#include <hip/hip_runtime.h>

#include "shs_lib_device.hpp"

namespace shs_internal {
// shadow = true: PassShadowMap's depth pass; false: rasterize_mesh + builtin programs.
hipError_t launch_lib_setup(const shs_dev::LibFrameParams &fp, const shs_dev::LibBuffers &fb, bool shadow, hipStream_t s);
int lib_raster_resident_blocks(int device, bool shadow);   // CUs x occupancy of k_lib_raster
hipError_t launch_lib_raster(const shs_dev::LibFrameParams &fp, const shs_dev::LibBuffers &fb, bool shadow, int grid,
                             hipStream_t s);
}  // namespace shs_internal
