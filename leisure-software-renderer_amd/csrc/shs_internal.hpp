// shs_internal.hpp -- kernel launch wrappers shared between shs_legacy.hip and shs_abi.cpp.
#pragma once
#include <hip/hip_runtime.h>

#include "shs_device.hpp"

namespace shs_internal {
hipError_t launch_setup(const shs_dev::FrameParams &fp, const shs_dev::FrameBuffers &fb, hipStream_t s);
hipError_t launch_scan(const shs_dev::FrameParams &fp, const shs_dev::FrameBuffers &fb, int n_tiles, hipStream_t s);
hipError_t launch_scatter(const shs_dev::FrameParams &fp, const shs_dev::FrameBuffers &fb, hipStream_t s);
hipError_t launch_raster(const shs_dev::FrameParams &fp, const shs_dev::FrameBuffers &fb, int n_owned_tiles,
                         hipStream_t s);
}  // namespace shs_internal
