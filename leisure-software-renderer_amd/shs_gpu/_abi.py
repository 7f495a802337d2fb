"""ctypes declarations of include/shs_gpu.h (libshs_gpu.so, built in-tree for gfx950).

The product path: every call goes through the C ABI into the HIP kernels.  There is no CPU
fallback -- if the shared library is missing or fails to load, importing this module raises.
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# SHS_GPU_LIB: another in-tree build of the library (timing experiments with compile-time variants)
LIB_PATH = os.environ.get("SHS_GPU_LIB") or os.path.join(HERE, "libshs_gpu.so")

SHS_OK = 0
SHS_ERR_INVALID = -1
SHS_ERR_HIP = -2
SHS_ERR_NO_DEVICE = -3
SHS_ERR_OVERFLOW = -4

SHADING_FLAT = 0
SHADING_GOURAUD = 1
SHADING_PHONG = 2
SHADING_BLINN_PHONG = 3
SHADING_NAMES = {"flat": 0, "gouraud": 1, "phong": 2, "blinn_phong": 3}

FRAME_PREQUANT = 1
FRAME_PRESENT = 2
OPT_BIN_CAPACITY = 1
OPT_RASTER_MODE = 2
OPT_TIMELINE = 3
OPT_RASTER_LOOP = 4
OPT_SPILL_CAPACITY = 5
OPT_FRAG_CAPACITY = 6
OPT_LIB_PART = 7
OPT_SHARD_CULL = 8
OPT_SHARD_LAYOUT = 9
SHARD_INTERLEAVED = 0
SHARD_REGIONS = 1
OPT_SHARD_ROOT_SHARE = 10
OPT_SHADOW_FOOTPRINT = 11
OPT_LEGACY_PIPELINE = 12


class LegacyDraw(ctypes.Structure):
    _fields_ = [
        ("mesh_id", ctypes.c_int32),
        ("shading", ctypes.c_int32),
        ("mvp", ctypes.c_float * 16),
        ("model", ctypes.c_float * 16),
        ("light_dir", ctypes.c_float * 3),
        ("camera_pos", ctypes.c_float * 3),
        ("color", ctypes.c_uint8 * 4),
    ]


class FrameDesc(ctypes.Structure):
    _fields_ = [
        ("width", ctypes.c_int32),
        ("height", ctypes.c_int32),
        ("ref_tile_w", ctypes.c_int32),
        ("ref_tile_h", ctypes.c_int32),
        ("shard_rank", ctypes.c_int32),
        ("shard_count", ctypes.c_int32),
        ("flags", ctypes.c_uint32),
        ("clear_color", ctypes.c_uint8 * 4),
    ]


class RasterStats(ctypes.Structure):
    _fields_ = [
        ("tri_input", ctypes.c_uint64),
        ("tri_setup", ctypes.c_uint64),
        ("tri_ghost", ctypes.c_uint64),
        ("bin_entries", ctypes.c_uint64),
        ("covered_pixels", ctypes.c_uint64),
        ("tri_ghost_unbounded", ctypes.c_uint64),
        ("spilled", ctypes.c_uint64),
        ("max_tile_bin", ctypes.c_uint64),
        ("ghost_fragments", ctypes.c_uint64),
    ]


# ---- library path (rasterize_mesh / PassShadowMap / PassPBRForward) ----
PROGRAM_PBR_MR = 0
PROGRAM_BLINN_PHONG = 1
PROGRAM_DEBUG_ALBEDO = 2
PROGRAM_DEBUG_NORMAL = 3
PROGRAM_DEBUG_DEPTH = 4
CULL_NONE, CULL_BACK, CULL_FRONT = 0, 1, 2
LIB_DEPTH_MOTION = 1
LIB_BG_GRADIENT = 2

_F16 = ctypes.c_float * 16
_F3 = ctypes.c_float * 3


class LibDrawC(ctypes.Structure):
    _fields_ = [
        ("mesh_id", ctypes.c_int32),
        ("program", ctypes.c_int32),
        ("cull_mode", ctypes.c_int32),
        ("front_face_ccw", ctypes.c_int32),
        ("model", _F16), ("viewproj", _F16), ("prev_model", _F16), ("prev_viewproj", _F16),
        ("light_dir_ws", _F3), ("light_color", _F3), ("light_intensity", ctypes.c_float), ("camera_pos", _F3),
        ("base_color", _F3), ("metallic", ctypes.c_float), ("roughness", ctypes.c_float), ("ao", ctypes.c_float),
        ("shadow", ctypes.c_int32),
        ("light_viewproj", _F16),
        ("shadow_bias_const", ctypes.c_float), ("shadow_bias_slope", ctypes.c_float),
        ("shadow_pcf_radius", ctypes.c_int32),
        ("shadow_pcf_step", ctypes.c_float), ("shadow_strength", ctypes.c_float),
        ("enable_motion_vectors", ctypes.c_int32),
        ("base_color_tex", ctypes.c_int32),
    ]


class LibFrameC(ctypes.Structure):
    _fields_ = [
        ("width", ctypes.c_int32), ("height", ctypes.c_int32),
        ("shard_rank", ctypes.c_int32), ("shard_count", ctypes.c_int32),
        ("flags", ctypes.c_uint32),
        ("zn", ctypes.c_float), ("zf", ctypes.c_float),
        ("clear_hdr", ctypes.c_float * 4),
    ]


class LibStats(ctypes.Structure):
    _fields_ = [
        ("tri_input", ctypes.c_uint64), ("tri_after_clip", ctypes.c_uint64), ("tri_raster", ctypes.c_uint64),
        ("covered_pixels", ctypes.c_uint64), ("max_tile_bin", ctypes.c_uint64), ("spilled", ctypes.c_uint64),
        ("clipped_extra", ctypes.c_uint64),
    ]


class ShadowCasterC(ctypes.Structure):
    _fields_ = [("mesh_id", ctypes.c_int32), ("model", _F16)]


PROGRAM_FORWARD_PLUS = 5
TONEMAP_LDR, TONEMAP_PRESENT = 1, 2


MOTION_BLUR_PRESENT = 1


class MotionBlurDescC(ctypes.Structure):
    _fields_ = [("enable", ctypes.c_int32), ("samples", ctypes.c_int32), ("strength", ctypes.c_float),
                ("max_velocity_px", ctypes.c_float), ("min_velocity_px", ctypes.c_float),
                ("depth_reject", ctypes.c_float), ("dt", ctypes.c_float), ("flags", ctypes.c_uint32)]


class OccluderC(ctypes.Structure):
    _fields_ = [("mesh_id", ctypes.c_int32), ("model", _F16), ("aabb_min", _F3), ("aabb_max", _F3)]


class OcclusionDescC(ctypes.Structure):
    _fields_ = [("width", ctypes.c_int32), ("height", ctypes.c_int32), ("view", _F16), ("view_proj", _F16),
                ("depth_epsilon", ctypes.c_float), ("enable", ctypes.c_int32)]


class DebugDrawDescC(ctypes.Structure):
    _fields_ = [("width", ctypes.c_int32), ("height", ctypes.c_int32), ("view_proj", _F16), ("camera_pos", _F3),
                ("light_dir_ws", _F3)]


class DebugMeshC(ctypes.Structure):
    _fields_ = [("mesh_id", ctypes.c_int32), ("model", _F16), ("base_color", _F3)]


class DebugTriangleC(ctypes.Structure):
    _fields_ = [("p0", ctypes.c_float * 2), ("p1", ctypes.c_float * 2), ("p2", ctypes.c_float * 2), ("z", _F3),
                ("rgba", ctypes.c_uint8 * 4)]


class CanvasMotionBlurDescC(ctypes.Structure):
    _fields_ = [("width", ctypes.c_int32), ("height", ctypes.c_int32), ("curr_view", _F16), ("curr_proj", _F16),
                ("prev_view", _F16), ("prev_proj", _F16), ("samples", ctypes.c_int32), ("strength", ctypes.c_float),
                ("w_obj", ctypes.c_float), ("w_cam", ctypes.c_float), ("soft_knee", ctypes.c_int32),
                ("knee_px", ctypes.c_float), ("max_px", ctypes.c_float)]


class CanvasDofDescC(ctypes.Structure):
    _fields_ = [("width", ctypes.c_int32), ("height", ctypes.c_int32), ("blur_iterations", ctypes.c_int32),
                ("autofocus_radius", ctypes.c_int32), ("focus_x", ctypes.c_int32), ("focus_y", ctypes.c_int32),
                ("range", ctypes.c_float), ("max_blur", ctypes.c_float)]


class TonemapDescC(ctypes.Structure):
    _fields_ = [("exposure", ctypes.c_float), ("gamma", ctypes.c_float), ("flags", ctypes.c_uint32)]
LIGHT_CULL_NONE, LIGHT_CULL_TILED, LIGHT_CULL_TILED_DEPTH, LIGHT_CULL_CLUSTERED = 0, 1, 2, 3
_F4 = ctypes.c_float * 4


class CullingLightC(ctypes.Structure):
    """CullingLightGPU (lighting/light_types.hpp:141-166), 160 B."""
    _fields_ = [("position_range", _F4), ("color_intensity", _F4), ("direction_spot", _F4), ("axis_spot_outer", _F4),
                ("up_shape_x", _F4), ("shape_attenuation", _F4), ("type_shape_flags", ctypes.c_uint32 * 4),
                ("cull_sphere", _F4), ("cull_aabb_min", _F4), ("cull_aabb_max", _F4)]


class LightCullDescC(ctypes.Structure):
    _fields_ = [("width", ctypes.c_int32), ("height", ctypes.c_int32), ("tile_size", ctypes.c_uint32),
                ("max_per_tile", ctypes.c_uint32), ("mode", ctypes.c_uint32), ("z_slices", ctypes.c_uint32),
                ("view", _F16), ("proj", _F16), ("zn", ctypes.c_float), ("zf", ctypes.c_float),
                ("depth_linear", ctypes.c_int32), ("shard_rank", ctypes.c_int32), ("shard_count", ctypes.c_int32)]


class LightBinDescC(ctypes.Structure):
    _fields_ = [("width", ctypes.c_int32), ("height", ctypes.c_int32), ("tile_size", ctypes.c_uint32),
                ("mode", ctypes.c_uint32), ("z_slices", ctypes.c_uint32), ("max_per_bin", ctypes.c_uint32),
                ("view_proj", _F16), ("z_near", ctypes.c_float), ("z_far", ctypes.c_float),
                ("tile_min_view_depth", ctypes.c_void_p), ("tile_max_view_depth", ctypes.c_void_p),
                ("n_depth_tiles", ctypes.c_int32)]


# (name, restype, argtypes) for every symbol include/shs_gpu.h declares.
_P = ctypes.c_void_p
_F = ctypes.POINTER(ctypes.c_float)
SIGNATURES = [
    ("shs_abi_version", ctypes.c_int, []),
    ("shs_gpu_tile_size", ctypes.c_int, []),
    ("shs_create", ctypes.c_int, [ctypes.c_int, ctypes.POINTER(_P)]),
    ("shs_destroy", ctypes.c_int, [_P]),
    ("shs_last_error", ctypes.c_char_p, [_P]),
    ("shs_set_stream", ctypes.c_int, [_P, _P]),
    ("shs_get_stream", _P, [_P]),
    ("shs_synchronize", ctypes.c_int, [_P]),
    ("shs_mesh_upload_soup", ctypes.c_int, [_P, _F, _F, ctypes.c_int32, ctypes.POINTER(ctypes.c_int32)]),
    ("shs_mesh_share", ctypes.c_int, [_P, _P, ctypes.c_int32, ctypes.POINTER(ctypes.c_int32)]),
    ("shs_mesh_release", ctypes.c_int, [_P, ctypes.c_int32]),
    ("shs_render_legacy", ctypes.c_int, [_P, ctypes.POINTER(FrameDesc), ctypes.POINTER(LegacyDraw), ctypes.c_int32]),
    ("shs_render_legacy_batch", ctypes.c_int, [_P, ctypes.POINTER(FrameDesc), ctypes.POINTER(LegacyDraw), ctypes.c_int32,
                                               ctypes.c_int32]),
    ("shs_resolve", ctypes.c_int, [_P, _P, _P]),
    ("shs_resolve_frame", ctypes.c_int, [_P, ctypes.c_int32, _P, _P]),
    ("shs_resolve_present", ctypes.c_int, [_P, ctypes.c_int32, _P, ctypes.c_int32]),
    ("shs_present_device", ctypes.c_int, [_P, ctypes.c_int32, ctypes.POINTER(_P)]),
    ("shs_resolve_prequant", ctypes.c_int, [_P, _P]),
    ("shs_resolve_prequant_frame", ctypes.c_int, [_P, ctypes.c_int32, _P]),
    ("shs_texture_upload", ctypes.c_int, [_P, _P, ctypes.c_int32, ctypes.c_int32, ctypes.POINTER(ctypes.c_int32)]),
    ("shs_texture_release", ctypes.c_int, [_P, ctypes.c_int32]),
    ("shs_device_framebuffers", ctypes.c_int, [_P, ctypes.POINTER(_P), ctypes.POINTER(_P)]),
    ("shs_get_stats", ctypes.c_int, [_P, ctypes.POINTER(RasterStats)]),
    ("shs_enable_timing", ctypes.c_int, [_P, ctypes.c_int]),
    ("shs_last_kernel_ms", ctypes.c_int, [_P, _F]),
    ("shs_timing_reset", ctypes.c_int, [_P]),
    ("shs_timing_read", ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int64)]),
    ("shs_debug_records", ctypes.c_int, [_P, _P, ctypes.c_int64, ctypes.POINTER(ctypes.c_int64)]),
    ("shs_set_option", ctypes.c_int, [_P, ctypes.c_int, ctypes.c_int64]),
    ("shs_debug_timeline", ctypes.c_int, [_P, _P, ctypes.c_int64, ctypes.POINTER(ctypes.c_int64)]),
    ("shs_lib_debug_timeline", ctypes.c_int, [_P, _P, ctypes.c_int64, ctypes.POINTER(ctypes.c_int64)]),
    ("shs_lib_debug_setup_timeline", ctypes.c_int, [_P, _P, ctypes.c_int64, ctypes.POINTER(ctypes.c_int64)]),
    ("shs_tonemap", ctypes.c_int, [_P, ctypes.POINTER(TonemapDescC)]),
    ("shs_lib_fuse_tonemap", ctypes.c_int, [_P, ctypes.POINTER(TonemapDescC)]),
    ("shs_resolve_ldr", ctypes.c_int, [_P, _P, _P]),
    ("shs_ldr_device_targets", ctypes.c_int, [_P, ctypes.POINTER(_P), ctypes.POINTER(_P)]),
    ("shs_tonemap_thresholds", ctypes.c_int, [ctypes.c_float, _F]),
    ("shs_occlusion_pass", ctypes.c_int, [_P, ctypes.POINTER(OcclusionDescC), ctypes.POINTER(OccluderC), ctypes.c_int32,
                                          _P, ctypes.c_int32, _P, _P, ctypes.POINTER(ctypes.c_int32), _P]),
    ("shs_debug_draw_meshes", ctypes.c_int, [_P, ctypes.POINTER(DebugDrawDescC), ctypes.POINTER(DebugMeshC), ctypes.c_int32,
                                             _P, _P, _P]),
    ("shs_debug_fill_triangles", ctypes.c_int, [_P, ctypes.c_int32, ctypes.c_int32, ctypes.POINTER(DebugTriangleC),
                                                ctypes.c_int32, _P, _P]),
    ("shs_canvas_motion_blur", ctypes.c_int, [_P, ctypes.POINTER(CanvasMotionBlurDescC), _P, _P, _P, _P, ctypes.c_uint32]),
    ("shs_canvas_gaussian_blur", ctypes.c_int, [_P, ctypes.c_int32, ctypes.c_int32, _P, _P, ctypes.c_int32, ctypes.c_uint32]),
    ("shs_canvas_dof", ctypes.c_int, [_P, ctypes.POINTER(CanvasDofDescC), _P, _P, _P, _F, ctypes.c_uint32]),
    ("shs_motion_blur", ctypes.c_int, [_P, ctypes.POINTER(MotionBlurDescC)]),
    ("shs_resolve_motion_blur", ctypes.c_int, [_P, _P, _P]),
    ("shs_camera3d", ctypes.c_int, [_F, ctypes.c_float, ctypes.c_float, ctypes.c_float, ctypes.c_float, ctypes.c_float, _F, _F]),
    ("shs_model_trs", ctypes.c_int, [_F, ctypes.c_float, _F, _F]),
    ("shs_mat4_mul", ctypes.c_int, [_F, _F, _F]),
    ("shs_mat4_inverse", ctypes.c_int, [_F, _F]),
    ("shs_mesh_upload", ctypes.c_int, [_P, _F, ctypes.c_int32, _F, ctypes.c_int32, _F, ctypes.c_int32,
                                       ctypes.POINTER(ctypes.c_uint32), ctypes.c_int64, ctypes.POINTER(ctypes.c_int32)]),
    ("shs_render_pbr_forward", ctypes.c_int, [_P, ctypes.POINTER(LibFrameC), ctypes.POINTER(LibDrawC), ctypes.c_int32]),
    ("shs_resolve_lib", ctypes.c_int, [_P, _P, _P, _P]),
    ("shs_get_lib_stats", ctypes.c_int, [_P, ctypes.POINTER(LibStats)]),
    ("shs_lib_device_targets", ctypes.c_int, [_P, ctypes.POINTER(_P), ctypes.POINTER(_P), ctypes.POINTER(_P)]),
    ("shs_lib_timing_reset", ctypes.c_int, [_P]),
    ("shs_lib_timing_read", ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int64)]),
    ("shs_render_shadow_map", ctypes.c_int, [_P, ctypes.c_int32, ctypes.c_int32, _F, ctypes.POINTER(ShadowCasterC),
                                             ctypes.c_int32, _F]),
    ("shs_resolve_shadow_map", ctypes.c_int, [_P, _P]),
    ("shs_get_shadow_region", ctypes.c_int, [_P, _P]),
    ("shs_shadow_footprint", ctypes.c_int, [_P, ctypes.c_int32, ctypes.c_int32, _P, ctypes.c_int32, ctypes.c_int32, _P, _P, _P,
                                            ctypes.c_int32, _P]),
    ("shs_shadow_footprint_rows", ctypes.c_int, [_P, ctypes.c_int32, ctypes.c_int32, _P, ctypes.c_int32, ctypes.c_int32, _P,
                                                 _P, _P, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, _P, _P]),
    ("shs_tiles_packed_words", ctypes.c_int, [_P, ctypes.c_int, ctypes.c_int32, ctypes.POINTER(ctypes.c_int64)]),
    ("shs_tiles_rank_words", ctypes.c_int, [_P, ctypes.c_int, ctypes.c_int32, ctypes.c_int32, ctypes.POINTER(ctypes.c_int64)]),
    ("shs_get_shard_regions", ctypes.c_int, [_P, ctypes.c_int32, ctypes.POINTER(ctypes.c_int32)]),
    ("shs_shard_balance_rects", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                               ctypes.c_int32, ctypes.POINTER(ctypes.c_int32)]),
    ("shs_tiles_pack", ctypes.c_int, [_P, ctypes.c_int, ctypes.c_int32, ctypes.c_int32, _P]),
    ("shs_tiles_unpack", ctypes.c_int, [_P, ctypes.c_int, ctypes.c_int32, ctypes.c_int32, _P]),
    ("shs_tiles_unpack_ranks", ctypes.c_int, [_P, ctypes.c_int, ctypes.c_int32, ctypes.POINTER(ctypes.c_void_p)]),
    ("shs_lights_upload", ctypes.c_int, [_P, ctypes.POINTER(CullingLightC), ctypes.c_int32]),
    ("shs_light_cull", ctypes.c_int, [_P, ctypes.POINTER(LightCullDescC)]),
    ("shs_light_bin_culling", ctypes.c_int, [_P, ctypes.POINTER(LightBinDescC), _P, ctypes.c_int32, _P, _P, _P]),
    ("shs_resolve_light_lists", ctypes.c_int, [_P, _P, _P, _P]),
    ("shs_look_at_lh", ctypes.c_int, [_F, _F, _F, _F]),
    ("shs_perspective_lh_no", ctypes.c_int, [ctypes.c_float, ctypes.c_float, ctypes.c_float, ctypes.c_float, _F]),
    ("shs_model_euler", ctypes.c_int, [_F, _F, _F, _F]),
    ("shs_dir_light_camera_aabb", ctypes.c_int, [_F, _F, _F, ctypes.c_float, ctypes.c_uint32, _F, _F, _F]),
    # multi-GPU from one host process
    ("shs_group_create", ctypes.c_int, [ctypes.POINTER(ctypes.c_int32), ctypes.c_int32, ctypes.POINTER(_P)]),
    ("shs_group_destroy", ctypes.c_int, [_P]),
    ("shs_group_last_error", ctypes.c_char_p, [_P]),
    ("shs_group_size", ctypes.c_int, [_P]),
    ("shs_group_context", ctypes.c_int, [_P, ctypes.c_int32, ctypes.POINTER(_P)]),
    ("shs_group_mesh_upload", ctypes.c_int, [_P, _F, ctypes.c_int32, _F, ctypes.c_int32, _F, ctypes.c_int32,
                                             ctypes.POINTER(ctypes.c_uint32), ctypes.c_int64, ctypes.POINTER(ctypes.c_int32)]),
    ("shs_group_mesh_upload_soup", ctypes.c_int, [_P, _F, _F, ctypes.c_int32, ctypes.POINTER(ctypes.c_int32)]),
    ("shs_group_texture_upload", ctypes.c_int, [_P, _P, ctypes.c_int32, ctypes.c_int32, ctypes.POINTER(ctypes.c_int32)]),
    ("shs_group_lights_upload", ctypes.c_int, [_P, ctypes.POINTER(CullingLightC), ctypes.c_int32]),
    ("shs_group_set_option", ctypes.c_int, [_P, ctypes.c_int, ctypes.c_int64]),
    ("shs_group_lib_fuse_tonemap", ctypes.c_int, [_P, ctypes.POINTER(TonemapDescC)]),
    ("shs_group_light_cull", ctypes.c_int, [_P, ctypes.POINTER(LightCullDescC)]),
    ("shs_group_render_shadow_map", ctypes.c_int, [_P, ctypes.c_int32, ctypes.c_int32, _F, ctypes.POINTER(ShadowCasterC),
                                                   ctypes.c_int32, _F]),
    ("shs_group_render_pbr_forward", ctypes.c_int, [_P, ctypes.POINTER(LibFrameC), ctypes.POINTER(LibDrawC), ctypes.c_int32]),
    ("shs_group_render_legacy", ctypes.c_int, [_P, ctypes.POINTER(FrameDesc), ctypes.POINTER(LegacyDraw), ctypes.c_int32]),
    ("shs_group_gather", ctypes.c_int, [_P, ctypes.c_int]),
    ("shs_group_synchronize", ctypes.c_int, [_P]),
]


def _share_torch_hip_runtime():
    """One HIP runtime per process.  PyTorch-ROCm wheels bundle their own libamdhip64.so /
    libhsa-runtime64.so and load them by file name from torch/lib; libshs_gpu.so asks the dynamic
    linker for the SONAMEs libamdhip64.so.7 / libhsa-runtime64.so.1.  If libshs_gpu.so is loaded first,
    the system ROCm runtime comes up, and a later `import torch` maps a second HIP + HSA runtime into
    the process whose device enumeration then fails ("No HIP GPUs are available" / hipErrorNoDevice:
    tools/diag_runtime.py).  Loading torch's runtime first (by path, RTLD_GLOBAL,
    without importing torch) makes libshs_gpu.so bind to it by SONAME, and torch later finds the same
    file already mapped.  Without torch the system runtime is used.  SHS_GPU_HIP_RUNTIME=system skips."""
    if os.environ.get("SHS_GPU_HIP_RUNTIME", "") == "system":
        return None
    import importlib.util
    try:
        spec = importlib.util.find_spec("torch")
    except (ImportError, ValueError):
        return None
    if spec is None or not spec.submodule_search_locations:
        return None
    for d in spec.submodule_search_locations:
        hip = os.path.join(d, "lib", "libamdhip64.so")
        if os.path.exists(hip):
            return ctypes.CDLL(hip, mode=ctypes.RTLD_GLOBAL)
    return None


def load(path: str = LIB_PATH) -> ctypes.CDLL:
    _share_torch_hip_runtime()
    if not os.path.exists(path):
        raise RuntimeError(
            f"libshs_gpu.so not found at {path}: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "(there is no CPU fallback for the raster path)")
    lib = ctypes.CDLL(path)
    for name, res, args in SIGNATURES:
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


_LIB = None


def lib() -> ctypes.CDLL:
    global _LIB
    if _LIB is None:
        _LIB = load()
    return _LIB
