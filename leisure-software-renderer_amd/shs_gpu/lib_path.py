"""Library-path host mirror: MeshData, the per-item ShaderUniforms of PassPBRForward, PassShadowMap casters.

Reference (shs-renderer-lib/include/shs/): `rasterize_mesh` (sw_render/rasterizer.hpp:181-442) called by
`PassPBRForward::execute` (passes/pass_pbr_forward.hpp:49-214) once per RenderItem, after
`PassShadowMap::execute` (passes/pass_shadow_map.hpp:44-206).  The std::function ShaderProgram becomes a
program id + the POD uniform block (`LibDraw`); everything runs through libshs_gpu's C ABI.
"""
import ctypes
from dataclasses import dataclass, field
from typing import Optional

import numpy as np

from . import _abi
from ._abi import (CULL_BACK, CULL_FRONT, CULL_NONE, LIB_BG_GRADIENT, LIB_DEPTH_MOTION, LIGHT_CULL_CLUSTERED,
                   LIGHT_CULL_NONE, LIGHT_CULL_TILED, LIGHT_CULL_TILED_DEPTH, PROGRAM_BLINN_PHONG, PROGRAM_DEBUG_ALBEDO,
                   PROGRAM_DEBUG_DEPTH, PROGRAM_DEBUG_NORMAL, PROGRAM_FORWARD_PLUS, PROGRAM_PBR_MR)

__all__ = [
    "LibMesh", "LibDraw", "Texture2D", "LibFrame", "ShadowCaster", "PROGRAM_PBR_MR", "PROGRAM_BLINN_PHONG", "PROGRAM_DEBUG_ALBEDO",
    "PROGRAM_DEBUG_NORMAL", "PROGRAM_DEBUG_DEPTH", "CULL_NONE", "CULL_BACK", "CULL_FRONT", "IDENTITY",
    "look_at_lh", "perspective_lh_no", "model_euler", "mat_mul", "dir_light_camera_aabb",
]

IDENTITY = np.eye(4, dtype=np.float32).reshape(16)


@dataclass(eq=False)
class LibMesh:
    """MeshData (resources/mesh.hpp:23-43).  indices None = non-indexed soup."""
    positions: np.ndarray                      # float32 [n, 3]
    normals: Optional[np.ndarray] = None       # float32 [k, 3], k <= n (missing -> (0,1,0))
    uvs: Optional[np.ndarray] = None           # float32 [k, 2]
    indices: Optional[np.ndarray] = None       # uint32 [3m]

    @property
    def n_tris(self):
        return int(self.indices.size // 3) if self.indices is not None else int(self.positions.shape[0] // 3)


@dataclass(eq=False)
class Texture2D:
    """Texture2DData (resources/texture.hpp:23-49): Color texels, rgba uint8 [h, w, 4], texel (x, y) at
    rgba[y, x].  Uploaded once per context (Context.upload_texture)."""
    rgba: np.ndarray


@dataclass
class LibDraw:
    """One rasterize_mesh call: ShaderUniforms (shader/types.hpp:87-116) + RasterizerConfig cull state."""
    mesh: object
    program: int = PROGRAM_PBR_MR
    model: np.ndarray = field(default_factory=lambda: IDENTITY.copy())
    viewproj: np.ndarray = field(default_factory=lambda: IDENTITY.copy())
    prev_model: Optional[np.ndarray] = None        # None -> model (no history)
    prev_viewproj: Optional[np.ndarray] = None     # None -> viewproj
    light_dir_ws: tuple = (-0.4, -1.0, -0.2)
    light_color: tuple = (1.0, 1.0, 1.0)
    light_intensity: float = 1.0
    camera_pos: tuple = (0.0, 0.0, 0.0)
    base_color: tuple = (1.0, 1.0, 1.0)
    metallic: float = 0.0
    roughness: float = 0.6
    ao: float = 1.0
    cull_mode: int = CULL_BACK
    front_face_ccw: bool = True
    shadow: bool = False
    light_viewproj: np.ndarray = field(default_factory=lambda: IDENTITY.copy())
    shadow_bias_const: float = 0.0008
    shadow_bias_slope: float = 0.0015
    shadow_pcf_radius: int = 2
    shadow_pcf_step: float = 1.0
    shadow_strength: float = 1.0
    enable_motion_vectors: bool = False
    base_color_tex: Optional[Texture2D] = None     # u.base_color_tex (None: albedo_tex = vec3(1))


@dataclass
class LibFrame:
    """RasterizerTarget: RT_ColorHDR (+ RT_ColorDepthMotion when depth_motion)."""
    width: int
    height: int
    depth_motion: bool = True
    zn: float = 0.1
    zf: float = 200.0
    bg_gradient: bool = True
    clear_hdr: tuple = (0.0, 0.0, 0.0, 1.0)
    shard_rank: int = 0
    shard_count: int = 1

    def desc(self):
        d = _abi.LibFrameC()
        d.width, d.height = self.width, self.height
        d.shard_rank, d.shard_count = self.shard_rank, self.shard_count
        d.flags = (LIB_DEPTH_MOTION if self.depth_motion else 0) | (LIB_BG_GRADIENT if self.bg_gradient else 0)
        d.zn, d.zf = self.zn, self.zf
        for i in range(4):
            d.clear_hdr[i] = self.clear_hdr[i]
        return d


@dataclass
class ShadowCaster:
    mesh: object
    model: np.ndarray


# CullingLightGPU (lighting/light_types.hpp:141-166) as a numpy record (160 B, the C-ABI layout)
LIGHT_DTYPE = np.dtype([("position_range", "<f4", 4), ("color_intensity", "<f4", 4), ("direction_spot", "<f4", 4),
                        ("axis_spot_outer", "<f4", 4), ("up_shape_x", "<f4", 4), ("shape_attenuation", "<f4", 4),
                        ("type_shape_flags", "<u4", 4), ("cull_sphere", "<f4", 4), ("cull_aabb_min", "<f4", 4),
                        ("cull_aabb_max", "<f4", 4)])
assert LIGHT_DTYPE.itemsize == 160

LIGHT_FLAGS_DEFAULT = 1 | 2 | 4      # LightFlagsDefault (light_types.hpp:56-63)
ATTEN_LINEAR, ATTEN_SMOOTH, ATTEN_INVERSE_SQUARE = 0, 1, 2


def make_point_lights(pos, rng_range, color, intensity, attenuation_model=ATTEN_SMOOTH, power=1.0, bias=0.05,
                      cutoff=0.0, flags=LIGHT_FLAGS_DEFAULT):
    """make_point_culling_light (light_types.hpp:327-349) over arrays: pos [n,3], range [n], color [n,3],
    intensity [n] -> LIGHT_DTYPE [n] (make_light_common's clamps included, light_runtime.hpp:167-180)."""
    f = np.float32
    pos = np.asarray(pos, f).reshape(-1, 3)
    n = pos.shape[0]
    rng_range = np.maximum(np.asarray(rng_range, f).reshape(n), f(0.001))           # make_light_common
    color = np.maximum(np.asarray(color, f).reshape(n, 3), f(0.0))
    intensity = np.maximum(np.asarray(intensity, f).reshape(n), f(0.0))
    out = np.zeros(n, LIGHT_DTYPE)
    out["position_range"][:, :3] = pos
    out["position_range"][:, 3] = np.maximum(rng_range, f(0.0))
    out["color_intensity"][:, :3] = color
    out["color_intensity"][:, 3] = intensity
    out["direction_spot"] = (0.0, -1.0, 0.0, 1.0)
    out["axis_spot_outer"] = (1.0, 0.0, 0.0, 0.0)
    out["up_shape_x"] = (0.0, 1.0, 0.0, 0.0)
    out["shape_attenuation"] = (0.0, max(power, 0.001), max(bias, 1e-5), max(cutoff, 0.0))
    out["type_shape_flags"] = (1, 0, flags, attenuation_model)     # Point, Sphere
    r = np.maximum(rng_range, f(0.0))                               # point_light_culling_sphere
    out["cull_sphere"][:, :3] = pos
    out["cull_sphere"][:, 3] = r
    out["cull_aabb_min"][:, :3] = pos - r[:, None]                  # aabb_from_sphere
    out["cull_aabb_max"][:, :3] = pos + r[:, None]
    out["cull_aabb_min"][:, 3] = 1.0
    out["cull_aabb_max"][:, 3] = 1.0
    return out


@dataclass
class LightCull:
    """The CameraUBO fields fp_stress_light_cull.comp reads (shs_light_cull_desc)."""
    width: int
    height: int
    view: np.ndarray
    proj: np.ndarray
    zn: float = 0.1
    zf: float = 200.0
    tile_size: int = 16               # frame/frame_params.hpp:83-84
    max_per_tile: int = 128
    mode: int = 1
    z_slices: int = 16
    depth_linear: bool = True
    shard_rank: int = 0
    shard_count: int = 1

    def desc(self):
        d = _abi.LightCullDescC()
        d.width, d.height = self.width, self.height
        d.tile_size, d.max_per_tile, d.mode, d.z_slices = self.tile_size, self.max_per_tile, self.mode, self.z_slices
        for k in range(16):
            d.view[k] = float(self.view[k])
            d.proj[k] = float(self.proj[k])
        d.zn, d.zf = self.zn, self.zf
        d.depth_linear = 1 if self.depth_linear else 0
        d.shard_rank, d.shard_count = self.shard_rank, self.shard_count
        return d

    @property
    def tiles(self):
        ts = self.tile_size
        return (self.width + ts - 1) // ts, (self.height + ts - 1) // ts

    @property
    def n_lists(self):
        tx, ty = self.tiles
        return tx * ty * (self.z_slices if self.mode == 3 else 1)


def fill_draw_struct(a, d: LibDraw, mesh_id: int, tex_id: int = 0):
    a.mesh_id = mesh_id
    a.base_color_tex = int(tex_id)
    a.program = int(d.program)
    a.cull_mode = int(d.cull_mode)
    a.front_face_ccw = 1 if d.front_face_ccw else 0
    pm = d.model if d.prev_model is None else d.prev_model
    pv = d.viewproj if d.prev_viewproj is None else d.prev_viewproj
    for k in range(16):
        a.model[k] = float(d.model[k])
        a.viewproj[k] = float(d.viewproj[k])
        a.prev_model[k] = float(pm[k])
        a.prev_viewproj[k] = float(pv[k])
        a.light_viewproj[k] = float(d.light_viewproj[k])
    for k in range(3):
        a.light_dir_ws[k] = float(d.light_dir_ws[k])
        a.light_color[k] = float(d.light_color[k])
        a.camera_pos[k] = float(d.camera_pos[k])
        a.base_color[k] = float(d.base_color[k])
    a.light_intensity = float(d.light_intensity)
    a.metallic, a.roughness, a.ao = float(d.metallic), float(d.roughness), float(d.ao)
    a.shadow = 1 if d.shadow else 0
    a.shadow_bias_const, a.shadow_bias_slope = float(d.shadow_bias_const), float(d.shadow_bias_slope)
    a.shadow_pcf_radius = int(d.shadow_pcf_radius)
    a.shadow_pcf_step, a.shadow_strength = float(d.shadow_pcf_step), float(d.shadow_strength)
    a.enable_motion_vectors = 1 if d.enable_motion_vectors else 0


# ---- GLM restatements (host, via libshs_gpu) -----------------------------------------------
def _fp(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))


def _v3(v):
    return np.ascontiguousarray(v, dtype=np.float32).reshape(3)


def look_at_lh(eye, center, up=(0.0, 1.0, 0.0)):
    out = np.zeros(16, np.float32)
    e, c, u = _v3(eye), _v3(center), _v3(up)
    assert _abi.lib().shs_look_at_lh(_fp(e), _fp(c), _fp(u), _fp(out)) == 0
    return out


def perspective_lh_no(fovy_radians, aspect, zn, zf):
    out = np.zeros(16, np.float32)
    assert _abi.lib().shs_perspective_lh_no(fovy_radians, aspect, zn, zf, _fp(out)) == 0
    return out


def model_euler(pos, rot_euler=(0.0, 0.0, 0.0), scl=(1.0, 1.0, 1.0)):
    out = np.zeros(16, np.float32)
    p, r, s = _v3(pos), _v3(rot_euler), _v3(scl)
    assert _abi.lib().shs_model_euler(_fp(p), _fp(r), _fp(s), _fp(out)) == 0
    return out


def mat_mul(a, b):
    out = np.zeros(16, np.float32)
    a = np.ascontiguousarray(a, dtype=np.float32)
    b = np.ascontiguousarray(b, dtype=np.float32)
    assert _abi.lib().shs_mat4_mul(_fp(a), _fp(b), _fp(out)) == 0
    return out


def dir_light_camera_aabb(sun_dir, mn, mx, margin=10.0, res=2048):
    v, p, vp = (np.zeros(16, np.float32) for _ in range(3))
    s, a, b = _v3(sun_dir), _v3(mn), _v3(mx)
    assert _abi.lib().shs_dir_light_camera_aabb(_fp(s), _fp(a), _fp(b), margin, res, _fp(v), _fp(p), _fp(vp)) == 0
    return v, p, vp


# ---- the software library's CPU light binning (build_light_bin_culling) ------
@dataclass
class LightBin:
    """LightBinCullingConfig + the call's view_proj / viewport (light_culling_runtime.hpp:29-36, 266-275).
    mode: 0 none, 1 tiled, 2 tiled + per-tile view-depth range, 3 clustered."""
    width: int
    height: int
    view_proj: np.ndarray
    mode: int = 1
    tile_size: int = 16
    z_slices: int = 16
    z_near: float = 0.1
    z_far: float = 1000.0
    max_per_bin: int = 0               # 0: unbounded (n_lights)
    tile_min_view_depth: np.ndarray = None
    tile_max_view_depth: np.ndarray = None

    def desc(self, n_lights, keep):
        d = _abi.LightBinDescC()
        d.width, d.height = self.width, self.height
        d.tile_size, d.mode, d.z_slices = self.tile_size, self.mode, self.z_slices
        d.max_per_bin = self.max_per_bin if self.max_per_bin > 0 else max(int(n_lights), 1)
        for k in range(16):
            d.view_proj[k] = float(self.view_proj[k])
        d.z_near, d.z_far = self.z_near, self.z_far
        if self.tile_min_view_depth is not None:
            mn = np.ascontiguousarray(self.tile_min_view_depth, dtype=np.float32)
            mx = np.ascontiguousarray(self.tile_max_view_depth, dtype=np.float32)
            keep += [mn, mx]
            d.tile_min_view_depth, d.tile_max_view_depth = mn.ctypes.data, mx.ctypes.data
            d.n_depth_tiles = int(mn.size)
        return d


def light_aabbs(lights):
    """World AABBs of point lights as Jolt sphere SceneShapes of radius = range: position -/+ range."""
    pr = np.asarray(lights["position_range"], np.float32)
    pos, r = pr[:, :3], pr[:, 3:4]
    return np.concatenate([pos - r, pos + r], axis=1).astype(np.float32)
