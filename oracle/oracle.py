"""ctypes wrapper of oracle/_build/libshs_oracle.so -- the CPU restatement of the reference path.

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg.  The product (libshs_gpu.so / shs_gpu) never imports this.  PARITY UNPINNED (see shs_oracle.h).
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "_build", "libshs_oracle.so")


class OraDraw(ctypes.Structure):
    _fields_ = [
        ("shading", ctypes.c_int32),
        ("n_tris", ctypes.c_int32),
        ("positions", ctypes.POINTER(ctypes.c_float)),
        ("normals", ctypes.POINTER(ctypes.c_float)),
        ("mvp", ctypes.c_float * 16),
        ("model", ctypes.c_float * 16),
        ("light_dir", ctypes.c_float * 3),
        ("camera_pos", ctypes.c_float * 3),
        ("color", ctypes.c_uint8 * 4),
    ]


_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = ctypes.CDLL(LIB)
        P = ctypes.c_void_p
        L.ora_render_legacy.restype = ctypes.c_int
        L.ora_render_legacy.argtypes = [ctypes.c_int] * 5 + [ctypes.POINTER(OraDraw), ctypes.c_int, P, P, P]
        L.ora_screen_coords.restype = ctypes.c_int
        L.ora_screen_coords.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.POINTER(OraDraw), P]
        L.ora_barycentric.restype = None
        L.ora_barycentric.argtypes = [P, ctypes.c_float, ctypes.c_float, P]
        L.ora_fnv1a64.restype = ctypes.c_uint64
        L.ora_fnv1a64.argtypes = [P, ctypes.c_uint64]
        L.ora_mat4_inverse.argtypes = [P, P]
        L.ora_mat4_mul.argtypes = [P, P, P]
        F = ctypes.c_float
        L.ora_camera3d.restype = None
        L.ora_camera3d.argtypes = [P, F, F, F, F, F, P, P]
        L.ora_model_trs.restype = None
        L.ora_model_trs.argtypes = [P, F, P, P]
        L.ora_look_at_lh.restype = None
        L.ora_look_at_lh.argtypes = [P, P, P, P]
        L.ora_perspective_lh_no.restype = None
        L.ora_perspective_lh_no.argtypes = [F, F, F, F, P]
        L.ora_legacy_mvp.restype = None
        L.ora_legacy_mvp.argtypes = [P, P, P, ctypes.c_int, P, P]
        _lib = L
    return _lib


def _draw_array(draws):
    """draws: objects with .mesh (.positions/.normals float32 [n,9]), .shading, .mvp, .model,
    .light_dir, .camera_pos, .color.  Returns (ctypes array, keepalive list)."""
    arr = (OraDraw * max(len(draws), 1))()
    keep = []
    for i, d in enumerate(draws):
        pos = np.ascontiguousarray(d.mesh.positions, dtype=np.float32)
        nrm = np.ascontiguousarray(d.mesh.normals, dtype=np.float32)
        keep += [pos, nrm]
        a = arr[i]
        a.shading = int(d.shading)
        a.n_tris = pos.shape[0]
        a.positions = pos.ctypes.data_as(ctypes.POINTER(ctypes.c_float))
        a.normals = nrm.ctypes.data_as(ctypes.POINTER(ctypes.c_float))
        for k in range(16):
            a.mvp[k] = float(d.mvp[k])
            a.model[k] = float(d.model[k])
        for k in range(3):
            a.light_dir[k] = float(d.light_dir[k])
            a.camera_pos[k] = float(d.camera_pos[k])
        for k in range(4):
            a.color[k] = int(d.color[k])
    return arr, keep


def render_legacy(width, height, draws, tile=(80, 80), threads=1, prequant=False):
    """-> (color uint8[H,W,4] canvas rows, depth float32[H,W] screen rows, prequant or None)."""
    arr, keep = _draw_array(draws)
    color = np.empty((height, width, 4), np.uint8)
    depth = np.empty((height, width), np.float32)
    pq = np.empty((height, width, 4), np.float32) if prequant else None
    rc = lib().ora_render_legacy(width, height, tile[0], tile[1], threads, arr, len(draws),
                                 color.ctypes.data, depth.ctypes.data, pq.ctypes.data if pq is not None else None)
    if rc != 0:
        raise RuntimeError(f"ora_render_legacy failed: {rc}")
    return color, depth, pq


def screen_coords(width, height, draw):
    arr, keep = _draw_array([draw])
    out = np.empty((arr[0].n_tris, 9), np.float32)
    lib().ora_screen_coords(width, height, arr, out.ctypes.data)
    return out


def barycentric(tri6, px, py):
    t = np.ascontiguousarray(tri6, dtype=np.float32)
    o = np.empty(3, np.float32)
    lib().ora_barycentric(t.ctypes.data, px, py, o.ctypes.data)
    return o


def fnv1a64(arr):
    a = np.ascontiguousarray(arr)
    return int(lib().ora_fnv1a64(a.ctypes.data, a.nbytes))


# ===== library path (shs_oracle_lib.c) ====================================================
_F16 = ctypes.c_float * 16
_F3 = ctypes.c_float * 3


class OraMesh(ctypes.Structure):
    _fields_ = [
        ("positions", ctypes.POINTER(ctypes.c_float)),
        ("normals", ctypes.POINTER(ctypes.c_float)),
        ("uvs", ctypes.POINTER(ctypes.c_float)),
        ("n_verts", ctypes.c_int32), ("n_normals", ctypes.c_int32), ("n_uvs", ctypes.c_int32),
        ("indices", ctypes.POINTER(ctypes.c_uint32)),
        ("n_indices", ctypes.c_int64),
    ]


class OraLibDraw(ctypes.Structure):
    _fields_ = [
        ("mesh", OraMesh),
        ("program", ctypes.c_int32), ("cull_mode", ctypes.c_int32), ("front_face_ccw", ctypes.c_int32),
        ("shadow", ctypes.c_int32),
        ("model", _F16), ("viewproj", _F16), ("prev_model", _F16), ("prev_viewproj", _F16),
        ("light_dir_ws", _F3), ("light_color", _F3), ("light_intensity", ctypes.c_float), ("camera_pos", _F3),
        ("base_color", _F3), ("metallic", ctypes.c_float), ("roughness", ctypes.c_float), ("ao", ctypes.c_float),
        ("light_viewproj", _F16),
        ("shadow_bias_const", ctypes.c_float), ("shadow_bias_slope", ctypes.c_float),
        ("shadow_pcf_radius", ctypes.c_int32),
        ("shadow_pcf_step", ctypes.c_float), ("shadow_strength", ctypes.c_float),
        ("enable_motion_vectors", ctypes.c_int32),
        ("base_color_tex", ctypes.c_void_p), ("tex_w", ctypes.c_int32), ("tex_h", ctypes.c_int32),
    ]


class OraLibTarget(ctypes.Structure):
    _fields_ = [
        ("W", ctypes.c_int32), ("H", ctypes.c_int32),
        ("zn", ctypes.c_float), ("zf", ctypes.c_float),
        ("bg_gradient", ctypes.c_int32),
        ("clear_hdr", ctypes.c_float * 4),
        ("hdr", ctypes.POINTER(ctypes.c_float)), ("depth", ctypes.POINTER(ctypes.c_float)),
        ("motion", ctypes.POINTER(ctypes.c_float)),
        ("shadow", ctypes.POINTER(ctypes.c_float)),
        ("shadow_w", ctypes.c_int32), ("shadow_h", ctypes.c_int32),
        ("lights", ctypes.c_void_p), ("n_lights", ctypes.c_int32),
        ("tile_counts", ctypes.c_void_p), ("tile_indices", ctypes.c_void_p),
        ("cull", ctypes.c_void_p),
    ]


class OraShadowCaster(ctypes.Structure):
    _fields_ = [("mesh", OraMesh), ("model", _F16)]


def _lib_lib():
    L = lib()
    if not getattr(L, "_lib_path_ready", False):
        P = ctypes.c_void_p
        L.ora_pbr_forward.restype = ctypes.c_int
        L.ora_pbr_forward.argtypes = [ctypes.POINTER(OraLibTarget), ctypes.POINTER(OraLibDraw), ctypes.c_int, P]
        L.ora_shadow_map.restype = ctypes.c_int
        L.ora_shadow_map.argtypes = [ctypes.c_int, ctypes.c_int, P, ctypes.POINTER(OraShadowCaster), ctypes.c_int, P, P]
        L.ora_dir_light_camera_aabb.restype = None
        L.ora_dir_light_camera_aabb.argtypes = [P, P, P, ctypes.c_float, ctypes.c_uint32, P, P, P]
        L.ora_mat4_determinant.restype = ctypes.c_float
        L.ora_mat4_determinant.argtypes = [P]
        L._lib_path_ready = True
    return L


def _fill_mesh(om, mesh, keep):
    pos = np.ascontiguousarray(mesh.positions, dtype=np.float32).reshape(-1, 3)
    keep.append(pos)
    om.positions = pos.ctypes.data_as(ctypes.POINTER(ctypes.c_float))
    om.n_verts = pos.shape[0]
    if mesh.normals is not None:
        n = np.ascontiguousarray(mesh.normals, dtype=np.float32).reshape(-1, 3)
        keep.append(n)
        om.normals = n.ctypes.data_as(ctypes.POINTER(ctypes.c_float))
        om.n_normals = n.shape[0]
    if mesh.uvs is not None:
        u = np.ascontiguousarray(mesh.uvs, dtype=np.float32).reshape(-1, 2)
        keep.append(u)
        om.uvs = u.ctypes.data_as(ctypes.POINTER(ctypes.c_float))
        om.n_uvs = u.shape[0]
    if mesh.indices is not None:
        i = np.ascontiguousarray(mesh.indices, dtype=np.uint32).reshape(-1)
        keep.append(i)
        om.indices = i.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32))
        om.n_indices = i.size


def _lib_draws(draws, keep):
    arr = (OraLibDraw * max(len(draws), 1))()
    for i, d in enumerate(draws):
        a = arr[i]
        _fill_mesh(a.mesh, d.mesh, keep)
        a.program, a.cull_mode, a.front_face_ccw = int(d.program), int(d.cull_mode), 1 if d.front_face_ccw else 0
        a.shadow = 1 if d.shadow else 0
        pm = d.model if d.prev_model is None else d.prev_model
        pv = d.viewproj if d.prev_viewproj is None else d.prev_viewproj
        for k in range(16):
            a.model[k], a.viewproj[k] = float(d.model[k]), float(d.viewproj[k])
            a.prev_model[k], a.prev_viewproj[k] = float(pm[k]), float(pv[k])
            a.light_viewproj[k] = float(d.light_viewproj[k])
        for k in range(3):
            a.light_dir_ws[k], a.light_color[k] = float(d.light_dir_ws[k]), float(d.light_color[k])
            a.camera_pos[k], a.base_color[k] = float(d.camera_pos[k]), float(d.base_color[k])
        a.light_intensity = float(d.light_intensity)
        a.metallic, a.roughness, a.ao = float(d.metallic), float(d.roughness), float(d.ao)
        a.shadow_bias_const, a.shadow_bias_slope = float(d.shadow_bias_const), float(d.shadow_bias_slope)
        a.shadow_pcf_radius = int(d.shadow_pcf_radius)
        a.shadow_pcf_step, a.shadow_strength = float(d.shadow_pcf_step), float(d.shadow_strength)
        a.enable_motion_vectors = 1 if d.enable_motion_vectors else 0
        tex = getattr(d, "base_color_tex", None)
        if tex is not None:   # lib_path.Texture2D: rgba uint8 [h, w, 4]
            t = np.ascontiguousarray(tex.rgba, dtype=np.uint8)
            keep.append(t)
            a.base_color_tex = t.ctypes.data
            a.tex_h, a.tex_w = int(t.shape[0]), int(t.shape[1])
    return arr


def pbr_forward(frame, draws, shadow_map=None):
    """PassPBRForward::execute (one rasterize_mesh per draw) -> (hdr [H,W,4], depth [H,W] | None,
    motion [H,W,2] | None, stats {tri_input, tri_after_clip, tri_raster}).  frame: shs_gpu.lib.LibFrame;
    draws: shs_gpu.lib.LibDraw with host meshes; shadow_map: float32 [h, w] sampled by draws with shadow."""
    keep = []
    arr = _lib_draws(draws, keep)
    W, H = frame.width, frame.height
    hdr = np.empty((H, W, 4), np.float32)
    depth = np.empty((H, W), np.float32) if frame.depth_motion else None
    motion = np.empty((H, W, 2), np.float32) if frame.depth_motion else None
    t = OraLibTarget()
    t.W, t.H, t.zn, t.zf = W, H, frame.zn, frame.zf
    t.bg_gradient = 1 if frame.bg_gradient else 0
    for i in range(4):
        t.clear_hdr[i] = frame.clear_hdr[i]
    fp = ctypes.POINTER(ctypes.c_float)
    t.hdr = hdr.ctypes.data_as(fp)
    if depth is not None:
        t.depth, t.motion = depth.ctypes.data_as(fp), motion.ctypes.data_as(fp)
    if shadow_map is not None:
        sm = np.ascontiguousarray(shadow_map, dtype=np.float32)
        keep.append(sm)
        t.shadow = sm.ctypes.data_as(fp)
        t.shadow_h, t.shadow_w = sm.shape
    if _FWD_CTX is not None:
        lights, cdesc, counts, idx = _FWD_CTX
        keep += [lights, cdesc, counts, idx]
        t.lights, t.n_lights = lights.ctypes.data, lights.shape[0]
        t.tile_counts, t.tile_indices = counts.ctypes.data, idx.ctypes.data
        t.cull = ctypes.addressof(cdesc)
    st = np.zeros(3, np.uint64)
    rc = _lib_lib().ora_pbr_forward(ctypes.byref(t), arr, len(draws), st.ctypes.data)
    if rc != 0:
        raise RuntimeError(f"ora_pbr_forward failed: {rc}")
    return hdr, depth, motion, {"tri_input": int(st[0]), "tri_after_clip": int(st[1]), "tri_raster": int(st[2])}


def shadow_map(size, sun_dir, casters):
    """PassShadowMap::execute -> (shadow map float32 [h, w], light viewproj float32[16])."""
    w, h = (size, size) if isinstance(size, int) else size
    keep = []
    arr = (OraShadowCaster * max(len(casters), 1))()
    for i, c in enumerate(casters):
        _fill_mesh(arr[i].mesh, c.mesh, keep)
        for k in range(16):
            arr[i].model[k] = float(c.model[k])
    sm = np.empty((h, w), np.float32)
    vp = np.zeros(16, np.float32)
    sd = np.ascontiguousarray(sun_dir, dtype=np.float32)
    rc = _lib_lib().ora_shadow_map(w, h, sd.ctypes.data, arr, len(casters), sm.ctypes.data, vp.ctypes.data)
    if rc != 0:
        raise RuntimeError(f"ora_shadow_map failed: {rc}")
    return sm, vp


def dir_light_camera_aabb(sun_dir, mn, mx, margin=10.0, res=2048):
    v, p, vp = (np.zeros(16, np.float32) for _ in range(3))
    a = [np.ascontiguousarray(x, dtype=np.float32) for x in (sun_dir, mn, mx)]
    _lib_lib().ora_dir_light_camera_aabb(a[0].ctypes.data, a[1].ctypes.data, a[2].ctypes.data, margin, res,
                                         v.ctypes.data, p.ctypes.data, vp.ctypes.data)
    return v, p, vp


# ===== Forward+ light lists (shs_oracle_light.c) ===========================================
class OraLightCullDesc(ctypes.Structure):
    _fields_ = [("width", ctypes.c_int32), ("height", ctypes.c_int32), ("tile_size", ctypes.c_uint32),
                ("max_per_tile", ctypes.c_uint32), ("mode", ctypes.c_uint32), ("z_slices", ctypes.c_uint32),
                ("view", _F16), ("proj", _F16), ("zn", ctypes.c_float), ("zf", ctypes.c_float),
                ("depth_linear", ctypes.c_int32)]


def _cull_desc(c):
    d = OraLightCullDesc()
    d.width, d.height = c.width, c.height
    d.tile_size, d.max_per_tile, d.mode, d.z_slices = c.tile_size, c.max_per_tile, c.mode, c.z_slices
    for k in range(16):
        d.view[k], d.proj[k] = float(c.view[k]), float(c.proj[k])
    d.zn, d.zf = c.zn, c.zf
    d.depth_linear = 1 if c.depth_linear else 0
    return d


def _light_lib():
    L = _lib_lib()
    if not getattr(L, "_light_ready", False):
        P = ctypes.c_void_p
        L.ora_light_cull.restype = None
        L.ora_light_cull.argtypes = [ctypes.POINTER(OraLightCullDesc), P, ctypes.c_int, P, P, P]
        L.ora_depth_reduce.restype = None
        L.ora_depth_reduce.argtypes = [ctypes.POINTER(OraLightCullDesc), P, P]
        L.ora_light_project.restype = None
        L.ora_light_project.argtypes = [ctypes.POINTER(OraLightCullDesc), P, ctypes.c_int, P]
        L._light_ready = True
    return L


def light_cull(cull, lights, depth=None):
    """fp_stress_light_cull.comp (+ fp_stress_depth_reduce.comp over `depth` for mode 2).  cull:
    shs_gpu.lib_path.LightCull; lights: LIGHT_DTYPE array -> (counts, indices [n_lists, maxp], ranges)."""
    L = _light_lib()
    d = _cull_desc(cull)
    lights = np.ascontiguousarray(lights)
    tx, ty = cull.tiles
    ranges = np.zeros((tx * ty, 2), np.float32)
    if cull.mode == 2:
        dep = np.ascontiguousarray(depth, dtype=np.float32)
        L.ora_depth_reduce(ctypes.byref(d), dep.ctypes.data, ranges.ctypes.data)
    counts = np.zeros(cull.n_lists, np.uint32)
    idx = np.zeros((cull.n_lists, cull.max_per_tile), np.uint32)
    L.ora_light_cull(ctypes.byref(d), lights.ctypes.data, lights.shape[0], ranges.ctypes.data, counts.ctypes.data,
                     idx.ctypes.data)
    return counts, idx, ranges


def light_project(cull, lights):
    L = _light_lib()
    d = _cull_desc(cull)
    lights = np.ascontiguousarray(lights)
    out = np.zeros((lights.shape[0], 8), np.float32)
    L.ora_light_project(ctypes.byref(d), lights.ctypes.data, lights.shape[0], out.ctypes.data)
    return out


def forward_plus(frame, draws, lights, cull, lists, shadow_map=None):
    """pbr_forward with the Forward+ program's light data: lists = (counts, indices) of light_cull."""
    global _FWD_CTX
    _FWD_CTX = (np.ascontiguousarray(lights), _cull_desc(cull), np.ascontiguousarray(lists[0], dtype=np.uint32),
                np.ascontiguousarray(lists[1], dtype=np.uint32))
    try:
        return pbr_forward(frame, draws, shadow_map)
    finally:
        _FWD_CTX = None


_FWD_CTX = None


def sample_texture(rgba, u, v):
    """sample_texture2d_bilinear_repeat_linear (builtin_shaders.hpp:33-55): rgba uint8 [h, w, 4] -> float32[3]."""
    L = lib()
    if not getattr(L, "_tex_ready", False):
        L.ora_sample_texture.restype = None
        L.ora_sample_texture.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_float, ctypes.c_float,
                                         ctypes.c_void_p]
        L._tex_ready = True
    t = np.ascontiguousarray(rgba, dtype=np.uint8)
    out = np.zeros(3, np.float32)
    L.ora_sample_texture(t.ctypes.data, t.shape[1], t.shape[0], float(u), float(v), out.ctypes.data)
    return out


def tonemap(hdr, exposure=1.0, gamma=2.2):
    """PassTonemap + upload_ldr_to_rgba8 over hdr float32 [H, W, 4] (rows y up) ->
    (ldr uint8 [H, W, 4] rows y up, present uint8 [H, W, 4] rows top-down)."""
    L = _lib_lib()
    if not getattr(L, "_post_ready", False):
        P = ctypes.c_void_p
        L.ora_tonemap.restype = None
        L.ora_tonemap.argtypes = [P, ctypes.c_int, ctypes.c_int, ctypes.c_float, ctypes.c_float, P, P]
        L.ora_tonemap_channel.restype = ctypes.c_uint8
        L.ora_tonemap_channel.argtypes = [ctypes.c_float, ctypes.c_float, ctypes.c_float]
        L._post_ready = True
    hdr = np.ascontiguousarray(hdr, dtype=np.float32)
    H, W = hdr.shape[:2]
    ldr = np.empty((H, W, 4), np.uint8)
    present = np.empty((H, W, 4), np.uint8)
    L.ora_tonemap(hdr.ctypes.data, W, H, float(exposure), float(gamma), ldr.ctypes.data, present.ctypes.data)
    return ldr, present


def tonemap_channel(s, exposure, inv_gamma):
    """One channel byte of PassTonemap (exposure / inv_gamma already clamped as the pass does)."""
    tonemap(np.zeros((1, 1, 4), np.float32))   # binds the signatures
    return int(_lib_lib().ora_tonemap_channel(float(s), float(exposure), float(inv_gamma)))


def motion_blur(src_ldr, depth, motion, enable=True, samples=10, strength=1.0, max_velocity_px=20.0,
                min_velocity_px=0.25, depth_reject=0.08, dt=1.0 / 60.0):
    """PassMotionBlur over an RT_ColorLDR (uint8 [H, W, 4], rows y up) with the depth [H, W] and motion
    [H, W, 2] planes -> uint8 [H, W, 4] (defaults: MotionBlurPassParams, frame_params.hpp:49-57)."""
    L = _lib_lib()
    if not getattr(L, "_mb_ready", False):
        P = ctypes.c_void_p
        L.ora_motion_blur.restype = None
        L.ora_motion_blur.argtypes = [P, P, P, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int] + \
            [ctypes.c_float] * 5 + [P]
        L._mb_ready = True
    src = np.ascontiguousarray(src_ldr, dtype=np.uint8)
    H, W = src.shape[:2]
    dep = np.ascontiguousarray(depth, dtype=np.float32)
    mot = np.ascontiguousarray(motion, dtype=np.float32)
    out = np.empty_like(src)
    L.ora_motion_blur(src.ctypes.data, dep.ctypes.data, mot.ctypes.data, W, H, 1 if enable else 0, int(samples),
                      float(strength), float(max_velocity_px), float(min_velocity_px), float(depth_reject), float(dt),
                      out.ctypes.data)
    return out


class OraOccObject(ctypes.Structure):
    _fields_ = [("pos", ctypes.c_void_p), ("n_verts", ctypes.c_int32), ("idx", ctypes.c_void_p), ("n_idx", ctypes.c_int32),
                ("model", _F16), ("aabb_min", ctypes.c_float * 3), ("aabb_max", ctypes.c_float * 3)]


def occlusion_pass(width, height, view, view_proj, objects, frustum_visible, depth_epsilon=1e-4, enable=True):
    """culling_sw::run_software_occlusion_pass restated -> (occluded uint8 [n], visible uint32 [k], depth)."""
    L = _lib_lib()
    if not getattr(L, "_occ_ready", False):
        P = ctypes.c_void_p
        L.ora_occlusion_pass.restype = ctypes.c_int
        L.ora_occlusion_pass.argtypes = [P, ctypes.c_int, P, ctypes.c_int, ctypes.c_int, P, ctypes.c_int, ctypes.c_int,
                                         P, P, ctypes.c_float, P, P]
        L._occ_ready = True
    n = len(objects)
    arr = (OraOccObject * max(n, 1))()
    keep = []
    for i, (mesh, model, mn, mx) in enumerate(objects):
        pos = np.ascontiguousarray(mesh.positions, dtype=np.float32)
        idx = np.ascontiguousarray(mesh.indices, dtype=np.uint32)
        keep += [pos, idx]
        a = arr[i]
        a.pos, a.n_verts, a.idx, a.n_idx = pos.ctypes.data, pos.shape[0], idx.ctypes.data, idx.size
        for k in range(16):
            a.model[k] = float(model[k])
        for k in range(3):
            a.aabb_min[k], a.aabb_max[k] = float(mn[k]), float(mx[k])
    fv = np.ascontiguousarray(frustum_visible, dtype=np.uint32)
    v16 = np.ascontiguousarray(view, dtype=np.float32)
    vp16 = np.ascontiguousarray(view_proj, dtype=np.float32)
    depth = np.ones((height, width), np.float32)
    occ = np.zeros(max(n, 1), np.uint8)
    vis = np.zeros(max(fv.size, 1), np.uint32)
    nv = L.ora_occlusion_pass(ctypes.addressof(arr), n, fv.ctypes.data, fv.size, 1 if enable else 0, depth.ctypes.data,
                              width, height, v16.ctypes.data, vp16.ctypes.data, float(depth_epsilon), occ.ctypes.data,
                              vis.ctypes.data)
    return occ[:n], vis[:nv], depth


# ---- camera / model matrices (shs_oracle_camera.c) -------------------------------------------------
def _f32(a, n):
    a = np.ascontiguousarray(a, dtype=np.float32).reshape(-1)
    assert a.size == n
    return a


def camera3d(position, yaw, pitch, fov=60.0, zn=0.1, zf=1000.0):
    """Camera3D::update (shs_renderer.hpp:1224-1236) -> (view, proj) float32[16], column-major."""
    L = lib()
    pos = _f32(position, 3)
    view = np.zeros(16, np.float32)
    proj = np.zeros(16, np.float32)
    L.ora_camera3d(pos.ctypes.data, yaw, pitch, fov, zn, zf, view.ctypes.data, proj.ctypes.data)
    return view, proj


def model_trs(position, rot_deg_y, scale):
    """MonkeyObject::get_world_matrix (blinn_phong_shading.cpp:122-128)."""
    L = lib()
    p, s = _f32(position, 3), _f32(scale, 3)
    out = np.zeros(16, np.float32)
    L.ora_model_trs(p.ctypes.data, rot_deg_y, s.ctypes.data, out.ctypes.data)
    return out


def look_at_lh(eye, center, up):
    out = np.zeros(16, np.float32)
    e, c, u = _f32(eye, 3), _f32(center, 3), _f32(up, 3)
    lib().ora_look_at_lh(e.ctypes.data, c.ctypes.data, u.ctypes.data, out.ctypes.data)
    return out


def perspective_lh_no(fovy, aspect, zn, zf):
    out = np.zeros(16, np.float32)
    lib().ora_perspective_lh_no(fovy, aspect, zn, zf, out.ctypes.data)
    return out


def legacy_mvp(view, proj, model, flat=False):
    """RendererSystem::process uniforms: mvp = (proj * view) * model, or for the Flat pipeline
    mv = view * model, mvp = proj * mv -> (mvp, mv or model)."""
    v, p, m = _f32(view, 16), _f32(proj, 16), _f32(model, 16)
    mvp = np.zeros(16, np.float32)
    mv = np.zeros(16, np.float32)
    lib().ora_legacy_mvp(v.ctypes.data, p.ctypes.data, m.ctypes.data, 1 if flat else 0, mvp.ctypes.data, mv.ctypes.data)
    return mvp, mv


def sdl_present(canvas_rgba):
    """Canvas::copy_to_SDLSurface (shs_renderer.hpp:833-848) into create_sdl_surface's RGBA32 surface
    (:850-856, little-endian masks R 0x000000ff .. A 0xff000000): surface row h-1-y = canvas row y,
    SDL_MapRGBA(r, g, b, a) = the Color bytes.  canvas_rgba: uint8 [H, W, 4] canvas rows -> uint8
    [H, W, 4] surface rows (top-down)."""
    c = np.ascontiguousarray(canvas_rgba, dtype=np.uint8)
    h, w = c.shape[:2]
    out = np.empty_like(c)
    for y in range(h):
        out[h - 1 - y] = c[y]
    return out



class OraLightBinDesc(ctypes.Structure):
    _fields_ = [("width", ctypes.c_int32), ("height", ctypes.c_int32), ("tile_size", ctypes.c_uint32),
                ("mode", ctypes.c_uint32), ("z_slices", ctypes.c_uint32), ("max_per_bin", ctypes.c_uint32),
                ("view_proj", _F16), ("z_near", ctypes.c_float), ("z_far", ctypes.c_float),
                ("tile_min_view_depth", ctypes.c_void_p), ("tile_max_view_depth", ctypes.c_void_p),
                ("n_depth_tiles", ctypes.c_int32)]


def light_bin_culling(lb, aabbs):
    """build_light_bin_culling (light_culling_runtime.hpp:266-371), oracle/shs_oracle_lightbin.c.
    lb: shs_gpu.lib_path.LightBin; aabbs float32 [n, 6] -> (bins_xyz, counts, indices [bins, cap])."""
    L = lib()
    if not getattr(L, "_lb_ready", False):
        L.ora_light_bin_culling.restype = ctypes.c_int
        L.ora_light_bin_culling.argtypes = [ctypes.POINTER(OraLightBinDesc), ctypes.c_void_p, ctypes.c_int,
                                            ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        L._lb_ready = True
    aabbs = np.ascontiguousarray(aabbs, dtype=np.float32).reshape(-1, 6)
    n = aabbs.shape[0]
    d = OraLightBinDesc()
    d.width, d.height, d.tile_size, d.mode, d.z_slices = lb.width, lb.height, lb.tile_size, lb.mode, lb.z_slices
    d.max_per_bin = lb.max_per_bin if lb.max_per_bin > 0 else max(n, 1)
    for k in range(16):
        d.view_proj[k] = float(lb.view_proj[k])
    d.z_near, d.z_far = lb.z_near, lb.z_far
    keep = []
    if lb.tile_min_view_depth is not None:
        mn = np.ascontiguousarray(lb.tile_min_view_depth, dtype=np.float32)
        mx = np.ascontiguousarray(lb.tile_max_view_depth, dtype=np.float32)
        keep += [mn, mx]
        d.tile_min_view_depth, d.tile_max_view_depth, d.n_depth_tiles = mn.ctypes.data, mx.ctypes.data, mn.size
    ts = max(lb.tile_size, 1)
    bx, by = (lb.width + ts - 1) // ts, (lb.height + ts - 1) // ts
    n_bins = bx * by * (max(lb.z_slices, 1) if lb.mode == 3 else 1)
    counts = np.zeros(n_bins, np.uint32)
    idx = np.zeros((n_bins, d.max_per_bin), np.uint32)
    bins = np.zeros(3, np.uint32)
    L.ora_light_bin_culling(ctypes.byref(d), aabbs.ctypes.data, n, bins.ctypes.data, counts.ctypes.data, idx.ctypes.data)
    return tuple(int(b) for b in bins), counts, idx


# ---- debug_draw (shs_oracle_debugdraw.c) -------------------------------------------------------------
class OraDDMesh(ctypes.Structure):
    _fields_ = [("pos", ctypes.c_void_p), ("n_verts", ctypes.c_int32), ("idx", ctypes.c_void_p), ("n_idx", ctypes.c_int32),
                ("model", _F16), ("base", ctypes.c_float * 3)]


def _dd_ready(L):
    if not getattr(L, "_dd_ready", False):
        P = ctypes.c_void_p
        L.ora_debug_draw_meshes.restype = ctypes.c_int
        L.ora_debug_draw_meshes.argtypes = [P, ctypes.c_int, ctypes.c_int, ctypes.c_int, P, P, P, P, P, P]
        L.ora_draw_filled_triangle.restype = None
        L.ora_draw_filled_triangle.argtypes = [P, P, ctypes.c_int, ctypes.c_int, P, ctypes.c_float, P, ctypes.c_float,
                                               P, ctypes.c_float, P]
        L._dd_ready = True


def debug_draw_meshes(width, height, view_proj, camera_pos, light_dir_ws, meshes, rgba=None, depth=None):
    """draw_mesh_blinn_phong_transformed (debug_draw.hpp:147-203) over meshes = [(mesh, model[16],
    base[3])] in order -> (rgba uint8 [H, W, 4], depth [H, W], tri_lit float32 [n_tris, 4])."""
    L = lib()
    _dd_ready(L)
    rgba = np.zeros((height, width, 4), np.uint8) if rgba is None else np.array(rgba, np.uint8, copy=True)
    depth = np.ones((height, width), np.float32) if depth is None else np.array(depth, np.float32, copy=True)
    n = len(meshes)
    arr = (OraDDMesh * max(n, 1))()
    keep = []
    n_tris = 0
    for i, (mesh, model, base) in enumerate(meshes):
        pos = np.ascontiguousarray(mesh.positions, dtype=np.float32)
        idx = np.ascontiguousarray(mesh.indices, dtype=np.uint32)
        keep += [pos, idx]
        a = arr[i]
        a.pos, a.n_verts, a.idx, a.n_idx = pos.ctypes.data, pos.shape[0], idx.ctypes.data, idx.size
        for k in range(16):
            a.model[k] = float(model[k])
        for k in range(3):
            a.base[k] = float(base[k])
        n_tris += idx.size // 3
    lit = np.zeros((max(n_tris, 1), 4), np.float32)
    vp, cam, ld = _f32(view_proj, 16), _f32(camera_pos, 3), _f32(light_dir_ws, 3)
    L.ora_debug_draw_meshes(ctypes.addressof(arr), n, width, height, vp.ctypes.data, cam.ctypes.data, ld.ctypes.data,
                            rgba.ctypes.data, depth.ctypes.data, lit.ctypes.data)
    return rgba, depth, lit[:n_tris]


def draw_filled_triangles(width, height, screen, z, colors, rgba=None, depth=None):
    """draw_filled_triangle (debug_draw.hpp:60-109) for each triangle in order."""
    L = lib()
    _dd_ready(L)
    rgba = np.zeros((height, width, 4), np.uint8) if rgba is None else np.array(rgba, np.uint8, copy=True)
    depth = np.ones((height, width), np.float32) if depth is None else np.array(depth, np.float32, copy=True)
    screen = np.ascontiguousarray(screen, np.float32).reshape(-1, 3, 2)
    z = np.ascontiguousarray(z, np.float32).reshape(-1, 3)
    colors = np.ascontiguousarray(colors, np.uint8).reshape(-1, 4)
    for t in range(screen.shape[0]):
        p = screen[t]
        L.ora_draw_filled_triangle(rgba.ctypes.data, depth.ctypes.data, width, height, p[0].ctypes.data, float(z[t, 0]),
                                   p[1].ctypes.data, float(z[t, 1]), p[2].ctypes.data, float(z[t, 2]),
                                   colors[t].ctypes.data)
    return rgba, depth


# ---- Canvas-API multi-pass extras (shs_oracle_canvas_post.c) ----------------------------------------
def _cp_ready(L):
    if not getattr(L, "_cp_ready", False):
        P, I, F = ctypes.c_void_p, ctypes.c_int, ctypes.c_float
        L.ora_canvas_motion_blur.restype = None
        L.ora_canvas_motion_blur.argtypes = [P, P, P, P, I, I, P, P, P, P, I, F, F, F, I, F, F]
        L.ora_canvas_gaussian.restype = None
        L.ora_canvas_gaussian.argtypes = [P, P, I, I, I]
        L.ora_canvas_autofocus.restype = F
        L.ora_canvas_autofocus.argtypes = [P, I, I, I, I, I]
        L.ora_canvas_dof.restype = F
        L.ora_canvas_dof.argtypes = [P, P, P, I, I, I, I, I, I, F, F]
        L._cp_ready = True


def canvas_motion_blur(src, depth, velocity, curr_view, curr_proj, prev_view, prev_proj, samples=12, strength=0.85,
                       w_obj=1.0, w_cam=0.35, soft_knee=True, knee_px=18.0, max_px=22.0):
    """combined_motion_blur_pass (hello_pbr.cpp:1128-1252): src uint8 [H, W, 4], depth float32 [H, W],
    velocity float32 [H, W, 2] -> dst uint8 [H, W, 4]."""
    L = lib()
    _cp_ready(L)
    src = np.ascontiguousarray(src, np.uint8)
    H, W = src.shape[:2]
    depth = np.ascontiguousarray(depth, np.float32)
    velocity = np.ascontiguousarray(velocity, np.float32)
    dst = np.zeros_like(src)
    m = [_f32(a, 16) for a in (curr_view, curr_proj, prev_view, prev_proj)]
    L.ora_canvas_motion_blur(src.ctypes.data, depth.ctypes.data, velocity.ctypes.data, dst.ctypes.data, W, H,
                             *[a.ctypes.data for a in m], int(samples), float(strength), float(w_obj), float(w_cam),
                             1 if soft_knee else 0, float(knee_px), float(max_px))
    return dst


def canvas_gaussian(src, horizontal):
    L = lib()
    _cp_ready(L)
    src = np.ascontiguousarray(src, np.uint8)
    dst = np.zeros_like(src)
    L.ora_canvas_gaussian(src.ctypes.data, dst.ctypes.data, src.shape[1], src.shape[0], 1 if horizontal else 0)
    return dst


def canvas_autofocus(depth, cx, cy, radius):
    L = lib()
    _cp_ready(L)
    depth = np.ascontiguousarray(depth, np.float32)
    return L.ora_canvas_autofocus(depth.ctypes.data, depth.shape[1], depth.shape[0], int(cx), int(cy), int(radius))


def canvas_dof(color, depth, iterations=3, radius=6, focus=None, range_=24.0, max_blur=0.6):
    """The DoF step of hello_depth_of_field.cpp:786-812 -> (composite, blur, focus_depth)."""
    L = lib()
    _cp_ready(L)
    out = np.array(color, np.uint8, copy=True)
    H, W = out.shape[:2]
    depth = np.ascontiguousarray(depth, np.float32)
    blur = np.zeros_like(out)
    cx, cy = (W // 2, H // 2) if focus is None else focus
    f = L.ora_canvas_dof(out.ctypes.data, depth.ctypes.data, blur.ctypes.data, W, H, int(iterations), int(radius),
                         int(cx), int(cy), float(range_), float(max_blur))
    return out, blur, f


def set_lib_threads(n):
    """rasterize_mesh's row-parallel split of big bboxes (rasterizer.hpp:424-436) on n host threads."""
    L = _lib_lib()
    L.ora_set_lib_threads.restype = None
    L.ora_set_lib_threads.argtypes = [ctypes.c_int]
    L.ora_set_lib_threads(int(n))
