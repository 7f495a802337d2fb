"""shs_gpu -- Python mirror of the shs_renderer legacy draw-call API over libshs_gpu.so.

The reference drives its hot path from C++ (`RendererSystem::process` -> `draw_triangle_tile`,
cpp-folders/src/hello-3d-primitives/hello_pipeline_blinn_phong_shading.cpp:244-313).  This module
is the thin host layer the tests and bench use: it owns a context (`shs_create`), uploads meshes
once (`shs_mesh_upload_soup`, the ModelGeometry soup), enqueues frames (`shs_render_legacy`) and
resolves framebuffers into the reference layouts (`shs_resolve`).  Every call goes through the C ABI
into the gfx950 kernels; there is no CPU path here.
"""
import ctypes
from dataclasses import dataclass, field

import numpy as np

from . import _abi
from ._abi import (FRAME_PREQUANT, FRAME_PRESENT, SHADING_BLINN_PHONG, SHADING_FLAT, SHADING_GOURAUD, SHADING_NAMES,
                   SHADING_PHONG, FrameDesc, LegacyDraw, RasterStats)

__all__ = [
    "ShsError", "Context", "Frame", "Draw", "SHADING_FLAT", "SHADING_GOURAUD", "SHADING_PHONG",
    "SHADING_BLINN_PHONG", "SHADING_NAMES", "FRAME_PREQUANT", "lib",
]

lib = _abi.lib


class ShsError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"shs_gpu error {code}: {msg}")
        self.code = code


def _fptr(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))


@dataclass
class Draw:
    """One object of the legacy scene loop: the reference's `Uniforms` + mesh + shading model."""
    mesh: object                 # Mesh (positions/normals float32 [n,9]) or an uploaded mesh id
    shading: int
    mvp: np.ndarray              # float32[16], column-major (glm::mat4 storage)
    model: np.ndarray            # float32[16] (Flat: Uniforms::mv)
    light_dir: np.ndarray        # float32[3]  (Flat: light_dir_view)
    camera_pos: np.ndarray       # float32[3]
    color: tuple = (60, 100, 200, 255)


@dataclass
class Frame:
    width: int
    height: int
    ref_tile: tuple = (80, 80)   # TILE_SIZE_X/Y of the legacy pipelines
    shard_rank: int = 0
    shard_count: int = 1
    clear_color: tuple = (0, 0, 0, 255)
    prequant: bool = False
    present: bool = False             # SHS_FRAME_PRESENT: also write the SDL staging
    debug_flags: int = 0         # timing experiments only (bits 8+, wrong images)

    def desc(self) -> FrameDesc:
        d = FrameDesc()
        d.width, d.height = self.width, self.height
        d.ref_tile_w, d.ref_tile_h = self.ref_tile
        d.shard_rank, d.shard_count = self.shard_rank, self.shard_count
        d.flags = (FRAME_PREQUANT if self.prequant else 0) | (FRAME_PRESENT if self.present else 0) | \
                  (int(self.debug_flags) & ~0xff)
        for i in range(4):
            d.clear_color[i] = self.clear_color[i]
        return d


class Context:
    """A libshs_gpu context bound to one HIP device (one host thread at a time)."""

    def __init__(self, device: int = 0):
        self._lib = lib()
        h = ctypes.c_void_p()
        rc = self._lib.shs_create(device, ctypes.byref(h))
        if rc != 0:
            raise ShsError(rc, f"shs_create(device={device}) failed (no gfx950 device?)")
        self._h = h
        self._meshes = {}
        self._frame = None
        self._lib_frame = None
        self._shadow_size = None

    def _check(self, rc):
        if rc != 0:
            raise ShsError(rc, self._lib.shs_last_error(self._h).decode(errors="replace"))

    def close(self):
        if getattr(self, "_h", None):
            self._lib.shs_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    # -- geometry -----------------------------------------------------------------------------
    def upload_mesh(self, mesh) -> int:
        key = id(mesh)
        if key in self._meshes:
            return self._meshes[key][0]
        pos = np.ascontiguousarray(mesh.positions, dtype=np.float32)
        nrm = np.ascontiguousarray(mesh.normals, dtype=np.float32)
        assert pos.shape == nrm.shape and pos.shape[-1] == 9
        mid = ctypes.c_int32()
        self._check(self._lib.shs_mesh_upload_soup(self._h, _fptr(pos), _fptr(nrm), pos.shape[0], ctypes.byref(mid)))
        self._meshes[key] = (mid.value, mesh)
        return mid.value

    # -- frames -------------------------------------------------------------------------------
    def _draw_array(self, draws):
        arr = (LegacyDraw * max(len(draws), 1))()
        for i, d in enumerate(draws):
            a = arr[i]
            a.mesh_id = d.mesh if isinstance(d.mesh, int) else self.upload_mesh(d.mesh)
            a.shading = int(d.shading)
            for k in range(16):
                a.mvp[k] = float(d.mvp[k])
                a.model[k] = float(d.model[k])
            for k in range(3):
                a.light_dir[k] = float(d.light_dir[k])
                a.camera_pos[k] = float(d.camera_pos[k])
            for k in range(4):
                a.color[k] = int(d.color[k])
        return arr

    def prepare(self, frame: Frame, draws):
        """Build the ctypes frame/draw arrays once (re-used by render_prepared in timed loops)."""
        return frame, frame.desc(), self._draw_array(draws), len(draws)

    def render_prepared(self, prepared):
        frame, desc, arr, n = prepared
        self._check(self._lib.shs_render_legacy(self._h, ctypes.byref(desc), arr, n))
        self._frame = frame

    def render(self, frame: Frame, draws):
        self.render_prepared(self.prepare(frame, draws))

    def prepare_batch(self, frame: Frame, frames_draws):
        """frames_draws: one draw list per frame (equal lengths and triangle counts) -> prepared batch."""
        n = len(frames_draws[0])
        assert all(len(d) == n for d in frames_draws), "every frame of a batch has the same number of draws"
        flat = [d for fd in frames_draws for d in fd]
        return frame, frame.desc(), self._draw_array(flat), n, len(frames_draws)

    def render_batch_prepared(self, prepared):
        frame, desc, arr, n, n_frames = prepared
        self._check(self._lib.shs_render_legacy_batch(self._h, ctypes.byref(desc), arr, n, n_frames))
        self._frame = frame
        self._n_frames = n_frames

    def render_batch(self, frame: Frame, frames_draws):
        """shs_render_legacy_batch: one k_setup + k_raster pair renders every frame of the batch."""
        self.render_batch_prepared(self.prepare_batch(frame, frames_draws))

    def resolve_frame(self, index: int):
        f = self._frame
        color = np.empty((f.height, f.width, 4), dtype=np.uint8)
        depth = np.empty((f.height, f.width), dtype=np.float32)
        self._check(self._lib.shs_resolve_frame(self._h, int(index), color.ctypes.data_as(ctypes.c_void_p),
                                                depth.ctypes.data_as(ctypes.c_void_p)))
        return color, depth

    def synchronize(self):
        self._check(self._lib.shs_synchronize(self._h))

    def resolve(self):
        f = self._frame
        color = np.empty((f.height, f.width, 4), dtype=np.uint8)
        depth = np.empty((f.height, f.width), dtype=np.float32)
        self._check(self._lib.shs_resolve(self._h, color.ctypes.data_as(ctypes.c_void_p),
                                          depth.ctypes.data_as(ctypes.c_void_p)))
        return color, depth

    def present_device(self, index: int = 0) -> int:
        """Device address of frame `index`'s SDL staging (SHS_FRAME_PRESENT); a batch's frames are
        contiguous, W * H * 4 bytes apart."""
        p = ctypes.c_void_p()
        self._check(self._lib.shs_present_device(self._h, int(index), ctypes.byref(p)))
        return p.value

    def resolve_present(self, index: int = 0, pitch: int = 0):
        """The SDL staging of frame `index` (Canvas::copy_to_SDLSurface): uint8 [H, W, 4], rows top-down.
        pitch > W*4 pads rows as an SDL surface would (returned array [H, pitch] bytes)."""
        f = self._frame
        pitch = pitch or f.width * 4
        out = np.zeros((f.height, pitch), dtype=np.uint8)
        self._check(self._lib.shs_resolve_present(self._h, int(index), out.ctypes.data_as(ctypes.c_void_p), pitch))
        return out if pitch != f.width * 4 else out.reshape(f.height, f.width, 4)

    def resolve_prequant(self, index: int = 0):
        """Pre-truncation shader floats of frame `index` of the last batch (SHS_FRAME_PREQUANT)."""
        f = self._frame
        pq = np.empty((f.height, f.width, 4), dtype=np.float32)
        self._check(self._lib.shs_resolve_prequant_frame(self._h, int(index), pq.ctypes.data_as(ctypes.c_void_p)))
        return pq

    def device_framebuffers(self):
        c, d = ctypes.c_void_p(), ctypes.c_void_p()
        self._check(self._lib.shs_device_framebuffers(self._h, ctypes.byref(c), ctypes.byref(d)))
        return c.value, d.value

    def stats(self) -> dict:
        s = RasterStats()
        self._check(self._lib.shs_get_stats(self._h, ctypes.byref(s)))
        return {k: int(getattr(s, k)) for k, _ in RasterStats._fields_}

    def enable_timing(self, on=True):
        self._check(self._lib.shs_enable_timing(self._h, 1 if on else 0))

    def kernel_ms(self):
        ms = (ctypes.c_float * 4)()
        self._check(self._lib.shs_last_kernel_ms(self._h, ms))
        return {"setup": ms[0], "raster": ms[3]}

    def timing_reset(self):
        self._check(self._lib.shs_timing_reset(self._h))

    def timing_read(self):
        """-> (frames, {kernel: mean ms}) over every frame since timing_reset()."""
        s = (ctypes.c_double * 4)()
        n = ctypes.c_int64()
        self._check(self._lib.shs_timing_read(self._h, s, ctypes.byref(n)))
        k = max(n.value, 1)
        return n.value, {"setup": s[0] / k, "raster": s[3] / k}

    # shs_dev::TriHot (64 B): word = draw | flags << 29
    TRIREC_DTYPE = np.dtype([
        ("ax", "<f4"), ("ay", "<f4"), ("v0x", "<f4"), ("v0y", "<f4"), ("v1x", "<f4"), ("v1y", "<f4"),
        ("d00", "<f4"), ("d01", "<f4"), ("d11", "<f4"), ("denom", "<f4"), ("z0", "<f4"), ("z1", "<f4"),
        ("z2", "<f4"), ("word", "<u4"), ("gbx", "<u4"), ("gby", "<u4")])

    def debug_records(self):
        """The last frame's per-triangle raster records (structured numpy array)."""
        n = ctypes.c_int64()
        self._check(self._lib.shs_debug_records(self._h, None, 0, ctypes.byref(n)))
        out = np.zeros(n.value, dtype=self.TRIREC_DTYPE)
        self._check(self._lib.shs_debug_records(self._h, out.ctypes.data_as(ctypes.c_void_p), n.value, ctypes.byref(n)))
        return out

    def set_raster_mode(self, mode: int):
        """0 auto, 1 scan (no bins), 2 bins."""
        self._check(self._lib.shs_set_option(self._h, _abi.OPT_RASTER_MODE, int(mode)))

    def set_raster_loop(self, loop: int):
        """Legacy raster inner loop: 1 (candidate, pixel) pair tasks (default), 0 per-pixel candidate loop."""
        self._check(self._lib.shs_set_option(self._h, _abi.OPT_RASTER_LOOP, int(loop)))

    def set_timeline(self, enable: bool, shadow: bool = False):
        """Workgroup timelines of the frames that follow; shadow: the library shadow pass's raster
        (lib_debug_timeline) instead of the camera pass's."""
        self._check(self._lib.shs_set_option(self._h, _abi.OPT_TIMELINE, (2 if shadow else 1) if enable else 0))

    # -- after the path: PassTonemap + present staging ------------------------------------------
    def tonemap(self, exposure: float = 1.0, gamma: float = 2.2, ldr: bool = True, present: bool = True):
        """PassTonemap (pass_tonemap.hpp:36-83) over the last camera pass's HDR target into the
        RT_ColorLDR layout and / or the SDL staging of upload_ldr_to_rgba8 (one launch)."""
        d = _abi.TonemapDescC()
        d.exposure, d.gamma = float(exposure), float(gamma)
        d.flags = (_abi.TONEMAP_LDR if ldr else 0) | (_abi.TONEMAP_PRESENT if present else 0)
        self._check(self._lib.shs_tonemap(self._h, ctypes.byref(d)))
        self._tonemap_flags = d.flags

    def fuse_tonemap(self, exposure: float = 1.0, gamma: float = 2.2, ldr: bool = True, present: bool = True,
                     enable: bool = True):
        """Fused PassTonemap: later camera passes also write the tonemap targets from their shading
        kernel (the same bytes as tonemap() after the pass); enable=False turns it off."""
        if not enable:
            self._check(self._lib.shs_lib_fuse_tonemap(self._h, None))
            return
        d = _abi.TonemapDescC()
        d.exposure, d.gamma = float(exposure), float(gamma)
        d.flags = (_abi.TONEMAP_LDR if ldr else 0) | (_abi.TONEMAP_PRESENT if present else 0)
        self._check(self._lib.shs_lib_fuse_tonemap(self._h, ctypes.byref(d)))
        self._tonemap_flags = d.flags

    def resolve_ldr(self):
        """-> (ldr uint8 [H, W, 4] rows y up or None, present uint8 [H, W, 4] rows top-down or None)."""
        f = self._lib_frame
        flags = getattr(self, "_tonemap_flags", 0)
        ldr = np.empty((f.height, f.width, 4), np.uint8) if flags & _abi.TONEMAP_LDR else None
        pre = np.empty((f.height, f.width, 4), np.uint8) if flags & _abi.TONEMAP_PRESENT else None
        self._check(self._lib.shs_resolve_ldr(self._h, None if ldr is None else ldr.ctypes.data_as(ctypes.c_void_p),
                                              None if pre is None else pre.ctypes.data_as(ctypes.c_void_p)))
        return ldr, pre

    def motion_blur(self, enable=True, samples=10, strength=1.0, max_velocity_px=20.0, min_velocity_px=0.25,
                    depth_reject=0.08, dt=1.0 / 60.0, present=True):
        """PassMotionBlur (pass_motion_blur.hpp:38-170) over the last tonemap's RT_ColorLDR with the
        camera pass's depth / motion planes (defaults: MotionBlurPassParams)."""
        d = _abi.MotionBlurDescC()
        d.enable, d.samples = 1 if enable else 0, int(samples)
        d.strength, d.max_velocity_px, d.min_velocity_px = float(strength), float(max_velocity_px), float(min_velocity_px)
        d.depth_reject, d.dt = float(depth_reject), float(dt)
        d.flags = _abi.MOTION_BLUR_PRESENT if present else 0
        self._check(self._lib.shs_motion_blur(self._h, ctypes.byref(d)))
        self._mb_present = bool(present)

    def resolve_motion_blur(self):
        """-> (blurred RT_ColorLDR uint8 [H, W, 4] rows y up, present staging or None)."""
        f = self._lib_frame
        ldr = np.empty((f.height, f.width, 4), np.uint8)
        pre = np.empty((f.height, f.width, 4), np.uint8) if getattr(self, "_mb_present", False) else None
        self._check(self._lib.shs_resolve_motion_blur(self._h, ldr.ctypes.data_as(ctypes.c_void_p),
                                                      None if pre is None else pre.ctypes.data_as(ctypes.c_void_p)))
        return ldr, pre

    def occlusion_pass(self, width, height, view, view_proj, objects, frustum_visible, depth_epsilon=1e-4,
                       enable=True):
        """culling_sw::run_software_occlusion_pass (culling_software.hpp:229-331).  objects: sequence of
        (LibMesh with indices, model float[16], aabb_min[3], aabb_max[3]) -> (occluded uint8 [n],
        visible uint32 [k] in visit order, depth float32 [height, width])."""
        n = len(objects)
        # shs_occluder records (int32 mesh_id, float model[16], aabb_min[3], aabb_max[3]) built in numpy
        arr = np.zeros((max(n, 1), ctypes.sizeof(_abi.OccluderC) // 4), np.float32)
        if n:
            arr[:n, 0].view(np.int32)[:] = [self.upload_lib_mesh(o[0]) for o in objects]
            arr[:n, 1:17] = np.asarray([o[1] for o in objects], np.float32).reshape(n, 16)
            arr[:n, 17:20] = np.asarray([o[2] for o in objects], np.float32).reshape(n, 3)
            arr[:n, 20:23] = np.asarray([o[3] for o in objects], np.float32).reshape(n, 3)
        d = _abi.OcclusionDescC()
        d.width, d.height = int(width), int(height)
        for k in range(16):
            d.view[k], d.view_proj[k] = float(view[k]), float(view_proj[k])
        d.depth_epsilon, d.enable = float(depth_epsilon), 1 if enable else 0
        fv = np.ascontiguousarray(frustum_visible, dtype=np.uint32)
        occ = np.zeros(max(n, 1), np.uint8)
        vis = np.zeros(max(fv.size, 1), np.uint32)
        nv = ctypes.c_int32()
        depth = np.zeros((height, width), np.float32)
        self._check(self._lib.shs_occlusion_pass(self._h, ctypes.byref(d), arr.ctypes.data_as(ctypes.POINTER(_abi.OccluderC)), n,
                                                 fv.ctypes.data_as(ctypes.c_void_p),
                                                 fv.size, occ.ctypes.data_as(ctypes.c_void_p),
                                                 vis.ctypes.data_as(ctypes.c_void_p), ctypes.byref(nv),
                                                 depth.ctypes.data_as(ctypes.c_void_p)))
        return occ[:n], vis[:nv.value], depth

    def debug_draw_meshes(self, width, height, view_proj, camera_pos, light_dir_ws, meshes, rgba=None, depth=None,
                          tri_lit=False):
        """debug_draw::draw_mesh_blinn_phong_transformed (sw_render/debug_draw.hpp:147-203) over meshes =
        sequence of (LibMesh with indices, model float[16], base_color[3]), in order.  rgba uint8
        [height, width, 4] (RT_ColorLDR, y * W + x) and depth float32 [height, width] are drawn into in
        place (defaults: cleared to 0 / 1.0).  Returns (rgba, depth) or, with tri_lit, (rgba, depth,
        float32 [n_tris, 4] lit rgb + area-test flag)."""
        rgba = np.zeros((height, width, 4), np.uint8) if rgba is None else rgba
        depth = np.ones((height, width), np.float32) if depth is None else depth
        assert rgba.shape == (height, width, 4) and rgba.dtype == np.uint8 and rgba.flags.c_contiguous
        assert depth.shape == (height, width) and depth.dtype == np.float32 and depth.flags.c_contiguous
        n = len(meshes)
        # shs_debug_mesh records (int32 mesh_id, float model[16], base_color[3]) built in numpy
        arr = np.zeros((max(n, 1), ctypes.sizeof(_abi.DebugMeshC) // 4), np.float32)
        n_tris = 0
        if n:
            arr[:n, 0].view(np.int32)[:] = [self.upload_lib_mesh(m[0]) for m in meshes]
            arr[:n, 1:17] = np.asarray([m[1] for m in meshes], np.float32).reshape(n, 16)
            arr[:n, 17:20] = np.asarray([m[2] for m in meshes], np.float32).reshape(n, 3)
            n_tris = sum(len(m[0].indices) // 3 for m in meshes)
        d = _abi.DebugDrawDescC()
        d.width, d.height = int(width), int(height)
        for k in range(16):
            d.view_proj[k] = float(view_proj[k])
        for k in range(3):
            d.camera_pos[k], d.light_dir_ws[k] = float(camera_pos[k]), float(light_dir_ws[k])
        lit = np.zeros((max(n_tris, 1), 4), np.float32) if tri_lit else None
        self._check(self._lib.shs_debug_draw_meshes(self._h, ctypes.byref(d), arr.ctypes.data_as(ctypes.POINTER(_abi.DebugMeshC)),
                                                    n, rgba.ctypes.data_as(ctypes.c_void_p),
                                                    depth.ctypes.data_as(ctypes.c_void_p),
                                                    None if lit is None else lit.ctypes.data_as(ctypes.c_void_p)))
        return (rgba, depth, lit[:n_tris]) if tri_lit else (rgba, depth)

    def debug_fill_triangles(self, width, height, screen, z, colors, rgba=None, depth=None):
        """debug_draw::draw_filled_triangle (debug_draw.hpp:60-109) for each triangle in order: screen
        float32 [n, 3, 2] points, z float32 [n, 3], colors uint8 [n, 4]."""
        rgba = np.zeros((height, width, 4), np.uint8) if rgba is None else rgba
        depth = np.ones((height, width), np.float32) if depth is None else depth
        assert rgba.shape == (height, width, 4) and rgba.dtype == np.uint8 and rgba.flags.c_contiguous
        assert depth.shape == (height, width) and depth.dtype == np.float32 and depth.flags.c_contiguous
        screen = np.asarray(screen, np.float32).reshape(-1, 6)
        n = screen.shape[0]
        rec = np.zeros((max(n, 1), ctypes.sizeof(_abi.DebugTriangleC) // 4), np.float32)
        rec[:n, 0:6] = screen
        rec[:n, 6:9] = np.asarray(z, np.float32).reshape(n, 3)
        rec[:n, 9].view(np.uint32)[:] = np.ascontiguousarray(colors, np.uint8).reshape(n, 4).view(np.uint32).reshape(n)
        self._check(self._lib.shs_debug_fill_triangles(self._h, int(width), int(height),
                                                       rec.ctypes.data_as(ctypes.POINTER(_abi.DebugTriangleC)), n,
                                                       rgba.ctypes.data_as(ctypes.c_void_p),
                                                       depth.ctypes.data_as(ctypes.c_void_p)))
        return rgba, depth

    CANVAS_DEVICE = 1

    def _on_torch_stream(self):
        """Device-tensor calls run on torch's current stream, so they are ordered after the torch work
        that wrote their inputs and before the torch work that reads their outputs (tensors allocated
        here, e.g. dst, belong to that stream too).  The context is re-pointed only when it is on
        another stream (shs_set_stream synchronises)."""
        import torch
        s = torch.cuda.current_stream().cuda_stream
        if self.stream != s:
            self.set_stream(s)

    def canvas_motion_blur(self, src, depth, velocity, curr_view, curr_proj, prev_view, prev_proj, samples=12,
                           strength=0.85, w_obj=1.0, w_cam=0.35, soft_knee=True, knee_px=18.0, max_px=22.0, dst=None):
        """combined_motion_blur_pass (hello_pbr.cpp:1128-1252).  Host arrays: src uint8 [H, W, 4], depth
        float32 [H, W] (view z), velocity float32 [H, W, 2] -> dst uint8 [H, W, 4].  torch CUDA tensors of
        the same shapes run on the device (asynchronous on the context stream)."""
        H, W = src.shape[:2]
        d = _abi.CanvasMotionBlurDescC()
        d.width, d.height = W, H
        for k in range(16):
            d.curr_view[k], d.curr_proj[k] = float(curr_view[k]), float(curr_proj[k])
            d.prev_view[k], d.prev_proj[k] = float(prev_view[k]), float(prev_proj[k])
        d.samples, d.strength, d.w_obj, d.w_cam = int(samples), float(strength), float(w_obj), float(w_cam)
        d.soft_knee, d.knee_px, d.max_px = 1 if soft_knee else 0, float(knee_px), float(max_px)
        dev = _is_device(src)
        if dev:
            self._on_torch_stream()
        if dst is None:
            dst = _empty_like(src)
        keep = (_host_c(src, np.uint8), _host_c(depth, np.float32), _host_c(velocity, np.float32), dst)
        self._check(self._lib.shs_canvas_motion_blur(self._h, ctypes.byref(d), *[_ptr(a) for a in keep],
                                                     self.CANVAS_DEVICE if dev else 0))
        return dst

    def canvas_gaussian_blur(self, src, horizontal, dst=None):
        """gaussian_blur_pass (hello_depth_of_field.cpp:175-251), one axis."""
        H, W = src.shape[:2]
        dev = _is_device(src)
        if dev:
            self._on_torch_stream()
        if dst is None:
            dst = _empty_like(src)
        src = _host_c(src, np.uint8)
        self._check(self._lib.shs_canvas_gaussian_blur(self._h, W, H, _ptr(src), _ptr(dst),
                                                       1 if horizontal else 0, self.CANVAS_DEVICE if dev else 0))
        return dst

    def canvas_dof(self, color, depth, iterations=3, radius=6, focus=None, range_=24.0, max_blur=0.6, blur=None):
        """The DoF step of hello_depth_of_field.cpp:786-812 on color (sharp in, composite out, in place)
        -> (color, blur, focus_depth)."""
        H, W = color.shape[:2]
        d = _abi.CanvasDofDescC()
        d.width, d.height, d.blur_iterations, d.autofocus_radius = W, H, int(iterations), int(radius)
        d.focus_x, d.focus_y = (W // 2, H // 2) if focus is None else focus
        d.range, d.max_blur = float(range_), float(max_blur)
        dev = _is_device(color)
        if dev:
            self._on_torch_stream()
        if blur is None:
            blur = _empty_like(color)
        f = ctypes.c_float()
        depth = _host_c(depth, np.float32)
        self._check(self._lib.shs_canvas_dof(self._h, ctypes.byref(d), _ptr(color), _ptr(depth),
                                             _ptr(blur), ctypes.byref(f), self.CANVAS_DEVICE if dev else 0))
        return color, blur, f.value

    def lib_device_targets(self):
        """Device pointers of the library targets: (hdr float4 W*H, depth W*H, motion float2 W*H)."""
        a, b, c = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p()
        self._check(self._lib.shs_lib_device_targets(self._h, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c)))
        return a.value, b.value, c.value

    def ldr_device_targets(self):
        a, b = ctypes.c_void_p(), ctypes.c_void_p()
        self._check(self._lib.shs_ldr_device_targets(self._h, ctypes.byref(a), ctypes.byref(b)))
        return a.value, b.value

    @staticmethod
    def tonemap_thresholds(gamma: float):
        """Host-side byte thresholds in x = c / (1 + c) (thr[0] = 0; +inf = byte never reached)."""
        thr = np.zeros(256, np.float32)
        rc = lib().shs_tonemap_thresholds(float(gamma), thr.ctypes.data_as(ctypes.POINTER(ctypes.c_float)))
        if rc != 0:
            raise ShsError(rc, "shs_tonemap_thresholds")
        return thr

    @staticmethod
    def shard_balance(blocks, width, height, count, root_share=1.0):
        """Host-side region balance (shs_shard_balance_rects): blocks uint32 [n, 4] as k_lib_setup writes them
        -> [(bx0, by0, bx1, by1)] per rank."""
        b = np.ascontiguousarray(np.asarray(blocks, np.uint32).reshape(-1, 4))
        out = np.zeros(4 * count, np.int32)
        rc = lib().shs_shard_balance_rects(b.ctypes.data if b.size else None, b.shape[0], int(width), int(height), int(count),
                                           int(round(root_share * 1000)), out.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)))
        if rc != 0:
            raise ShsError(rc, "shs_shard_balance_rects")
        return [tuple(int(v) for v in out[4 * r:4 * r + 4]) for r in range(count)]

    @staticmethod
    def shadow_footprint(light_vp, sm_size, camera_vp, width, height, px_rect, world_min, world_max, reach):
        """Host-side footprint (shs_shadow_footprint): the texel rectangle (x0, y0, x1, y1), inclusive, of an
        sm_size = (w, h) shadow map that PCF of `reach` texels reads from the points of the world box whose
        camera projection lands on px_rect (x0, y0, x1, y1; rows y up) of a width x height frame."""
        sw, sh = (sm_size, sm_size) if isinstance(sm_size, int) else sm_size
        f16 = lambda m: np.ascontiguousarray(np.asarray(m, np.float32).reshape(16))
        f3 = lambda v: np.ascontiguousarray(np.asarray(v, np.float32).reshape(3))
        lv, cv, b0, b1 = f16(light_vp), f16(camera_vp), f3(world_min), f3(world_max)
        px = np.ascontiguousarray(np.asarray(px_rect, np.int32).reshape(4))
        out = np.zeros(4, np.int32)
        rc = lib().shs_shadow_footprint(lv.ctypes.data, int(sw), int(sh), cv.ctypes.data, int(width), int(height),
                                        px.ctypes.data, b0.ctypes.data, b1.ctypes.data, int(reach), out.ctypes.data)
        if rc != 0:
            raise ShsError(rc, "shs_shadow_footprint")
        return tuple(int(v) for v in out)

    @staticmethod
    def shadow_footprint_rows(light_vp, sm_size, camera_vp, width, height, px_rect, world_min, world_max, reach,
                              row_h=32):
        """shs_shadow_footprint_rows: per row of row_h texels the read texel columns -> (x0[], x1[]) int32
        arrays (x1 < x0: none), from the footprint polytope's convex light-space image."""
        sw, sh = (sm_size, sm_size) if isinstance(sm_size, int) else sm_size
        f16 = lambda m: np.ascontiguousarray(np.asarray(m, np.float32).reshape(16))
        f3 = lambda v: np.ascontiguousarray(np.asarray(v, np.float32).reshape(3))
        lv, cv, b0, b1 = f16(light_vp), f16(camera_vp), f3(world_min), f3(world_max)
        px = np.ascontiguousarray(np.asarray(px_rect, np.int32).reshape(4))
        n_rows = (int(sh) + row_h - 1) // row_h
        x0, x1 = np.zeros(n_rows, np.int32), np.zeros(n_rows, np.int32)
        rc = lib().shs_shadow_footprint_rows(lv.ctypes.data, int(sw), int(sh), cv.ctypes.data, int(width), int(height),
                                             px.ctypes.data, b0.ctypes.data, b1.ctypes.data, int(reach), int(row_h),
                                             n_rows, x0.ctypes.data, x1.ctypes.data)
        if rc != 0:
            raise ShsError(rc, "shs_shadow_footprint_rows")
        return x0, x1

    LIB_TIMELINE_FIELDS = ("start", "end", "gather", "pairs", "shade", "clear", "n_busy", "n_clear", "chunks",
                           "n_pairs", "n_cand", "max_tile", "stage", "seg", "tiles", "last",
                           "mt_rt", "mt_items", "mt_rounds", "mt_passes", "mt_staged", "mt_pairs", "mt_gather",
                           "mt_breaks")

    def lib_debug_timeline(self):
        """Last camera pass's k_lib_raster workgroup timeline: uint64 [grid, 24] (LIB_TIMELINE_FIELDS;
        times in 10-ns ticks; mt_*: the workgroup's longest busy tile)."""
        n = ctypes.c_int64()
        self._check(self._lib.shs_lib_debug_timeline(self._h, None, 0, ctypes.byref(n)))
        out = np.zeros(n.value, dtype=np.uint64)
        self._check(self._lib.shs_lib_debug_timeline(self._h, out.ctypes.data_as(ctypes.c_void_p), n.value, ctypes.byref(n)))
        return out.reshape(-1, len(self.LIB_TIMELINE_FIELDS))

    def lib_debug_setup_timeline(self):
        """Last camera pass's k_lib_setup workgroup timeline: uint64 [blocks, 8] (start, triangles done,
        deferred marks done, end in 10-ns ticks; large primitives; deferred union w*h; tile-sharded cull
        front end done (0 without it); kept triangles)."""
        n = ctypes.c_int64()
        self._check(self._lib.shs_lib_debug_setup_timeline(self._h, None, 0, ctypes.byref(n)))
        out = np.zeros(n.value, dtype=np.uint64)
        self._check(self._lib.shs_lib_debug_setup_timeline(self._h, out.ctypes.data_as(ctypes.c_void_p), n.value,
                                                           ctypes.byref(n)))
        return out.reshape(-1, 8)

    def debug_timeline(self):
        """Last frame's workgroup timeline: (header dict, setup [n,2], raster [n,2]) in 10-ns ticks."""
        n = ctypes.c_int64()
        self._check(self._lib.shs_debug_timeline(self._h, None, 0, ctypes.byref(n)))
        out = np.zeros(n.value, dtype=np.uint64)
        self._check(self._lib.shs_debug_timeline(self._h, out.ctypes.data_as(ctypes.c_void_p), n.value, ctypes.byref(n)))
        hs, hr, stride = int(out[0]), int(out[1]), int(out[5])
        head = {"setup_grid": hs, "raster_grid": hr, "setup_blocks": int(out[2]), "ghost_blocks": int(out[3]),
                "clear_blocks": int(out[4])}
        slots = out[8:].reshape(-1, stride)
        return head, slots[:hs], slots[hs:hs + hr]

    def set_bin_capacity(self, cap: int):
        self._check(self._lib.shs_set_option(self._h, _abi.OPT_BIN_CAPACITY, int(cap)))

    def set_lib_part(self, part: int):
        """Camera-pass raster work split (SHS_OPT_LIB_PART): -1 auto (512 when sharded), 0 off (default), else the part size."""
        self._check(self._lib.shs_set_option(self._h, _abi.OPT_LIB_PART, int(part)))

    def set_shard_cull(self, on: bool):
        """SHS_OPT_SHARD_CULL: tile-sharded camera passes set up only the rank's triangles (default off)."""
        self._check(self._lib.shs_set_option(self._h, _abi.OPT_SHARD_CULL, 1 if on else 0))

    def set_shard_layout(self, regions: bool):
        """SHS_OPT_SHARD_LAYOUT: tile-sharded library frames own interleaved 32x32 tiles (default) or one
        cost-balanced rectangle per rank (regions=True)."""
        self._check(self._lib.shs_set_option(self._h, _abi.OPT_SHARD_LAYOUT,
                                             _abi.SHARD_REGIONS if regions else _abi.SHARD_INTERLEAVED))

    def set_shard_root_share(self, share: float):
        """SHS_OPT_SHARD_ROOT_SHARE: rank 0's share of a region layout relative to the others (0..1)."""
        self._check(self._lib.shs_set_option(self._h, _abi.OPT_SHARD_ROOT_SHARE, int(round(share * 1000))))

    def set_legacy_pipeline(self, on: bool):
        """SHS_OPT_LEGACY_PIPELINE: a multi-draw scan-mode batch's raster runs in the next batch's launch
        (or at the next call that reads frames); results identical, frames final only after such a call."""
        self._check(self._lib.shs_set_option(self._h, _abi.OPT_LEGACY_PIPELINE, 1 if on else 0))

    def set_shadow_footprint(self, on: bool):
        """SHS_OPT_SHADOW_FOOTPRINT: shadow passes are recorded and rendered by the next camera pass over
        only the shadow-map tiles its pixels' PCF can read (default off: the whole map when called)."""
        self._check(self._lib.shs_set_option(self._h, _abi.OPT_SHADOW_FOOTPRINT, 1 if on else 0))

    def shadow_region(self):
        """The last enqueued shadow pass's bin tiles (bx0, by0, bx1, by1), inclusive; bx1 < bx0: none."""
        arr = (ctypes.c_int32 * 4)()
        self._check(self._lib.shs_get_shadow_region(self._h, arr))
        return tuple(arr)

    def shard_regions(self, count):
        """The last region-sharded camera pass's layout: [(bx0, by0, bx1, by1)] per rank (bin tiles, inclusive)."""
        arr = (ctypes.c_int32 * (4 * count))()
        self._check(self._lib.shs_get_shard_regions(self._h, count, arr))
        return [tuple(arr[4 * r:4 * r + 4]) for r in range(count)]

    def set_overflow_capacities(self, spill: int = 0, frags: int = 0):
        """Tests: shrink the legacy bin-spill / ghost-fragment lists (0 = leave) to force overflows."""
        if spill:
            self._check(self._lib.shs_set_option(self._h, _abi.OPT_SPILL_CAPACITY, int(spill)))
        if frags:
            self._check(self._lib.shs_set_option(self._h, _abi.OPT_FRAG_CAPACITY, int(frags)))

    def set_stream(self, hip_stream):
        self._check(self._lib.shs_set_stream(self._h, ctypes.c_void_p(hip_stream)))

    # -- library path (rasterize_mesh / PassShadowMap / PassPBRForward) ---------------------------
    def share_lib_mesh(self, src, mesh) -> int:
        """A handle to src's device copy of library mesh `mesh` (uploaded there if it is not yet), so
        that later draws of `mesh` on this context read src's buffers (shs_mesh_share: frames in flight
        on several contexts keep one copy).  src must outlive this context's use of it."""
        key = ("lib", id(mesh))
        if key in self._meshes:
            return self._meshes[key][0]
        sid = src.upload_lib_mesh(mesh)
        mid = ctypes.c_int32()
        self._check(self._lib.shs_mesh_share(self._h, src._h, sid, ctypes.byref(mid)))
        self._meshes[key] = (mid.value, mesh)
        return mid.value

    def upload_lib_mesh(self, mesh) -> int:
        key = ("lib", id(mesh))
        if key in self._meshes:
            return self._meshes[key][0]
        pos = np.ascontiguousarray(mesh.positions, dtype=np.float32).reshape(-1, 3)
        nrm = None if mesh.normals is None else np.ascontiguousarray(mesh.normals, dtype=np.float32).reshape(-1, 3)
        uv = None if mesh.uvs is None else np.ascontiguousarray(mesh.uvs, dtype=np.float32).reshape(-1, 2)
        idx = None if mesh.indices is None else np.ascontiguousarray(mesh.indices, dtype=np.uint32).reshape(-1)
        mid = ctypes.c_int32()
        self._check(self._lib.shs_mesh_upload(
            self._h, _fptr(pos), pos.shape[0],
            _fptr(nrm) if nrm is not None else None, 0 if nrm is None else nrm.shape[0],
            _fptr(uv) if uv is not None else None, 0 if uv is None else uv.shape[0],
            idx.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)) if idx is not None else None,
            0 if idx is None else idx.size, ctypes.byref(mid)))
        self._meshes[key] = (mid.value, mesh)
        return mid.value

    def render_shadow_map(self, size, sun_dir, casters):
        """PassShadowMap::execute -> the light camera's viewproj (float32[16])."""
        from ._abi import ShadowCasterC
        w, h = (size, size) if isinstance(size, int) else size
        arr = (ShadowCasterC * max(len(casters), 1))()
        for i, c in enumerate(casters):
            arr[i].mesh_id = c.mesh if isinstance(c.mesh, int) else self.upload_lib_mesh(c.mesh)
            for k in range(16):
                arr[i].model[k] = float(c.model[k])
        sd = np.ascontiguousarray(sun_dir, dtype=np.float32).reshape(3)
        vp = np.zeros(16, np.float32)
        self._check(self._lib.shs_render_shadow_map(self._h, w, h, _fptr(sd), arr, len(casters), _fptr(vp)))
        self._shadow_size = (w, h)
        return vp

    def resolve_shadow_map(self):
        w, h = self._shadow_size
        out = np.empty((h, w), np.float32)
        self._check(self._lib.shs_resolve_shadow_map(self._h, out.ctypes.data_as(ctypes.c_void_p)))
        return out

    def upload_texture(self, tex) -> int:
        """shs_texture_upload of a lib_path.Texture2D (cached per object) -> texture id (>= 1)."""
        key = ("tex", id(tex))
        if key in self._meshes:
            return self._meshes[key][0]
        rgba = np.ascontiguousarray(tex.rgba, dtype=np.uint8)
        assert rgba.ndim == 3 and rgba.shape[2] == 4
        tid = ctypes.c_int32()
        self._check(self._lib.shs_texture_upload(self._h, rgba.ctypes.data_as(ctypes.c_void_p), rgba.shape[1],
                                                 rgba.shape[0], ctypes.byref(tid)))
        self._meshes[key] = (tid.value, tex)
        return tid.value

    def prepare_lib(self, frame, draws):
        from ._abi import LibDrawC
        from .lib_path import fill_draw_struct
        arr = (LibDrawC * max(len(draws), 1))()
        for i, d in enumerate(draws):
            tex = getattr(d, "base_color_tex", None)
            fill_draw_struct(arr[i], d, d.mesh if isinstance(d.mesh, int) else self.upload_lib_mesh(d.mesh),
                             0 if tex is None else self.upload_texture(tex))
        return frame, frame.desc(), arr, len(draws)

    def render_pbr_forward_prepared(self, prepared):
        frame, desc, arr, n = prepared
        self._check(self._lib.shs_render_pbr_forward(self._h, ctypes.byref(desc), arr, n))
        self._lib_frame = frame

    def render_pbr_forward(self, frame, draws):
        """PassPBRForward::execute: clears + one rasterize_mesh per draw (asynchronous)."""
        self.render_pbr_forward_prepared(self.prepare_lib(frame, draws))

    def resolve_lib(self):
        """-> (hdr float32[H,W,4], depth float32[H,W] or None, motion float32[H,W,2] or None), rows y-up."""
        f = self._lib_frame
        hdr = np.empty((f.height, f.width, 4), np.float32)
        depth = np.empty((f.height, f.width), np.float32) if f.depth_motion else None
        motion = np.empty((f.height, f.width, 2), np.float32) if f.depth_motion else None
        vp = ctypes.c_void_p
        self._check(self._lib.shs_resolve_lib(self._h, hdr.ctypes.data_as(vp),
                                              depth.ctypes.data_as(vp) if depth is not None else None,
                                              motion.ctypes.data_as(vp) if motion is not None else None))
        return hdr, depth, motion

    def synchronize_lib(self):
        """Wait for the enqueued library passes (re-issues a pass whose capacity overflowed)."""
        from ._abi import LibStats
        if self._lib_frame is not None:
            self._check(self._lib.shs_get_lib_stats(self._h, ctypes.byref(LibStats())))
        elif self._shadow_size is not None:
            self.resolve_shadow_map()

    # -- tile shards (multi-GPU gather) ----------------------------------------------------------
    TARGET_LEGACY, TARGET_LIB, TARGET_PRESENT, TARGET_LIB_PRESENT = 0, 1, 2, 3

    def tiles_packed_words(self, target, count):
        """Packed words of the largest rank's tiles (a buffer size every rank's tiles fit)."""
        n = ctypes.c_int64()
        self._check(self._lib.shs_tiles_packed_words(self._h, target, count, ctypes.byref(n)))
        return n.value

    def tiles_rank_words(self, target, rank, count):
        """Packed words of rank's own tiles (region layouts differ per rank)."""
        n = ctypes.c_int64()
        self._check(self._lib.shs_tiles_rank_words(self._h, target, rank, count, ctypes.byref(n)))
        return n.value

    def tiles_pack(self, target, rank, count, dst_ptr):
        """Pack rank's owned tiles into the device buffer at dst_ptr (e.g. tensor.data_ptr())."""
        self._check(self._lib.shs_tiles_pack(self._h, target, rank, count, ctypes.c_void_p(dst_ptr)))

    def tiles_unpack(self, target, rank, count, src_ptr):
        self._check(self._lib.shs_tiles_unpack(self._h, target, rank, count, ctypes.c_void_p(src_ptr)))

    def tiles_unpack_ranks(self, target, count, src_ptrs):
        """shs_tiles_unpack_ranks: every rank's packed device buffer (src_ptrs[r]; 0 / None skips rank r)
        unpacked into this context's frame by one launch."""
        arr = (ctypes.c_void_p * count)(*[int(p) if p else None for p in src_ptrs])
        self._check(self._lib.shs_tiles_unpack_ranks(self._h, int(target), int(count), arr))

    def upload_lights(self, lights):
        """lights: numpy LIGHT_DTYPE array (CullingLightGPU records)."""
        from ._abi import CullingLightC
        arr = np.ascontiguousarray(lights)
        self._check(self._lib.shs_lights_upload(self._h, arr.ctypes.data_as(ctypes.POINTER(CullingLightC)), arr.shape[0]))
        self._n_lights = arr.shape[0]

    def light_cull(self, cull):
        """fp_stress_light_cull.comp (+ depth reduce for mode 2) into the context's tile lists."""
        self._cull = cull
        self._check(self._lib.shs_light_cull(self._h, ctypes.byref(cull.desc())))

    def resolve_light_lists(self):
        """-> (counts uint32[n_lists], indices uint32[n_lists, max_per_tile], ranges float32[tiles, 2])."""
        c = self._cull
        counts = np.empty(c.n_lists, np.uint32)
        idx = np.empty((c.n_lists, c.max_per_tile), np.uint32)
        tx, ty = c.tiles
        ranges = np.empty((ty * tx, 2), np.float32)
        vp = ctypes.c_void_p
        self._check(self._lib.shs_resolve_light_lists(self._h, counts.ctypes.data_as(vp), idx.ctypes.data_as(vp),
                                                      ranges.ctypes.data_as(vp)))
        return counts, idx, ranges

    def light_bin_culling(self, lb, aabbs):
        """build_light_bin_culling on the GPU: lb = lib_path.LightBin, aabbs float32 [n, 6] (min, max) ->
        (bins_xyz, counts uint32 [bins], indices uint32 [bins, cap])."""
        aabbs = np.ascontiguousarray(aabbs, dtype=np.float32).reshape(-1, 6)
        keep = []
        d = lb.desc(aabbs.shape[0], keep)
        ts = max(lb.tile_size, 1)
        bx, by = (lb.width + ts - 1) // ts, (lb.height + ts - 1) // ts
        n_bins = bx * by * (max(lb.z_slices, 1) if lb.mode == 3 else 1)
        counts = np.zeros(n_bins, np.uint32)
        idx = np.zeros((n_bins, d.max_per_bin), np.uint32)
        bins = np.zeros(3, np.uint32)
        self._check(self._lib.shs_light_bin_culling(self._h, ctypes.byref(d), aabbs.ctypes.data, aabbs.shape[0],
                                                    bins.ctypes.data, counts.ctypes.data, idx.ctypes.data))
        return tuple(int(b) for b in bins), counts, idx

    def lib_timing_reset(self):
        self._check(self._lib.shs_lib_timing_reset(self._h))

    def lib_timing_read(self):
        """-> ({shadow, camera} pass counts, {kernel: mean ms}) since lib_timing_reset()."""
        s = (ctypes.c_double * 4)()
        n = (ctypes.c_int64 * 2)()
        self._check(self._lib.shs_lib_timing_read(self._h, s, n))
        ns, nc = max(n[0], 1), max(n[1], 1)
        return {"shadow": n[0], "camera": n[1]}, {"shadow_setup": s[0] / ns, "shadow_raster": s[1] / ns,
                                                    "setup": s[2] / nc, "raster": s[3] / nc}

    def lib_stats(self) -> dict:
        from ._abi import LibStats
        s = LibStats()
        self._check(self._lib.shs_get_lib_stats(self._h, ctypes.byref(s)))
        return {k: int(getattr(s, k)) for k, _ in LibStats._fields_}

    @property
    def stream(self):
        return self._lib.shs_get_stream(self._h)


def _is_device(a):
    return hasattr(a, "is_cuda") and a.is_cuda


def _empty_like(a):
    if _is_device(a):
        import torch
        return torch.empty_like(a)
    return np.empty_like(a)


def _host_c(a, dtype):
    return a if _is_device(a) else np.ascontiguousarray(a, dtype=dtype)


def _ptr(a):
    if _is_device(a):
        assert a.is_contiguous()
        return ctypes.c_void_p(a.data_ptr())
    assert a.flags.c_contiguous
    return a.ctypes.data_as(ctypes.c_void_p)
