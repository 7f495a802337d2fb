"""Multi-GPU from one host process: the shs_group_* C ABI (include/shs_gpu.h).

n contexts (rank r on devices[r]; a device may repeat) render the interleaved 32x32 tiles of every
frame (tile % n == r); `gather(target)` composes the frame on rank 0's context with peer copies
(xGMI between MI355X devices), after which rank 0's context resolves the full frame with the usual
single-context calls.  This is the path a single-process C++ host (the reference's render loop,
hello_pipeline_blinn_phong_shading.cpp:369-455) uses; `shard.py` is the one-process-per-GPU variant.
"""
import ctypes

import numpy as np

from . import Context, ShsError, _abi, _fptr
from .lib_path import fill_draw_struct


class _RankContext(Context):
    """A non-owning view of a group rank's context (the group destroys it)."""

    def __init__(self, lib, handle):  # noqa: D401  (no shs_create)
        self._lib = lib
        self._h = handle
        self._meshes = {}
        self._frame = None
        self._lib_frame = None
        self._shadow_size = None

    def close(self):
        self._h = None


class Group:
    def __init__(self, devices):
        self._lib = _abi.lib()
        devs = (ctypes.c_int32 * len(devices))(*devices)
        h = ctypes.c_void_p()
        rc = self._lib.shs_group_create(devs, len(devices), ctypes.byref(h))
        if rc != 0:
            raise ShsError(rc, f"shs_group_create({list(devices)}) failed")
        self._h = h
        self.n = len(devices)
        self._ids = {}
        self.ranks = []
        for r in range(self.n):
            c = ctypes.c_void_p()
            self._check(self._lib.shs_group_context(self._h, r, ctypes.byref(c)))
            self.ranks.append(_RankContext(self._lib, c))

    def _check(self, rc):
        if rc != 0:
            raise ShsError(rc, self._lib.shs_group_last_error(self._h).decode(errors="replace"))

    def close(self):
        if getattr(self, "_h", None):
            for r in self.ranks:
                r.close()
            self._lib.shs_group_destroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def root(self) -> Context:
        """Rank 0's context: resolves the composed frame after gather()."""
        return self.ranks[0]

    # -- replicated uploads -----------------------------------------------------------------------
    def upload_lib_mesh(self, mesh) -> int:
        key = ("lib", id(mesh))
        if key in self._ids:
            return self._ids[key][0]
        pos = np.ascontiguousarray(mesh.positions, dtype=np.float32).reshape(-1, 3)
        nrm = None if mesh.normals is None else np.ascontiguousarray(mesh.normals, dtype=np.float32).reshape(-1, 3)
        uv = None if mesh.uvs is None else np.ascontiguousarray(mesh.uvs, dtype=np.float32).reshape(-1, 2)
        idx = None if mesh.indices is None else np.ascontiguousarray(mesh.indices, dtype=np.uint32).reshape(-1)
        mid = ctypes.c_int32()
        self._check(self._lib.shs_group_mesh_upload(
            self._h, _fptr(pos), pos.shape[0], _fptr(nrm) if nrm is not None else None, 0 if nrm is None else nrm.shape[0],
            _fptr(uv) if uv is not None else None, 0 if uv is None else uv.shape[0],
            idx.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)) if idx is not None else None,
            0 if idx is None else idx.size, ctypes.byref(mid)))
        self._ids[key] = (mid.value, mesh)
        return mid.value

    def upload_mesh(self, mesh) -> int:
        key = ("soup", id(mesh))
        if key in self._ids:
            return self._ids[key][0]
        pos = np.ascontiguousarray(mesh.positions, dtype=np.float32)
        nrm = np.ascontiguousarray(mesh.normals, dtype=np.float32)
        mid = ctypes.c_int32()
        self._check(self._lib.shs_group_mesh_upload_soup(self._h, _fptr(pos), _fptr(nrm), pos.shape[0], ctypes.byref(mid)))
        self._ids[key] = (mid.value, mesh)
        return mid.value

    def upload_texture(self, tex) -> int:
        key = ("tex", id(tex))
        if key in self._ids:
            return self._ids[key][0]
        rgba = np.ascontiguousarray(tex.rgba, dtype=np.uint8)
        tid = ctypes.c_int32()
        self._check(self._lib.shs_group_texture_upload(self._h, rgba.ctypes.data_as(ctypes.c_void_p), rgba.shape[1],
                                                       rgba.shape[0], ctypes.byref(tid)))
        self._ids[key] = (tid.value, tex)
        return tid.value

    def upload_lights(self, lights):
        arr = np.ascontiguousarray(lights)
        self._check(self._lib.shs_group_lights_upload(self._h, arr.ctypes.data_as(ctypes.POINTER(_abi.CullingLightC)),
                                                      arr.shape[0]))

    def fuse_tonemap(self, exposure=1.0, gamma=2.2, ldr=True, present=True):
        d = _abi.TonemapDescC()
        d.exposure, d.gamma = float(exposure), float(gamma)
        d.flags = (_abi.TONEMAP_LDR if ldr else 0) | (_abi.TONEMAP_PRESENT if present else 0)
        self._check(self._lib.shs_group_lib_fuse_tonemap(self._h, ctypes.byref(d)))
        for r in self.ranks:
            r._tonemap_flags = d.flags

    def set_option(self, option, value):
        """shs_group_set_option: shs_set_option on every rank's context."""
        self._check(self._lib.shs_group_set_option(self._h, int(option), int(value)))

    def set_shard_layout(self, regions: bool, root_share: float = None):
        """SHS_OPT_SHARD_LAYOUT on every rank: interleaved tiles (default) or one cost-balanced rectangle
        per rank; root_share: SHS_OPT_SHARD_ROOT_SHARE (rank 0's share, it also composes the gather)."""
        self.set_option(_abi.OPT_SHARD_LAYOUT, _abi.SHARD_REGIONS if regions else _abi.SHARD_INTERLEAVED)
        if root_share is not None:
            self.set_option(_abi.OPT_SHARD_ROOT_SHARE, int(round(root_share * 1000)))

    # -- sharded passes ---------------------------------------------------------------------------
    def light_cull(self, cull):
        self._check(self._lib.shs_group_light_cull(self._h, ctypes.byref(cull.desc())))
        for r in self.ranks:
            r._cull = cull

    def render_shadow_map(self, size, sun_dir, casters):
        w, h = (size, size) if isinstance(size, int) else size
        arr = (_abi.ShadowCasterC * max(len(casters), 1))()
        for i, c in enumerate(casters):
            arr[i].mesh_id = self.upload_lib_mesh(c.mesh)
            for k in range(16):
                arr[i].model[k] = float(c.model[k])
        sd = np.ascontiguousarray(sun_dir, dtype=np.float32).reshape(3)
        vp = np.zeros(16, np.float32)
        self._check(self._lib.shs_group_render_shadow_map(self._h, w, h, _fptr(sd), arr, len(casters), _fptr(vp)))
        for r in self.ranks:
            r._shadow_size = (w, h)
        return vp

    def prepare_lib(self, frame, draws):
        arr = (_abi.LibDrawC * max(len(draws), 1))()
        for i, d in enumerate(draws):
            tex = getattr(d, "base_color_tex", None)
            fill_draw_struct(arr[i], d, self.upload_lib_mesh(d.mesh), 0 if tex is None else self.upload_texture(tex))
        return frame, frame.desc(), arr, len(draws)

    def render_pbr_forward_prepared(self, prepared):
        frame, desc, arr, n = prepared
        self._check(self._lib.shs_group_render_pbr_forward(self._h, ctypes.byref(desc), arr, n))
        for r in self.ranks:
            r._lib_frame = frame

    def render_pbr_forward(self, frame, draws):
        self.render_pbr_forward_prepared(self.prepare_lib(frame, draws))

    def render(self, frame, draws):
        """Sharded legacy frame (shs_render_legacy on every rank)."""
        arr = (_abi.LegacyDraw * max(len(draws), 1))()
        for i, d in enumerate(draws):
            a = arr[i]
            a.mesh_id = self.upload_mesh(d.mesh)
            a.shading = int(d.shading)
            for k in range(16):
                a.mvp[k], a.model[k] = float(d.mvp[k]), float(d.model[k])
            for k in range(3):
                a.light_dir[k], a.camera_pos[k] = float(d.light_dir[k]), float(d.camera_pos[k])
            for k in range(4):
                a.color[k] = int(d.color[k])
        desc = frame.desc()
        self._check(self._lib.shs_group_render_legacy(self._h, ctypes.byref(desc), arr, len(draws)))
        for r in self.ranks:
            r._frame = frame

    def gather(self, target):
        self._check(self._lib.shs_group_gather(self._h, int(target)))

    def synchronize(self):
        self._check(self._lib.shs_group_synchronize(self._h))
