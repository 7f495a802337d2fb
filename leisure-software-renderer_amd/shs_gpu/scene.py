"""Synthetic scenes for BASELINE.json configs, built with the reference's own scene constants.

Configs (BASELINE.json "configs"):
  C1  Suzanne Blinn-Phong + z-buffer, 800x600            (hello_pipeline_blinn_phong_shading.cpp:152-153)
  C2  Suzanne Blinn-Phong + z-buffer, 1920x1080
  C3  64-instance Suzanne grid, Phong, 1920x1080        (grid generalising hello_flat_shading_xsimd.cpp:125-128,
                                                          Phong light from hello_pipeline_phong_shading.cpp:163)
Camera: shs::Viewer((0,5,-20), 50, W, H) -> Camera3D fov 60, zn 0.1, zf 1000, aspect 4/3 (sic,
shs_renderer.hpp:1234, 1323-1337).  Uniform matrices are built by the GLM restatement in
libshs_gpu (shs_camera3d / shs_model_trs / shs_mat4_mul); vector normalisations below follow
glm::normalize in float32 (v * (1/sqrt(dot(v,v))), dot = (x*x + y*y) + z*z).
"""
import ctypes
import os
import struct
from dataclasses import dataclass

import numpy as np

from . import _abi
from . import Draw, Frame, SHADING_BLINN_PHONG, SHADING_FLAT, SHADING_GOURAUD, SHADING_PHONG

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
ASSETS = os.path.join(REPO, "assets")

f32 = np.float32


@dataclass(eq=False)
class Mesh:
    positions: np.ndarray   # float32 [n, 9]
    normals: np.ndarray     # float32 [n, 9]

    @property
    def n_tris(self):
        return int(self.positions.shape[0])


_MONKEY = None


def load_soup(path):
    with open(path, "rb") as fh:
        magic = fh.read(8)
        if magic != b"SHSSOUP1":
            raise ValueError(f"{path}: not a SHSSOUP1 file")
        n, _ = struct.unpack("<II", fh.read(8))
        pos = np.frombuffer(fh.read(36 * n), dtype="<f4").reshape(n, 9).astype(np.float32)
        nrm = np.frombuffer(fh.read(36 * n), dtype="<f4").reshape(n, 9).astype(np.float32)
    return Mesh(pos, nrm)


def monkey() -> Mesh:
    """Suzanne (967 triangles) from assets/monkey.soup.bin (tools/convert_obj.py)."""
    global _MONKEY
    if _MONKEY is None:
        _MONKEY = load_soup(os.path.join(ASSETS, "monkey.soup.bin"))
    return _MONKEY


# ---- float32 GLM helpers ------------------------------------------------------------------
def glm_normalize(v):
    x, y, z = (f32(c) for c in v)
    d = (x * x + y * y) + z * z
    inv = f32(1.0) / np.sqrt(d)
    return np.array([x * inv, y * inv, z * inv], dtype=np.float32)


def glm_m4v4(m, v):
    """glm mat4 * vec4: (m0*x + m1*y) + (m2*z + m3*w)."""
    m = np.asarray(m, dtype=np.float32)
    x, y, z, w = (f32(c) for c in v)
    return np.array([(m[0 + r] * x + m[4 + r] * y) + (m[8 + r] * z + m[12 + r] * w) for r in range(4)], dtype=np.float32)


def _fp(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))


def camera(position=(0.0, 5.0, -20.0), yaw=0.0, pitch=0.0, fov=60.0, zn=0.1, zf=1000.0):
    """Camera3D::update via the library's GLM restatement -> (view, proj) float32[16]."""
    lib = _abi.lib()
    pos = np.asarray(position, dtype=np.float32)
    view = np.zeros(16, np.float32)
    proj = np.zeros(16, np.float32)
    rc = lib.shs_camera3d(_fp(pos), yaw, pitch, fov, zn, zf, _fp(view), _fp(proj))
    assert rc == 0
    return view, proj


def model_trs(position, rot_deg_y, scale):
    lib = _abi.lib()
    p = np.asarray(position, dtype=np.float32)
    s = np.asarray(scale, dtype=np.float32)
    out = np.zeros(16, np.float32)
    assert lib.shs_model_trs(_fp(p), rot_deg_y, _fp(s), _fp(out)) == 0
    return out


def mat_mul(a, b):
    lib = _abi.lib()
    a = np.ascontiguousarray(a, dtype=np.float32)
    b = np.ascontiguousarray(b, dtype=np.float32)
    out = np.zeros(16, np.float32)
    assert lib.shs_mat4_mul(_fp(a), _fp(b), _fp(out)) == 0
    return out


def make_draw(mesh, shading, model, view, proj, light_world, camera_pos, color):
    """Uniforms exactly as RendererSystem::process builds them (blinn_phong_shading.cpp:277-282;
    flat_shading.cpp:282-286 for the Flat pipeline's mv / light_dir_view)."""
    pv = mat_mul(proj, view)
    if shading == SHADING_FLAT:
        mv = mat_mul(view, model)
        mvp = mat_mul(proj, mv)
        ldv = glm_normalize(glm_m4v4(view, (*light_world, 0.0))[:3])
        return Draw(mesh, shading, mvp, mv, ldv, np.asarray(camera_pos, np.float32), tuple(color))
    mvp = mat_mul(pv, model)
    return Draw(mesh, shading, mvp, model, np.asarray(light_world, np.float32), np.asarray(camera_pos, np.float32),
                tuple(color))


CAM_POS = (0.0, 5.0, -20.0)
LIGHT_BLINN = (-1.0, -0.4, 1.0)   # blinn_phong_shading.cpp:152 (also Gouraud :148)
LIGHT_PHONG = (1.0, 1.0, -1.0)    # phong_shading.cpp:163 (also Flat :153)
COLOR_BLUE = (60, 100, 200, 255)  # blinn_phong_shading.cpp:153
COLOR_FLAT = (100, 150, 255, 255) # flat_shading.cpp:156


def monkey_scene(width, height, shading=SHADING_BLINN_PHONG, yaw=0.0, pitch=0.0, rotation=0.0, cam_pos=CAM_POS):
    """C1/C2 (and the Phong/Gouraud/Flat single-monkey demos): one Suzanne at (0,0,10), scale 4."""
    mesh = monkey()
    view, proj = camera(cam_pos, yaw, pitch)
    model = model_trs((0.0, 0.0, 10.0), rotation, (4.0, 4.0, 4.0))
    if shading in (SHADING_BLINN_PHONG, SHADING_GOURAUD):
        light, color = LIGHT_BLINN, COLOR_BLUE
    elif shading == SHADING_PHONG:
        light, color = LIGHT_PHONG, COLOR_BLUE
    else:
        light, color = LIGHT_PHONG, COLOR_FLAT
    light = glm_normalize(light)
    return Frame(width, height), [make_draw(mesh, shading, model, view, proj, light, cam_pos, color)]


def grid_scene(width=1920, height=1080, n=8, step=15.0, scale=5.0, shading=SHADING_PHONG, yaw=0.0, pitch=0.0,
               cam_pos=CAM_POS):
    """C3: n x n Suzanne instances at (i*step - off, 0, j*step + 20), off = step*(n-1)/2 (the xsimd demo's
    2x2 grid has off = 7.5), i outer / j inner submission order, scale 5, Phong."""
    mesh = monkey()
    view, proj = camera(cam_pos, yaw, pitch)
    off = step * (n - 1) / 2.0
    light = glm_normalize(LIGHT_PHONG)
    draws = []
    for i in range(n):
        for j in range(n):
            model = model_trs((i * step - off, 0.0, j * step + 20.0), 0.0, (scale, scale, scale))
            draws.append(make_draw(mesh, shading, model, view, proj, light, cam_pos, COLOR_BLUE))
    return Frame(width, height), draws


def config(name, **kw):
    name = name.lower()
    if name == "c1":
        return monkey_scene(800, 600, SHADING_BLINN_PHONG, **kw)
    if name == "c2":
        return monkey_scene(1920, 1080, SHADING_BLINN_PHONG, **kw)
    if name == "c3":
        return grid_scene(1920, 1080, **kw)
    raise KeyError(name)


def build_named(spec):
    """Rebuild a scene from a JSON-able spec (used by tests/golden fixtures):
    {"kind": "config", "name": "c1"} or
    {"kind": "monkey", "width", "height", "shading", "yaw", "pitch", "rotation", "cam"} or
    {"kind": "grid", "width", "height", "n", "shading"}."""
    k = spec["kind"]
    if k == "config":
        return config(spec["name"])
    if k == "monkey":
        return monkey_scene(spec["width"], spec["height"], spec["shading"], yaw=spec.get("yaw", 0.0),
                            pitch=spec.get("pitch", 0.0), rotation=spec.get("rotation", 0.0),
                            cam_pos=tuple(spec.get("cam", CAM_POS)))
    if k == "grid":
        return grid_scene(spec["width"], spec["height"], n=spec.get("n", 8), shading=spec.get("shading", SHADING_PHONG))
    raise KeyError(k)
