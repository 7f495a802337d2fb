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
