#!/usr/bin/env python3
"""Convert the reference's Suzanne mesh (.obj text) into the triangle-soup binary the bench and
tests load on the GPU box (where /root/reference does not exist).

Data only: the output holds the expanded triangle soup exactly as shs::ModelGeometry lays it out
(cpp-folders/src/hello-shs-renderer/shs_renderer.hpp:1265-1298: one entry per face corner, in face
order, positions / normals / uvs in separate arrays).  Floats are parsed with libc strtof, the
documented source of vertex floats (assimp's own float parser is unpinned).

Output format (little endian):
    8 bytes magic b"SHSSOUP1", u32 n_tris, u32 reserved,
    f32 positions[9*n_tris], f32 normals[9*n_tris], f32 uvs[6*n_tris]

Usage: python tools/convert_obj.py /root/reference/cpp-folders/src/assets/obj/monkey/monkey.rawobj assets/monkey.soup.bin
"""
import ctypes
import struct
import sys

import numpy as np

_libc = ctypes.CDLL(None)
_libc.strtof.restype = ctypes.c_float
_libc.strtof.argtypes = [ctypes.c_char_p, ctypes.POINTER(ctypes.c_char_p)]


def _f(tok: str) -> float:
    return _libc.strtof(tok.encode(), None)


def read_obj_soup(path):
    v, vt, vn = [], [], []
    pos, nrm, uv = [], [], []
    with open(path, "r") as fh:
        for line in fh:
            parts = line.split()
            if not parts:
                continue
            tag = parts[0]
            if tag == "v":
                v.append([_f(t) for t in parts[1:4]])
            elif tag == "vt":
                vt.append([_f(t) for t in parts[1:3]])
            elif tag == "vn":
                vn.append([_f(t) for t in parts[1:4]])
            elif tag == "f":
                corners = parts[1:]
                if len(corners) != 3:  # ModelGeometry skips non-triangles (shs_renderer.hpp:1270)
                    continue
                for c in corners:
                    idx = c.split("/")
                    vi = int(idx[0]) - 1
                    ti = int(idx[1]) - 1 if len(idx) > 1 and idx[1] else -1
                    ni = int(idx[2]) - 1 if len(idx) > 2 and idx[2] else -1
                    pos.append(v[vi])
                    uv.append(vt[ti] if ti >= 0 else [0.0, 0.0])
                    nrm.append(vn[ni] if ni >= 0 else [0.0, 1.0, 0.0])
    p = np.asarray(pos, dtype=np.float32).reshape(-1, 9)
    n = np.asarray(nrm, dtype=np.float32).reshape(-1, 9)
    t = np.asarray(uv, dtype=np.float32).reshape(-1, 6)
    return p, n, t


def write_soup(path, p, n, t):
    with open(path, "wb") as fh:
        fh.write(b"SHSSOUP1")
        fh.write(struct.pack("<II", p.shape[0], 0))
        fh.write(p.astype("<f4").tobytes())
        fh.write(n.astype("<f4").tobytes())
        fh.write(t.astype("<f4").tobytes())


if __name__ == "__main__":
    src, dst = sys.argv[1], sys.argv[2]
    p, n, t = read_obj_soup(src)
    write_soup(dst, p, n, t)
    print(f"{dst}: {p.shape[0]} triangles")
