#!/usr/bin/env python3
"""Generate tests/golden/legacy_golden.json: oracle outputs (FNV-1a of colour and depth, covered
pixel count) for fixed scenes, with every draw's uniforms stored as float32 bit patterns so the
fixture is self-contained.  The oracle is the CPU restatement of the reference (parity unpinned:
the reference cannot be built here and ships no fixtures for this path).

Usage: python tests/golden/make_golden.py          (legacy_golden.json)
       python tests/golden/make_golden.py --lib    (lib_golden.json: library path, C5-small scene)
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "leisure-software-renderer_amd"))

import numpy as np  # noqa: E402

from oracle import oracle  # noqa: E402
from shs_gpu import scene  # noqa: E402

SPECS = [
    ("c1_blinn_phong_800x600", {"kind": "config", "name": "c1"}),
    ("c2_blinn_phong_1920x1080", {"kind": "config", "name": "c2"}),
    ("c3_grid_phong_1920x1080", {"kind": "config", "name": "c3"}),
]
for sh, nm in enumerate(["flat", "gouraud", "phong", "blinn_phong"]):
    SPECS.append((f"monkey_{nm}_640x480_cam", {"kind": "monkey", "width": 640, "height": 480, "shading": sh,
                                               "yaw": 17.0, "pitch": -9.0, "rotation": 23.0 * sh,
                                               "cam": [0.0, 5.0, -12.0]}))


def bits(a):
    return np.asarray(a, np.float32).view(np.uint32).tolist()


def main():
    frames = []
    for name, spec in SPECS:
        frame, draws = scene.build_named(spec)
        c, d, _ = oracle.render_legacy(frame.width, frame.height, draws, tile=frame.ref_tile, threads=8)
        frames.append({
            "name": name, "scene": spec, "width": frame.width, "height": frame.height, "tile": list(frame.ref_tile),
            "draws": [{"shading": int(x.shading), "color": list(x.color), "mvp": bits(x.mvp), "model": bits(x.model),
                       "light_dir": bits(x.light_dir), "camera_pos": bits(x.camera_pos)} for x in draws],
            "color_fnv1a64": hex(oracle.fnv1a64(c)), "depth_fnv1a64": hex(oracle.fnv1a64(d)),
            "covered": int((d < np.finfo(np.float32).max).sum()),
        })
        print(name, frames[-1]["covered"], frames[-1]["depth_fnv1a64"])
    with open(os.path.join(HERE, "legacy_golden.json"), "w") as fh:
        json.dump({"generator": "tests/golden/make_golden.py", "oracle": "oracle/shs_oracle.c",
                   "mesh": "assets/monkey.soup.bin (tools/convert_obj.py from the reference's monkey.rawobj)",
                   "frames": frames}, fh, indent=1)


def main_lib():
    """C5-small through the library-path oracle (PassShadowMap 128^2 + PassPBRForward 320x180)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from test_lib_oracle import _c5_small_outputs
    sm, hdr, d, m, st = _c5_small_outputs(oracle)
    rng = np.random.default_rng(0)
    cov = np.argwhere(d < 1.0)
    probes = cov[rng.choice(len(cov), 24, replace=False)].tolist() + [[0, 0], [179, 319]]
    out = {"generator": "tests/golden/make_golden.py --lib", "oracle": "oracle/shs_oracle_lib.c",
           "scene": "shs_gpu.scene_lib.c5_scene(320, 180), shadow 128", "stats": st,
           "shadow_fnv": hex(oracle.fnv1a64(sm)), "depth_fnv": hex(oracle.fnv1a64(d)), "covered": int(len(cov)),
           "probe_px": probes, "probe_hdr": [hdr[y, x].tolist() for y, x in probes]}
    with open(os.path.join(HERE, "lib_golden.json"), "w") as fh:
        json.dump(out, fh, indent=1)
    print("lib", st, out["covered"], out["depth_fnv"])


if __name__ == "__main__":
    main_lib() if "--lib" in sys.argv else main()
