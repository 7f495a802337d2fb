"""The product library ignores the timing-experiment switches.

SHS_* environment variables and the frame's DBG_* bits (bench --debug-flags) attribute kernel time in
tools/ runs; several of them give wrong images.  Only the -DSHS_TIMING_EXPERIMENTS build
(`make -C leisure-software-renderer_amd exp` -> libshs_gpu_exp.so, loaded through SHS_GPU_LIB) reads
them.  CPU: the switch names are not in the product library at all.  GPU: a child process with every
switch set (and the DBG bits in the frame flags) renders the oracle's frames."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "leisure-software-renderer_amd", "shs_gpu", "libshs_gpu.so")

SWITCHES = {
    "SHS_LIB_EXP": "0xffff", "SHS_LIB_SCAN_MAX": "0", "SHS_LIB_XCD_ST": "7", "SHS_LIB_DEEP": "1",
    "SHS_LIB_STATIC_DIV": "0", "SHS_LIB_HEAVY": "1", "SHS_GHOST_LIST": "1", "SHS_GHOST_INLINE": "0",
    "SHS_LEGACY_NORECS": "1", "SHS_LEGACY_SHARE_VARY": "0", "SHS_LEGACY_XCD_ROWS": "0",
    "SHS_RASTER_PER_CU": "1", "SHS_OCC_PROF": "1",
}


def test_product_library_has_no_switch_names():
    blob = open(LIB, "rb").read()
    for name in SWITCHES:
        assert name.encode() + b"\0" not in blob, f"{name} is read by the product library"


CHILD = r"""
import os, sys
import numpy as np
sys.path.insert(0, os.path.join(sys.argv[1], "leisure-software-renderer_amd"))
sys.path.insert(0, os.path.join(sys.argv[1], "tests"))
sys.path.insert(0, sys.argv[1])
import shs_gpu
from shs_gpu import scene, scene_lib
from oracle import oracle
from helpers import assert_color_parity, assert_depth_bitexact, assert_float_close
with shs_gpu.Context(0) as ctx:
    for cfg in ("c1", "c3"):
        frame, draws = scene.config(cfg)
        frame.prequant = True
        frame.debug_flags = 0x7f00          # every DBG_* bit: skip ghost / shade / pairs, clear only ...
        ctx.render(frame, draws)
        gc, gd = ctx.resolve()
        gpq = ctx.resolve_prequant()
        rc, rd, rpq = oracle.render_legacy(frame.width, frame.height, draws, tile=frame.ref_tile,
                                           threads=8, prequant=True)
        assert_depth_bitexact(gd, rd)
        assert_color_parity(gc, rc, gpq, rpq)
    frame, draws, casters, sun, _ = scene_lib.c5_scene(480, 270, program=0)
    scene_lib.wire_shadow(draws, np.eye(4, dtype=np.float32).reshape(16))
    lvp = ctx.render_shadow_map(256, sun, casters)
    sm_ref, _ = oracle.shadow_map(256, sun, casters)
    for d in draws:
        if d.shadow:
            d.light_viewproj = lvp
    ctx.render_pbr_forward(frame, draws)
    gh, gd, gm = ctx.resolve_lib()
    rh, rd, rm, _ = oracle.pbr_forward(frame, draws, sm_ref)
    assert_depth_bitexact(gd, rd)
    assert_float_close(gh, rh, what="hdr")
    assert_float_close(gm, rm, what="motion")
print("switches ignored")
"""


@pytest.mark.gpu
def test_switches_do_not_change_frames():
    env = dict(os.environ)
    env.update(SWITCHES)
    env.pop("SHS_GPU_LIB", None)
    r = subprocess.run([sys.executable, "-c", CHILD, ROOT], env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "switches ignored" in r.stdout
