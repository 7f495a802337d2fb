"""Forward+ debugging aid (GPU box): renders the small tiled-mode Forward+ scene of
tests/test_light_parity.py on the GPU and with the oracle and lists the 16x4 resolve blocks whose HDR
differs beyond 1e-5 (with their light lists), e.g. to bisect a resolve-kernel change with
SHS_GPU_LIB=<variant build>.  usage: python tools/dbg_forward_plus.py"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "leisure-software-renderer_amd"), ROOT]
import shs_gpu
from shs_gpu import scene_lib
from oracle import oracle
frame, draws, lights, cull = scene_lib.c4_scene(480, 270, n_objects=60, tris_per_object=200, n_lights=64, mode=1, tile_size=16, max_per_tile=128)
ctx = shs_gpu.Context(0)
ctx.upload_lights(lights)
ctx.light_cull(cull)
ctx.render_pbr_forward(frame, draws)
gh, gd, _ = ctx.resolve_lib()
rc, ri = oracle.light_cull(cull, lights)[:2]
rh, rd, _, _ = oracle.forward_plus(frame, draws, lights, cull, (rc, ri))
bad = np.abs(gh - rh) > 1e-5
ys, xs = np.nonzero(bad.any(-1))
print('bad px', len(ys))
blocks = set((y//4, x//16) for y, x in zip(ys, xs))
print('blocks', len(blocks))
H, W = 270, 480
for (by, bx) in sorted(blocks)[:12]:
    y0, x0 = by*4, bx*16
    lists = set()
    for y in range(y0, min(y0+4, H)):
        for x in range(x0, x0+16):
            lists.add(min((H-1-y)//16, 16)*30 + min(x//16, 29))
    nb = int(bad[y0:y0+4, x0:x0+16].any(-1).sum())
    print('block', (y0, x0), 'lists', [(l, int(rc[l])) for l in lists], 'bad', nb, 'maxerr', float(np.abs(gh-rh)[y0:y0+4, x0:x0+16].max()))
