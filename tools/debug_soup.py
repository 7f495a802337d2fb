"""Diagnose random-soup mismatches: which 32x8 raster tiles differ, and their candidate / pair counts."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "leisure-software-renderer_amd"), ROOT, os.path.join(ROOT, "tests")]
import shs_gpu
from shs_gpu.scene import Mesh
from oracle import oracle
from test_gpu_parity import _ndc_soup, _identity_draw

rng = np.random.default_rng(1)
W, H = 333, 241
pos, nrm = _ndc_soup(rng, W, H, 1500)
frame = shs_gpu.Frame(W, H)
draws = [_identity_draw(Mesh(pos, nrm), shading=1)]
ctx = shs_gpu.Context(0)
ctx.render(frame, draws)
c, d = ctx.resolve()
recs = ctx.debug_records()
oc, od, _ = oracle.render_legacy(W, H, draws, threads=8)
bad = d.view(np.uint32) != od.view(np.uint32)
print("bad", bad.sum())
lo = lambda v: (v.astype(np.int64) & 0xffff).astype(np.int16).astype(np.int64)
hi = lambda v: ((v.astype(np.int64) >> 16) & 0xffff).astype(np.int16).astype(np.int64)
gx0, gx1, gy0, gy1 = lo(recs["gbx"]), hi(recs["gbx"]), lo(recs["gby"]), hi(recs["gby"])
ys, xs = np.nonzero(bad)
tiles = sorted(set(zip((ys // 8).tolist(), (xs // 32).tolist())))
for (ty, tx) in tiles[:12]:
    X0, Y0 = tx * 32, ty * 8
    X1, Y1 = X0 + 31, Y0 + 7
    m = (recs["flags"] & 1 == 0) & (gx1 >= X0) & (gx0 <= X1) & (gy1 >= Y0) & (gy0 <= Y1) & (gx0 <= gx1)
    idx = np.nonzero(m)[0]
    areas = [(min(gx1[i], X1) - max(gx0[i], X0) + 1) * (min(gy1[i], Y1) - max(gy0[i], Y0) + 1) for i in idx]
    nb = int(bad[Y0:Y1 + 1, X0:X1 + 1].sum())
    print(f"tile ({ty},{tx}) bad {nb} cand {len(idx)} pairs {sum(areas)} per-wave {[sum(areas[w::4]) for w in range(4)]}")
good_tiles = 0
