"""Host model of the region layout (shs_abi_shard.cpp) for the C4 / C5 camera pass: the setup blocks'
chunk bounds as k_lib_setup computes them (numpy restatement), the balancer's bisection, and each rank's
share of the cost terms (pixels, triangles spread over block bounds, triangle x tile coverage).  Used to
fit the cost weights against measured per-rank kernel times (tools/trace_ranks.py).
usage: python tools/region_model.py [c4|c5] [N] [regions literal or None] [px_w covered_px_w cov_w]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "leisure-software-renderer_amd"), ROOT]
from shs_gpu import scene_lib  # noqa: E402

T = 32


def block_rects(frame, draws):
    W, H = frame.width, frame.height
    tx, ty = (W + T - 1) // T, (H + T - 1) // T
    out = []
    base = 0
    spans = []
    for d in draws:
        n = d.mesh.n_tris
        spans.append((base, base + n, d))
        base += n
    n_tris = base
    for b in range((n_tris + 255) // 256):
        t0, t1 = b * 256, min(b * 256 + 255, n_tris - 1)
        ds = [s for s in spans if s[0] <= t0 < s[1]]
        s0, s1, d = ds[0]
        if t1 >= s1:
            out.append((0, tx - 1, 0, ty - 1, t1 - t0 + 1, 0))
            continue
        pos = d.mesh.positions
        idx = d.mesh.indices
        lo, hi = t0 - s0, t1 - s0
        c0, c1 = lo >> 8, hi >> 8
        pts = []
        for c in range(c0, c1 + 1):
            tr = np.arange(c * 256, min((c + 1) * 256, d.mesh.n_tris))
            v = idx.reshape(-1, 3)[tr].reshape(-1) if idx is not None else (3 * tr[:, None] + np.arange(3)).reshape(-1)
            p = pos[v]
            mn, mx = p.min(0), p.max(0)
            for k in range(8):
                pts.append([mx[0] if k & 1 else mn[0], mx[1] if k & 2 else mn[1], mx[2] if k & 4 else mn[2], 1.0])
        P = np.array(pts, np.float32)
        M = np.asarray(d.model, np.float32).reshape(4, 4).T
        V = np.asarray(d.viewproj, np.float32).reshape(4, 4).T
        c = (V @ (M @ P.T)).T
        if (c[:, 3] <= 0).any():
            out.append((0, tx - 1, 0, ty - 1, t1 - t0 + 1, 0))
            continue
        sx = (c[:, 0] / c[:, 3] * 0.5 + 0.5) * (W - 1)
        sy = (c[:, 1] / c[:, 3] * 0.5 + 0.5) * (H - 1)
        x0, x1, y0, y1 = sx.min(), sx.max(), sy.min(), sy.max()
        if not (x1 >= -2 and y1 >= -2 and x0 <= W + 1 and y0 <= H + 1):
            out.append((1, 0, 1, 0, t1 - t0 + 1, 1))
            continue
        bx0 = max(0, int(max(x0 - 2, 0)) // T); bx1 = min(tx - 1, int(min(x1 + 2, W - 1)) // T)
        by0 = max(0, int(max(y0 - 2, 0)) // T); by1 = min(ty - 1, int(min(y1 + 2, H - 1)) // T)
        out.append((bx0, bx1, by0, by1, t1 - t0 + 1, 1))
    return np.array(out, np.int64), tx, ty


def cost_maps(rects, tx, ty, W, H):
    """-> px (pixels per tile), tri (triangles spread over their block bounds), cov (triangles x
    covering blocks: each covering block adds its triangle count)."""
    px = np.zeros((ty, tx))
    for y in range(ty):
        for x in range(tx):
            px[y, x] = min(T, W - T * x) * min(T, H - T * y)
    tri = np.zeros((ty, tx))
    cov = np.zeros((ty, tx))
    for x0, x1, y0, y1, n, bounded in rects:
        if x1 < x0 or y1 < y0:
            continue
        a = (x1 - x0 + 1) * (y1 - y0 + 1)
        tri[y0:y1 + 1, x0:x1 + 1] += n / a
        if bounded:
            cov[y0:y1 + 1, x0:x1 + 1] += n
    covpx = px * (cov > 0)
    return px, tri, cov, covpx


def bisect(S, x0, y0, x1, y1, r0, n, out):
    def ssum(a, b, c, d):
        return S[d + 1, c + 1] - S[b, c + 1] - S[d + 1, a] + S[b, a]
    if n == 1:
        out[r0] = (x0, y0, x1, y1)
        return
    w, h = x1 - x0 + 1, y1 - y0 + 1
    if w <= 0 or h <= 0 or (w == 1 and h == 1):
        out[r0] = (x0, y0, x1, y1)
        for r in range(1, n):
            out[r0 + r] = (1, 1, 0, 0)
        return
    n1 = n // 2
    along_x = h == 1 or (w > 1 and w >= h)
    total = ssum(x0, y0, x1, y1)
    want = total * n1 / n
    lo, hi = (x0, x1) if along_x else (y0, y1)
    best, err = lo + 1, -1
    for c in range(lo + 1, hi + 1):
        left = ssum(x0, y0, c - 1, y1) if along_x else ssum(x0, y0, x1, c - 1)
        e = abs(left - want)
        if err < 0 or e < err:
            best, err = c, e
        if left >= want:
            break
    if along_x:
        bisect(S, x0, y0, best - 1, y1, r0, n1, out)
        bisect(S, best, y0, x1, y1, r0 + n1, n - n1, out)
    else:
        bisect(S, x0, y0, x1, best - 1, r0, n1, out)
        bisect(S, x0, best, x1, y1, r0 + n1, n - n1, out)


def balance(cost, n):
    ty, tx = cost.shape
    S = np.zeros((ty + 1, tx + 1))
    S[1:, 1:] = cost.cumsum(0).cumsum(1)
    out = [None] * n
    bisect(S, 0, 0, tx - 1, ty - 1, 0, n, out)
    return out


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c4"
    N = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    if cfg == "c4":
        frame, draws, _, _ = scene_lib.c4_scene(3840, 2160)
    else:
        frame, draws, _, _, _ = scene_lib.c5_scene(3840, 2160, 2048)
    rects, tx, ty = block_rects(frame, draws)
    px, tri, cov, covpx = cost_maps(rects, tx, ty, frame.width, frame.height)
    print(f"blocks {len(rects)} unbounded {(rects[:, 5] == 0).sum()} sum(n*area) {cov.sum():.4g}")
    regs = eval(sys.argv[3]) if len(sys.argv) > 3 else None
    if regs is None:
        w = [float(x) for x in sys.argv[4:7]] if len(sys.argv) > 6 else [5.0, 15.0, 1.0]   # shs_abi_shard.cpp
        regs = balance(px * w[0] + covpx * w[1] + cov * w[2], N)
    print("regions", regs)
    for r, (x0, y0, x1, y1) in enumerate(regs):
        s = (slice(y0, y1 + 1), slice(x0, x1 + 1))
        # setup blocks the rank runs: bounds meeting its rectangle, or unbounded (never skipped)
        hit = (rects[:, 5] == 0) | ((rects[:, 0] <= x1) & (rects[:, 1] >= x0) & (rects[:, 2] <= y1) & (rects[:, 3] >= y0)
                                    & (rects[:, 0] <= rects[:, 1]))
        print(f"rank {r}: px {px[s].sum() / 1e6:7.3f}M covered px {covpx[s].sum() / 1e6:7.3f}M tri {tri[s].sum() / 1e3:8.1f}K "
              f"cov {cov[s].sum() / 1e6:8.2f}M setup blocks {int(hit.sum())}")


if __name__ == "__main__":
    main()
