"""The library raster's conservative row spans (shs_lib.hip lib_row_span): every pixel that passes
lib_test's float inside test (rasterizer.hpp:167-179, :338 -- u, v, w >= 0 from the record's float
values, no contraction) must lie inside its row's span, or the raster would drop a fragment.  This
restates the span arithmetic in numpy float32 (IEEE per operation, as the kernel's -ffp-contract=off
build) and checks it against the per-pixel test over small, large, sliver and pixel-centre-aligned
triangles.  The kernel itself is covered by the -m gpu parity tests (depth bit-exact)."""
import math

import numpy as np

f = np.float32


def _inside(ax, ay, v0x, v0y, v1x, v1y, idn, px, py):
    vpx = f(f(f(px) + f(0.5)) - ax)
    vpy = f(f(f(py) + f(0.5)) - ay)
    v = f(f(f(vpx * v1y) - f(v1x * vpy)) * idn)
    w = f(f(f(v0x * vpy) - f(vpx * v0y)) * idn)
    u = f(f(f(1.0) - v) - w)
    return not (u < 0 or v < 0 or w < 0)


def _span(ax, ay, v0x, v0y, v1x, v1y, idn, py, bx0, bx1):
    E = f(2.0 ** -18)
    dy = f(f(f(py) + f(0.5)) - ay)
    ady = abs(dy)
    T = f(max(abs(f(f(bx0) + f(0.5)) - ax), abs(f(f(bx1) + f(0.5)) - ax)))
    aid = abs(idn)
    mv = f(aid * f(f(abs(v1y) * T) + f(abs(v1x) * ady)))
    mw = f(aid * f(f(abs(v0y) * T) + f(abs(v0x) * ady)))
    lo, hi = f(-1e30), f(1e30)

    def edge(a, c, e):
        nonlocal lo, hi
        b = f(-e - c)
        if a > 0:
            lo = max(lo, f(b / a))
        elif a < 0:
            hi = min(hi, f(b / a))
        elif b > 0:
            lo, hi = f(1e30), f(-1e30)

    with np.errstate(all="ignore"):
        edge(f(idn * v1y), f(f(-idn * v1x) * dy), f(E * mv))
        edge(f(-idn * v0y), f(f(idn * v0x) * dy), f(E * mw))
        edge(f(idn * f(v0y - v1y)), f(f(1.0) + f(f(idn * f(v1x - v0x)) * dy)), f(E * f(f(1.0) + f(f(2.0) * f(mv + mw)))))
        flo, fhi = f(f(lo + ax) - f(0.5)), f(f(hi + ax) - f(0.5))
        slo = f(f(2.0 ** -12) * f(f(abs(lo) + abs(ax)) + f(1.0)))
        shi = f(f(2.0 ** -12) * f(f(abs(hi) + abs(ax)) + f(1.0)))
        a, b = f(flo - slo), f(fhi + shi)
    a = 1e9 if np.isnan(a) else min(max(float(a), -1e9), 1e9)   # fminf / fmaxf drop a NaN operand
    b = 1e9 if np.isnan(b) else min(max(float(b), -1e9), 1e9)
    return max(bx0, math.ceil(a)), min(bx1, math.floor(b))


def test_row_spans_hold_every_inside_pixel():
    rng = np.random.default_rng(0x5BA7)
    missed = excluded = total = 0
    for it in range(240):
        kind = it % 4
        base = rng.uniform(0, 4000, 2)
        if kind == 0:
            pts = base + rng.uniform(-8, 8, (3, 2))
        elif kind == 1:
            pts = base + rng.uniform(-40, 40, (3, 2))
        elif kind == 2:   # sliver: a corner within ~1e-3 px of the opposite edge
            d = rng.uniform(-30, 30, 2)
            pts = np.array([base, base + d, base + d * rng.uniform(0.2, 0.8) + rng.normal(0, 1e-3, 2)])
        else:
            pts = base + rng.uniform(-3000, 3000, (3, 2))
        if it % 3 == 0:
            pts = np.round(pts) + 0.5   # corners on pixel centres: edges through centres
        elif it % 3 == 1:
            pts = np.round(pts)
        pts = pts.astype(f)
        ax, ay = pts[0]
        v0, v1 = (pts[1] - pts[0]).astype(f), (pts[2] - pts[0]).astype(f)
        den = f(f(v0[0] * v1[1]) - f(v1[0] * v0[1]))
        if abs(den) < 1e-8:
            continue
        idn = f(f(1.0) / den)
        cx, cy = pts.mean(0)
        tx0, ty0 = int(max(0, cx - 16)) // 32 * 32, int(max(0, cy - 4)) // 8 * 8
        for py in range(ty0, ty0 + 8):
            s0, s1 = _span(ax, ay, v0[0], v0[1], v1[0], v1[1], idn, py, tx0, tx0 + 31)
            for px in range(tx0, tx0 + 32):
                total += 1
                if s0 <= px <= s1:
                    continue
                excluded += 1
                if _inside(ax, ay, v0[0], v0[1], v1[0], v1[1], idn, px, py):
                    missed += 1
    assert missed == 0, f"{missed} inside pixels outside their row span"
    assert excluded > total // 4, "the spans exclude almost nothing"
