"""The legacy raster's conservative row spans (shs_legacy.hip legacy_row_span): every pixel that passes
barycentric_coordinate's float test (hello-shs-renderer/shs_renderer.hpp:802-821 -- the Gram form
v = (d11 d20 - d01 d21) / denom, w = (d00 d21 - d01 d20) / denom, u = 1 - v - w, all >= 0, at
P = (px + 0.5, py + 0.5): hello_pipeline_blinn_phong_shading.cpp:227-229) must lie inside its row's
span, or the raster would drop a fragment.  Pixels outside the triangle's bbox are tested too: the
80x80 tile clamp makes the reference test them for slivers, and the span must hold
them as well.  The numpy float32 restatement below follows the kernel's operation order (IEEE per
operation, -ffp-contract=off); the kernel itself is covered by the -m gpu parity tests."""
import math

import numpy as np

f = np.float32


def _record(pts):
    """rec_from_screen's Gram terms (shs_device.hpp TriRec) from float32 screen corners."""
    ax, ay = pts[0]
    v0x, v0y = f(pts[1][0] - ax), f(pts[1][1] - ay)
    v1x, v1y = f(pts[2][0] - ax), f(pts[2][1] - ay)
    d00 = f(f(v0x * v0x) + f(v0y * v0y))
    d01 = f(f(v0x * v1x) + f(v0y * v1y))
    d11 = f(f(v1x * v1x) + f(v1y * v1y))
    den = f(f(d00 * d11) - f(d01 * d01))
    return ax, ay, v0x, v0y, v1x, v1y, d00, d01, d11, den


def _inside(rec, px, py):
    """bary_pass (shs_device.hpp), the reference's test."""
    ax, ay, v0x, v0y, v1x, v1y, d00, d01, d11, den = rec
    with np.errstate(all="ignore"):
        vpx = f(f(f(px) + f(0.5)) - ax)
        vpy = f(f(f(py) + f(0.5)) - ay)
        d20 = f(f(vpx * v0x) + f(vpy * v0y))
        d21 = f(f(vpx * v1x) + f(vpy * v1y))
        nv = f(f(d11 * d20) - f(d01 * d21))
        nw = f(f(d00 * d21) - f(d01 * d20))
        v = f(nv / den)
        w = f(nw / den)
        u = f(f(f(1.0) - v) - w)
    return not (u < 0 or v < 0 or w < 0)


def legacy_span(rec, py, bx0, bx1):
    """legacy_row_span: the pixels of row py in [bx0, bx1] that can pass _inside."""
    ax, ay, v0x, v0y, v1x, v1y, d00, d01, d11, den = rec
    vals = (ax, ay, v0x, v0y, v1x, v1y, d00, d01, d11, den)
    if not all(np.isfinite(x) for x in vals) or not abs(den) > 0:
        return bx0, bx1
    E = f(2.0 ** -18)
    with np.errstate(all="ignore"):
        Y = f(f(f(py) + f(0.5)) - ay)
        aY = abs(Y)
        T = max(abs(f(f(f(bx0) + f(0.5)) - ax)), abs(f(f(f(bx1) + f(0.5)) - ax)))
        idn = f(f(1.0) / den)
        aid = abs(idn)
        s0 = f(f(abs(v0x) * T) + f(abs(v0y) * aY))
        s1 = f(f(abs(v1x) * T) + f(abs(v1y) * aY))
        mv = f(aid * f(f(abs(d11) * s0) + f(abs(d01) * s1)))
        mw = f(aid * f(f(abs(d00) * s1) + f(abs(d01) * s0)))
        av = f(f(f(d11 * v0x) - f(d01 * v1x)) * idn)
        cv = f(f(f(f(d11 * v0y) - f(d01 * v1y)) * idn) * Y)
        aw = f(f(f(d00 * v1x) - f(d01 * v0x)) * idn)
        cw = f(f(f(f(d00 * v1y) - f(d01 * v0y)) * idn) * Y)
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

        edge(av, cv, f(E * mv))
        edge(aw, cw, f(E * mw))
        edge(f(-f(av + aw)), f(f(1.0) - f(cv + cw)), f(E * f(f(1.0) + f(f(2.0) * f(mv + mw)))))
        flo, fhi = f(f(lo + ax) - f(0.5)), f(f(hi + ax) - f(0.5))
        slo = f(f(2.0 ** -12) * f(f(abs(lo) + abs(ax)) + f(1.0)))
        shi = f(f(2.0 ** -12) * f(f(abs(hi) + abs(ax)) + f(1.0)))
        a, b = f(flo - slo), f(fhi + shi)
    a = 1e9 if np.isnan(a) else min(max(float(a), -1e9), 1e9)   # fminf / fmaxf drop a NaN operand
    b = 1e9 if np.isnan(b) else min(max(float(b), -1e9), 1e9)
    return max(bx0, math.ceil(a)), min(bx1, math.floor(b))


def _triangles(rng, n):
    for it in range(n):
        kind = it % 5
        base = rng.uniform(0, 1900, 2)
        if kind == 0:
            pts = base + rng.uniform(-6, 6, (3, 2))
        elif kind == 1:
            pts = base + rng.uniform(-40, 40, (3, 2))
        elif kind == 2:   # sliver: a corner within ~1e-3 px of the opposite edge
            d = rng.uniform(-30, 30, 2)
            pts = np.array([base, base + d, base + d * rng.uniform(0.2, 0.8) + rng.normal(0, 1e-3, 2)])
        elif kind == 3:   # hair-thin and long (the tile-clamp slivers of DESIGN.md 5)
            d = rng.uniform(-300, 300, 2)
            pts = np.array([base, base + d, base + d * rng.uniform(0.1, 0.9) + rng.normal(0, 1e-4, 2)])
        else:
            pts = base + rng.uniform(-2000, 2000, (3, 2))
        if it % 3 == 0:
            pts = np.round(pts) + 0.5   # corners on pixel centres: edges through centres
        elif it % 3 == 1:
            pts = np.round(pts)
        if rng.uniform() < 0.5:
            pts = pts[::-1]             # both windings
        yield pts.astype(f)


def test_legacy_row_spans_hold_every_inside_pixel():
    rng = np.random.default_rng(0x1E6A)
    missed = excluded = total = 0
    for pts in _triangles(rng, 400):
        rec = _record(pts)
        if not abs(rec[-1]) >= 1e-5:    # barycentric_coordinate rejects every pixel
            continue
        # a 32x8 tile at the centroid, and one at the first corner (pixels outside the bbox)
        for cx, cy in (pts.mean(0), pts[0]):
            tx0, ty0 = int(max(0, cx - 16)) // 32 * 32, int(max(0, cy - 4)) // 8 * 8
            for py in range(ty0, ty0 + 8):
                s0, s1 = legacy_span(rec, py, tx0, tx0 + 31)
                for px in range(tx0, tx0 + 32):
                    total += 1
                    if s0 <= px <= s1:
                        continue
                    excluded += 1
                    if _inside(rec, px, py):
                        missed += 1
    assert missed == 0, f"{missed} inside pixels outside their row span"
    assert excluded > total // 4, "the spans exclude almost nothing"


def test_legacy_row_spans_sliver_rows_exhaustive():
    """Slivers over their whole bbox plus a 3-px margin (the ghost pixels): every passing pixel in span."""
    rng = np.random.default_rng(77)
    missed = passing = 0
    for it in range(60):
        base = rng.uniform(10, 1000, 2)
        d = rng.uniform(-60, 60, 2)
        pts = np.array([base, base + d, base + d * rng.uniform(0.05, 0.95) + rng.normal(0, 10.0 ** -rng.uniform(2, 5), 2)])
        pts = pts.astype(f)
        rec = _record(pts)
        if not abs(rec[-1]) >= 1e-5:
            continue
        x0, x1 = int(pts[:, 0].min()) - 3, int(pts[:, 0].max()) + 3
        y0, y1 = int(pts[:, 1].min()) - 3, int(pts[:, 1].max()) + 3
        for py in range(y0, y1 + 1):
            s0, s1 = legacy_span(rec, py, x0, x1)
            for px in range(x0, x1 + 1):
                if _inside(rec, px, py):
                    passing += 1
                    missed += not (s0 <= px <= s1)
    assert missed == 0
    assert passing > 100


def _inside_vec(rec, px, py):
    """_inside over arrays of pixels (float32, the same operation order)."""
    ax, ay, v0x, v0y, v1x, v1y, d00, d01, d11, den = rec
    with np.errstate(all="ignore"):
        vpx = (px.astype(f) + f(0.5)).astype(f) - ax
        vpy = (py.astype(f) + f(0.5)).astype(f) - ay
        d20 = (vpx * v0x).astype(f) + (vpy * v0y).astype(f)
        d21 = (vpx * v1x).astype(f) + (vpy * v1y).astype(f)
        nv = (d11 * d20).astype(f) - (d01 * d21).astype(f)
        nw = (d00 * d21).astype(f) - (d01 * d20).astype(f)
        v = (nv / den).astype(f)
        w = (nw / den).astype(f)
        u = ((f(1.0) - v).astype(f) - w).astype(f)
    return ~((u < 0) | (v < 0) | (w < 0))


def _classify(n_rt, rts, extent, fmin, fmax):
    """classify_axis (shs_legacy.hip): reference-tile columns before / after [fmin, fmax], the span of the rest."""
    before = sum(1 for c in range(n_rt) if f(min(c * rts + rts, extent) - 1) < fmin)
    after = sum(1 for c in range(n_rt) if f(c * rts) > fmax)
    lo, hi = 0, -1
    if before + after < n_rt:
        c0, c1 = before, n_rt - 1 - after
        lo = int(max(f(c0 * rts), fmin))
        hi = int(min(f(min(c1 * rts + rts, extent) - 1), fmax))
    return before, after, lo, hi


def _edge(i, before, n_rt, after, rts, extent):
    return min((i + 1) * rts, extent) - 1 if i < before else (n_rt - after + (i - before)) * rts


def test_legacy_spans_hold_tile_clamp_lines():
    """sliver_pixels (shs_legacy.hip) walks an unbounded sliver's tile-clamp pixels line by line and
    tests only each line's span: a row's is legacy_row_span of the record, a column's that of the
    record with x and y swapped (every Gram term and computed barycentric is bit-identical under the
    swap).  Every visited pixel that passes the reference's test must lie in its line's span, however
    far from the bbox the reference tile's edge line is (80x80 tiles over 1920x1080)."""
    rng = np.random.default_rng(4242)
    W, H, T = 1920, 1080, 80
    rt_x, rt_y = (W + T - 1) // T, (H + T - 1) // T
    passing = missed = lines = 0
    for it in range(120):
        base = rng.uniform(40, 1880, 2).astype(np.float64)
        d = rng.uniform(-900, 900, 2)
        # near-degenerate slivers: the third corner within ~1e-3..1e-5 px of the first edge's line
        pts = np.array([base, base + d, base + d * rng.uniform(0.05, 0.95) + rng.normal(0, 10.0 ** -rng.uniform(3, 5), 2)])
        pts = np.clip(pts, -50, [W + 50, H + 50]).astype(f)
        rec = _record(pts)
        if not abs(rec[-1]) >= 1e-5:
            continue
        recs = _record(pts[:, ::-1])   # x <-> y
        fminx, fmaxx = f(pts[:, 0].min()), f(pts[:, 0].max())
        fminy, fmaxy = f(pts[:, 1].min()), f(pts[:, 1].max())
        ix0, ix1 = max(0, int(np.floor(fminx))), min(W - 1, int(np.floor(fmaxx)))
        iy0, iy1 = max(0, int(np.floor(fminy))), min(H - 1, int(np.floor(fmaxy)))
        cl, cr, xi0, xi1 = _classify(rt_x, T, W, fminx, fmaxx)
        ru, rd, yi0, yi1 = _classify(rt_y, T, H, fminy, fmaxy)
        yout = [_edge(j, ru, rt_y, rd, T, H) for j in range(ru + rd)]
        ys = np.array(yout + list(range(yi0, yi1 + 1)), dtype=np.int64)
        if len(ys):
            y_lo, y_hi = int(ys.min()), int(ys.max())
            for i in range(cl + cr):   # edge columns over Yout u Yin
                x = _edge(i, cl, rt_x, cr, T, W)
                lines += 1
                ok = _inside_vec(rec, np.full(len(ys), x), ys)
                out = ~((x >= ix0) & (x <= ix1) & (ys >= iy0) & (ys <= iy1))
                s0, s1 = legacy_span(recs, x, y_lo, y_hi)
                hit = ok & out
                passing += int(hit.sum())
                missed += int((hit & ((ys < s0) | (ys > s1))).sum())
        if xi0 <= xi1:
            xs = np.arange(xi0, xi1 + 1)
            for y in yout:   # edge rows over Xin
                lines += 1
                ok = _inside_vec(rec, xs, np.full(len(xs), y))
                out = ~((xs >= ix0) & (xs <= ix1) & (y >= iy0) & (y <= iy1))
                s0, s1 = legacy_span(rec, y, xi0, xi1)
                hit = ok & out
                passing += int(hit.sum())
                missed += int((hit & ((xs < s0) | (xs > s1))).sum())
    assert lines > 500
    assert missed == 0, f"{missed} of {passing} passing tile-clamp pixels outside their line's span"
