// shs_footprint.hpp -- host-only: which shadow-map texels a camera pass can read (SHS_OPT_SHADOW_FOOTPRINT).
//
// PassPBRForward's programs read the shadow map only through shadow_visibility_dir
// (lighting/shadow_sample.hpp:65-104): the shaded point's world position, projected with the draw's
// light_viewproj, rounded to a texel (cx, cy), and the (2r+1)^2 PCF taps cx + ox*step, cy + oy*step,
// clamped to the map.  The shaded point of a pixel is the perspective-correct interpolation of one of
// the draw's triangles (rasterizer.hpp:365-387), so it lies (up to rounding) in
//   * the draw's world box (the model transform of the mesh's model-space box), and
//   * the camera frustum slice of the pixels the pass shades: the rank's rectangle of pixel centres,
//     NDC x / y between the rectangle's bounds and -w <= z <= w (rasterize_mesh clips to the frustum).
// Both are intersections of half-spaces, so their intersection is a convex polytope; every one of its
// vertices is the intersection of three of the twelve planes, found here by enumerating the triples.
// An orthographic (or any w > 0) light projection maps the polytope to a convex set whose bounds are
// the bounds of its projected vertices.  The texel rectangle adds the PCF reach and 2 texels of
// margin for the rounding of the shader's own arithmetic; everything is computed in double.
//
// A tile-sharded rank then renders only the 32x32 shadow-map bin tiles of that rectangle (a region of
// the shadow pass, shs_shard.hpp) -- no shadow map is exchanged between ranks.
#pragma once
#include <math.h>
#include <stdint.h>

#include <algorithm>

namespace shs_fp {

struct TexelRect {
    int x0 = 0, y0 = 0, x1 = -1, y1 = -1;   // inclusive; x1 < x0 or y1 < y0: no texel
    bool empty() const { return x1 < x0 || y1 < y0; }
};

inline TexelRect unite(const TexelRect &a, const TexelRect &b) {
    if (a.empty()) return b;
    if (b.empty()) return a;
    return {std::min(a.x0, b.x0), std::min(a.y0, b.y0), std::max(a.x1, b.x1), std::max(a.y1, b.y1)};
}

// Row i of a column-major 4x4 matrix (glm layout: m[col * 4 + row]).
inline void mat_row(const float *m, int i, double out[4]) {
    for (int c = 0; c < 4; ++c) out[c] = (double)m[c * 4 + i];
}

// The texels of an sm_w x sm_h shadow map that the PCF of a point in (world box [bmin, bmax]) ∩
// (camera frustum slice of the pixel rectangle px = {x0, y0, x1, y1}, inclusive, rows y up, of a W x H
// frame) can read, for a light projection light_vp and a PCF reach of `reach` texels.  Anything that
// cannot be bounded (non-finite input, a polytope point with light w <= 0) gives the whole map.
// (pts / n_pts, when given: the polytope's vertices projected to texel space, at most 220 of them;
// n_pts = -1 when the result is the whole map for lack of a bound.)
inline TexelRect shadow_footprint(const float light_vp[16], int sm_w, int sm_h, const float camera_vp[16], int W, int H,
                                  const int px[4], const double bmin[3], const double bmax[3], int reach,
                                  double (*pts)[2] = nullptr, int *n_pts = nullptr) {
    if (n_pts) *n_pts = -1;
    TexelRect full{0, 0, sm_w - 1, sm_h - 1};
    if (sm_w <= 0 || sm_h <= 0) { if (n_pts) *n_pts = 0; return TexelRect{}; }
    if (px[2] < px[0] || px[3] < px[1]) { if (n_pts) *n_pts = 0; return TexelRect{}; }   // no pixel: nothing is read
    double pl[12][4];
    int n = 0;
    for (int a = 0; a < 3; ++a) {   // the world box: x - min >= 0, max - x >= 0
        double *p = pl[n++];
        p[0] = p[1] = p[2] = 0.0; p[a] = 1.0; p[3] = -bmin[a];
        double *q = pl[n++];
        q[0] = q[1] = q[2] = 0.0; q[a] = -1.0; q[3] = bmax[a];
    }
    double r[4][4];
    for (int i = 0; i < 4; ++i) mat_row(camera_vp, i, r[i]);
    // pixel centres px+0.5 with one pixel of margin, screen = (ndc * 0.5 + 0.5) * (size - 1)
    for (int axis = 0; axis < 2; ++axis) {
        const int size = axis == 0 ? W : H;
        double lo = -1.0, hi = 1.0;
        if (size > 1) {
            lo = 2.0 * ((double)px[axis] + 0.5 - 1.0) / (double)(size - 1) - 1.0;
            hi = 2.0 * ((double)px[axis + 2] + 0.5 + 1.0) / (double)(size - 1) - 1.0;
        }
        lo = std::max(lo, -1.0);   // and inside the clip volume: -w <= x, y <= w
        hi = std::min(hi, 1.0);
        double *p = pl[n++], *q = pl[n++];
        for (int c = 0; c < 4; ++c) {
            p[c] = r[axis][c] - lo * r[3][c];   // ndc >= lo  <=>  c - lo w >= 0 (w > 0)
            q[c] = hi * r[3][c] - r[axis][c];   // ndc <= hi
        }
    }
    {
        double *p = pl[n++], *q = pl[n++];
        for (int c = 0; c < 4; ++c) {
            p[c] = r[2][c] + r[3][c];   // z >= -w
            q[c] = r[3][c] - r[2][c];   // z <= w
        }
    }
    for (int i = 0; i < n; ++i)
        for (int c = 0; c < 4; ++c)
            if (!isfinite(pl[i][c])) return full;
    double lv[4][4];
    for (int i = 0; i < 4; ++i) mat_row(light_vp, i, lv[i]);
    double ux0 = INFINITY, ux1 = -INFINITY, uy0 = INFINITY, uy1 = -INFINITY;
    bool any = false;
    int np_ = 0;
    for (int i = 0; i < n; ++i)
        for (int j = i + 1; j < n; ++j)
            for (int k = j + 1; k < n; ++k) {
                const double *a = pl[i], *b = pl[j], *c = pl[k];
                // a.xyz . p = -a.w etc.: Cramer's rule
                const double det = a[0] * (b[1] * c[2] - b[2] * c[1]) - a[1] * (b[0] * c[2] - b[2] * c[0]) +
                                   a[2] * (b[0] * c[1] - b[1] * c[0]);
                const double na = sqrt(a[0] * a[0] + a[1] * a[1] + a[2] * a[2]);
                const double nb = sqrt(b[0] * b[0] + b[1] * b[1] + b[2] * b[2]);
                const double nc = sqrt(c[0] * c[0] + c[1] * c[1] + c[2] * c[2]);
                if (!(fabs(det) > 1e-12 * na * nb * nc)) continue;
                const double ra = -a[3], rb = -b[3], rc = -c[3];
                const double x = (ra * (b[1] * c[2] - b[2] * c[1]) - a[1] * (rb * c[2] - b[2] * rc) + a[2] * (rb * c[1] - b[1] * rc)) / det;
                const double y = (a[0] * (rb * c[2] - b[2] * rc) - ra * (b[0] * c[2] - b[2] * c[0]) + a[2] * (b[0] * rc - rb * c[0])) / det;
                const double z = (a[0] * (b[1] * rc - rb * c[1]) - a[1] * (b[0] * rc - rb * c[0]) + ra * (b[0] * c[1] - b[1] * c[0])) / det;
                if (!(isfinite(x) && isfinite(y) && isfinite(z))) continue;
                bool inside = true;
                const double mag = fabs(x) + fabs(y) + fabs(z) + 1.0;
                for (int m = 0; m < n && inside; ++m) {
                    const double *p = pl[m];
                    const double s = p[0] * x + p[1] * y + p[2] * z + p[3];
                    const double tol = 1e-9 * (fabs(p[0]) + fabs(p[1]) + fabs(p[2]) + fabs(p[3])) * mag;
                    inside = s >= -tol;
                }
                if (!inside) continue;
                const double w = lv[3][0] * x + lv[3][1] * y + lv[3][2] * z + lv[3][3];
                if (!(w > 1e-8)) return full;
                const double u = ((lv[0][0] * x + lv[0][1] * y + lv[0][2] * z + lv[0][3]) / w) * 0.5 + 0.5;
                const double v = ((lv[1][0] * x + lv[1][1] * y + lv[1][2] * z + lv[1][3]) / w) * 0.5 + 0.5;
                if (!(isfinite(u) && isfinite(v))) return full;
                ux0 = std::min(ux0, u * (sm_w - 1)); ux1 = std::max(ux1, u * (sm_w - 1));
                uy0 = std::min(uy0, v * (sm_h - 1)); uy1 = std::max(uy1, v * (sm_h - 1));
                if (pts && np_ < 220) { pts[np_][0] = u * (sm_w - 1); pts[np_][1] = v * (sm_h - 1); }
                ++np_;
                any = true;
            }
    if (n_pts) *n_pts = std::min(np_, 220);
    if (!any) return TexelRect{};   // the box misses the pixels' frustum slice: no point, no read
    const double m = (double)reach + 2.0;
    auto clampi = [](double v, int hi) { return (int)std::min<double>(std::max<double>(v, 0.0), (double)hi); };
    TexelRect t;
    t.x0 = clampi(floor(ux0 - m), sm_w - 1);
    t.x1 = clampi(ceil(ux1 + m), sm_w - 1);
    t.y0 = clampi(floor(uy0 - m), sm_h - 1);
    t.y1 = clampi(ceil(uy1 + m), sm_h - 1);
    return t;
}

// Per row of `row_h` texels (row r: texel rows r * row_h .. r * row_h + row_h - 1), the texel columns the
// PCF can read: the x extent of the convex hull of the projected vertices (the polytope's image is that
// hull) within the row's band widened by the reach + 2 margin above and below, widened by the same margin
// left and right, clamped to the map.  x1 < x0: nothing in that row is read.  Rows are united into
// x0[] / x1[] (min / max), so several draws' spans can be gathered into one table.  Since round 6: the
// region-sharded shadow pass renders only these tiles of its rectangle.
inline void footprint_rows(const double (*pts)[2], int n, int sm_w, int sm_h, int reach, int row_h, int n_rows, int *x0,
                           int *x1) {
    if (n <= 0) return;
    // Andrew's monotone chain over the points (n <= 220)
    int idx[220];
    const int m_ = std::min(n, 220);
    for (int i = 0; i < m_; ++i) idx[i] = i;
    std::sort(idx, idx + m_, [&](int a, int b) {
        return pts[a][0] < pts[b][0] || (pts[a][0] == pts[b][0] && pts[a][1] < pts[b][1]);
    });
    int hull[441], k = 0;
    auto cross = [&](int o, int a, int b) {
        return (pts[a][0] - pts[o][0]) * (pts[b][1] - pts[o][1]) - (pts[a][1] - pts[o][1]) * (pts[b][0] - pts[o][0]);
    };
    for (int i = 0; i < m_; ++i) {
        while (k >= 2 && cross(hull[k - 2], hull[k - 1], idx[i]) <= 0.0) --k;
        hull[k++] = idx[i];
    }
    for (int i = m_ - 2, lo = k + 1; i >= 0; --i) {
        while (k >= lo && cross(hull[k - 2], hull[k - 1], idx[i]) <= 0.0) --k;
        hull[k++] = idx[i];
    }
    if (k > 1) --k;   // the last point repeats the first
    const double mg = (double)reach + 2.0;
    for (int r = 0; r < n_rows; ++r) {
        const double b0 = (double)r * row_h - mg, b1 = (double)r * row_h + (row_h - 1) + mg;
        double lo = INFINITY, hi = -INFINITY;
        for (int e = 0; e < k; ++e) {   // each hull edge (a single point: a degenerate edge) clipped to the band
            const double *p = pts[hull[e]], *q = pts[hull[(e + 1) % k]];
            double t0 = 0.0, t1 = 1.0;
            const double dy = q[1] - p[1];
            if (dy == 0.0) {
                if (p[1] < b0 || p[1] > b1) continue;
            } else {
                double ta = (b0 - p[1]) / dy, tb = (b1 - p[1]) / dy;
                if (ta > tb) std::swap(ta, tb);
                t0 = std::max(t0, ta);
                t1 = std::min(t1, tb);
                if (t0 > t1) continue;
            }
            const double xa = p[0] + t0 * (q[0] - p[0]), xb = p[0] + t1 * (q[0] - p[0]);
            lo = std::min(lo, std::min(xa, xb));
            hi = std::max(hi, std::max(xa, xb));
        }
        if (!(lo <= hi)) continue;
        const int a = (int)std::min<double>(std::max<double>(floor(lo - mg), 0.0), (double)(sm_w - 1));
        const int b = (int)std::min<double>(std::max<double>(ceil(hi + mg), 0.0), (double)(sm_w - 1));
        if (x1[r] < x0[r]) { x0[r] = a; x1[r] = b; }
        else { x0[r] = std::min(x0[r], a); x1[r] = std::max(x1[r], b); }
    }
    (void)sm_h;
}

// The world box of a mesh's model-space box [b0, b1] under a model matrix (column-major), in double and
// widened by 1e-6 of its magnitude: it contains the float transforms of every vertex of the mesh.
inline void world_box(const float *M, const float b0[3], const float b1[3], double out_min[3], double out_max[3]) {
    for (int a = 0; a < 3; ++a) { out_min[a] = INFINITY; out_max[a] = -INFINITY; }
    for (int k = 0; k < 8; ++k) {
        const double p[3] = {(k & 1) ? b1[0] : b0[0], (k & 2) ? b1[1] : b0[1], (k & 4) ? b1[2] : b0[2]};
        for (int a = 0; a < 3; ++a) {
            const double v = (double)M[a] * p[0] + (double)M[4 + a] * p[1] + (double)M[8 + a] * p[2] + (double)M[12 + a];
            out_min[a] = std::min(out_min[a], v);
            out_max[a] = std::max(out_max[a], v);
        }
    }
    for (int a = 0; a < 3; ++a) {
        const double e = 1e-6 * (fabs(out_min[a]) + fabs(out_max[a]) + 1.0);
        out_min[a] -= e;
        out_max[a] += e;
    }
}

}  // namespace shs_fp
