/* shs_oracle_lightbin.c -- TEST INFRASTRUCTURE ONLY (the oracle): the software library's CPU light
 * binning, restated from the reference (paths under cpp-folders/src/shs-renderer-lib/include/shs/):
 *
 *   build_light_bin_culling          lighting/light_culling_runtime.hpp:266-371 (mode dispatch, z clamps)
 *   cull_lights_tiled                 lighting/jolt_light_culling.hpp:135-187
 *   cull_lights_tiled_view_depth_range                             :261-324
 *   cull_lights_clustered                                          :341-412 (log depth slices)
 *   make_screen_tile_cell / unproject_ndc / make_oriented_plane_from_points / ndc_from_view_depth_lh_no
 *                                                                  :36-133
 *   extract_frustum_planes / make_plane_from_vec4   geometry/frustum_culling.hpp:32-65
 *   classify_sphere_vs_cell / classify_aabb_vs_cell / classify_*_vs_frustum / classify_vs_cell
 *                                                   geometry/jolt_culling.hpp:129-257 (tolerance 1e-5)
 *
 * The lights are Jolt SceneShapes (geometry/scene_shape.hpp:56-81); the binning reads only their world
 * AABB and the bounding sphere Jolt derives from it: centre 0.5 * (min + max), radius |0.5 * (max - min)|
 * (JPH::AABox::GetCenter / GetExtent / Vec3::Length, Jolt v5.2.0 -- absent here, its published
 * algorithm restated; "parity unpinned" like the rest of the oracle).  A Jolt sphere of radius r at p
 * has the AABB p -/+ r, so its bounding sphere has radius ~sqrt(3) r.  GLM (absent) is restated in its
 * scalar operation order: dot (x + y) + z, normalize v * (1 / sqrt(dot)), mat4 * vec4
 * (m0 x + m1 y) + (m2 z + m3 w), vec / scalar per component. */
#include <math.h>
#include <stdint.h>
#include <string.h>

#include "shs_oracle.h"

typedef struct { float x, y, z; } v3;
typedef struct { v3 n; float d; } plane_t;

static v3 v3_add(v3 a, v3 b) { v3 r = {a.x + b.x, a.y + b.y, a.z + b.z}; return r; }
static v3 v3_sub(v3 a, v3 b) { v3 r = {a.x - b.x, a.y - b.y, a.z - b.z}; return r; }
static v3 v3_mul(v3 a, float s) { v3 r = {a.x * s, a.y * s, a.z * s}; return r; }
static float v3_dot(v3 a, v3 b) { const float x = a.x * b.x, y = a.y * b.y, z = a.z * b.z; return (x + y) + z; }
static v3 v3_cross(v3 a, v3 b) {
    v3 r = {a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y};
    return r;
}
static v3 v3_normalize(v3 a) { return v3_mul(a, 1.0f / sqrtf(v3_dot(a, a))); }
static float fmaxf_std(float a, float b) { return (a < b) ? b : a; }   /* std::max(a, b) */
static float fminf_std(float a, float b) { return (b < a) ? b : a; }   /* std::min(a, b) */

/* make_plane_from_vec4 (frustum_culling.hpp:32-46) */
static plane_t plane_from_vec4(float x, float y, float z, float w) {
    plane_t p;
    const v3 n = {x, y, z};
    const float len = sqrtf(v3_dot(n, n));
    if (len <= 1e-8f) {
        p.n.x = 0.0f; p.n.y = 1.0f; p.n.z = 0.0f;
        p.d = w;
        return p;
    }
    p.n.x = n.x / len; p.n.y = n.y / len; p.n.z = n.z / len;
    p.d = w / len;
    return p;
}

/* extract_frustum_planes (frustum_culling.hpp:48-65): rows of the column-major view_proj */
static void frustum_planes(const float *m, plane_t out[6]) {
    float r[4][4];
    for (int row = 0; row < 4; ++row)
        for (int c = 0; c < 4; ++c) r[row][c] = m[4 * c + row];
    for (int k = 0; k < 3; ++k) {
        out[2 * k] = plane_from_vec4(r[3][0] + r[k][0], r[3][1] + r[k][1], r[3][2] + r[k][2], r[3][3] + r[k][3]);
        out[2 * k + 1] = plane_from_vec4(r[3][0] - r[k][0], r[3][1] - r[k][1], r[3][2] - r[k][2], r[3][3] - r[k][3]);
    }
}

static float signed_distance(const plane_t *p, v3 q) { return v3_dot(p->n, q) + p->d; }

enum { CC_OUTSIDE = 0, CC_INTERSECTING = 1, CC_INSIDE = 2 };

/* classify_sphere_vs_cell / _vs_frustum (jolt_culling.hpp:129-145, 187-201) */
static int classify_sphere(v3 c, float radius, const plane_t *pl, int n) {
    const float r = fmaxf_std(radius, 0.0f);
    int fully_inside = 1;
    for (int i = 0; i < n; ++i) {
        const float dist = signed_distance(&pl[i], c);
        if (dist < -(r + 1e-5f)) return CC_OUTSIDE;
        if (dist < (r + 1e-5f)) fully_inside = 0;
    }
    return fully_inside ? CC_INSIDE : CC_INTERSECTING;
}

/* classify_aabb_vs_cell / _vs_frustum (:151-181, 207-229): p- and n-vertices */
static int classify_aabb(v3 mn, v3 mx, const plane_t *pl, int n) {
    int fully_inside = 1;
    for (int i = 0; i < n; ++i) {
        const plane_t *p = &pl[i];
        const v3 pv = {p->n.x >= 0.0f ? mx.x : mn.x, p->n.y >= 0.0f ? mx.y : mn.y, p->n.z >= 0.0f ? mx.z : mn.z};
        if (signed_distance(p, pv) < -1e-5f) return CC_OUTSIDE;
        const v3 nv = {p->n.x >= 0.0f ? mn.x : mx.x, p->n.y >= 0.0f ? mn.y : mx.y, p->n.z >= 0.0f ? mn.z : mx.z};
        if (signed_distance(p, nv) < 1e-5f) fully_inside = 0;
    }
    return fully_inside ? CC_INSIDE : CC_INTERSECTING;
}

/* classify_vs_cell / classify_vs_frustum (:241-257, 260-275): the bounding sphere first, then the AABB */
static int classify_shape(const v3 *mn, const v3 *mx, const plane_t *pl, int n) {
    const v3 c = v3_mul(v3_add(*mn, *mx), 0.5f);
    const v3 e = v3_mul(v3_sub(*mx, *mn), 0.5f);
    const float radius = sqrtf(v3_dot(e, e));
    const int b = classify_sphere(c, radius, pl, n);
    if (b != CC_INTERSECTING) return b;
    return classify_aabb(*mn, *mx, pl, n);
}

/* unproject_ndc (jolt_light_culling.hpp:52-58): inv_vp * vec4(ndc, 1), xyz / w */
static v3 unproject(const float *m, float x, float y, float z) {
    float c[4];
    for (int r = 0; r < 4; ++r) c[r] = (m[r] * x + m[4 + r] * y) + (m[8 + r] * z + m[12 + r] * 1.0f);
    v3 o = {c[0] / c[3], c[1] / c[3], c[2] / c[3]};
    return o;
}

/* make_oriented_plane_from_points (:36-50) */
static plane_t oriented_plane(v3 a, v3 b, v3 c, v3 inside) {
    plane_t p;
    p.n = v3_normalize(v3_cross(v3_sub(b, a), v3_sub(c, a)));
    p.d = -v3_dot(p.n, a);
    if (v3_dot(p.n, inside) + p.d < 0.0f) {
        p.n.x = -p.n.x; p.n.y = -p.n.y; p.n.z = -p.n.z;
        p.d = -p.d;
    }
    return p;
}

/* make_screen_tile_cell (:95-133) */
static void tile_cell(uint32_t tx, uint32_t ty, uint32_t ts, uint32_t W, uint32_t H, const float *inv, float zn_ndc,
                      float zf_ndc, plane_t out[6]) {
    const float x0 = (float)(tx * ts) / (float)W * 2.0f - 1.0f;
    const uint32_t xe = (tx + 1) * ts < W ? (tx + 1) * ts : W;
    const float x1 = (float)xe / (float)W * 2.0f - 1.0f;
    const float y_top = 1.0f - (float)(ty * ts) / (float)H * 2.0f;
    const uint32_t ye = (ty + 1) * ts < H ? (ty + 1) * ts : H;
    const float y_bottom = 1.0f - (float)ye / (float)H * 2.0f;
    const v3 nbl = unproject(inv, x0, y_bottom, zn_ndc), nbr = unproject(inv, x1, y_bottom, zn_ndc);
    const v3 ntl = unproject(inv, x0, y_top, zn_ndc), ntr = unproject(inv, x1, y_top, zn_ndc);
    const v3 fbl = unproject(inv, x0, y_bottom, zf_ndc), fbr = unproject(inv, x1, y_bottom, zf_ndc);
    const v3 ftl = unproject(inv, x0, y_top, zf_ndc), ftr = unproject(inv, x1, y_top, zf_ndc);
    const v3 inside = v3_mul(v3_add(v3_add(v3_add(nbl, ntr), fbl), ftr), 0.25f);
    out[0] = oriented_plane(nbl, nbr, ntr, inside);   /* near */
    out[1] = oriented_plane(fbr, fbl, ftl, inside);   /* far */
    out[2] = oriented_plane(nbl, ntl, ftl, inside);   /* left */
    out[3] = oriented_plane(nbr, fbr, ftr, inside);   /* right */
    out[4] = oriented_plane(nbl, fbl, fbr, inside);   /* bottom */
    out[5] = oriented_plane(ntl, ntr, ftr, inside);   /* top */
}

/* ndc_from_view_depth_lh_no (:84-92) */
static float ndc_from_view_depth(float view_depth, float z_near, float z_far) {
    const float n = fmaxf_std(z_near, 1e-4f);
    const float f = fmaxf_std(z_far, n + 1e-3f);
    const float z = view_depth < n ? n : (f < view_depth ? f : view_depth);   /* std::clamp */
    const float denom = fmaxf_std(f - n, 1e-6f);
    return ((f + n) / denom) - ((2.0f * f * n) / (denom * z));
}

int ora_light_bin_culling(const ora_light_bin_desc *d, const float *aabbs, int n_lights, uint32_t *bins_xyz,
                          uint32_t *counts, uint32_t *indices) {
    const uint32_t ts = d->tile_size > 1u ? d->tile_size : 1u;
    const float zn = fmaxf_std(d->z_near, 1e-4f);
    const float zf = fmaxf_std(d->z_far, zn + 1e-3f);
    const uint32_t bx = ((uint32_t)d->width + ts - 1u) / ts, by = ((uint32_t)d->height + ts - 1u) / ts;
    const uint32_t slices = d->mode == 3u ? (d->z_slices > 1u ? d->z_slices : 1u) : 1u;
    /* mode None or no lights: no bins (LightBinCullingData's defaults, light_culling_runtime.hpp:285-301) */
    bins_xyz[0] = bins_xyz[1] = bins_xyz[2] = 0u;
    if (d->mode == 0u || n_lights <= 0) return 0;
    bins_xyz[0] = bx; bins_xyz[1] = by; bins_xyz[2] = slices;
    const size_t n_bins = (size_t)bx * by * slices;
    memset(counts, 0, n_bins * sizeof(uint32_t));
    float inv[16];
    ora_mat4_inverse(d->view_proj, inv);
    plane_t fr[6];
    frustum_planes(d->view_proj, fr);
    unsigned char *vis = (unsigned char *)__builtin_alloca((size_t)n_lights);
    for (int li = 0; li < n_lights; ++li) {
        const v3 mn = {aabbs[6 * li], aabbs[6 * li + 1], aabbs[6 * li + 2]};
        const v3 mx = {aabbs[6 * li + 3], aabbs[6 * li + 4], aabbs[6 * li + 5]};
        vis[li] = classify_shape(&mn, &mx, fr, 6) != CC_OUTSIDE;
    }
    const int depth_ok = d->mode == 2u && d->tile_min_view_depth && d->tile_max_view_depth &&
                         d->n_depth_tiles == (int32_t)(bx * by);
    const float log_ratio = logf(zf / zn);
    for (uint32_t cz = 0; cz < slices; ++cz) {
        float s_near = -1.0f, s_far = 1.0f;
        if (d->mode == 3u) {
            const float slice_near = zn * expf(log_ratio * (float)cz / (float)slices);
            const float slice_far = zn * expf(log_ratio * (float)(cz + 1) / (float)slices);
            s_near = ndc_from_view_depth(slice_near, zn, zf);
            s_far = ndc_from_view_depth(slice_far, zn, zf);
        }
        for (uint32_t ty = 0; ty < by; ++ty)
            for (uint32_t tx = 0; tx < bx; ++tx) {
                const uint32_t tile = ty * bx + tx;
                float n_ndc = s_near, f_ndc = s_far;
                if (depth_ok) {
                    n_ndc = ndc_from_view_depth(d->tile_min_view_depth[tile], zn, zf);
                    f_ndc = ndc_from_view_depth(d->tile_max_view_depth[tile], zn, zf);
                }
                plane_t cell[6];
                tile_cell(tx, ty, ts, (uint32_t)d->width, (uint32_t)d->height, inv, n_ndc, f_ndc, cell);
                const size_t bin = (size_t)cz * bx * by + tile;
                uint32_t k = 0;
                for (int li = 0; li < n_lights; ++li) {
                    if (!vis[li]) continue;
                    const v3 mn = {aabbs[6 * li], aabbs[6 * li + 1], aabbs[6 * li + 2]};
                    const v3 mx = {aabbs[6 * li + 3], aabbs[6 * li + 4], aabbs[6 * li + 5]};
                    if (classify_shape(&mn, &mx, cell, 6) != CC_OUTSIDE) {
                        if (k < d->max_per_bin) indices[bin * d->max_per_bin + k] = (uint32_t)li;
                        ++k;
                    }
                }
                counts[bin] = k;
            }
    }
    (void)fminf_std;
    return 0;
}
