/* shs_oracle_post.c -- TEST INFRASTRUCTURE ONLY (the oracle; never linked by the product).
 *
 * CPU restatement of the passes right after the raster path, for the parity tests:
 *   PassTonemap::execute   shs-renderer-lib/include/shs/passes/pass_tonemap.hpp:36-83
 *     exposure = max(0.0001, fp.exposure), inv_gamma = 1 / max(0.001, fp.gamma); per channel
 *     c = max(0, s * exposure); c = c / (1 + c); c = pow(c, inv_gamma);
 *     byte = clamp((int)lround(c * 255), 0, 255); alpha 255.
 *   upload_ldr_to_rgba8    exp-plumbing/hello_pass_basics.cpp:102-119
 *     the RGBA8 staging of the SDL texture: canvas rows (y up) flipped to screen rows, alpha 255.
 * Paths relative to /root/reference/cpp-folders/src/.  std::max/std::clamp semantics are kept
 * ((a < b) ? b : a; NaN in the second argument of max(0, v) gives 0), std::pow(float, float) is
 * powf and std::lround is lround, so the bytes are the reference's on this libm (glibc). */
#include <math.h>
#include <stddef.h>
#include <stdint.h>
#include <stdlib.h>

#include "shs_oracle.h"

static inline float std_max(float a, float b) { return (a < b) ? b : a; }

/* One channel of PassTonemap (pass_tonemap.hpp:63-79). */
uint8_t ora_tonemap_channel(float s, float exposure, float inv_gamma) {
    float c = std_max(0.0f, s * exposure);
    c = c / (1.0f + c);
    c = powf(c, inv_gamma);
    int v = (int)lround(c * 255.0f);
    if (v < 0) v = 0;
    if (v > 255) v = 255;
    return (uint8_t)v;
}

/* hdr: W*H*4 floats (RT_ColorHDR, rows y up); ldr (RT_ColorLDR, rows y up) and present
 * (upload_ldr_to_rgba8, rows top-down) W*H*4 bytes each, either may be NULL. */
void ora_tonemap(const float *hdr, int W, int H, float exposure_param, float gamma_param, uint8_t *ldr,
                 uint8_t *present) {
    const float exposure = std_max(0.0001f, exposure_param);
    const float inv_gamma = 1.0f / std_max(0.001f, gamma_param);
    for (int y = 0; y < H; ++y) {
        for (int x = 0; x < W; ++x) {
            const float *s = hdr + ((size_t)y * W + x) * 4;
            uint8_t px[4];
            px[0] = ora_tonemap_channel(s[0], exposure, inv_gamma);
            px[1] = ora_tonemap_channel(s[1], exposure, inv_gamma);
            px[2] = ora_tonemap_channel(s[2], exposure, inv_gamma);
            px[3] = 255;
            if (ldr) {
                uint8_t *d = ldr + ((size_t)y * W + x) * 4;
                for (int k = 0; k < 4; ++k) d[k] = px[k];
            }
            if (present) {
                uint8_t *d = present + ((size_t)(H - 1 - y) * W + x) * 4;
                for (int k = 0; k < 4; ++k) d[k] = px[k];
            }
        }
    }
}

/* PassMotionBlur::execute (shs-renderer-lib/include/shs/passes/pass_motion_blur.hpp:38-170) on one
 * RT_ColorLDR (src, rows y up) with the RT_ColorDepthMotion depth / motion planes (rows y up) into
 * dst (W*H*4 bytes).  samples / strength / velocities / depth_reject are FrameParams::pass.motion_blur,
 * dt is FrameParams::dt.  enable = 0 copies src. */
static inline int clampi_(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }
static inline float clampf_(float v, float lo, float hi) { return (v < lo) ? lo : ((hi < v) ? hi : v); }

void ora_motion_blur(const uint8_t *src, const float *depth, const float *motion, int W, int H, int enable,
                     int samples_param, float strength_param, float max_vel_param, float min_vel_param,
                     float depth_reject_param, float dt, uint8_t *dst) {
    if (!enable) {
        for (size_t i = 0; i < (size_t)W * H * 4; ++i) dst[i] = src[i];
        return;
    }
    const int samples = clampi_(samples_param, 4, 32);
    const float strength = std_max(0.0f, strength_param);
    const float max_vel = std_max(1.0f, max_vel_param);
    const float min_vel = std_max(0.0f, min_vel_param);
    const float depth_eps = std_max(0.0f, depth_reject_param);
    const float dt_scale = clampf_(std_max(dt, 1e-4f) * 60.0f, 0.5f, 2.5f);
    for (int y = 0; y < H; ++y) {
        for (int x = 0; x < W; ++x) {
            const size_t o = (size_t)y * W + x;
            uint8_t *d = dst + o * 4;
            const uint8_t *c0 = src + o * 4;
            float vx = motion[2 * o] * strength * dt_scale;
            float vy = motion[2 * o + 1] * strength * dt_scale;
            const float len = sqrtf(vx * vx + vy * vy);
            if (len < min_vel) {
                for (int k = 0; k < 4; ++k) d[k] = c0[k];
                continue;
            }
            if (len > max_vel && len > 1e-6f) {
                const float s = max_vel / len;
                vx *= s;
                vy *= s;
            }
            const float center_depth = depth[o];
            float ar = 0.0f, ag = 0.0f, ab = 0.0f, aw = 0.0f;
            for (int i = 0; i < samples; ++i) {
                const float t = ((float)i / (float)(samples - 1) - 0.5f);
                const int sx = clampi_((int)lround((float)x + vx * t), 0, W - 1);
                const int sy = clampi_((int)lround((float)y + vy * t), 0, H - 1);
                const float sd = depth[(size_t)sy * W + sx];
                if (fabsf(sd - center_depth) > depth_eps) continue;
                const uint8_t *sc = src + ((size_t)sy * W + sx) * 4;
                ar += (float)sc[0];
                ag += (float)sc[1];
                ab += (float)sc[2];
                aw += 1.0f;
            }
            if (aw < 1.0f) {
                for (int k = 0; k < 4; ++k) d[k] = c0[k];
                continue;
            }
            d[0] = (uint8_t)clampi_((int)lround(ar / aw), 0, 255);
            d[1] = (uint8_t)clampi_((int)lround(ag / aw), 0, 255);
            d[2] = (uint8_t)clampi_((int)lround(ab / aw), 0, 255);
            d[3] = 255;
        }
    }
}

/* ---- software occlusion ---------------------------------------------------
 * culling_sw::run_software_occlusion_pass (shs-renderer-lib/include/shs/geometry/culling_software.hpp
 * :229-331) as scene_culling.hpp:187-219 drives it: the frustum-visible objects sorted by the view z of
 * their world AABB centre (view_depth_of_aabb_center :220-227; ties keep the input order), each tested
 * with project_aabb_to_screen_rect (:137-197) + is_rect_occluded (:199-218) against the occlusion depth
 * and, when visible, rasterized into it by rasterize_mesh_depth_transformed (:111-135) ->
 * rasterize_depth_triangle (:65-109), project_world_to_screen (:44-63).  GLM op order as elsewhere:
 * mat4 * vec4 = (m0 x + m1 y) + (m2 z + m3 w); std::min / std::max keep their (a, b) semantics. */
static inline float std_min(float a, float b) { return (b < a) ? b : a; }

static void m4v_(const float *m, const float *v, float *o) {
    for (int r = 0; r < 4; ++r) o[r] = (m[r] * v[0] + m[4 + r] * v[1]) + (m[8 + r] * v[2] + m[12 + r] * v[3]);
}

static inline float edge_fn(const float *a, const float *b, const float *p) {
    return (p[0] - a[0]) * (b[1] - a[1]) - (p[1] - a[1]) * (b[0] - a[0]);
}

static int project_w2s(const float *world, const float *vp, int W, int H, float *xy, float *z01) {
    const float w4[4] = {world[0], world[1], world[2], 1.0f};
    float c[4];
    m4v_(vp, w4, c);
    if (c[3] <= 0.001f) return 0;
    const float nx = c[0] / c[3], ny = c[1] / c[3], nz = c[2] / c[3];
    if (nz < -1.0f || nz > 1.0f) return 0;
    xy[0] = (nx + 1.0f) * 0.5f * (float)W;
    xy[1] = (ny + 1.0f) * 0.5f * (float)H;
    *z01 = nz * 0.5f + 0.5f;
    return 1;
}

static void raster_depth_tri(float *depth, int W, int H, const float *p0, float z0, const float *p1, float z1,
                             const float *p2, float z2) {
    const float area = edge_fn(p0, p1, p2);
    if (fabsf(area) <= 1e-6f) return;
    const float min_xf = std_min(p0[0], std_min(p1[0], p2[0])), min_yf = std_min(p0[1], std_min(p1[1], p2[1]));
    const float max_xf = std_max(p0[0], std_max(p1[0], p2[0])), max_yf = std_max(p0[1], std_max(p1[1], p2[1]));
    int min_x = (int)floorf(min_xf), min_y = (int)floorf(min_yf), max_x = (int)ceilf(max_xf), max_y = (int)ceilf(max_yf);
    min_x = min_x < 0 ? 0 : min_x;
    min_y = min_y < 0 ? 0 : min_y;
    max_x = max_x > W - 1 ? W - 1 : max_x;
    max_y = max_y > H - 1 ? H - 1 : max_y;
    if (min_x > max_x || min_y > max_y) return;
    const int ccw = area > 0.0f;
    for (int y = min_y; y <= max_y; ++y) {
        for (int x = min_x; x <= max_x; ++x) {
            const float p[2] = {(float)x + 0.5f, (float)y + 0.5f};
            const float w0 = edge_fn(p1, p2, p), w1 = edge_fn(p2, p0, p), w2 = edge_fn(p0, p1, p);
            const int inside = ccw ? (w0 >= 0.0f && w1 >= 0.0f && w2 >= 0.0f) : (w0 <= 0.0f && w1 <= 0.0f && w2 <= 0.0f);
            if (!inside) continue;
            const float d = (w0 / area) * z0 + (w1 / area) * z1 + (w2 / area) * z2;
            if (d < 0.0f || d > 1.0f) continue;
            float *dst = depth + (size_t)y * W + x;
            if (d < *dst) *dst = d;
        }
    }
}

/* project_aabb_to_screen_rect: rect4 = {x_min, y_min, x_max, y_max}; returns valid, *z_near */
static int aabb_rect(const float *mn, const float *mx, const float *vp, int W, int H, int *rect4, float *z_near) {
    float min_x = (float)W, min_y = (float)H, max_x = -1.0f, max_y = -1.0f, near_depth = 1.0f;
    int any = 0;
    for (int i = 0; i < 8; ++i) {
        const float c[4] = {(i & 1) ? mx[0] : mn[0], (i & 2) ? mx[1] : mn[1], (i & 4) ? mx[2] : mn[2], 1.0f};
        float clip[4];
        m4v_(vp, c, clip);
        if (clip[3] <= 0.001f) continue;
        const float nx = clip[0] / clip[3], ny = clip[1] / clip[3], nz = clip[2] / clip[3];
        const float z01 = nz * 0.5f + 0.5f;
        if (z01 < 0.0f || z01 > 1.0f) continue;
        const float sx = (nx + 1.0f) * 0.5f * (float)W, sy = (ny + 1.0f) * 0.5f * (float)H;
        min_x = std_min(min_x, sx);
        min_y = std_min(min_y, sy);
        max_x = std_max(max_x, sx);
        max_y = std_max(max_y, sy);
        near_depth = std_min(near_depth, z01);
        any = 1;
    }
    if (!any) return 0;
    int x0 = (int)floorf(min_x), y0 = (int)floorf(min_y), x1 = (int)ceilf(max_x), y1 = (int)ceilf(max_y);
    rect4[0] = x0 < 0 ? 0 : x0;
    rect4[1] = y0 < 0 ? 0 : y0;
    rect4[2] = x1 > W - 1 ? W - 1 : x1;
    rect4[3] = y1 > H - 1 ? H - 1 : y1;
    *z_near = (near_depth < 0.0f) ? 0.0f : ((1.0f < near_depth) ? 1.0f : near_depth);
    return rect4[0] <= rect4[2] && rect4[1] <= rect4[3];
}

int ora_occlusion_pass(const ora_occ_object *objs, int n_objects, const uint32_t *frustum_visible, int n_fv, int enable,
                       float *depth, int W, int H, const float *view16, const float *vp16, float eps,
                       uint8_t *occluded, uint32_t *visible_out) {
    int n_vis = 0;
    for (int i = 0; i < n_objects; ++i) occluded[i] = 0;
    if (!enable) {
        for (int k = 0; k < n_fv; ++k)
            if ((int)frustum_visible[k] < n_objects) visible_out[n_vis++] = frustum_visible[k];
        return n_vis;
    }
    for (size_t i = 0; i < (size_t)W * H; ++i) depth[i] = 1.0f;
    /* sort by the view z of the AABB centre (stable: equal keys keep the input order) */
    uint32_t *order = (uint32_t *)malloc(sizeof(uint32_t) * (size_t)(n_fv > 0 ? n_fv : 1));
    float *key = (float *)malloc(sizeof(float) * (size_t)(n_fv > 0 ? n_fv : 1));
    int n = 0;
    for (int k = 0; k < n_fv; ++k) {
        const uint32_t idx = frustum_visible[k];
        if ((int)idx >= n_objects) continue;
        const ora_occ_object *o = &objs[idx];
        const float c[4] = {0.5f * (o->aabb_min[0] + o->aabb_max[0]), 0.5f * (o->aabb_min[1] + o->aabb_max[1]),
                            0.5f * (o->aabb_min[2] + o->aabb_max[2]), 1.0f};
        float v[4];
        m4v_(view16, c, v);
        /* insertion into the sorted prefix (stable) */
        int j = n;
        while (j > 0 && v[2] < key[j - 1]) {
            key[j] = key[j - 1];
            order[j] = order[j - 1];
            --j;
        }
        key[j] = v[2];
        order[j] = idx;
        ++n;
    }
    for (int s = 0; s < n; ++s) {
        const ora_occ_object *o = &objs[order[s]];
        int rect[4];
        float z_near = 1.0f;
        int occ = 0;
        if (aabb_rect(o->aabb_min, o->aabb_max, vp16, W, H, rect, &z_near)) {
            occ = 1;
            for (int y = rect[1]; y <= rect[3] && occ; ++y)
                for (int x = rect[0]; x <= rect[2]; ++x)
                    if (z_near <= depth[(size_t)y * W + x] + eps) { occ = 0; break; }
        }
        occluded[order[s]] = (uint8_t)occ;
        if (occ) continue;
        visible_out[n_vis++] = order[s];
        for (int t = 0; t + 2 < o->n_idx; t += 3) {
            float sp[3][2], sz[3];
            int ok = 1;
            for (int k = 0; k < 3 && ok; ++k) {
                const uint32_t vi = o->idx[t + k];
                if ((int)vi >= o->n_verts) { ok = 0; break; }
                const float lp[4] = {o->pos[3 * vi], o->pos[3 * vi + 1], o->pos[3 * vi + 2], 1.0f};
                float wp[4];
                m4v_(o->model, lp, wp);
                ok = project_w2s(wp, vp16, W, H, sp[k], &sz[k]);
            }
            if (ok) raster_depth_tri(depth, W, H, sp[0], sz[0], sp[1], sz[1], sp[2], sz[2]);
        }
    }
    free(order);
    free(key);
    return n_vis;
}
