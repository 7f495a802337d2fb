/* shs_oracle_canvas_post.c -- TEST INFRASTRUCTURE ONLY (the checker of SURVEY.md 8f row 4's
 * Canvas-API extras; never linked into the product).  Sequential CPU restatements, paths relative to
 * /root/reference/cpp-folders/src/hello-render-target/:
 *   ora_canvas_motion_blur   combined_motion_blur_pass (hello_pbr.cpp:1128-1252) with
 *                            viewz_to_ndcz / canvas_to_ndc_xy / ndc_to_screen_xy /
 *                            compute_camera_velocity_canvas_fast (:1051-1109), apply_soft_knee (:1111-1122);
 *   ora_canvas_gaussian      gaussian_blur_pass (hello_depth_of_field.cpp:175-251);
 *   ora_canvas_autofocus     autofocus_depth_median_center (:257-285), nth_element as a sort;
 *   ora_canvas_dof           the DoF step of :786-812 with dof_composite_pass (:287-343).
 * Matrices: curr_vp = proj * view and glm::inverse via this oracle's own ora_mat4_mul /
 * ora_mat4_inverse.  Colours are 4 bytes per pixel, buffers y * W + x. */
#include <float.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "shs_oracle.h"

static void cp_m4v(const float *m, float x, float y, float z, float w, float *o) {
    for (int r = 0; r < 4; ++r) o[r] = (m[r] * x + m[4 + r] * y) + (m[8 + r] * z + m[12 + r] * w);
}
static int cp_clampi(int v, int lo, int hi) { return (v < lo) ? lo : (v > hi ? hi : v); }
static float cp_clampf(float v, float lo, float hi) {
    if (v < lo) return lo;
    if (v > hi) return hi;
    return v;
}

static void cam_velocity(int x, int y, float view_z, int W, int H, const float *prev_vp, const float *inv_vp,
                         const float *proj, float *v) {
    v[0] = v[1] = 0.0f;
    if (view_z == FLT_MAX) return;
    const int py_screen = (H - 1) - y;
    const float fx = ((float)x + 0.5f) / (float)W;
    const float fy = ((float)py_screen + 0.5f) / (float)H;
    const float ndc_x = fx * 2.0f - 1.0f, ndc_y = 1.0f - fy * 2.0f;
    float c[4];
    cp_m4v(proj, 0.0f, 0.0f, view_z, 1.0f, c);
    const float ndc_z = (fabsf(c[3]) < 1e-6f) ? 0.0f : c[2] / c[3];
    float wh[4];
    cp_m4v(inv_vp, ndc_x, ndc_y, ndc_z, 1.0f, wh);
    if (fabsf(wh[3]) < 1e-6f) return;
    const float world[3] = {wh[0] / wh[3], wh[1] / wh[3], wh[2] / wh[3]};
    float pc[4];
    cp_m4v(prev_vp, world[0], world[1], world[2], 1.0f, pc);
    if (fabsf(pc[3]) < 1e-6f) return;
    const float pn[2] = {pc[0] / pc[3], pc[1] / pc[3]};
    const float psx = (pn[0] * 0.5f + 0.5f) * (float)(W - 1);
    const float psy = (1.0f - (pn[1] * 0.5f + 0.5f)) * (float)(H - 1);
    const float vs[2] = {(float)x - psx, (float)py_screen - psy};
    v[0] = vs[0];
    v[1] = -vs[1];
}

void ora_canvas_motion_blur(const uint8_t *src, const float *depth, const float *vel, uint8_t *dst, int W, int H,
                            const float *curr_view, const float *curr_proj, const float *prev_view,
                            const float *prev_proj, int samples, float strength, float w_obj, float w_cam,
                            int soft_knee, float knee, float max_px) {
    float curr_vp[16], prev_vp[16], inv_vp[16];
    ora_mat4_mul(curr_proj, curr_view, curr_vp);
    ora_mat4_mul(prev_proj, prev_view, prev_vp);
    ora_mat4_inverse(curr_vp, inv_vp);
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
            const size_t i = (size_t)y * W + x;
            float vc[2];
            cam_velocity(x, y, depth[i], W, H, prev_vp, inv_vp, curr_proj, vc);
            const float vo[2] = {vel[2 * i] - vc[0], vel[2 * i + 1] - vc[1]};
            float vt[2] = {w_obj * vo[0] + w_cam * vc[0], w_obj * vo[1] + w_cam * vc[1]};
            vt[0] *= strength;
            vt[1] *= strength;
            if (soft_knee) {
                const float len = sqrtf(vt[0] * vt[0] + vt[1] * vt[1]);
                if (!(len <= 1e-6f) && !(len <= knee)) {
                    const float den = max_px - knee;
                    const float t = (len - knee) / ((1e-6f < den) ? den : 1e-6f);   /* std::max(1e-6f, den) */
                    const float t2 = t / (1.0f + t);
                    const float new_len = knee + (max_px - knee) * t2;
                    const float s = new_len / len;
                    vt[0] *= s;
                    vt[1] *= s;
                }
            }
            float len = sqrtf(vt[0] * vt[0] + vt[1] * vt[1]);
            if (len > max_px && len > 1e-6f) {
                const float s = max_px / len;
                vt[0] *= s;
                vt[1] *= s;
                len = max_px;
            }
            if (len < 0.001f || samples <= 1) {
                memcpy(dst + 4 * i, src + 4 * i, 4);
                continue;
            }
            const float dir[2] = {vt[0] / len, vt[1] / len};
            float r = 0, g = 0, b = 0, wsum = 0.0f;
            for (int k = 0; k < samples; ++k) {
                const float t = (samples == 1) ? 0.0f : ((float)k / (float)(samples - 1));
                const float a = (t - 0.5f) * 2.0f;
                const float p[2] = {(float)x + dir[0] * (a * len), (float)y + dir[1] * (a * len)};
                const float rx = roundf(p[0]), ry = roundf(p[1]);
                /* (int) of NaN: x86 gives INT_MIN, which the clamp maps to 0 */
                const int sx = cp_clampi(rx == rx ? (int)rx : INT32_MIN, 0, W - 1);
                const int sy = cp_clampi(ry == ry ? (int)ry : INT32_MIN, 0, H - 1);
                const float wgt = 1.0f - fabsf(a);
                const uint8_t *c = src + 4 * ((size_t)sy * W + sx);
                r += wgt * (float)c[0];
                g += wgt * (float)c[1];
                b += wgt * (float)c[2];
                wsum += wgt;
            }
            if (wsum < 0.0001f) wsum = 1.0f;
            uint8_t *o = dst + 4 * i;
            o[0] = (uint8_t)cp_clampi((int)(r / wsum), 0, 255);
            o[1] = (uint8_t)cp_clampi((int)(g / wsum), 0, 255);
            o[2] = (uint8_t)cp_clampi((int)(b / wsum), 0, 255);
            o[3] = 255;
        }
}

void ora_canvas_gaussian(const uint8_t *src, uint8_t *dst, int W, int H, int horizontal) {
    const float w0 = 0.06136f, w1 = 0.24477f, w2 = 0.38774f;
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
            const uint8_t *c[5];
            for (int k = 0; k < 5; ++k) {
                const int sx = horizontal ? cp_clampi(x + k - 2, 0, W - 1) : x;
                const int sy = horizontal ? y : cp_clampi(y + k - 2, 0, H - 1);
                c[k] = src + 4 * ((size_t)sy * W + sx);
            }
            for (int ch = 0; ch < 4; ++ch) {
                float v = w0 * c[0][ch] + w1 * c[1][ch] + w2 * c[2][ch] + w1 * c[3][ch] + w0 * c[4][ch];
                v = (0.0f < v) ? v : 0.0f;
                v = (v < 255.0f) ? v : 255.0f;
                dst[4 * ((size_t)y * W + x) + ch] = (uint8_t)v;
            }
        }
}

static int cp_cmpf(const void *a, const void *b) {
    const float x = *(const float *)a, y = *(const float *)b;
    return (x < y) ? -1 : (y < x ? 1 : 0);
}

float ora_canvas_autofocus(const float *depth, int W, int H, int cx, int cy, int radius) {
    const int side = 2 * radius + 1;
    float *s = (float *)malloc(sizeof(float) * (size_t)side * side);
    int n = 0;
    for (int dy = -radius; dy <= radius; ++dy)
        for (int dx = -radius; dx <= radius; ++dx) {
            const int x = cx + dx, y = cy + dy;
            const float d = (x >= 0 && x < W && y >= 0 && y < H) ? depth[(size_t)y * W + x] : FLT_MAX;
            if (d == FLT_MAX) continue;
            s[n++] = d;
        }
    float out;
    if (n == 0) {
        const float d = (cx >= 0 && cx < W && cy >= 0 && cy < H) ? depth[(size_t)cy * W + cx] : FLT_MAX;
        out = (d == FLT_MAX) ? 15.0f : d;
    } else {
        qsort(s, (size_t)n, sizeof(float), cp_cmpf);   /* the element nth_element leaves at n / 2 */
        out = s[n / 2];
    }
    free(s);
    return out;
}

float ora_canvas_dof(uint8_t *color, const float *depth, uint8_t *blur_out, int W, int H, int iterations, int radius,
                     int cx, int cy, float range, float max_blur) {
    const size_t n = (size_t)W * H * 4;
    uint8_t *sharp = (uint8_t *)malloc(n), *pong = (uint8_t *)malloc(n);
    memcpy(sharp, color, n);
    memcpy(pong, sharp, n);
    for (int i = 0; i < iterations; ++i) {
        ora_canvas_gaussian(pong, color, W, H, 1);   /* pong -> ping */
        ora_canvas_gaussian(color, pong, W, H, 0);   /* ping -> pong */
    }
    const float focus = ora_canvas_autofocus(depth, W, H, cx, cy, radius);
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
            const size_t i = (size_t)y * W + x;
            float d = depth[i];
            if (d == FLT_MAX) d = focus + range;
            const float coc = fabsf(d - focus) / range;
            float t = cp_clampf(coc, 0.0f, 1.0f);
            t = t * t * (3.0f - 2.0f * t);
            t = cp_clampf(t * max_blur, 0.0f, 1.0f);
            t = cp_clampf(t, 0.0f, 1.0f);
            const float ia = 1.0f - t;
            for (int ch = 0; ch < 3; ++ch) color[4 * i + ch] = (uint8_t)(int)(ia * sharp[4 * i + ch] + t * pong[4 * i + ch]);
            color[4 * i + 3] = 255;
        }
    if (blur_out) memcpy(blur_out, pong, n);
    free(sharp);
    free(pong);
    return focus;
}
