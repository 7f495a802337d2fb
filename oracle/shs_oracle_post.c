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
