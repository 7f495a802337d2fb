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
