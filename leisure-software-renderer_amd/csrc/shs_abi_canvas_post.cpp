// shs_abi_canvas_post.cpp -- C ABI of the Canvas-API multi-pass extras (include/shs_gpu.h, SURVEY.md
// 8f row 4), paths relative to /root/reference/cpp-folders/src/hello-render-target/:
//   shs_canvas_motion_blur    combined_motion_blur_pass (hello_pbr.cpp:1128-1252) as the PASS2 step of
//                             hello_pbr.cpp:1695-1725 calls it (curr / prev camera matrices);
//   shs_canvas_gaussian_blur  gaussian_blur_pass (hello_depth_of_field.cpp:175-251);
//   shs_canvas_dof            the depth-of-field chain of hello_depth_of_field.cpp:786-812: the blur
//                             iterations (horizontal pong -> ping, vertical ping -> pong), the
//                             autofocus median (:257-285) and dof_composite_pass (:287-343).
// The host derives the pass's matrices (curr_vp, prev_vp, glm::inverse(curr_vp)) with the GLM
// restatement in shs_glm.hpp.  Buffers are host memory (synchronous) or, with SHS_CANVAS_DEVICE,
// device memory (enqueued on the context stream).
#include <cstring>

#include "shs_canvas_post_internal.hpp"
#include "shs_ctx.hpp"
#include "shs_glm.hpp"

namespace {

bool size_ok(shs_ctx *ctx, int W, int H) {
    if (W > 0 && H > 0 && W <= 32767 && H <= 32767) return true;
    ctx->err = "canvas size: 1 .. 32767 per side";
    return false;
}

bool flags_ok(shs_ctx *ctx, uint32_t flags) {
    if (!(flags & ~SHS_CANVAS_DEVICE)) return true;
    ctx->err = "canvas pass flags: SHS_CANVAS_DEVICE only";
    return false;
}

}  // namespace

extern "C" {

int shs_canvas_motion_blur(shs_ctx *ctx, const shs_canvas_motion_blur_desc *d, const uint8_t *src, const float *depth,
                           const float *velocity, uint8_t *dst, uint32_t flags) {
    if (!ctx || !d || !src || !depth || !velocity || !dst) return SHS_ERR_INVALID;
    if (!size_ok(ctx, d->width, d->height) || !flags_ok(ctx, flags)) return SHS_ERR_INVALID;
    if (set_dev(ctx)) return SHS_ERR_HIP;
    const size_t npx = (size_t)d->width * d->height;
    shs_dev::CanvasMBParams p{};
    p.W = d->width;
    p.H = d->height;
    float curr_vp[16];
    shs_host::mul(d->curr_proj, d->curr_view, curr_vp);
    shs_host::mul(d->prev_proj, d->prev_view, p.prev_vp);
    shs_host::inverse(curr_vp, p.inv_curr_vp);
    std::memcpy(p.curr_proj, d->curr_proj, sizeof p.curr_proj);
    p.samples = d->samples;
    p.soft_knee = d->soft_knee != 0;
    p.strength = d->strength;
    p.w_obj = d->w_obj;
    p.w_cam = d->w_cam;
    p.knee = d->knee_px;
    p.max_px = d->max_px;
    if (flags & SHS_CANVAS_DEVICE) {
        p.src = reinterpret_cast<const uint32_t *>(src);
        p.depth = depth;
        p.velocity = reinterpret_cast<const float2 *>(velocity);
        p.dst = reinterpret_cast<uint32_t *>(dst);
        HIP_TRY(ctx, shs_internal::launch_canvas_motion_blur(p, ctx->stream));
        return SHS_OK;
    }
    if (ensure(ctx, ctx->cp_a, npx) || ensure(ctx, ctx->cp_b, npx) || ensure(ctx, ctx->cp_depth, npx) ||
        ensure(ctx, ctx->cp_vel, 2 * npx))
        return SHS_ERR_HIP;
    HIP_TRY(ctx, hipMemcpyAsync(ctx->cp_a.p, src, npx * 4, hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(ctx, hipMemcpyAsync(ctx->cp_depth.p, depth, npx * 4, hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(ctx, hipMemcpyAsync(ctx->cp_vel.p, velocity, npx * 8, hipMemcpyHostToDevice, ctx->stream));
    p.src = ctx->cp_a.p;
    p.depth = ctx->cp_depth.p;
    p.velocity = reinterpret_cast<const float2 *>(ctx->cp_vel.p);
    p.dst = ctx->cp_b.p;
    HIP_TRY(ctx, shs_internal::launch_canvas_motion_blur(p, ctx->stream));
    HIP_TRY(ctx, hipMemcpyAsync(dst, ctx->cp_b.p, npx * 4, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    return SHS_OK;
}

int shs_canvas_gaussian_blur(shs_ctx *ctx, int32_t width, int32_t height, const uint8_t *src, uint8_t *dst,
                             int32_t horizontal, uint32_t flags) {
    if (!ctx || !src || !dst) return SHS_ERR_INVALID;
    if (!size_ok(ctx, width, height) || !flags_ok(ctx, flags)) return SHS_ERR_INVALID;
    if (set_dev(ctx)) return SHS_ERR_HIP;
    const size_t npx = (size_t)width * height;
    if (flags & SHS_CANVAS_DEVICE) {
        HIP_TRY(ctx, shs_internal::launch_canvas_gaussian(reinterpret_cast<const uint32_t *>(src),
                                                          reinterpret_cast<uint32_t *>(dst), width, height,
                                                          horizontal != 0, ctx->stream));
        return SHS_OK;
    }
    if (ensure(ctx, ctx->cp_a, npx) || ensure(ctx, ctx->cp_b, npx)) return SHS_ERR_HIP;
    HIP_TRY(ctx, hipMemcpyAsync(ctx->cp_a.p, src, npx * 4, hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(ctx, shs_internal::launch_canvas_gaussian(ctx->cp_a.p, ctx->cp_b.p, width, height, horizontal != 0, ctx->stream));
    HIP_TRY(ctx, hipMemcpyAsync(dst, ctx->cp_b.p, npx * 4, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    return SHS_OK;
}

int shs_canvas_dof(shs_ctx *ctx, const shs_canvas_dof_desc *d, uint8_t *color, const float *depth, uint8_t *blur_out,
                   float *focus_depth, uint32_t flags) {
    if (!ctx || !d || !color || !depth) return SHS_ERR_INVALID;
    if (!size_ok(ctx, d->width, d->height) || !flags_ok(ctx, flags)) return SHS_ERR_INVALID;
    if (d->blur_iterations < 0 || d->autofocus_radius < 0 || d->autofocus_radius > SHS_CANVAS_MAX_AUTOFOCUS_RADIUS) {
        ctx->err = "dof: blur_iterations >= 0, autofocus_radius 0 .. SHS_CANVAS_MAX_AUTOFOCUS_RADIUS";
        return SHS_ERR_INVALID;
    }
    if (set_dev(ctx)) return SHS_ERR_HIP;
    const int W = d->width, H = d->height;
    const size_t npx = (size_t)W * H;
    const bool dev = (flags & SHS_CANVAS_DEVICE) != 0;
    if (ensure(ctx, ctx->cp_a, npx) || ensure(ctx, ctx->cp_b, npx) || ensure(ctx, ctx->cp_focus, 1)) return SHS_ERR_HIP;
    uint32_t *sharp = reinterpret_cast<uint32_t *>(color);
    const float *z = depth;
    if (!dev) {
        if (ensure(ctx, ctx->cp_src, npx) || ensure(ctx, ctx->cp_depth, npx)) return SHS_ERR_HIP;
        HIP_TRY(ctx, hipMemcpyAsync(ctx->cp_src.p, color, npx * 4, hipMemcpyHostToDevice, ctx->stream));
        HIP_TRY(ctx, hipMemcpyAsync(ctx->cp_depth.p, depth, npx * 4, hipMemcpyHostToDevice, ctx->stream));
        sharp = ctx->cp_src.p;
        z = ctx->cp_depth.p;
    }
    // pong = sharp; per iteration: horizontal pong -> ping, vertical ping -> pong (ping = cp_b, pong = cp_a)
    const uint32_t *pong = sharp;
    if (d->blur_iterations == 0) {   // pong.color = sharp_copy, kept apart from the composite written over ping
        HIP_TRY(ctx, hipMemcpyAsync(ctx->cp_a.p, sharp, npx * 4, hipMemcpyDeviceToDevice, ctx->stream));
        pong = ctx->cp_a.p;
    }
    for (int it = 0; it < d->blur_iterations; ++it) {
        HIP_TRY(ctx, shs_internal::launch_canvas_gaussian(pong, ctx->cp_b.p, W, H, true, ctx->stream));
        HIP_TRY(ctx, shs_internal::launch_canvas_gaussian(ctx->cp_b.p, ctx->cp_a.p, W, H, false, ctx->stream));
        pong = ctx->cp_a.p;
    }
    shs_dev::CanvasDofParams p{};
    p.sharp = sharp;
    p.blur = pong;
    p.depth = z;
    p.out = sharp;   // ping.color: each pixel reads its own sharp value before writing
    p.focus = ctx->cp_focus.p;
    p.W = W;
    p.H = H;
    p.cx = d->focus_x;
    p.cy = d->focus_y;
    p.radius = d->autofocus_radius;
    p.range = d->range;
    p.max_blur = d->max_blur;
    HIP_TRY(ctx, shs_internal::launch_canvas_autofocus(p, ctx->stream));
    HIP_TRY(ctx, shs_internal::launch_canvas_dof_composite(p, ctx->stream));
    if (blur_out) {
        const hipMemcpyKind k = dev ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
        HIP_TRY(ctx, hipMemcpyAsync(blur_out, pong, npx * 4, k, ctx->stream));
    }
    if (!dev) HIP_TRY(ctx, hipMemcpyAsync(color, ctx->cp_src.p, npx * 4, hipMemcpyDeviceToHost, ctx->stream));
    if (focus_depth) HIP_TRY(ctx, hipMemcpyAsync(focus_depth, ctx->cp_focus.p, sizeof(float), hipMemcpyDeviceToHost, ctx->stream));
    if (!dev || focus_depth) HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    return SHS_OK;
}

}  // extern "C"
