// shs_abi_post.cpp -- C ABI of the passes after the raster path (include/shs_gpu.h):
// PassTonemap (shs-renderer-lib/include/shs/passes/pass_tonemap.hpp:36-83) and the SDL texture
// staging upload_ldr_to_rgba8 (exp-plumbing/hello_pass_basics.cpp:102-119) and PassMotionBlur
// (shs-renderer-lib/include/shs/passes/pass_motion_blur.hpp:38-170), paths relative to
// /root/reference/cpp-folders/src/.
#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>

#include "shs_ctx.hpp"
#include "shs_post_internal.hpp"

namespace {

// The reference's byte of one channel once c / (1 + c) = x is known (pass_tonemap.hpp:73-79):
// std::pow(float, float) and std::lround of this host's libm, exactly as the pass runs them.
int ref_byte(float x, float inv_gamma) {
    const float c = std::pow(x, inv_gamma);
    const int v = (int)std::lround(c * 255.0f);
    return v < 0 ? 0 : (v > 255 ? 255 : v);
}

float bits_float(uint32_t b) {
    float f;
    std::memcpy(&f, &b, 4);
    return f;
}

uint32_t float_bits(float f) {
    uint32_t b;
    std::memcpy(&b, &f, 4);
    return b;
}

// thr[k] = the smallest float x in [0, 1] with ref_byte(x) >= k (+inf if none), k = 1..255:
// a binary search over the bit patterns of [0, 1] (ordered like the values).
void tonemap_thresholds(float gamma_param, float thr[256]) {
    const float inv_gamma = 1.0f / std::max(0.001f, gamma_param);
    const uint32_t one = float_bits(1.0f);
    thr[0] = 0.0f;
    for (int k = 1; k < 256; ++k) {
        if (ref_byte(1.0f, inv_gamma) < k) {
            thr[k] = std::numeric_limits<float>::infinity();
            continue;
        }
        uint32_t lo = 0, hi = one;   // ref_byte(bits(hi)) >= k
        while (lo < hi) {
            const uint32_t mid = lo + (hi - lo) / 2;
            if (ref_byte(bits_float(mid), inv_gamma) >= k) hi = mid; else lo = mid + 1;
        }
        thr[k] = bits_float(lo);
    }
}

int enqueue_tonemap(shs_ctx *ctx) {
    const shs_tonemap_desc &d = ctx->tm_desc;
    const int W = ctx->lib_frame.width, H = ctx->lib_frame.height;
    const size_t npx = (size_t)W * H;
    if ((d.flags & SHS_TONEMAP_LDR) && ensure(ctx, ctx->lib_ldr, npx)) return SHS_ERR_HIP;
    if ((d.flags & SHS_TONEMAP_PRESENT) && ensure(ctx, ctx->lib_present, npx)) return SHS_ERR_HIP;
    // the thresholds depend on the clamped gamma only (pass_tonemap.hpp: 1 / max(0.001, gamma))
    const float g = std::max(0.001f, d.gamma);
    if (!ctx->tm_thr_valid || ctx->tm_gamma != g) {
        tonemap_thresholds(g, ctx->tm_thr);
        ctx->tm_gamma = g;
        ctx->tm_thr_valid = true;
    }
    shs_dev::TonemapParams p{};
    p.hdr = ctx->lib_hdr.p;
    p.ldr = (d.flags & SHS_TONEMAP_LDR) ? ctx->lib_ldr.p : nullptr;
    p.present = (d.flags & SHS_TONEMAP_PRESENT) ? ctx->lib_present.p : nullptr;
    p.W = W;
    p.H = H;
    // a tile-sharded camera pass wrote only its own tiles: map only those (the others stay undefined,
    // like the HDR target's)
    p.rank = ctx->lib_frame.shard_count > 1 ? ctx->lib_frame.shard_rank : 0;
    p.count = std::max(1, ctx->lib_frame.shard_count);
    if (p.count > 1 && ctx->reg_last_count == p.count) p.reg = ctx->reg_last[(size_t)p.rank];
    p.exposure = std::max(0.0001f, d.exposure);
    p.inv_gamma = 1.0f / std::max(0.001f, d.gamma);
    std::memcpy(p.thr, ctx->tm_thr, sizeof p.thr);
    HIP_TRY(ctx, shs_internal::launch_tonemap(p, ctx->stream));
    return SHS_OK;
}

int enqueue_motion_blur(shs_ctx *ctx) {
    const shs_motion_blur_desc &d = ctx->mb_desc;
    const int W = ctx->lib_frame.width, H = ctx->lib_frame.height;
    const size_t npx = (size_t)W * H;
    if (ensure(ctx, ctx->lib_mb, npx)) return SHS_ERR_HIP;
    if ((d.flags & SHS_MOTION_BLUR_PRESENT) && ensure(ctx, ctx->lib_mb_present, npx)) return SHS_ERR_HIP;
    shs_dev::MotionBlurParams p{};
    p.src = ctx->lib_ldr.p;
    p.depth = ctx->lib_depth.p;
    p.motion = ctx->lib_motion.p;
    p.dst = ctx->lib_mb.p;
    p.present = (d.flags & SHS_MOTION_BLUR_PRESENT) ? ctx->lib_mb_present.p : nullptr;
    p.W = W;
    p.H = H;
    // the pass's parameter clamps (pass_motion_blur.hpp:76-81), the same float expressions
    p.enable = d.enable != 0;
    p.samples = std::min(std::max(d.samples, 4), 32);
    p.strength = std::max(0.0f, d.strength);
    p.max_vel = std::max(1.0f, d.max_velocity_px);
    p.min_vel = std::max(0.0f, d.min_velocity_px);
    p.depth_eps = std::max(0.0f, d.depth_reject);
    const float dts = std::max(d.dt, 1e-4f) * 60.0f;
    p.dt_scale = dts < 0.5f ? 0.5f : (2.5f < dts ? 2.5f : dts);   // std::clamp
    HIP_TRY(ctx, shs_internal::launch_motion_blur(p, ctx->stream));
    return SHS_OK;
}

}  // namespace

int shs_tonemap_reissue(shs_ctx *ctx) {
    const int rc = enqueue_tonemap(ctx);
    if (rc || !ctx->have_mb) return rc;
    return enqueue_motion_blur(ctx);
}

extern "C" {

int shs_lib_fuse_tonemap(shs_ctx *ctx, const shs_tonemap_desc *desc) {
    if (!ctx) return SHS_ERR_INVALID;
    if (!desc) {
        ctx->tm_fuse = false;
        return SHS_OK;
    }
    if (!(desc->flags & (SHS_TONEMAP_LDR | SHS_TONEMAP_PRESENT)) || (desc->flags & ~(SHS_TONEMAP_LDR | SHS_TONEMAP_PRESENT))) {
        ctx->err = "tonemap flags: SHS_TONEMAP_LDR and / or SHS_TONEMAP_PRESENT";
        return SHS_ERR_INVALID;
    }
    if (!std::isfinite(desc->exposure) || !std::isfinite(desc->gamma)) {
        ctx->err = "tonemap exposure / gamma must be finite";
        return SHS_ERR_INVALID;
    }
    ctx->tm_fuse = true;
    ctx->tm_fuse_desc = *desc;
    return SHS_OK;
}

int shs_tonemap_thresholds(float gamma, float thr[256]) {
    if (!thr) return SHS_ERR_INVALID;
    tonemap_thresholds(gamma, thr);
    return SHS_OK;
}

int shs_tonemap(shs_ctx *ctx, const shs_tonemap_desc *desc) {
    if (!ctx || !desc) return SHS_ERR_INVALID;
    if (!ctx->have_lib_frame) { ctx->err = "no library frame rendered"; return SHS_ERR_INVALID; }
    if (!(desc->flags & (SHS_TONEMAP_LDR | SHS_TONEMAP_PRESENT)) || (desc->flags & ~(SHS_TONEMAP_LDR | SHS_TONEMAP_PRESENT))) {
        ctx->err = "tonemap flags: SHS_TONEMAP_LDR and / or SHS_TONEMAP_PRESENT";
        return SHS_ERR_INVALID;
    }
    if (!std::isfinite(desc->exposure) || !std::isfinite(desc->gamma)) {
        ctx->err = "tonemap exposure / gamma must be finite";
        return SHS_ERR_INVALID;
    }
    if (set_dev(ctx)) return SHS_ERR_HIP;
    ctx->tm_desc = *desc;
    const int rc = enqueue_tonemap(ctx);
    if (rc) return rc;
    ctx->have_ldr = true;
    ctx->have_mb = false;
    return SHS_OK;
}

int shs_motion_blur(shs_ctx *ctx, const shs_motion_blur_desc *desc) {
    if (!ctx || !desc) return SHS_ERR_INVALID;
    if (!ctx->have_ldr || !(ctx->tm_desc.flags & SHS_TONEMAP_LDR)) {
        ctx->err = "motion blur needs a tonemap with SHS_TONEMAP_LDR after the camera pass";
        return SHS_ERR_INVALID;
    }
    if (!(ctx->lib_frame.flags & SHS_LIB_DEPTH_MOTION)) {
        ctx->err = "motion blur needs the depth_motion target (SHS_LIB_DEPTH_MOTION)";
        return SHS_ERR_INVALID;
    }
    if (desc->flags & ~SHS_MOTION_BLUR_PRESENT) { ctx->err = "motion blur flags"; return SHS_ERR_INVALID; }
    if (set_dev(ctx)) return SHS_ERR_HIP;
    ctx->mb_desc = *desc;
    const int rc = enqueue_motion_blur(ctx);
    if (rc) return rc;
    ctx->have_mb = true;
    return SHS_OK;
}

int shs_resolve_motion_blur(shs_ctx *ctx, uint8_t *ldr, uint8_t *present) {
    if (!ctx) return SHS_ERR_INVALID;
    if (!ctx->have_mb) { ctx->err = "no motion blur since the last camera pass"; return SHS_ERR_INVALID; }
    if (present && !(ctx->mb_desc.flags & SHS_MOTION_BLUR_PRESENT)) { ctx->err = "no present staging written"; return SHS_ERR_INVALID; }
    if (set_dev(ctx)) return SHS_ERR_HIP;
    const int rc = shs_resolve_lib(ctx, nullptr, nullptr, nullptr);   // finishes (re-issues) the pass chain
    if (rc) return rc;
    const size_t n = (size_t)ctx->lib_frame.width * ctx->lib_frame.height * 4;
    if (ldr) HIP_TRY(ctx, hipMemcpy(ldr, ctx->lib_mb.p, n, hipMemcpyDeviceToHost));
    if (present) HIP_TRY(ctx, hipMemcpy(present, ctx->lib_mb_present.p, n, hipMemcpyDeviceToHost));
    return SHS_OK;
}

int shs_resolve_ldr(shs_ctx *ctx, uint8_t *ldr, uint8_t *present) {
    if (!ctx) return SHS_ERR_INVALID;
    if (!ctx->have_ldr) { ctx->err = "no tonemap since the last camera pass"; return SHS_ERR_INVALID; }
    if ((ldr && !(ctx->tm_desc.flags & SHS_TONEMAP_LDR)) || (present && !(ctx->tm_desc.flags & SHS_TONEMAP_PRESENT))) {
        ctx->err = "target not written by the last tonemap";
        return SHS_ERR_INVALID;
    }
    if (set_dev(ctx)) return SHS_ERR_HIP;
    // the camera pass may still be re-issued (capacity overflow): shs_resolve_lib finishes it
    const int rc = shs_resolve_lib(ctx, nullptr, nullptr, nullptr);
    if (rc) return rc;
    const size_t n = (size_t)ctx->lib_frame.width * ctx->lib_frame.height * 4;
    if (ldr) HIP_TRY(ctx, hipMemcpy(ldr, ctx->lib_ldr.p, n, hipMemcpyDeviceToHost));
    if (present) HIP_TRY(ctx, hipMemcpy(present, ctx->lib_present.p, n, hipMemcpyDeviceToHost));
    return SHS_OK;
}

int shs_ldr_device_targets(shs_ctx *ctx, void **ldr_dev, void **present_dev) {
    if (!ctx) return SHS_ERR_INVALID;
    if (!ctx->have_ldr) { ctx->err = "no tonemap since the last camera pass"; return SHS_ERR_INVALID; }
    if (set_dev(ctx)) return SHS_ERR_HIP;
    const int rc = shs_resolve_lib(ctx, nullptr, nullptr, nullptr);   // finishes (re-issues) the pass chain
    if (rc) return rc;
    if (ldr_dev) *ldr_dev = (ctx->tm_desc.flags & SHS_TONEMAP_LDR) ? ctx->lib_ldr.p : nullptr;
    if (present_dev) *present_dev = (ctx->tm_desc.flags & SHS_TONEMAP_PRESENT) ? ctx->lib_present.p : nullptr;
    return SHS_OK;
}

}  // extern "C"
