// abi_legacy.cpp -- a C++ host compiled with g++ against include/shs_gpu.h alone, driving the legacy
// path the way the Seam-1 adapter does (integration/shs_gpu_seams.hpp, LegacyRendererSystemGPU):
// create -> upload the ModelGeometry soup -> shs_render_legacy -> shs_resolve into caller-owned
// Canvas / ZBuffer-layout buffers, plus a frame batch (shs_render_legacy_batch / shs_resolve_frame).
// Every frame is compared with the CPU oracle (oracle/shs_oracle.h, TEST INFRASTRUCTURE): depth bit
// for bit, colour exactly except a +-1 byte where both pre-truncation floats agree within 1e-5 * 255.
//
// Scene: hello_pipeline_blinn_phong_shading.cpp:152-153 (Suzanne at (0,0,10), scale 4, colour
// {60,100,200}, light normalize(-1,-0.4,1)) seen by Viewer((0,5,-20)) (shs_renderer.hpp:1323-1337), at
// 800x600 (config 1) and 1920x1080 (config 2), with camera poses and all four shading models.
// Exit status 0 = every comparison passed.  Run by tests/test_abi_c.py (-m gpu).
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "shs_gpu.h"
#include "shs_oracle.h"

namespace {

struct Soup {
    std::vector<float> pos, nrm;
    int32_t n = 0;
};

bool load_soup(const std::string &path, Soup &s) {
    FILE *f = std::fopen(path.c_str(), "rb");
    if (!f) return false;
    char magic[8];
    uint32_t hdr[2];
    bool ok = std::fread(magic, 1, 8, f) == 8 && std::memcmp(magic, "SHSSOUP1", 8) == 0 && std::fread(hdr, 4, 2, f) == 2;
    if (ok) {
        s.n = (int32_t)hdr[0];
        s.pos.resize((size_t)s.n * 9);
        s.nrm.resize((size_t)s.n * 9);
        ok = std::fread(s.pos.data(), 36, s.n, f) == (size_t)s.n && std::fread(s.nrm.data(), 36, s.n, f) == (size_t)s.n;
    }
    std::fclose(f);
    return ok;
}

// glm::normalize(vec3) in float: v * (1 / sqrt((x*x + y*y) + z*z))
void normalize3(const float in[3], float out[3]) {
    const float x = in[0] * in[0], y = in[1] * in[1], z = in[2] * in[2];
    const float inv = 1.0f / std::sqrt((x + y) + z);
    for (int k = 0; k < 3; ++k) out[k] = in[k] * inv;
}

int g_fail = 0;

#define EXPECT(cond, ...)                                                                                    \
    do {                                                                                                     \
        if (!(cond)) {                                                                                       \
            std::printf("FAIL %s:%d: ", __FILE__, __LINE__);                                                 \
            std::printf(__VA_ARGS__);                                                                        \
            std::printf("\n");                                                                               \
            ++g_fail;                                                                                        \
        }                                                                                                    \
    } while (0)

#define SHS_CHECK(ctx, call)                                                                                 \
    do {                                                                                                     \
        const int rc_ = (call);                                                                              \
        if (rc_ != SHS_OK) {                                                                                 \
            std::printf("FAIL %s -> %d: %s\n", #call, rc_, shs_last_error(ctx));                            \
            return 2;                                                                                        \
        }                                                                                                    \
    } while (0)

struct Pose {
    float yaw, pitch;
    int shading;
};

// The per-object Uniforms RendererSystem::process builds (blinn_phong_shading.cpp:277-282; the Flat
// demo's mv / light_dir_view, flat_shading.cpp:256, 284-287), with the ABI's GLM host helpers.
void make_draw(int32_t mesh_id, const Pose &p, shs_legacy_draw &d, ora_draw &o, const Soup &soup) {
    const float cam[3] = {0.0f, 5.0f, -20.0f}, mpos[3] = {0.0f, 0.0f, 10.0f}, mscl[3] = {4.0f, 4.0f, 4.0f};
    float view[16], proj[16], model[16], pv[16], mvp[16], mv[16];
    shs_camera3d(cam, p.yaw, p.pitch, 60.0f, 0.1f, 1000.0f, view, proj);
    shs_model_trs(mpos, 0.0f, mscl, model);
    std::memset(&d, 0, sizeof d);
    d.mesh_id = mesh_id;
    d.shading = p.shading;
    const float blinn[3] = {-1.0f, -0.4f, 1.0f}, phong[3] = {1.0f, 1.0f, -1.0f};
    float light[3];
    normalize3(p.shading == SHS_SHADING_BLINN_PHONG || p.shading == SHS_SHADING_GOURAUD ? blinn : phong, light);
    if (p.shading == SHS_SHADING_FLAT) {
        shs_mat4_mul(view, model, mv);
        shs_mat4_mul(proj, mv, mvp);
        std::memcpy(d.model, mv, 64);
        // light_dir_view = normalize(vec3(view * vec4(light, 0))): (m0*x + m1*y) + (m2*z + m3*0)
        float lv[3];
        for (int r = 0; r < 3; ++r) lv[r] = (view[r] * light[0] + view[4 + r] * light[1]) + (view[8 + r] * light[2] + view[12 + r] * 0.0f);
        normalize3(lv, d.light_dir);
        d.color[0] = 100; d.color[1] = 150; d.color[2] = 255; d.color[3] = 255;   // flat_shading.cpp:156
    } else {
        shs_mat4_mul(proj, view, pv);
        shs_mat4_mul(pv, model, mvp);
        std::memcpy(d.model, model, 64);
        std::memcpy(d.light_dir, light, 12);
        d.color[0] = 60; d.color[1] = 100; d.color[2] = 200; d.color[3] = 255;    // blinn_phong_shading.cpp:153
    }
    std::memcpy(d.mvp, mvp, 64);
    std::memcpy(d.camera_pos, cam, 12);
    std::memset(&o, 0, sizeof o);
    o.shading = d.shading;
    o.n_tris = soup.n;
    o.positions = soup.pos.data();
    o.normals = soup.nrm.data();
    std::memcpy(o.mvp, d.mvp, 64);
    std::memcpy(o.model, d.model, 64);
    std::memcpy(o.light_dir, d.light_dir, 12);
    std::memcpy(o.camera_pos, d.camera_pos, 12);
    std::memcpy(o.color, d.color, 4);
}

// Depth bit-exact; colour exact except +-1 where both pre-truncation floats agree within 1e-5*255.
void compare(const char *what, int W, int H, const std::vector<uint8_t> &gc, const std::vector<float> &gd,
             const std::vector<float> *gpq, const std::vector<uint8_t> &rc, const std::vector<float> &rd,
             const std::vector<float> &rpq) {
    size_t bad_depth = 0, bad_color = 0, boundary = 0, covered = 0;
    for (size_t i = 0; i < (size_t)W * H; ++i) {
        uint32_t a, b;
        std::memcpy(&a, &gd[i], 4);
        std::memcpy(&b, &rd[i], 4);
        bad_depth += a != b;
        covered += rd[i] < 3.4028234e38f;
    }
    for (size_t i = 0; i < (size_t)W * H * 4; ++i) {
        if (gc[i] == rc[i]) continue;
        const int dd = std::abs((int)gc[i] - (int)rc[i]);
        const bool explained = dd == 1 && gpq && (i % 4) < 3 && std::fabs((*gpq)[i] - rpq[i]) <= 1e-5f * 255.0f;
        if (explained) ++boundary; else ++bad_color;
    }
    std::printf("%-34s %dx%d covered=%zu depth_mismatch=%zu colour_mismatch=%zu boundary_bytes=%zu\n", what, W, H, covered,
                bad_depth, bad_color, boundary);
    EXPECT(bad_depth == 0, "%s: %zu depth words differ", what, bad_depth);
    EXPECT(bad_color == 0, "%s: %zu colour bytes differ", what, bad_color);
    EXPECT(covered > 1000, "%s: only %zu covered pixels", what, covered);
}

}  // namespace

int main(int argc, char **argv) {
    const std::string root = argc > 1 ? argv[1] : ".";
    Soup soup;
    if (!load_soup(root + "/assets/monkey.soup.bin", soup)) {
        std::printf("FAIL cannot read %s/assets/monkey.soup.bin\n", root.c_str());
        return 2;
    }
    shs_ctx *ctx = nullptr;
    if (shs_create(0, &ctx) != SHS_OK) {
        std::printf("FAIL shs_create: no gfx950 device\n");
        return 3;
    }
    int32_t mesh = -1;
    SHS_CHECK(ctx, shs_mesh_upload_soup(ctx, soup.pos.data(), soup.nrm.data(), soup.n, &mesh));

    const Pose poses[] = {{0.0f, 0.0f, SHS_SHADING_BLINN_PHONG}, {17.0f, -9.0f, SHS_SHADING_PHONG},
                          {-33.0f, 12.5f, SHS_SHADING_GOURAUD}, {8.0f, 4.0f, SHS_SHADING_FLAT}};
    const int sizes[2][2] = {{800, 600}, {1920, 1080}};
    for (const auto &sz : sizes) {
        const int W = sz[0], H = sz[1];
        for (const Pose &p : poses) {
            shs_legacy_draw d;
            ora_draw o;
            make_draw(mesh, p, d, o, soup);
            shs_frame_desc f{};
            f.width = W; f.height = H;
            f.ref_tile_w = 80; f.ref_tile_h = 80;
            f.shard_rank = 0; f.shard_count = 1;
            f.flags = SHS_FRAME_PREQUANT;
            f.clear_color[3] = 255;
            SHS_CHECK(ctx, shs_render_legacy(ctx, &f, &d, 1));
            std::vector<uint8_t> gc((size_t)W * H * 4);   // Canvas::buffer() layout
            std::vector<float> gd((size_t)W * H), gpq((size_t)W * H * 4);
            SHS_CHECK(ctx, shs_resolve(ctx, gc.data(), gd.data()));
            SHS_CHECK(ctx, shs_resolve_prequant(ctx, gpq.data()));
            shs_raster_stats st{};
            SHS_CHECK(ctx, shs_get_stats(ctx, &st));
            EXPECT(st.tri_input == (uint64_t)soup.n, "tri_input %llu", (unsigned long long)st.tri_input);
            std::vector<uint8_t> rc((size_t)W * H * 4);
            std::vector<float> rd((size_t)W * H), rpq((size_t)W * H * 4);
            EXPECT(ora_render_legacy(W, H, 80, 80, 8, &o, 1, rc.data(), rd.data(), rpq.data()) == 0, "oracle failed");
            char what[96];
            std::snprintf(what, sizeof what, "single yaw=%g pitch=%g shading=%d", p.yaw, p.pitch, p.shading);
            compare(what, W, H, gc, gd, &gpq, rc, rd, rpq);
            size_t cov = 0;
            for (float z : rd) cov += z < 3.4028234e38f;
            EXPECT(st.covered_pixels == cov, "covered_pixels %llu vs %zu", (unsigned long long)st.covered_pixels, cov);
        }
    }

    // A batch of the four poses at 1920x1080: every frame equals the oracle's (colour with the frame's
    // own pre-truncation floats, shs_resolve_prequant_frame).
    {
        const int W = 1920, H = 1080, F = 4;
        std::vector<shs_legacy_draw> draws(F);
        std::vector<ora_draw> odraws(F);
        for (int k = 0; k < F; ++k) make_draw(mesh, poses[k], draws[k], odraws[k], soup);
        shs_frame_desc f{};
        f.width = W; f.height = H;
        f.ref_tile_w = 80; f.ref_tile_h = 80;
        f.shard_rank = 0; f.shard_count = 1;
        f.flags = SHS_FRAME_PREQUANT;
        f.clear_color[3] = 255;
        SHS_CHECK(ctx, shs_render_legacy_batch(ctx, &f, draws.data(), 1, F));
        for (int k = 0; k < F; ++k) {
            std::vector<uint8_t> gc((size_t)W * H * 4), rc((size_t)W * H * 4);
            std::vector<float> gd((size_t)W * H), rd((size_t)W * H), gpq((size_t)W * H * 4), rpq((size_t)W * H * 4);
            SHS_CHECK(ctx, shs_resolve_frame(ctx, k, gc.data(), gd.data()));
            SHS_CHECK(ctx, shs_resolve_prequant_frame(ctx, k, gpq.data()));
            EXPECT(ora_render_legacy(W, H, 80, 80, 8, &odraws[k], 1, rc.data(), rd.data(), rpq.data()) == 0, "oracle failed");
            char what[64];
            std::snprintf(what, sizeof what, "batch frame %d/%d", k, F);
            compare(what, W, H, gc, gd, &gpq, rc, rd, rpq);
        }
        EXPECT(shs_resolve_frame(ctx, F, nullptr, nullptr) == SHS_ERR_INVALID, "frame index past the batch accepted");
    }
    shs_destroy(ctx);
    std::printf(g_fail ? "abi_legacy: %d FAILED\n" : "abi_legacy: all passed\n", g_fail);
    return g_fail ? 1 : 0;
}
