// abi_group.cpp -- a single-process C++ host using several GPUs through the C ABI alone (g++ against
// include/shs_gpu.h): a shs_group of N contexts renders the interleaved 32x32 tile shards of a frame,
// shs_group_gather composes it on rank 0 (peer copies), and rank 0 resolves the full frame.  Every
// composed frame must equal, bit for bit, the frame one unsharded context renders:
//   legacy (Seam 1): Suzanne Blinn-Phong at 1920x1080, colour + depth and the SDL present staging;
//   library (Seam 3): a seeded soup + floor, PassPBRForward (PBR, motion) at 1280x720, HDR + depth +
//   motion, then with the fused PassTonemap into the present staging;
//   three frames back to back with no host wait between gathers (double-buffered receive buffers).
// usage: abi_group ROOT [N] [device list, e.g. 0,0,0]  (default: N = 8 contexts on device 0).
// Exit status 0 = every comparison passed; 3 = no device.  Run by tests/test_abi_c.py (-m gpu).
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "shs_gpu.h"

namespace {

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

#define CK(call)                                                                                             \
    do {                                                                                                     \
        const int rc_ = (call);                                                                              \
        if (rc_ != SHS_OK) {                                                                                 \
            std::printf("FAIL %s -> %d: %s\n", #call, rc_, err_of());                                       \
            return 2;                                                                                        \
        }                                                                                                    \
    } while (0)

shs_ctx *g_ctx = nullptr;
shs_group *g_grp = nullptr;
const char *err_of() {
    static std::string s;
    s = std::string("ctx: ") + (g_ctx ? shs_last_error(g_ctx) : "-") + " | group: " + (g_grp ? shs_group_last_error(g_grp) : "-");
    return s.c_str();
}

bool load_soup(const std::string &path, std::vector<float> &pos, std::vector<float> &nrm, int32_t &n) {
    FILE *f = std::fopen(path.c_str(), "rb");
    if (!f) return false;
    char magic[8];
    uint32_t hdr[2];
    bool ok = std::fread(magic, 1, 8, f) == 8 && std::memcmp(magic, "SHSSOUP1", 8) == 0 && std::fread(hdr, 4, 2, f) == 2;
    if (ok) {
        n = (int32_t)hdr[0];
        pos.resize((size_t)n * 9);
        nrm.resize((size_t)n * 9);
        ok = std::fread(pos.data(), 36, n, f) == (size_t)n && std::fread(nrm.data(), 36, n, f) == (size_t)n;
    }
    std::fclose(f);
    return ok;
}

template <typename T>
size_t count_diff(const std::vector<T> &a, const std::vector<T> &b) {
    size_t n = 0;
    const uint8_t *pa = reinterpret_cast<const uint8_t *>(a.data()), *pb = reinterpret_cast<const uint8_t *>(b.data());
    for (size_t i = 0; i < a.size() * sizeof(T); i += sizeof(T)) n += std::memcmp(pa + i, pb + i, sizeof(T)) != 0;
    return n;
}

uint32_t g_seed = 0x5EEDu;
float frand() {   // xorshift32 in [0, 1)
    g_seed ^= g_seed << 13; g_seed ^= g_seed >> 17; g_seed ^= g_seed << 5;
    return (float)(g_seed >> 8) * (1.0f / 16777216.0f);
}

void legacy_draw(int32_t mesh, float yaw, shs_legacy_draw &d) {
    const float cam[3] = {0.0f, 5.0f, -20.0f}, mpos[3] = {0.0f, 0.0f, 10.0f}, mscl[3] = {4.0f, 4.0f, 4.0f};
    float view[16], proj[16], model[16], pv[16];
    shs_camera3d(cam, yaw, 0.0f, 60.0f, 0.1f, 1000.0f, view, proj);
    shs_model_trs(mpos, 0.0f, mscl, model);
    std::memset(&d, 0, sizeof d);
    d.mesh_id = mesh;
    d.shading = SHS_SHADING_BLINN_PHONG;
    shs_mat4_mul(proj, view, pv);
    shs_mat4_mul(pv, model, d.mvp);
    std::memcpy(d.model, model, 64);
    d.light_dir[0] = -0.6963106f; d.light_dir[1] = -0.2785242f; d.light_dir[2] = 0.6963106f;
    std::memcpy(d.camera_pos, cam, 12);
    d.color[0] = 60; d.color[1] = 100; d.color[2] = 200; d.color[3] = 255;
}

void lib_draws(int32_t soup, int32_t floor, float yaw, int W, int H, shs_lib_draw d[2]) {
    const float eye[3] = {0.0f, 6.0f, -18.0f}, at[3] = {0.0f, 1.0f, 0.0f}, up[3] = {0.0f, 1.0f, 0.0f};
    float view[16], proj[16], vp[16];
    shs_look_at_lh(eye, at, up, view);
    shs_perspective_lh_no(1.0471976f, (float)W / (float)H, 0.1f, 200.0f, proj);
    shs_mat4_mul(proj, view, vp);
    const float pos[3] = {0.0f, 1.0f, 0.0f}, rot[3] = {0.0f, yaw, 0.0f}, prot[3] = {0.0f, yaw - 0.05f, 0.0f};
    const float scl[3] = {1.0f, 1.0f, 1.0f}, zero[3] = {0.0f, 0.0f, 0.0f};
    for (int k = 0; k < 2; ++k) {
        shs_lib_draw &x = d[k];
        std::memset(&x, 0, sizeof x);
        x.mesh_id = k == 0 ? floor : soup;
        x.program = SHS_PROGRAM_PBR_MR;
        x.cull_mode = SHS_CULL_NONE;
        x.front_face_ccw = 1;
        shs_model_euler(k == 0 ? zero : pos, k == 0 ? zero : rot, scl, x.model);
        shs_model_euler(k == 0 ? zero : pos, k == 0 ? zero : prot, scl, x.prev_model);
        std::memcpy(x.viewproj, vp, 64);
        std::memcpy(x.prev_viewproj, vp, 64);
        x.light_dir_ws[0] = 0.4668f; x.light_dir_ws[1] = -0.3487f; x.light_dir_ws[2] = 0.8127f;
        x.light_color[0] = x.light_color[1] = x.light_color[2] = 1.0f;
        x.light_intensity = 5.0f;
        std::memcpy(x.camera_pos, eye, 12);
        x.base_color[0] = k ? 0.8f : 0.6f; x.base_color[1] = k ? 0.5f : 0.6f; x.base_color[2] = k ? 0.2f : 0.6f;
        x.metallic = 0.1f; x.roughness = 0.5f; x.ao = 1.0f;
        x.enable_motion_vectors = 1;
    }
}

}  // namespace

int main(int argc, char **argv) {
    const std::string root = argc > 1 ? argv[1] : ".";
    const int n = argc > 2 ? std::atoi(argv[2]) : 8;
    std::vector<int32_t> devs(n, 0);
    if (argc > 3) {   // "0,1,2,..."
        const char *p = argv[3];
        for (int r = 0; r < n && *p; ++r) {
            devs[r] = (int32_t)std::strtol(p, const_cast<char **>(&p), 10);
            if (*p == ',') ++p;
        }
    }
    std::vector<float> pos, nrm;
    int32_t n_tris = 0;
    if (!load_soup(root + "/assets/monkey.soup.bin", pos, nrm, n_tris)) { std::printf("FAIL no monkey soup\n"); return 2; }
    if (shs_create(devs[0], &g_ctx) != SHS_OK) { std::printf("FAIL shs_create: no gfx950 device\n"); return 3; }
    CK(shs_group_create(devs.data(), n, &g_grp));
    EXPECT(shs_group_size(g_grp) == n, "group size");
    shs_ctx *root0 = nullptr;
    CK(shs_group_context(g_grp, 0, &root0));

    // ---- legacy (Seam 1): colour + depth, then the SDL staging ----
    {
        const int W = 1920, H = 1080;
        int32_t m1 = -1, mg = -1;
        CK(shs_mesh_upload_soup(g_ctx, pos.data(), nrm.data(), n_tris, &m1));
        CK(shs_group_mesh_upload_soup(g_grp, pos.data(), nrm.data(), n_tris, &mg));
        for (float yaw : {0.0f, 11.0f, -7.5f}) {
            shs_legacy_draw d1, dg;
            legacy_draw(m1, yaw, d1);
            legacy_draw(mg, yaw, dg);
            shs_frame_desc f{};
            f.width = W; f.height = H; f.ref_tile_w = 80; f.ref_tile_h = 80; f.shard_count = 1;
            f.flags = SHS_FRAME_PRESENT;
            f.clear_color[3] = 255;
            CK(shs_render_legacy(g_ctx, &f, &d1, 1));
            std::vector<uint8_t> c1((size_t)W * H * 4), cg(c1.size()), p1(c1.size()), pg(c1.size());
            std::vector<float> z1((size_t)W * H), zg(z1.size());
            CK(shs_resolve(g_ctx, c1.data(), z1.data()));
            CK(shs_resolve_present(g_ctx, 0, p1.data(), W * 4));
            CK(shs_group_render_legacy(g_grp, &f, &dg, 1));
            CK(shs_group_gather(g_grp, SHS_TARGET_LEGACY));
            CK(shs_resolve(root0, cg.data(), zg.data()));
            CK(shs_group_gather(g_grp, SHS_TARGET_PRESENT));
            CK(shs_resolve_present(root0, 0, pg.data(), W * 4));
            const size_t dc = count_diff(c1, cg), dz = count_diff(z1, zg), dp = count_diff(p1, pg);
            std::printf("legacy  yaw=%5.1f %d ranks: colour %zu / depth %zu / present %zu differing\n", yaw, n, dc, dz, dp);
            EXPECT(dc == 0 && dz == 0 && dp == 0, "legacy sharded frame differs (yaw %g)", yaw);
        }
    }

    // ---- library (Seam 3): PBR + motion, then the fused tonemap's present staging ----
    {
        const int W = 1280, H = 720, NT = 20000;
        std::vector<float> sp((size_t)NT * 9), sn((size_t)NT * 9);
        for (int t = 0; t < NT; ++t) {
            const float cx = frand() * 8.0f - 4.0f, cy = frand() * 4.0f, cz = frand() * 8.0f - 4.0f;
            for (int k = 0; k < 3; ++k) {
                sp[t * 9 + 3 * k] = cx + frand() * 0.6f - 0.3f;
                sp[t * 9 + 3 * k + 1] = cy + frand() * 0.6f - 0.3f;
                sp[t * 9 + 3 * k + 2] = cz + frand() * 0.6f - 0.3f;
                sn[t * 9 + 3 * k] = 0.0f; sn[t * 9 + 3 * k + 1] = 1.0f; sn[t * 9 + 3 * k + 2] = 0.0f;
            }
        }
        const float fl[12] = {-30.0f, 0.0f, -30.0f, 30.0f, 0.0f, -30.0f, 30.0f, 0.0f, 30.0f, -30.0f, 0.0f, 30.0f};
        const float fn[12] = {0, 1, 0, 0, 1, 0, 0, 1, 0, 0, 1, 0};
        const uint32_t fi[6] = {0, 2, 1, 0, 3, 2};
        int32_t s1, f1, sg, fg;
        CK(shs_mesh_upload(g_ctx, sp.data(), NT * 3, sn.data(), NT * 3, nullptr, 0, nullptr, 0, &s1));
        CK(shs_mesh_upload(g_ctx, fl, 4, fn, 4, nullptr, 0, fi, 6, &f1));
        CK(shs_group_mesh_upload(g_grp, sp.data(), NT * 3, sn.data(), NT * 3, nullptr, 0, nullptr, 0, &sg));
        CK(shs_group_mesh_upload(g_grp, fl, 4, fn, 4, nullptr, 0, fi, 6, &fg));
        shs_lib_frame f{};
        f.width = W; f.height = H; f.shard_count = 1;
        f.flags = SHS_LIB_DEPTH_MOTION | SHS_LIB_BG_GRADIENT;
        f.zn = 0.1f; f.zf = 200.0f;
        const size_t np = (size_t)W * H;
        for (int lay = 0; lay < 4; ++lay) {   // (interleaved, regions) x (raw targets, fused tonemap)
            const int layout = lay < 2 ? SHS_SHARD_INTERLEAVED : SHS_SHARD_REGIONS, fused = lay & 1;
            const char *lname = layout == SHS_SHARD_REGIONS ? "regions" : "interleaved";
            CK(shs_group_set_option(g_grp, SHS_OPT_SHARD_LAYOUT, layout));
            shs_tonemap_desc tm{1.0f, 2.2f, SHS_TONEMAP_PRESENT};
            CK(shs_lib_fuse_tonemap(g_ctx, fused ? &tm : nullptr));
            CK(shs_group_lib_fuse_tonemap(g_grp, fused ? &tm : nullptr));
            std::vector<float> h1(np * 4), hg(np * 4), z1(np), zg(np), m1(np * 2), mgv(np * 2);
            std::vector<uint8_t> p1(np * 4), pg(np * 4);
            // three frames back to back: the group gathers each without a host wait in between
            const float yaws[3] = {0.0f, 0.4f, 1.1f};
            for (float yaw : yaws) {
                shs_lib_draw dg[2];
                lib_draws(sg, fg, yaw, W, H, dg);
                CK(shs_group_render_pbr_forward(g_grp, &f, dg, 2));
                CK(shs_group_gather(g_grp, fused ? SHS_TARGET_LIB_PRESENT : SHS_TARGET_LIB));
            }
            shs_lib_draw d1[2];
            lib_draws(s1, f1, yaws[2], W, H, d1);
            CK(shs_render_pbr_forward(g_ctx, &f, d1, 2));
            if (fused) {
                CK(shs_resolve_ldr(g_ctx, nullptr, p1.data()));
                CK(shs_resolve_ldr(root0, nullptr, pg.data()));
                const size_t dp = count_diff(p1, pg);
                std::printf("library fused tonemap %d ranks (%s), 3rd frame: present %zu differing\n", n, lname, dp);
                EXPECT(dp == 0, "sharded present staging differs");
            } else {
                CK(shs_resolve_lib(g_ctx, h1.data(), z1.data(), m1.data()));
                CK(shs_resolve_lib(root0, hg.data(), zg.data(), mgv.data()));
                const size_t dh = count_diff(h1, hg), dz = count_diff(z1, zg), dm = count_diff(m1, mgv);
                size_t cov = 0;
                for (float z : z1) cov += z < 1.0f;
                std::printf("library %d ranks (%s), 3rd frame: hdr %zu / depth %zu / motion %zu differing, %zu covered px\n", n,
                            lname, dh, dz, dm, cov);
                EXPECT(dh == 0 && dz == 0 && dm == 0, "sharded library frame differs");
                EXPECT(cov > 10000, "library frame nearly empty");
            }
            if (layout == SHS_SHARD_REGIONS) {   // the rectangles every rank used tile the bin grid exactly
                std::vector<int32_t> rects((size_t)4 * n);
                CK(shs_get_shard_regions(root0, n, rects.data()));
                const int tx = (W + 31) / 32, ty = (H + 31) / 32;
                std::vector<int> cover((size_t)tx * ty, 0);
                for (int r = 0; r < n; ++r)
                    for (int y = rects[4 * r + 1]; y <= rects[4 * r + 3]; ++y)
                        for (int x = rects[4 * r]; x <= rects[4 * r + 2]; ++x)
                            if (x >= 0 && x < tx && y >= 0 && y < ty) cover[(size_t)y * tx + x]++;
                size_t bad = 0;
                for (int c : cover) bad += c != 1;
                EXPECT(bad == 0, "region layout does not tile the bin grid (%zu tiles)", bad);
            }
        }
    }
    CK(shs_group_synchronize(g_grp));
    shs_group_destroy(g_grp);
    shs_destroy(g_ctx);
    std::printf(g_fail ? "abi_group: %d FAILED\n" : "abi_group: all passed\n", g_fail);
    return g_fail ? 1 : 0;
}
