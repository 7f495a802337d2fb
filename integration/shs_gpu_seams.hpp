// shs_gpu_seams.hpp -- drop-in adapters that route the reference's hot path through libshs_gpu.
//
// Header-only C++20 for the reference tree (sharavsambuu/leisure-software-renderer); it includes the
// reference's own headers and glm, so it compiles there, not in this repository's image (glm, SDL2
// and assimp are absent here -- SURVEY.md 8c).  The C ABI it calls (include/shs_gpu.h) is compiled
// and exercised here by tests/abi_c/abi_legacy.cpp.  Paths below are relative to
// /root/reference/cpp-folders/src/.
//
//   Seam 1  LegacyRendererSystemGPU<SceneT, ObjectT, SHADING>: replaces RendererSystem of
//           hello-3d-primitives/hello_pipeline_{blinn_phong,phong,gouraud,flat}_shading.cpp
//           (the 80x80 tile-job loop of process(), :244-313 in the Blinn-Phong demo).
//   Seam 3  PassShadowMapGPU / PassPBRForwardGPU: IRenderPass implementations with the ids,
//           contracts and resource I/O of PassShadowMapAdapter / PassPBRForwardAdapter
//           (shs-renderer-lib/include/shs/pipeline/pass_adapters.hpp:356-394, 1005-1062), registered
//           under "shadow_map" / "pbr_forward" by register_gpu_passes() over the standard registry
//           (make_standard_pass_factory_registry, pass_adapters.hpp:1497-1568).
#pragma once

#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

#include <glm/glm.hpp>
#include <glm/gtc/matrix_transform.hpp>
#include <glm/gtc/type_ptr.hpp>

#include "shs_gpu.h"

namespace shs_gpu_seams {

inline void check(shs_ctx *ctx, int rc) {
    if (rc != SHS_OK) throw std::runtime_error(ctx ? shs_last_error(ctx) : "shs_gpu: no context");
}

// One device context per host render thread (a context is used by one thread).
struct Device {
    shs_ctx *ctx = nullptr;
    explicit Device(int device_index = 0) {
        if (shs_create(device_index, &ctx) != SHS_OK) throw std::runtime_error("shs_gpu: no gfx950 device");
    }
    ~Device() { shs_destroy(ctx); }
    Device(const Device &) = delete;
    Device &operator=(const Device &) = delete;
};

// =====================================================================================================
// Seam 1 -- the legacy Canvas / ZBuffer / draw-call path.
//
// Maintainer edit in a hello_pipeline_*_shading.cpp demo (SystemProcessor, :327-360 of the Blinn-Phong
// demo): declare the member as `shs::AbstractSystem *renderer_system;` and construct
//     this->renderer_system = new shs_gpu_seams::LegacyRendererSystemGPU<HelloScene, MonkeyObject,
//                                                                      SHS_SHADING_BLINN_PHONG>(scene);
// (SHS_SHADING_PHONG / _GOURAUD / _FLAT in the other three demos).  Everything else -- the scene,
// the LogicSystem / Viewer camera update, Canvas::fill_pixel, copy_to_SDLSurface and the SDL loop --
// is unchanged.  The job system is no longer used for rendering.
//
// SceneT must provide what RendererSystem reads (HelloScene, blinn_phong_shading.cpp:144-163):
//   std::vector<shs::AbstractObject3D*> scene_objects; shs::Canvas *canvas; shs::Viewer *viewer;
//   glm::vec3 light_direction;
// ObjectT (MonkeyObject, :110-141): ModelGeometry *geometry; shs::Color color; get_world_matrix().
// =====================================================================================================
template <class SceneT, class ObjectT, int SHADING>
class LegacyRendererSystemGPU : public shs::AbstractSystem {
public:
    static constexpr int kTileX = 80, kTileY = 80;   // TILE_SIZE_X / _Y (blinn_phong_shading.cpp:29-30)

    explicit LegacyRendererSystemGPU(SceneT *scene, int device_index = 0)
        : scene_(scene), dev_(device_index),
          // the same ZBuffer RendererSystem allocates in its constructor (:176-181)
          z_buffer_(scene->canvas->get_width(), scene->canvas->get_height(), scene->viewer->camera->z_near,
                    scene->viewer->camera->z_far) {}

    // RendererSystem::process(dt) (:244-313): clear z, rasterise every object, join -- one enqueue plus
    // one resolve into the caller-owned Canvas / ZBuffer in their own layouts.
    void process(float /*delta_time*/) override {
        shs::Canvas &canvas = *scene_->canvas;
        const glm::mat4 view = scene_->viewer->camera->view_matrix;
        const glm::mat4 proj = scene_->viewer->camera->projection_matrix;
        // flat_shading.cpp:256: the Flat pipeline's view-space light direction
        const glm::vec3 light_dir_view = glm::normalize(glm::vec3(view * glm::vec4(scene_->light_direction, 0.0f)));

        draws_.clear();
        for (shs::AbstractObject3D *object : scene_->scene_objects) {
            auto *obj = dynamic_cast<ObjectT *>(object);   // the demo's `if (!monkey) continue;`
            if (!obj) continue;
            shs_legacy_draw d{};
            d.mesh_id = mesh_id(obj);
            d.shading = SHADING;
            if constexpr (SHADING == SHS_SHADING_FLAT) {
                // Uniforms{mv, mvp, light_dir_view, color} (flat_shading.cpp:284-287)
                const glm::mat4 mv = view * obj->get_world_matrix();
                const glm::mat4 mvp = proj * mv;
                std::memcpy(d.mvp, glm::value_ptr(mvp), sizeof d.mvp);
                std::memcpy(d.model, glm::value_ptr(mv), sizeof d.model);
                std::memcpy(d.light_dir, glm::value_ptr(light_dir_view), sizeof d.light_dir);
            } else {
                // Uniforms{model, mvp = proj * view * model, light_dir, camera_pos, color} (:277-282)
                const glm::mat4 model = obj->get_world_matrix();
                const glm::mat4 mvp = proj * view * model;
                std::memcpy(d.mvp, glm::value_ptr(mvp), sizeof d.mvp);
                std::memcpy(d.model, glm::value_ptr(model), sizeof d.model);
                std::memcpy(d.light_dir, glm::value_ptr(scene_->light_direction), sizeof d.light_dir);
                std::memcpy(d.camera_pos, glm::value_ptr(scene_->viewer->position), sizeof d.camera_pos);
            }
            d.color[0] = obj->color.r; d.color[1] = obj->color.g; d.color[2] = obj->color.b; d.color[3] = obj->color.a;
            draws_.push_back(d);
        }

        shs_frame_desc f{};
        f.width = canvas.get_width();
        f.height = canvas.get_height();
        f.ref_tile_w = kTileX;   // the reference's tile-clamp pixels are reproduced exactly
        f.ref_tile_h = kTileY;
        f.shard_rank = 0;
        f.shard_count = 1;
        // main() clears the canvas black before render (:441, Canvas::fill_pixel); the GPU frame
        // writes every pixel, clear included
        f.clear_color[0] = 0; f.clear_color[1] = 0; f.clear_color[2] = 0; f.clear_color[3] = 255;
        check(dev_.ctx, shs_render_legacy(dev_.ctx, &f, draws_.data(), static_cast<int32_t>(draws_.size())));
        // Canvas::buffer() (Buffer<Color>, canvas rows bottom-up, RGBA8 -- shs_renderer.hpp:308-342, 753-796)
        // and ZBuffer::buffer() (screen rows as the legacy pipelines index it, :652-702)
        check(dev_.ctx, shs_resolve(dev_.ctx, reinterpret_cast<uint8_t *>(canvas.buffer().raw()), z_buffer_.buffer().raw()));
    }

    shs::ZBuffer &z_buffer() { return z_buffer_; }   // RendererSystem keeps it private; exposed here
    shs_ctx *context() { return dev_.ctx; }

private:
    // ModelGeometry's soup (shs_renderer.hpp:1296-1298): triangles[i] / normals[i], 3 corners per
    // triangle; uploaded once per geometry and kept device resident.
    int32_t mesh_id(ObjectT *obj) {
        auto it = mesh_ids_.find(obj->geometry);
        if (it != mesh_ids_.end()) return it->second;
        const auto &tri = obj->geometry->triangles;
        const auto &nrm = obj->geometry->normals;
        static_assert(sizeof(glm::vec3) == 12, "ModelGeometry vectors are packed float triples");
        int32_t id = -1;
        check(dev_.ctx, shs_mesh_upload_soup(dev_.ctx, glm::value_ptr(tri[0]), glm::value_ptr(nrm[0]),
                                             static_cast<int32_t>(tri.size() / 3), &id));
        mesh_ids_.emplace(obj->geometry, id);
        return id;
    }

    SceneT *scene_;
    Device dev_;
    shs::ZBuffer z_buffer_;
    std::vector<shs_legacy_draw> draws_;
    std::unordered_map<const void *, int32_t> mesh_ids_;
};

// =====================================================================================================
// Seam 3 -- the library's plugin pipeline (shs-renderer-lib/include/shs/pipeline/).
// =====================================================================================================
}  // namespace shs_gpu_seams

#if __has_include("shs/pipeline/pass_adapters.hpp")
#include "shs/pipeline/pass_adapters.hpp"

namespace shs_gpu_seams {

// Device-resident MeshData (resources/mesh.hpp:23-43), uploaded on first use.
class GpuMeshes {
public:
    explicit GpuMeshes(shs_ctx *ctx) : ctx_(ctx) {}
    int32_t id(const shs::MeshData &m) {
        auto it = ids_.find(&m);
        if (it != ids_.end()) return it->second;
        int32_t id = -1;
        check(ctx_, shs_mesh_upload(ctx_, glm::value_ptr(m.positions[0]), static_cast<int32_t>(m.positions.size()),
                                    m.normals.empty() ? nullptr : glm::value_ptr(m.normals[0]),
                                    static_cast<int32_t>(m.normals.size()),
                                    m.uvs.empty() ? nullptr : glm::value_ptr(m.uvs[0]), static_cast<int32_t>(m.uvs.size()),
                                    m.indices.empty() ? nullptr : m.indices.data(), static_cast<int64_t>(m.indices.size()),
                                    &id));
        ids_.emplace(&m, id);
        return id;
    }

private:
    shs_ctx *ctx_;
    std::unordered_map<const shs::MeshData *, int32_t> ids_;
};

// Device-resident Texture2DData (resources/texture.hpp:23-49), uploaded on first use; an invalid one
// (Texture2DData::valid() false) maps to 0 -- the sampler's vec3(1) (builtin_shaders.hpp:35).
class GpuTextures {
public:
    explicit GpuTextures(shs_ctx *ctx) : ctx_(ctx) {}
    int32_t id(const shs::Texture2DData *t) {
        if (!t || !t->valid()) return 0;
        auto it = ids_.find(t);
        if (it != ids_.end()) return it->second;
        int32_t id = 0;
        check(ctx_, shs_texture_upload(ctx_, &t->texels[0].r, t->w, t->h, &id));
        ids_.emplace(t, id);
        return id;
    }

private:
    shs_ctx *ctx_;
    std::unordered_map<const shs::Texture2DData *, int32_t> ids_;
};

// Shared by the passes of one pipeline: the device context, its meshes and textures, and whether the
// device shadow map belongs to the current frame.
struct GpuPassRuntime {
    Device device;
    GpuMeshes meshes;
    GpuTextures textures;
    bool resolve_shadow_to_host = false;   // also fill RT_ShadowDepth (for CPU consumers: shadow debug)
    explicit GpuPassRuntime(int device_index = 0) : device(device_index), meshes(device.ctx), textures(device.ctx) {}
};

// RenderItem transform, as both passes build it (pass_shadow_map.hpp:56-64, pass_pbr_forward.hpp:136-141).
inline glm::mat4 item_model(const shs::RenderItem &item) {
    glm::mat4 model(1.0f);
    model = glm::translate(model, item.tr.pos);
    model = glm::rotate(model, item.tr.rot_euler.x, glm::vec3(1.0f, 0.0f, 0.0f));
    model = glm::rotate(model, item.tr.rot_euler.y, glm::vec3(0.0f, 1.0f, 0.0f));
    model = glm::rotate(model, item.tr.rot_euler.z, glm::vec3(0.0f, 0.0f, 1.0f));
    model = glm::scale(model, item.tr.scl);
    return model;
}

// PassShadowMap::execute (passes/pass_shadow_map.hpp:44-206) on the GPU: scene AABB of the casters'
// mesh bounds, build_dir_light_camera_aabb (camera/light_camera.hpp:33-98), the depth pass.  Sets
// ctx.shadow exactly as the CPU pass does; the depth map stays on the device for PassPBRForwardGPU.
class PassShadowMapGPU final : public shs::IRenderPass {
public:
    PassShadowMapGPU(std::shared_ptr<GpuPassRuntime> rt, shs::RT_Shadow rt_shadow) : rt_(std::move(rt)), rt_shadow_(rt_shadow) {}

    const char *id() const override { return "shadow_map"; }
    shs::RenderBackendType preferred_backend() const override { return shs::RenderBackendType::Software; }
    bool supports_backend(shs::RenderBackendType b) const override { return b == shs::RenderBackendType::Software; }
    shs::TechniquePassContract describe_contract() const override { return shs::PassShadowMapAdapter(rt_shadow_).describe_contract(); }
    shs::PassIODesc describe_io() const override { return shs::PassShadowMapAdapter(rt_shadow_).describe_io(); }

    shs::PassExecutionResult execute_resolved(shs::Context &ctx, const shs::PassExecutionRequest &request) override {
        if (!request.valid || !request.inputs.scene || !request.inputs.frame || !request.inputs.registry)
            return shs::PassExecutionResult::not_executed();
        const shs::Scene &scene = *request.inputs.scene;
        const shs::FrameParams &fp = *request.inputs.frame;
        ctx.shadow.reset();
        if (!rt_shadow_.valid() || !fp.pass.shadow.enable) return shs::PassExecutionResult::executed_no_outputs();
        auto *shadow = static_cast<shs::RT_ShadowDepth *>(request.inputs.registry->get(rt_shadow_));
        if (!shadow || shadow->w <= 0 || shadow->h <= 0) return shs::PassExecutionResult::executed_no_outputs();

        casters_.clear();
        for (const auto &item : scene.items) {
            if (!item.visible || !item.casts_shadow || !scene.resources) continue;
            const shs::MeshData *mesh = scene.resources->get_mesh((shs::MeshAssetHandle)item.mesh);
            if (!mesh || mesh->positions.empty()) continue;
            shs_shadow_caster c{};
            c.mesh_id = rt_->meshes.id(*mesh);
            const glm::mat4 model = item_model(item);
            std::memcpy(c.model, glm::value_ptr(model), sizeof c.model);
            casters_.push_back(c);
        }
        shs_ctx *dctx = rt_->device.ctx;
        float light_vp[16];
        check(dctx, shs_render_shadow_map(dctx, shadow->w, shadow->h, glm::value_ptr(scene.sun.dir_ws), casters_.data(),
                                          static_cast<int32_t>(casters_.size()), light_vp));
        ctx.shadow.map = shadow;
        ctx.shadow.light_viewproj = glm::make_mat4(light_vp);
        ctx.shadow.valid = true;
        if (rt_->resolve_shadow_to_host) check(dctx, shs_resolve_shadow_map(dctx, shadow->depth.data()));
        return shs::PassExecutionResult::executed_no_outputs();
    }

private:
    std::shared_ptr<GpuPassRuntime> rt_;
    shs::RT_Shadow rt_shadow_{};
    std::vector<shs_shadow_caster> casters_;
};

// PassPBRForward::execute (passes/pass_pbr_forward.hpp:49-214) on the GPU: one shs_lib_draw per visible
// item with the ShaderUniforms the pass builds, the program it binds (:100-108), the motion history
// (:123-155), then one resolve into RT_ColorHDR / RT_ColorDepthMotion (PixelBuffer2D rows, y up).
class PassPBRForwardGPU final : public shs::IRenderPass {
public:
    PassPBRForwardGPU(std::shared_ptr<GpuPassRuntime> rt, shs::RTHandle rt_hdr, shs::RT_Motion rt_motion, shs::RTHandle rt_shadow)
        : rt_(std::move(rt)), rt_hdr_(rt_hdr), rt_motion_(rt_motion), rt_shadow_(rt_shadow) {}

    const char *id() const override { return "pbr_forward"; }
    shs::RenderBackendType preferred_backend() const override { return shs::RenderBackendType::Software; }
    bool supports_backend(shs::RenderBackendType b) const override { return b == shs::RenderBackendType::Software; }
    shs::TechniquePassContract describe_contract() const override {
        return shs::PassPBRForwardAdapter(rt_hdr_, rt_motion_, rt_shadow_).describe_contract();
    }
    shs::PassIODesc describe_io() const override { return shs::PassPBRForwardAdapter(rt_hdr_, rt_motion_, rt_shadow_).describe_io(); }

    shs::PassExecutionResult execute_resolved(shs::Context &ctx, const shs::PassExecutionRequest &request) override {
        if (!request.valid || !request.inputs.scene || !request.inputs.frame || !request.inputs.registry)
            return shs::PassExecutionResult::not_executed();
        const shs::Scene &scene = *request.inputs.scene;
        const shs::FrameParams &fp = *request.inputs.frame;
        shs::RTRegistry &rtr = *request.inputs.registry;
        if (!rt_hdr_.valid()) return shs::PassExecutionResult::not_executed();
        auto *hdr = static_cast<shs::RT_ColorHDR *>(rtr.get(rt_hdr_));
        if (!hdr || hdr->w <= 0 || hdr->h <= 0) return shs::PassExecutionResult::not_executed();
        auto *motion = rt_motion_.valid() ? static_cast<shs::RT_ColorDepthMotion *>(rtr.get(rt_motion_)) : nullptr;
        auto *shadow = rt_shadow_.valid() ? static_cast<shs::RT_ShadowDepth *>(rtr.get(rt_shadow_)) : nullptr;
        const bool depth_motion = motion && motion->w == hdr->w && motion->h == hdr->h;
        // The GPU pass draws the no-sky gradient background (:64-85); a sky model is outside its scope.
        if (scene.sky) unsupported("sky model backgrounds");

        int32_t program = SHS_PROGRAM_PBR_MR;
        if (fp.shading_model == shs::ShadingModel::BlinnPhong) program = SHS_PROGRAM_BLINN_PHONG;
        if (fp.debug_view == shs::DebugViewMode::Albedo) program = SHS_PROGRAM_DEBUG_ALBEDO;
        if (fp.debug_view == shs::DebugViewMode::Normal) program = SHS_PROGRAM_DEBUG_NORMAL;
        if (fp.debug_view == shs::DebugViewMode::Depth) program = SHS_PROGRAM_DEBUG_DEPTH;
        const int32_t cull = fp.cull_mode == shs::CullMode::None    ? SHS_CULL_NONE
                             : fp.cull_mode == shs::CullMode::Front ? SHS_CULL_FRONT
                                                                    : SHS_CULL_BACK;

        std::unordered_map<uint64_t, glm::mat4> next_prev{};
        draws_.clear();
        for (size_t item_index = 0; item_index < scene.items.size(); ++item_index) {
            const auto &item = scene.items[item_index];
            if (!item.visible || !scene.resources) continue;
            const shs::MeshData *mesh = scene.resources->get_mesh((shs::MeshAssetHandle)item.mesh);
            if (!mesh || mesh->empty()) continue;
            const shs::MaterialData *mat = scene.resources->get_material((shs::MaterialAssetHandle)item.mat);
            // u.base_color_tex (:173-176): the registry's Texture2DData, sampled on the device
            const int32_t tex_id = (mat && mat->base_color_tex != 0)
                                       ? rt_->textures.id(scene.resources->get_texture(mat->base_color_tex))
                                       : 0;
            const glm::mat4 model = item_model(item);
            uint64_t key = item.object_id;                                         // :143-148
            if (key == 0) {
                key = ((uint64_t)item.mesh << 32) ^ (uint64_t)item.mat ^ ((uint64_t)item_index + 1u);
                if (key == 0) key = 1;
            }
            glm::mat4 prev_model = model;
            const auto it = ctx.history.prev_model_by_object.find(key);
            if (ctx.history.has_prev_frame && it != ctx.history.prev_model_by_object.end()) prev_model = it->second;
            next_prev[key] = model;

            shs_lib_draw d{};
            d.mesh_id = rt_->meshes.id(*mesh);
            d.program = program;
            d.cull_mode = cull;
            d.front_face_ccw = fp.front_face_ccw ? 1 : 0;
            const glm::mat4 prev_vp = ctx.history.has_prev_frame ? scene.cam.prev_viewproj : scene.cam.viewproj;
            std::memcpy(d.model, glm::value_ptr(model), 64);
            std::memcpy(d.viewproj, glm::value_ptr(scene.cam.viewproj), 64);
            std::memcpy(d.prev_model, glm::value_ptr(prev_model), 64);
            std::memcpy(d.prev_viewproj, glm::value_ptr(prev_vp), 64);
            std::memcpy(d.light_dir_ws, glm::value_ptr(scene.sun.dir_ws), 12);
            std::memcpy(d.light_color, glm::value_ptr(scene.sun.color), 12);
            d.light_intensity = scene.sun.intensity;
            std::memcpy(d.camera_pos, glm::value_ptr(scene.cam.pos), 12);
            const glm::vec3 base = mat ? mat->base_color : glm::vec3(0.8f, 0.5f, 0.2f);   // :175-181
            std::memcpy(d.base_color, glm::value_ptr(base), 12);
            d.metallic = mat ? mat->metallic : 0.1f;
            d.roughness = mat ? mat->roughness : 0.5f;
            d.ao = mat ? mat->ao : 1.0f;
            if (fp.pass.shadow.enable && shadow && ctx.shadow.valid) {                    // :184-193
                d.shadow = 1;
                std::memcpy(d.light_viewproj, glm::value_ptr(ctx.shadow.light_viewproj), 64);
                d.shadow_bias_const = fp.pass.shadow.bias_const;
                d.shadow_bias_slope = fp.pass.shadow.bias_slope;
                d.shadow_pcf_radius = fp.pass.shadow.pcf_radius;
                d.shadow_pcf_step = fp.pass.shadow.pcf_step;
                d.shadow_strength = fp.pass.shadow.strength;
            }
            d.enable_motion_vectors = fp.pass.motion_vectors.enable ? 1 : 0;
            d.base_color_tex = tex_id;
            draws_.push_back(d);
        }

        shs_lib_frame f{};
        f.width = hdr->w;
        f.height = hdr->h;
        f.shard_rank = 0;
        f.shard_count = 1;
        f.flags = SHS_LIB_BG_GRADIENT | (depth_motion ? SHS_LIB_DEPTH_MOTION : 0u);
        f.zn = depth_motion ? motion->zn : 0.1f;
        f.zf = depth_motion ? motion->zf : 1000.0f;
        shs_ctx *dctx = rt_->device.ctx;
        check(dctx, shs_render_pbr_forward(dctx, &f, draws_.data(), static_cast<int32_t>(draws_.size())));
        check(dctx, shs_resolve_lib(dctx, &hdr->color.data[0].r, depth_motion ? motion->depth.data.data() : nullptr,
                                    depth_motion ? &motion->motion.data[0].x : nullptr));
        shs_lib_stats st{};
        check(dctx, shs_get_lib_stats(dctx, &st));
        ctx.debug.tri_input = st.tri_input;
        ctx.debug.tri_after_clip = st.tri_after_clip;
        ctx.debug.tri_raster = st.tri_raster;
        ctx.history.prev_model_by_object.swap(next_prev);
        ctx.history.has_prev_frame = true;
        return shs::PassExecutionResult::executed_no_outputs();
    }

private:
    // Inputs outside the GPU pass's scope (DESIGN.md "Out of scope") fail loudly: no silent CPU path.
    [[noreturn]] static void unsupported(const char *what) {
        throw std::runtime_error(std::string("PassPBRForwardGPU: ") + what + " are not supported on the GPU path");
    }

    std::shared_ptr<GpuPassRuntime> rt_;
    shs::RTHandle rt_hdr_{};
    shs::RT_Motion rt_motion_{};
    shs::RTHandle rt_shadow_{};
    std::vector<shs_lib_draw> draws_;
};

// Replace the standard registry's "shadow_map" and "pbr_forward" factories with the GPU passes
// (PassFactoryRegistry::register_factory overwrites by id, pass_registry.hpp:52-63); every other pass
// keeps the reference's implementation.  Usage:
//   auto reg = shs::make_standard_pass_factory_registry(rt_shadow, rt_hdr, rt_motion, rt_ldr, t0, t1);
//   auto gpu = std::make_shared<shs_gpu_seams::GpuPassRuntime>(0);
//   shs_gpu_seams::register_gpu_passes(reg, gpu, rt_shadow, rt_hdr, rt_motion);
inline void register_gpu_passes(shs::PassFactoryRegistry &reg, std::shared_ptr<GpuPassRuntime> rt, shs::RT_Shadow rt_shadow,
                                shs::RTHandle rt_hdr, shs::RT_Motion rt_motion) {
    reg.register_factory(shs::PassId::ShadowMap, [=]() { return std::make_unique<PassShadowMapGPU>(rt, rt_shadow); });
    reg.register_factory(shs::PassId::PBRForward, [=]() {
        return std::make_unique<PassPBRForwardGPU>(rt, rt_hdr, rt_motion, shs::RTHandle{rt_shadow.id});
    });
}

}  // namespace shs_gpu_seams
#endif
