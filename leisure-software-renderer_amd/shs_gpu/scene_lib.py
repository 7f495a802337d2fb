"""Synthetic library-path scenes (BASELINE.json configs[4], "C5": PBR Cook-Torrance + shadow-map pass).

C5: Suzanne + a floor plane, PassShadowMap (2048^2, sun normalize(0.4668,-0.3487,0.8127),
hello_pbr.cpp:110) then PassPBRForward with make_pbr_mr_program at 3840x2160.  Reference defaults are used
where the scene does not say otherwise: DirectionalLight colour 1 / intensity 5 (scene/scene_types.hpp:65-73),
ShadowPassParams bias 0.0008 / 0.0015, PCF radius 2 (frame/frame_params.hpp:25-33), Camera fov 60,
zn 0.1, zf 200 (scene_types.hpp:43-60), the no-material fallback (0.8,0.5,0.2) metallic 0.1 roughness 0.5
(pass_pbr_forward.hpp:178-184) for Suzanne and a grey plastic floor.
"""
import numpy as np

from .lib_path import (CULL_BACK, CULL_NONE, PROGRAM_PBR_MR, LibDraw, LibFrame, LibMesh, ShadowCaster, Texture2D, look_at_lh,
                       mat_mul, model_euler, perspective_lh_no)
from .scene import monkey

f32 = np.float32
SUN_DIR = (0.4668, -0.3487, 0.8127)   # normalised by build_dir_light_camera_aabb and the FS


def _glm_normalize(v):
    v = np.asarray(v, dtype=np.float32)
    d = (v[0] * v[0] + v[1] * v[1]) + v[2] * v[2]
    return (v * (f32(1.0) / np.sqrt(d, dtype=np.float32))).astype(np.float32)


_MONKEY_LIB = None


def monkey_lib() -> LibMesh:
    """Suzanne as an indexed MeshData: identical (position, normal) corners of the soup joined
    (the assimp JoinIdenticalVertices step of the reference's loader), first-seen order."""
    global _MONKEY_LIB
    if _MONKEY_LIB is None:
        soup = monkey()
        corners = np.concatenate([soup.positions.reshape(-1, 3), soup.normals.reshape(-1, 3)], axis=1)
        _, first, inv = np.unique(corners.view(np.uint32), axis=0, return_index=True, return_inverse=True)
        order = np.argsort(first)
        remap = np.empty_like(order)
        remap[order] = np.arange(order.size)
        verts = corners[first[order]]
        _MONKEY_LIB = LibMesh(positions=np.ascontiguousarray(verts[:, :3]), normals=np.ascontiguousarray(verts[:, 3:]),
                              uvs=None, indices=remap[inv.reshape(-1)].astype(np.uint32))
    return _MONKEY_LIB


def make_plane(width=10.0, depth=10.0, seg_x=10, seg_z=10) -> LibMesh:
    """make_plane(PlaneDesc) (geometry/primitives_builders.hpp:56-114) in float32, including
    add_triangle_match_normals' winding fix-up."""
    sx, sz = max(1, seg_x), max(1, seg_z)
    hw, hz = f32(width) * f32(0.5), f32(depth) * f32(0.5)
    origin = np.array([-hw, 0.0, -hz], np.float32)
    au = np.array([width, 0.0, 0.0], np.float32)
    av = np.array([0.0, 0.0, depth], np.float32)
    n = np.array([0.0, 1.0, 0.0], np.float32)
    pos, uv = [], []
    for y in range(sz + 1):
        fv = f32(y) / f32(sz)
        for x in range(sx + 1):
            fu = f32(x) / f32(sx)
            pos.append((origin + au * fu) + av * fv)
            uv.append((fu, fv))
    pos = np.asarray(pos, np.float32)
    idx = []
    stride = sx + 1

    def add(a, b, c):
        fn = np.cross(pos[b] - pos[a], pos[c] - pos[a])
        if float(np.dot(fn, n + n + n)) < 0.0:
            b, c = c, b
        idx.extend((a, b, c))

    for y in range(sz):
        for x in range(sx):
            i00 = y * stride + x
            i10, i01 = i00 + 1, i00 + stride
            add(i00, i01, i10)
            add(i10, i01, i00 + stride + 1)
    return LibMesh(positions=pos, normals=np.tile(n, (pos.shape[0], 1)), uvs=np.asarray(uv, np.float32),
                   indices=np.asarray(idx, np.uint32))


def noise_texture(w, h, seed) -> Texture2D:
    """A seeded RGBA8 Texture2DData of w x h texels (any size, 1x1 included)."""
    rng = np.random.default_rng(seed)
    return Texture2D(rgba=rng.integers(0, 256, size=(h, w, 4), dtype=np.uint8))


def monkey_lib_uv() -> LibMesh:
    """Suzanne with a synthetic UV0 (cylindrical projection of the positions, u wrapping past 1)."""
    m = monkey_lib()
    p = m.positions
    u = (np.arctan2(p[:, 0], p[:, 2]) / np.float32(np.pi) * np.float32(1.5)).astype(np.float32)
    v = (p[:, 1] * np.float32(0.7) + np.float32(0.5)).astype(np.float32)
    return LibMesh(positions=p, normals=m.normals, uvs=np.stack([u, v], axis=1).astype(np.float32), indices=m.indices)


def c5_scene(width=3840, height=2160, shadow_size=2048, program=PROGRAM_PBR_MR, motion=True, yaw=0.0, floor_seg=16,
             textured=False, floor_tex=(37, 23), monkey_tex=(1, 1)):
    """-> (frame, draws without shadow wiring, casters, sun_dir, shadow_size).  Call
    `wire_shadow(draws, light_viewproj)` after the shadow pass.
    textured: the materials carry a base_color_tex (pass_pbr_forward.hpp:173-176) -- the floor a
    floor_tex-sized noise texture with UVs running from -2.25 to 4.25 (repeat wrap, negative UVs), clipped
    at the frustum; Suzanne a monkey_tex-sized one over a cylindrical UV0."""
    zn, zf = 0.1, 200.0
    ang = np.deg2rad(yaw)
    eye = (f32(16.0 * np.sin(ang)), f32(7.0), f32(-16.0 * np.cos(ang)))
    view = look_at_lh(eye, (0.0, 1.5, 0.0))
    proj = perspective_lh_no(f32(np.deg2rad(60.0)), f32(width) / f32(height), zn, zf)
    vp = mat_mul(proj, view)
    eye_p = (f32(16.0 * np.sin(ang - 0.02)), f32(7.0), f32(-16.0 * np.cos(ang - 0.02)))
    prev_vp = mat_mul(proj, look_at_lh(eye_p, (0.0, 1.5, 0.0)))
    m_monkey = model_euler((0.0, 2.2, 0.0), (0.0, 0.0, 0.0), (2.0, 2.0, 2.0))
    pm_monkey = model_euler((0.0, 2.2, 0.0), (0.0, -0.05, 0.0), (2.0, 2.0, 2.0))
    m_floor = model_euler((0.0, 0.0, 0.0))
    floor = make_plane(55.0, 140.0, floor_seg, floor_seg)
    mk = monkey_lib()
    if textured:
        floor = LibMesh(positions=floor.positions, normals=floor.normals,
                        uvs=(floor.uvs * np.float32(6.5) - np.float32(2.25)).astype(np.float32), indices=floor.indices)
        mk = monkey_lib_uv()
    common = dict(viewproj=vp, prev_viewproj=prev_vp, light_dir_ws=SUN_DIR, light_color=(1.0, 1.0, 1.0),
                  light_intensity=5.0, camera_pos=eye, program=program, enable_motion_vectors=motion)
    draws = [
        LibDraw(mesh=floor, model=m_floor, base_color=(0.6, 0.6, 0.6), metallic=0.0, roughness=0.8, ao=1.0,
                cull_mode=CULL_NONE, **common),
        LibDraw(mesh=mk, model=m_monkey, prev_model=pm_monkey, base_color=(0.8, 0.5, 0.2), metallic=0.1,
                roughness=0.5, ao=1.0, cull_mode=CULL_NONE, **common),
    ]
    if textured:
        draws[0].base_color_tex = noise_texture(*floor_tex, seed=0x7E1)
        draws[1].base_color_tex = noise_texture(*monkey_tex, seed=0x7E2)
    casters = [ShadowCaster(floor, m_floor), ShadowCaster(mk, m_monkey)]
    frame = LibFrame(width, height, depth_motion=True, zn=zn, zf=zf, bg_gradient=True)
    return frame, draws, casters, SUN_DIR, shadow_size


def wire_shadow(draws, light_viewproj):
    for d in draws:
        d.shadow = True
        d.light_viewproj = np.asarray(light_viewproj, np.float32)
    return draws


# ---- C4: Forward+ tiled (BASELINE.json configs[3]) ---------------------------------------------
C4_BOX_MIN = (-30.0, 0.0, 8.0)
C4_BOX_MAX = (30.0, 12.0, 90.0)


def c4_geometry(n_objects=1000, tris_per_object=1000, n_draws=16, seed=0x5EED):
    """`n_objects` seeded objects of `tris_per_object` small triangles (soup, fp32
    position + face normal), all in front of the near plane, grouped into `n_draws` draws (materials).
    numpy PCG64 with the survey's seed stands in for its mt19937 (synthetic data either way)."""
    rng = np.random.default_rng(seed)
    lo, hi = np.array(C4_BOX_MIN, np.float32), np.array(C4_BOX_MAX, np.float32)
    centers = rng.uniform(lo, hi, size=(n_objects, 3)).astype(np.float32)
    radius = rng.uniform(0.6, 2.0, size=(n_objects, 1, 1)).astype(np.float32)
    # per triangle: a point in the object's ball + three corners within 0.35 world units
    p = centers[:, None, :] + radius * rng.normal(size=(n_objects, tris_per_object, 3)).astype(np.float32) * f32(0.45)
    corners = p[:, :, None, :] + rng.uniform(-0.35, 0.35, size=(n_objects, tris_per_object, 3, 3)).astype(np.float32)
    e1 = corners[:, :, 1] - corners[:, :, 0]
    e2 = corners[:, :, 2] - corners[:, :, 0]
    nrm = np.cross(e1, e2)
    nrm /= np.maximum(np.linalg.norm(nrm, axis=-1, keepdims=True), 1e-12)
    nrm = np.repeat(nrm[:, :, None, :], 3, axis=2).astype(np.float32)
    groups = np.array_split(np.arange(n_objects), n_draws)
    meshes = []
    for g in groups:
        pos = corners[g].reshape(-1, 3)
        meshes.append(LibMesh(positions=np.ascontiguousarray(pos), normals=np.ascontiguousarray(nrm[g].reshape(-1, 3))))
    colors = rng.uniform(0.25, 0.95, size=(n_draws, 3)).astype(np.float32)
    return meshes, colors


def c4_lights(n_lights=256, seed=0x11A7):
    """256 point lights: position in the scene box, range U[2,8], colour U[0.2,1]^3, intensity
    U[0.5,2], Smooth attenuation with the reference defaults (light_types.hpp:95-106)."""
    from .lib_path import make_point_lights
    rng = np.random.default_rng(seed)
    pos = rng.uniform(C4_BOX_MIN, C4_BOX_MAX, size=(n_lights, 3))
    return make_point_lights(pos, rng.uniform(2.0, 8.0, n_lights), rng.uniform(0.2, 1.0, (n_lights, 3)),
                             rng.uniform(0.5, 2.0, n_lights))


def c4_scene(width=3840, height=2160, n_objects=1000, tris_per_object=1000, n_draws=16, n_lights=256, mode=1,
             tile_size=16, max_per_tile=128, yaw=0.0):
    """-> (frame, draws, lights, cull).  Forward+ program (SHS_PROGRAM_FORWARD_PLUS), no culling."""
    from .lib_path import PROGRAM_FORWARD_PLUS, LightCull
    zn, zf = 0.1, 200.0
    meshes, colors = c4_geometry(n_objects, tris_per_object, n_draws)
    ang = np.deg2rad(yaw)
    eye = (f32(12.0 * np.sin(ang)), f32(8.0), f32(-12.0 * np.cos(ang)))
    view = look_at_lh(eye, (0.0, 4.0, 40.0))
    proj = perspective_lh_no(f32(np.deg2rad(60.0)), f32(width) / f32(height), zn, zf)
    vp = mat_mul(proj, view)
    draws = [LibDraw(mesh=m, program=PROGRAM_FORWARD_PLUS, viewproj=vp, camera_pos=eye, base_color=tuple(c),
                     cull_mode=CULL_NONE) for m, c in zip(meshes, colors)]
    frame = LibFrame(width, height, depth_motion=True, zn=zn, zf=zf, bg_gradient=True)
    cull = LightCull(width, height, view, proj, zn=zn, zf=zf, tile_size=tile_size, max_per_tile=max_per_tile, mode=mode)
    return frame, draws, c4_lights(n_lights), cull


# ---- software occlusion scene (hello_occlusion_culling_sw.cpp lineage) --------

def box_mesh(hx=0.5, hy=0.5, hz=0.5) -> LibMesh:
    """An indexed box (8 corners, 12 triangles), a DebugMesh like the Jolt box shape's."""
    p = np.array([[sx * hx, sy * hy, sz * hz] for sz in (-1, 1) for sy in (-1, 1) for sx in (-1, 1)], np.float32)
    q = [(0, 1, 3, 2), (4, 6, 7, 5), (0, 4, 5, 1), (2, 3, 7, 6), (0, 2, 6, 4), (1, 5, 7, 3)]
    idx = np.array([[a, b, c, a, c, d] for a, b, c, d in q], np.uint32).reshape(-1)
    return LibMesh(positions=p, indices=idx)


def sphere_mesh(r=0.5, seg=12, rings=8) -> LibMesh:
    v = []
    for i in range(rings + 1):
        th = np.pi * i / rings
        for j in range(seg):
            ph = 2.0 * np.pi * j / seg
            v.append((r * np.sin(th) * np.cos(ph), r * np.cos(th), r * np.sin(th) * np.sin(ph)))
    idx = []
    for i in range(rings):
        for j in range(seg):
            a, b = i * seg + j, i * seg + (j + 1) % seg
            c, d = a + seg, b + seg
            idx += [a, c, b, b, c, d]
    return LibMesh(positions=np.array(v, np.float32), indices=np.array(idx, np.uint32))


def world_aabb(mesh, model):
    m = np.asarray(model, np.float32).reshape(4, 4).T   # column-major storage -> row-major matrix
    p = np.c_[mesh.positions, np.ones(len(mesh.positions), np.float32)] @ m.T
    return p[:, :3].min(0).astype(np.float32), p[:, :3].max(0).astype(np.float32)


def occlusion_scene(n_objects=300, seed=7, width=300, height=225, walls=3):
    """-> (objects [(mesh, model, aabb_min, aabb_max)], view, view_proj, width, height).  Random boxes
    and spheres on a field, a few wide walls close to the camera occluding part of it, some objects
    behind the camera (their corners fail the clip.w test)."""
    rng = np.random.default_rng(seed)
    box, sph = box_mesh(), sphere_mesh()
    objs = []
    for i in range(n_objects):
        pos = (f32(rng.uniform(-30, 30)), f32(rng.uniform(0.0, 3.0)), f32(rng.uniform(-8, 70)))
        rot = tuple(f32(a) for a in rng.uniform(-np.pi, np.pi, 3))
        s = f32(rng.uniform(0.5, 3.0))
        model = model_euler(pos, rot, (s, s, s))
        mesh = box if i % 2 == 0 else sph
        mn, mx = world_aabb(mesh, model)
        objs.append((mesh, model, mn, mx))
    for w in range(walls):
        model = model_euler((f32(-12.0 + 12.0 * w), f32(2.0), f32(8.0 + 3.0 * w)), (0.0, 0.0, 0.0), (f32(7.0), f32(6.0), f32(0.5)))
        mn, mx = world_aabb(box, model)
        objs.append((box, model, mn, mx))
    view = look_at_lh((0.0, 3.0, -4.0), (0.0, 2.0, 30.0))
    proj = perspective_lh_no(f32(np.deg2rad(60.0)), f32(width) / f32(height), f32(0.1), f32(1000.0))
    return objs, view, mat_mul(proj, view), width, height
