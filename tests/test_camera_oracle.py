"""Camera and model matrices: the product's host helpers (shs_camera3d,
shs_model_trs, shs_mat4_mul in libshs_gpu, csrc/shs_glm.hpp) against the oracle's independent
restatement of Camera3D::update + glm::perspectiveLH + glm::lookAtLH (shs_renderer.hpp:1224-1236) and
MonkeyObject::get_world_matrix (blinn_phong_shading.cpp:122-128), bit for bit, over a yaw / pitch /
position sweep that includes every camera pose the GPU parity tests and the bench render.  Also
the GLM identities the reference relies on (orthonormal view basis, the 4/3 aspect, w = view z).
CPU only: host code on both sides."""
import itertools

import numpy as np
import pytest

from shs_gpu import scene

POSES = [(0.0, 0.0), (17.0, -9.0), (-33.0, 12.5), (3.0, 0.0), (-12.0, -3.0), (12.0, 3.0), (-20.0, -4.0),
         (90.0, 0.0), (-90.0, 45.0), (180.0, -89.0), (45.0, 89.0), (1e-3, -1e-3), (359.5, 30.0), (-137.25, -61.0)]
POSITIONS = [(0.0, 5.0, -20.0), (0.0, 5.0, -12.0), (0.0, 0.0, -5.0), (3.5, -2.25, 7.0), (-100.0, 40.0, 250.0)]


def _bits(a):
    return np.ascontiguousarray(a, dtype=np.float32).view(np.uint32)


@pytest.mark.parametrize("pos", POSITIONS)
def test_camera3d_matches_oracle_bitwise(oracle_mod, pos):
    for yaw, pitch in POSES:
        v1, p1 = scene.camera(pos, yaw, pitch)
        v2, p2 = oracle_mod.camera3d(pos, yaw, pitch)
        assert np.array_equal(_bits(v1), _bits(v2)), f"view differs at pos={pos} yaw={yaw} pitch={pitch}"
        assert np.array_equal(_bits(p1), _bits(p2)), f"proj differs at pos={pos} yaw={yaw} pitch={pitch}"


def test_camera_sweep_dense(oracle_mod):
    rng = np.random.default_rng(2024)
    for _ in range(400):
        pos = rng.uniform(-50, 50, size=3).astype(np.float32)
        yaw, pitch = float(rng.uniform(-360, 360)), float(rng.uniform(-89.9, 89.9))
        fov = float(rng.choice([45.0, 60.0, 75.0]))
        zn, zf = float(rng.choice([0.1, 0.5])), float(rng.choice([100.0, 1000.0]))
        v1, p1 = scene.camera(pos, yaw, pitch, fov=fov, zn=zn, zf=zf)
        v2, p2 = oracle_mod.camera3d(pos, yaw, pitch, fov, zn, zf)
        assert np.array_equal(_bits(v1), _bits(v2)) and np.array_equal(_bits(p1), _bits(p2))


def test_model_matrix_matches_oracle_bitwise(oracle_mod):
    rng = np.random.default_rng(7)
    cases = [((0.0, 0.0, 10.0), 0.0, (4.0, 4.0, 4.0))] + [
        ((i * 15.0 - 52.5, 0.0, j * 15.0 + 20.0), 0.0, (5.0, 5.0, 5.0)) for i, j in itertools.product(range(8), range(8))]
    for _ in range(100):
        cases.append((tuple(rng.uniform(-30, 30, 3)), float(rng.uniform(-720, 720)), tuple(rng.uniform(0.1, 9, 3))))
    for k in range(4):
        cases.append(((0.0, 0.0, 10.0), 23.0 * k, (4.0, 4.0, 4.0)))   # test_shading_models_camera_sweep rotations
    for pos, rot, scl in cases:
        a = scene.model_trs(pos, rot, scl)
        b = oracle_mod.model_trs(pos, rot, scl)
        assert np.array_equal(_bits(a), _bits(b)), f"model differs at {pos} {rot} {scl}"


@pytest.mark.parametrize("cfg", ["c1", "c2", "c3"])
def test_config_uniforms_from_oracle_matrices(oracle_mod, cfg):
    """Every draw of the BASELINE configs (and the bench's pose sweep) has the MVP / model the oracle's
    independent matrices give (mvp = (P * V) * M)."""
    for yaw, pitch in [(0.0, 0.0), (-12.0, -3.0), (11.5, 2.9)]:
        frame, draws = scene.config(cfg, yaw=yaw, pitch=pitch)
        view, proj = oracle_mod.camera3d(scene.CAM_POS, yaw, pitch)
        for d in draws:
            mvp, _ = oracle_mod.legacy_mvp(view, proj, d.model)
            assert np.array_equal(_bits(d.mvp), _bits(mvp))


def test_flat_pipeline_uniforms(oracle_mod):
    """Flat pipeline (flat_shading.cpp:284-285): mv = view * model, mvp = proj * mv."""
    from shs_gpu import SHADING_FLAT
    frame, draws = scene.monkey_scene(640, 480, SHADING_FLAT, yaw=17.0, pitch=-9.0, rotation=0.0)
    view, proj = oracle_mod.camera3d(scene.CAM_POS, 17.0, -9.0)
    model = oracle_mod.model_trs((0.0, 0.0, 10.0), 0.0, (4.0, 4.0, 4.0))
    mvp, mv = oracle_mod.legacy_mvp(view, proj, model, flat=True)
    assert np.array_equal(_bits(draws[0].mvp), _bits(mvp)) and np.array_equal(_bits(draws[0].model), _bits(mv))


def test_glm_identities(oracle_mod):
    """Properties of the restated GLM: the view's rotation rows are orthonormal (to float rounding),
    the projection hard-codes aspect 4/3 (shs_renderer.hpp:1234), clip w = view z (LH), and the camera
    looks along +z at yaw = pitch = 0 with no rotation."""
    view, proj = oracle_mod.camera3d((0.0, 5.0, -20.0), 0.0, 0.0)
    V = view.reshape(4, 4).T   # row-major
    assert np.array_equal(V[:3, :3], np.eye(3, dtype=np.float32))
    assert V[2, 3] == np.float32(20.0) and V[1, 3] == np.float32(-5.0)
    P = proj.reshape(4, 4).T
    assert P[3, 2] == 1.0 and P[3, 3] == 0.0
    assert P[1, 1] / P[0, 0] == pytest.approx(4.0 / 3.0, rel=1e-6)
    view, _ = oracle_mod.camera3d((1.0, 2.0, 3.0), 37.0, -21.0)
    R = view.reshape(4, 4).T[:3, :3].astype(np.float64)
    assert np.allclose(R @ R.T, np.eye(3), atol=1e-6)
    # perspectiveLH maps zn -> -1 and zf -> +1 in NDC
    p = oracle_mod.perspective_lh_no(np.float32(np.pi / 3), 4.0 / 3.0, 0.1, 1000.0).reshape(4, 4).T
    for z, want in [(0.1, -1.0), (1000.0, 1.0)]:
        c = p @ np.array([0, 0, z, 1], np.float32)
        assert c[2] / c[3] == pytest.approx(want, abs=1e-5)
