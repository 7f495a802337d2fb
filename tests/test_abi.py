"""CPU checks of the C-ABI boundary: the library loads, exports every symbol include/shs_gpu.h
declares, the ctypes layouts match the C structs, argument validation fails loudly, and the host
GLM helpers agree bit-for-bit with the oracle's independent restatement."""
import ctypes
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "shs_gpu.h")


def _declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\s*\*?\s*(shs_\w+)\s*\(", src, flags=re.M)))


def test_header_symbols_exported():
    import shs_gpu
    from shs_gpu import _abi
    lib = shs_gpu.lib()
    names = _declared_functions()
    assert len(names) >= 20
    bound = {n for n, _, _ in _abi.SIGNATURES}
    for n in names:
        assert hasattr(lib, n), f"{n} declared in shs_gpu.h but not exported"
        assert n in bound, f"{n} declared in shs_gpu.h but not bound in _abi.SIGNATURES"


def test_struct_layouts():
    from shs_gpu import _abi
    assert ctypes.sizeof(_abi.LegacyDraw) == 4 + 4 + 64 + 64 + 12 + 12 + 4
    assert ctypes.sizeof(_abi.FrameDesc) == 7 * 4 + 4
    assert ctypes.sizeof(_abi.RasterStats) == 9 * 8


def test_invalid_arguments_fail_loudly():
    import shs_gpu
    lib = shs_gpu.lib()
    assert lib.shs_destroy(None) == -1
    assert lib.shs_synchronize(None) == -1
    assert lib.shs_render_legacy(None, None, None, 0) == -1
    assert lib.shs_abi_version() == 1
    assert lib.shs_gpu_tile_size() in (8, 16, 32, 64)


def test_create_without_gpu_returns_no_device():
    """In this container there is no GPU: shs_create must return SHS_ERR_NO_DEVICE (never a CPU
    fallback context).  On a GPU box it succeeds."""
    import shs_gpu
    lib = shs_gpu.lib()
    h = ctypes.c_void_p()
    rc = lib.shs_create(0, ctypes.byref(h))
    if rc == 0:
        assert lib.shs_destroy(h) == 0
    else:
        assert rc == -3
        with pytest.raises(shs_gpu.ShsError):
            shs_gpu.Context(0)


def test_host_glm_matches_oracle_restatement(oracle_mod):
    """shs_mat4_mul / shs_mat4_inverse (product host code) vs ora_mat4_mul / ora_mat4_inverse
    (oracle): two independent restatements of GLM's operation order, bit-exact."""
    import shs_gpu
    lib = shs_gpu.lib()
    rng = np.random.default_rng(3)
    fp = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))
    for _ in range(200):
        a = rng.normal(size=16).astype(np.float32)
        b = rng.normal(size=16).astype(np.float32)
        o1 = np.zeros(16, np.float32)
        o2 = np.zeros(16, np.float32)
        assert lib.shs_mat4_mul(fp(a), fp(b), fp(o1)) == 0
        oracle_mod.lib().ora_mat4_mul(a.ctypes.data, b.ctypes.data, o2.ctypes.data)
        assert np.array_equal(o1.view(np.uint32), o2.view(np.uint32))
        assert lib.shs_mat4_inverse(fp(a), fp(o1)) == 0
        oracle_mod.lib().ora_mat4_inverse(a.ctypes.data, o2.ctypes.data)
        assert np.array_equal(o1.view(np.uint32), o2.view(np.uint32))


def test_camera3d_reference_viewer():
    """Viewer((0,5,-20)): yaw = pitch = 0 looks down +z; lookAtLH gives an axis-aligned view with
    translation (0,-5,20); perspectiveLH_NO(60 deg, 4/3 (sic), 0.1, 1000)."""
    from shs_gpu import scene
    view, proj = scene.camera((0.0, 5.0, -20.0), 0.0, 0.0)
    V = view.reshape(4, 4)  # V[c][r]
    assert np.array_equal(V[:3, :3], np.eye(3, dtype=np.float32))
    assert V[3, 0] == 0.0 and V[3, 1] == -5.0 and V[3, 2] == 20.0
    P = proj.reshape(4, 4)
    t = np.float32(np.tan(np.float32(np.float32(60.0) * np.float32(0.01745329251994329576923690768489)) / np.float32(2)))
    assert P[2, 3] == 1.0 and P[3, 3] == 0.0
    assert P[1, 1] == np.float32(1.0) / t
    assert P[0, 0] == np.float32(1.0) / (np.float32(4.0 / 3.0) * t)


def test_model_trs_reference_monkey():
    """MonkeyObject::get_world_matrix, position (0,0,10), rotation 0, scale 4: T*R*S."""
    from shs_gpu import scene
    m = scene.model_trs((0.0, 0.0, 10.0), 0.0, (4.0, 4.0, 4.0)).reshape(4, 4)
    expect = np.diag([4.0, 4.0, 4.0, 1.0]).astype(np.float32)
    expect[3, 2] = 10.0
    assert np.array_equal(m, expect)


def test_submodules_do_not_shadow_lib():
    """Importing the scene / library-path helpers keeps shs_gpu.lib the loader function."""
    import shs_gpu
    from shs_gpu import lib_path, scene, scene_lib  # noqa: F401
    assert callable(shs_gpu.lib) and shs_gpu.lib().shs_abi_version() == 1
