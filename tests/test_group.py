"""shs_group (one host process, N contexts, peer-copy gather) from the Python host mirror: the C4 /
C5 frames rendered as N tile shards and gathered on rank 0 equal the unsharded frame bit for bit, for
the library targets (HDR + depth + motion, fused-tonemap present staging) and Forward+ light lists."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n", [2, 5, 8])
def test_group_c5_composes(n):
    import shs_gpu
    from shs_gpu import scene_lib
    from shs_gpu.group import Group
    frame, draws, casters, sun, S = scene_lib.c5_scene(640, 360, 512, textured=True)
    single = shs_gpu.Context(0)
    g = Group([0] * n)
    try:
        lvp = single.render_shadow_map(S, sun, casters)
        lvp_g = g.render_shadow_map(S, sun, casters)
        assert np.array_equal(lvp.view(np.uint32), lvp_g.view(np.uint32))
        scene_lib.wire_shadow(draws, lvp)
        single.render_pbr_forward(frame, draws)
        want = single.resolve_lib()
        g.render_pbr_forward(frame, draws)
        g.gather(single.TARGET_LIB)
        got = g.root.resolve_lib()
        for a, b in zip(got, want):
            assert np.array_equal(a.view(np.uint32), b.view(np.uint32))
    finally:
        g.close()
        single.close()


@pytest.mark.parametrize("n", [3, 8])
def test_group_c4_forward_plus_present(n):
    import shs_gpu
    from shs_gpu import scene_lib
    from shs_gpu.group import Group
    frame, draws, lights, cull = scene_lib.c4_scene(960, 540, n_objects=60, tris_per_object=500)
    single = shs_gpu.Context(0)
    g = Group([0] * n)
    try:
        single.upload_lights(lights)
        single.light_cull(cull)
        single.fuse_tonemap(1.0, 2.2, ldr=False, present=True)
        single.render_pbr_forward(frame, draws)
        _, want = single.resolve_ldr()
        g.upload_lights(lights)
        g.fuse_tonemap(1.0, 2.2, ldr=False, present=True)
        for _ in range(3):   # back to back: the gathers' receive buffers alternate
            g.light_cull(cull)
            g.render_pbr_forward(frame, draws)
            g.gather(single.TARGET_LIB_PRESENT)
        _, got = g.root.resolve_ldr()
        assert np.array_equal(got, want)
    finally:
        g.close()
        single.close()


def test_group_legacy_present():
    import shs_gpu
    from shs_gpu import scene
    from shs_gpu.group import Group
    frame, draws = scene.monkey_scene(1920, 1080, 3)
    frame.present = True
    single = shs_gpu.Context(0)
    g = Group([0, 0, 0, 0])
    try:
        single.render(frame, draws)
        want = single.resolve_present(0)
        g.render(frame, draws)
        g.gather(single.TARGET_PRESENT)
        assert np.array_equal(g.root.resolve_present(0), want)
    finally:
        g.close()
        single.close()
