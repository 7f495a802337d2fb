"""shs_mesh_share: frames in flight on several contexts read one device copy of each mesh.  A context
that borrows another's meshes renders bit for bit what the owner renders (the same buffers and the same
arithmetic), and releasing or destroying the borrower frees nothing of the owner's."""
import numpy as np
import pytest


def _frame(ctx, frame, draws, lights, cull):
    ctx.upload_lights(lights)
    ctx.light_cull(cull)
    ctx.render_pbr_forward(frame, draws)
    return ctx.resolve_lib()


@pytest.mark.gpu
def test_shared_meshes_render_identically():
    import shs_gpu
    from shs_gpu import scene_lib
    frame, draws, lights, cull = scene_lib.c4_scene(320, 192, n_objects=24, tris_per_object=300, n_draws=4,
                                                    n_lights=16)
    owner, borrower = shs_gpu.Context(0), shs_gpu.Context(0)
    try:
        ids = [borrower.share_lib_mesh(owner, d.mesh) for d in draws]
        assert len(set(ids)) == len(draws)
        ref = _frame(owner, frame, draws, lights, cull)
        got = _frame(borrower, frame, draws, lights, cull)
        for a, b in zip(ref, got):
            np.testing.assert_array_equal(np.asarray(a).view(np.uint32), np.asarray(b).view(np.uint32))
        # the borrower lets go of its handles; the owner still renders from its buffers
        for i in ids:
            borrower._check(borrower._lib.shs_mesh_release(borrower._h, i))
        borrower.close()
        again = _frame(owner, frame, draws, lights, cull)
        for a, b in zip(ref, again):
            np.testing.assert_array_equal(np.asarray(a).view(np.uint32), np.asarray(b).view(np.uint32))
    finally:
        borrower.close()
        owner.close()


@pytest.mark.gpu
def test_share_rejects_bad_handles():
    import ctypes
    import shs_gpu
    a, b = shs_gpu.Context(0), shs_gpu.Context(0)
    try:
        mid = ctypes.c_int32()
        assert a._lib.shs_mesh_share(b._h, a._h, 7, ctypes.byref(mid)) != 0        # no such mesh
        assert a._lib.shs_mesh_share(a._h, a._h, 0, ctypes.byref(mid)) != 0        # a context with itself
    finally:
        b.close()
        a.close()
