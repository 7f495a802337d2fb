"""Software occlusion pass: shs_occlusion_pass against the oracle restatement
of culling_sw::run_software_occlusion_pass (geometry/culling_software.hpp:229-331), bit-exact: the
same occluded flags, the same visible list in visit order and the same occlusion depth buffer."""
import numpy as np
import pytest


def _scene(**kw):
    from shs_gpu import scene_lib
    return scene_lib.occlusion_scene(**kw)


def test_oracle_occlusion_scene_properties(oracle_mod):
    """The committed scene exercises both outcomes; with the pass disabled everything frustum-visible
    stays visible in input order; the occluded flags partition the frustum-visible set."""
    objs, view, vp, W, H = _scene()
    fv = np.arange(len(objs), dtype=np.uint32)[::-1].copy()
    occ, vis, depth = oracle_mod.occlusion_pass(W, H, view, vp, objs, fv)
    assert 0 < occ.sum() < len(objs)
    assert sorted(vis.tolist() + np.nonzero(occ)[0].tolist()) == list(range(len(objs)))
    assert depth.min() >= 0.0 and depth.max() <= 1.0 and (depth < 1.0).any()
    occ0, vis0, _ = oracle_mod.occlusion_pass(W, H, view, vp, objs, fv, enable=False)
    assert occ0.sum() == 0 and np.array_equal(vis0, fv)


@pytest.mark.gpu
@pytest.mark.parametrize("seed,n,eps", [(7, 300, 1e-4), (11, 600, 1e-4), (3, 120, 0.0), (5, 300, 0.01)])
def test_occlusion_pass_exact(oracle_mod, seed, n, eps):
    import shs_gpu
    objs, view, vp, W, H = _scene(n_objects=n, seed=seed)
    rng = np.random.default_rng(seed)
    fv = rng.permutation(len(objs))[: len(objs) - 7].astype(np.uint32)   # a frustum-visible subset
    fv = np.r_[fv, np.uint32(len(objs) + 5)]                               # out of range: dropped
    want = oracle_mod.occlusion_pass(W, H, view, vp, objs, fv, depth_epsilon=eps)
    with shs_gpu.Context(0) as ctx:
        got = ctx.occlusion_pass(W, H, view, vp, objs, fv, depth_epsilon=eps)
    assert np.array_equal(got[0], want[0]), f"occluded flags differ at {np.nonzero(got[0] != want[0])[0][:8]}"
    assert np.array_equal(got[1], want[1])
    assert np.array_equal(got[2].view(np.uint32), want[2].view(np.uint32))
    if eps <= 1e-4:   # a coarse epsilon keeps every object visible (z_near <= depth + eps everywhere)
        assert 0 < want[0].sum() < len(objs)


@pytest.mark.gpu
def test_occlusion_pass_large_buffer_and_disabled(oracle_mod):
    """A 4x larger buffer (1200x900, beyond the reference demo's 300x225), enable = 0, a side over 65535."""
    import shs_gpu
    objs, view, vp, _, _ = _scene(n_objects=200, seed=19, width=1200, height=900)
    fv = np.arange(len(objs), dtype=np.uint32)
    want = oracle_mod.occlusion_pass(1200, 900, view, vp, objs, fv)
    with shs_gpu.Context(0) as ctx:
        got = ctx.occlusion_pass(1200, 900, view, vp, objs, fv)
        off = ctx.occlusion_pass(1200, 900, view, vp, objs, fv, enable=False)
    assert np.array_equal(got[0], want[0]) and np.array_equal(got[1], want[1])
    assert np.array_equal(got[2].view(np.uint32), want[2].view(np.uint32))
    assert off[0].sum() == 0 and np.array_equal(off[1], fv)
    with shs_gpu.Context(0) as ctx, pytest.raises(shs_gpu.ShsError):
        ctx.occlusion_pass(65536, 2, view, vp, objs, fv)   # sides are limited to 16 bits


@pytest.mark.gpu
def test_occlusion_pass_resize_sequence(oracle_mod):
    """One context through buffer sizes down to 1x1 and a single column (the depth buffer and the
    per-object work are sized per call)."""
    import shs_gpu
    with shs_gpu.Context(0) as ctx:
        for seed, (W, H) in enumerate([(300, 225), (300, 200), (64, 48), (1, 1), (7, 300), (300, 225)]):
            objs, view, vp, _, _ = _scene(n_objects=150, seed=30 + seed, width=W, height=H)
            fv = np.arange(len(objs), dtype=np.uint32)
            want = oracle_mod.occlusion_pass(W, H, view, vp, objs, fv)
            got = ctx.occlusion_pass(W, H, view, vp, objs, fv)
            assert np.array_equal(got[0], want[0]) and np.array_equal(got[1], want[1]), (W, H)
            assert np.array_equal(got[2].view(np.uint32), want[2].view(np.uint32)), (W, H)
