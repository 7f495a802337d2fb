"""PassTonemap + present staging: shs_tonemap against the oracle restatement of
pass_tonemap.hpp:36-83 and hello_pass_basics.cpp:102-119 (oracle/shs_oracle_post.c).

CPU: the library's host-side byte thresholds reproduce the reference expression (glibc powf / lround)
on dense float samples around every threshold, with the kernel's decision (count of thresholds <= x)
emulated in numpy.  GPU: bit-exact LDR and present bytes for rendered and synthetic HDR targets."""
import numpy as np
import pytest


def _x_of(s, exposure):
    """The kernel's x = c / (1 + c), c = std::max(0, s * exposure), in float32."""
    e = np.float32(s) * np.float32(exposure)
    c = np.where(np.float32(0) < e, e, np.float32(0)).astype(np.float32)
    with np.errstate(invalid="ignore", over="ignore"):
        return (c / (np.float32(1) + c)).astype(np.float32)


def _emulate(s, exposure, thr):
    x = _x_of(s, exposure)
    out = np.zeros(x.shape, np.int64)
    ok = x >= 0   # NaN -> 0
    out[ok] = np.searchsorted(thr[1:], x[ok], side="right")
    return out


@pytest.mark.parametrize("gamma", [2.2, 1.0, 1.8, 0.5, 0.0, -1.0])
def test_thresholds_match_reference_bytes(oracle_mod, gamma):
    import shs_gpu
    thr = shs_gpu.Context.tonemap_thresholds(gamma)
    assert np.all(np.diff(thr[1:]) >= 0)
    inv_gamma = np.float32(1.0) / np.float32(max(0.001, gamma))
    # s values whose x lands within +-40 ulps of each finite threshold, plus a uniform sweep
    samples = [np.linspace(-1.0, 50.0, 4001, dtype=np.float32)]
    for t in thr[1:]:
        if not np.isfinite(t) or t <= 0 or t >= 1:
            continue
        s0 = np.float32(t / (1.0 - t))
        samples.append(s0 + np.arange(-40, 41, dtype=np.float32) * np.spacing(s0))
    s = np.concatenate(samples).astype(np.float32)
    want = np.array([oracle_mod.tonemap_channel(v, 1.0, inv_gamma) for v in s])
    got = _emulate(s, 1.0, thr)
    bad = np.nonzero(want != got)[0]
    assert bad.size == 0, f"{bad.size} mismatches, e.g. s={s[bad[:5]]} want={want[bad[:5]]} got={got[bad[:5]]}"


def test_oracle_edge_values(oracle_mod):
    """NaN and negative inputs give 0; +inf gives 0 (inf / inf = NaN, lround(NaN) casts to 0 on x86-64);
    a huge finite value gives 255; alpha is 255; present is the y-flip of ldr."""
    hdr = np.array([[[np.nan, -1.0, 1e30, 1.0], [np.inf, 0.0, 1.0, 0.5]],
                    [[0.25, 0.5, 4.0, 1.0], [-np.inf, 1e-30, 2.0, 1.0]]], np.float32)
    ldr, pre = oracle_mod.tonemap(hdr, 1.0, 2.2)
    assert ldr[0, 0, 0] == 0 and ldr[0, 0, 1] == 0 and ldr[0, 0, 2] == 255 and ldr[0, 1, 0] == 0
    assert np.all(ldr[..., 3] == 255)
    assert np.array_equal(pre, ldr[::-1])


# ---- GPU ------------------------------------------------------------------------------------------

def _c5(W, H):
    from shs_gpu import scene_lib
    frame, draws, casters, sun, S = scene_lib.c5_scene(W, H)
    return frame, draws


@pytest.mark.gpu
@pytest.mark.parametrize("exposure,gamma", [(1.0, 2.2), (2.5, 2.2), (0.7, 1.0), (1.0, 1.6), (1.0, -1.0), (3.0, 0.0)])
def test_tonemap_rendered_frame_exact(oracle_mod, exposure, gamma):
    import shs_gpu
    frame, draws = _c5(352, 200)
    with shs_gpu.Context(0) as ctx:
        ctx.render_pbr_forward(frame, draws)
        ctx.tonemap(exposure, gamma)
        ldr, pre = ctx.resolve_ldr()
        hdr, _, _ = ctx.resolve_lib()
    want_ldr, want_pre = oracle_mod.tonemap(hdr, exposure, gamma)
    assert np.array_equal(ldr, want_ldr)
    assert np.array_equal(pre, want_pre)


@pytest.mark.gpu
def test_tonemap_synthetic_hdr_exact(oracle_mod):
    """Every byte boundary, NaN / inf / negative / denormal / huge inputs, written straight into the
    device HDR target."""
    import torch
    import shs_gpu
    W, H = 256, 64
    frame, draws = _c5(W, H)
    thr = shs_gpu.Context.tonemap_thresholds(2.2)
    vals = []
    for t in thr[1:]:
        if np.isfinite(t) and 0 < t < 1:
            s0 = np.float32(t / (1.0 - t))
            vals += list(s0 + np.arange(-6, 7, dtype=np.float32) * np.spacing(s0))
    vals += [np.nan, np.inf, -np.inf, -0.0, 0.0, 1e-45, 1e-38, 3e38, -5.0, 1e6]
    rng = np.random.default_rng(3)
    flat = np.array(vals, np.float32)
    hdr = rng.uniform(-0.5, 8.0, size=(H, W, 4)).astype(np.float32)
    n = min(flat.size, H * W * 3)
    rgb = hdr[..., :3].reshape(-1).copy()
    rgb[:n] = flat[:n]
    hdr[..., :3] = rgb.reshape(H, W, 3)
    hdr[..., 3] = 1.0
    assert np.isnan(hdr).any() and np.isinf(hdr).any()
    with shs_gpu.Context(0) as ctx:
        ctx.render_pbr_forward(frame, draws)
        ctx.synchronize_lib()
        dev = ctx.lib_device_targets()[0]
        src = torch.from_numpy(hdr.reshape(-1)).to("cuda:0")
        torch.cuda.synchronize()
        _memcpy_d2d(dev, src.data_ptr(), hdr.nbytes)
        ctx.tonemap(1.0, 2.2)
        ldr, pre = ctx.resolve_ldr()
    want_ldr, want_pre = oracle_mod.tonemap(hdr, 1.0, 2.2)
    bad = np.argwhere(ldr != want_ldr)
    assert bad.size == 0, f"{len(bad)} mismatches, first {bad[:4]}"
    assert np.array_equal(pre, want_pre)


def _memcpy_d2d(dst, src, nbytes):
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so.7")   # by SONAME: the runtime already mapped (shs_gpu._abi.load)
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    rc = hip.hipMemcpy(ctypes.c_void_p(dst), ctypes.c_void_p(src), nbytes, 3)   # hipMemcpyDeviceToDevice
    assert rc == 0, rc


@pytest.mark.gpu
def test_tonemap_follows_new_pass_and_validates(oracle_mod):
    import shs_gpu
    from shs_gpu import ShsError
    frame, draws = _c5(160, 96)
    with shs_gpu.Context(0) as ctx:
        with pytest.raises(ShsError):
            ctx.tonemap()                     # no camera pass yet
        ctx.render_pbr_forward(frame, draws)
        with pytest.raises(ShsError):
            ctx.resolve_ldr()                 # no tonemap since the pass
        with pytest.raises(ShsError):
            ctx.tonemap(ldr=False, present=False)
        ctx.tonemap(ldr=False, present=True)
        ldr, pre = ctx.resolve_ldr()
        assert ldr is None and pre is not None
        hdr, _, _ = ctx.resolve_lib()
        _, want_pre = oracle_mod.tonemap(hdr, 1.0, 2.2)
        assert np.array_equal(pre, want_pre)


@pytest.mark.gpu
def test_post_chain_resize_sequence(oracle_mod):
    """One context through frame sizes down to 1x1 and single rows / columns: the fused tonemap, the
    PassTonemap and PassMotionBlur after it (each sized and cached per frame) vs the oracle."""
    import shs_gpu
    with shs_gpu.Context(0) as ctx:
        for i, (W, H) in enumerate([(96, 64), (96, 56), (1, 1), (37, 1), (1, 29), (17, 9), (96, 64)]):
            frame, draws = _c5(W, H)
            fused = i % 2 == 0
            ctx.fuse_tonemap(1.3, 2.2, ldr=True, present=True, enable=fused)
            ctx.render_pbr_forward(frame, draws)
            if not fused:
                ctx.tonemap(1.3, 2.2, ldr=True, present=True)
            ldr, pre = ctx.resolve_ldr()
            hdr, depth, motion = ctx.resolve_lib()
            want_ldr, want_pre = oracle_mod.tonemap(hdr, 1.3, 2.2)
            assert np.array_equal(ldr, want_ldr), (W, H, fused)
            assert np.array_equal(pre, want_pre), (W, H, fused)
            ctx.motion_blur(min_velocity_px=0.0)
            got, _ = ctx.resolve_motion_blur()
            want = oracle_mod.motion_blur(ldr, depth, motion, min_velocity_px=0.0)
            assert np.array_equal(got, want), (W, H)
        ctx.fuse_tonemap(enable=False)


# ---- PassMotionBlur ------------------------------------------------------------

def test_oracle_motion_blur_identities(oracle_mod):
    """No motion (below min_velocity) or enable = 0 leaves the image unchanged; a uniform image with
    equal depths stays uniform whatever the motion (every tap is accepted)."""
    rng = np.random.default_rng(5)
    H, W = 24, 40
    src = rng.integers(0, 256, size=(H, W, 4), dtype=np.uint8)
    src[..., 3] = 255
    depth = rng.uniform(0.2, 0.9, size=(H, W)).astype(np.float32)
    zero = np.zeros((H, W, 2), np.float32)
    assert np.array_equal(oracle_mod.motion_blur(src, depth, zero), src)
    mot = rng.uniform(-30, 30, size=(H, W, 2)).astype(np.float32)
    assert np.array_equal(oracle_mod.motion_blur(src, depth, mot, enable=False), src)
    flat = np.full_like(src, 77)
    flat[..., 3] = 255
    out = oracle_mod.motion_blur(flat, np.full((H, W), 0.5, np.float32), mot)
    assert np.array_equal(out, flat)


MB_CASES = [dict(), dict(samples=4), dict(samples=32, strength=2.5), dict(dt=1.0 / 30.0, min_velocity_px=0.0),
            dict(depth_reject=0.002, max_velocity_px=6.0), dict(enable=False), dict(samples=100, strength=-1.0)]


@pytest.mark.gpu
@pytest.mark.parametrize("case", range(len(MB_CASES)))
def test_motion_blur_exact(oracle_mod, case):
    import shs_gpu
    params = MB_CASES[case]
    frame, draws = _c5(352, 200)
    with shs_gpu.Context(0) as ctx:
        ctx.render_pbr_forward(frame, draws)
        ctx.tonemap(1.0, 2.2, ldr=True, present=False)
        ctx.motion_blur(**params)
        got, pre = ctx.resolve_motion_blur()
        ldr, _ = ctx.resolve_ldr()
        _, depth, motion = ctx.resolve_lib()
    assert np.abs(motion).max() > 1.0, "scene has no motion to blur"
    want = oracle_mod.motion_blur(ldr, depth, motion, **params)
    bad = np.argwhere(got != want)
    assert bad.size == 0, f"{len(bad)} byte mismatches, first {bad[:4]}"
    assert np.array_equal(pre, want[::-1])
    if params.get("enable", True) and params.get("strength", 1.0) > 0:
        assert not np.array_equal(got, ldr), "blur changed nothing"


@pytest.mark.gpu
def test_motion_blur_requires_inputs():
    import shs_gpu
    from shs_gpu import ShsError
    frame, draws = _c5(96, 64)
    with shs_gpu.Context(0) as ctx:
        ctx.render_pbr_forward(frame, draws)
        with pytest.raises(ShsError):
            ctx.motion_blur()                         # no tonemap yet
        ctx.tonemap(ldr=False, present=True)
        with pytest.raises(ShsError):
            ctx.motion_blur()                         # the tonemap wrote no RT_ColorLDR


@pytest.mark.gpu
def test_motion_blur_nonfinite_motion_exact(oracle_mod):
    """NaN / +-inf / huge motion vectors: the taps' lround of a NaN coordinate is x86-64's
    LONG_MIN cast to int (0), restated explicitly in the kernel."""
    import torch
    import shs_gpu
    frame, draws = _c5(160, 96)
    H, W = frame.height, frame.width
    rng = np.random.default_rng(11)
    mot = rng.uniform(-40, 40, size=(H, W, 2)).astype(np.float32)
    special = np.array([np.nan, np.inf, -np.inf, 3e38, -3e38, 1e20, np.nan, 0.0], np.float32)
    sel = rng.integers(0, special.size, size=(H, W, 2))
    mask = rng.random((H, W, 2)) < 0.3
    mot[mask] = special[sel[mask]]
    with shs_gpu.Context(0) as ctx:
        ctx.render_pbr_forward(frame, draws)
        ctx.synchronize_lib()
        dev_motion = ctx.lib_device_targets()[2]
        src = torch.from_numpy(mot.reshape(-1)).to("cuda:0")
        torch.cuda.synchronize()
        _memcpy_d2d(dev_motion, src.data_ptr(), mot.nbytes)
        ctx.tonemap(1.0, 2.2, ldr=True, present=False)
        ctx.motion_blur(min_velocity_px=0.0)
        got, _ = ctx.resolve_motion_blur()
        ldr, _ = ctx.resolve_ldr()
        _, depth, motion = ctx.resolve_lib()
    assert np.array_equal(motion.view(np.uint32), mot.view(np.uint32)), "injected motion was overwritten"
    want = oracle_mod.motion_blur(ldr, depth, motion, min_velocity_px=0.0)
    bad = np.argwhere(got != want)
    assert bad.size == 0, f"{len(bad)} byte mismatches, first {bad[:4]}"


# ---- fused PassTonemap (shs_lib_fuse_tonemap: the camera pass's shading kernel writes the bytes) ----

@pytest.mark.gpu
@pytest.mark.parametrize("exposure,gamma,ldr,present", [(1.0, 2.2, True, True), (2.5, 2.2, False, True),
                                                        (0.7, 1.0, True, False), (3.0, 0.0, True, True)])
def test_fused_tonemap_matches_pass(oracle_mod, exposure, gamma, ldr, present):
    """The fused bytes equal the oracle's PassTonemap of the same pass's HDR target, and a following
    frame without fusion needs shs_tonemap again."""
    import shs_gpu
    from shs_gpu import ShsError
    frame, draws = _c5(352, 200)
    with shs_gpu.Context(0) as ctx:
        ctx.fuse_tonemap(exposure, gamma, ldr=ldr, present=present)
        ctx.render_pbr_forward(frame, draws)
        got_ldr, got_pre = ctx.resolve_ldr()
        hdr, _, _ = ctx.resolve_lib()
        want_ldr, want_pre = oracle_mod.tonemap(hdr, exposure, gamma)
        if ldr:
            assert np.array_equal(got_ldr, want_ldr)
        else:
            assert got_ldr is None
        if present:
            assert np.array_equal(got_pre, want_pre)
        else:
            assert got_pre is None
        ctx.fuse_tonemap(enable=False)
        ctx.render_pbr_forward(frame, draws)
        with pytest.raises(ShsError):
            ctx.resolve_ldr()


@pytest.mark.gpu
def test_fused_tonemap_forward_plus_sharded(oracle_mod):
    """Forward+ (the C4 program) with the fused tonemap: the whole frame's present bytes, and each
    rank's tiles of a 3-way tile-sharded pass, equal the separate tonemap's."""
    import shs_gpu
    from shs_gpu import scene_lib
    frame, draws, lights, cull = scene_lib.c4_scene(640, 352, n_objects=60, tris_per_object=200)
    with shs_gpu.Context(0) as ctx:
        ctx.upload_lights(lights)
        ctx.light_cull(cull)
        ctx.render_pbr_forward(frame, draws)
        ctx.tonemap(1.0, 2.2, ldr=True, present=True)
        want_ldr, want_pre = ctx.resolve_ldr()
        ctx.fuse_tonemap(1.0, 2.2, ldr=True, present=True)
        ctx.render_pbr_forward(frame, draws)
        got_ldr, got_pre = ctx.resolve_ldr()
        assert np.array_equal(got_ldr, want_ldr) and np.array_equal(got_pre, want_pre)
        H, W = frame.height, frame.width
        ty, tx = np.mgrid[0:H, 0:W]
        tile = (ty // 32) * ((W + 31) // 32) + tx // 32          # rows y up (RT_ColorLDR)
        for r in range(3):
            frame.shard_rank, frame.shard_count = r, 3
            cull.shard_rank, cull.shard_count = r, 3
            ctx.light_cull(cull)
            ctx.render_pbr_forward(frame, draws)
            sl, _ = ctx.resolve_ldr()
            own = tile % 3 == r
            assert np.array_equal(sl[own], want_ldr[own]), f"rank {r}"
