"""Capacity overflows never reach an asynchronous consumer.

A legacy batch whose bin-spill or ghost-fragment list overflowed is incomplete until it is re-issued
with grown lists.  shs_present_device finishes the batch before it hands out the staging pointer, so a
D2H copy queued on the context stream behind it reads the final frame; a batch superseded by the next
render call has its overflow word read first (re-issued if set).  The lists are shrunk to a few
entries (SHS_OPT_SPILL_CAPACITY / SHS_OPT_FRAG_CAPACITY) so both overflow in the first pass."""
import ctypes

import numpy as np
import pytest

from helpers import assert_color_parity, assert_depth_bitexact
from test_gpu_parity import _hair_soup, _identity_draw

pytestmark = pytest.mark.gpu

W, H = 400, 300


def _frames(seeds, n=3000):
    from shs_gpu.scene import Mesh
    fds = []
    for seed in seeds:
        rng = np.random.default_rng(seed)
        pos, nrm = _hair_soup(rng, W, H, n)
        fds.append([_identity_draw(Mesh(pos, nrm), seed % 4)])
    return fds


def _hip():
    import torch  # noqa: F401  (maps torch's HIP runtime, the one libshs_gpu binds)
    hip = ctypes.CDLL("libamdhip64.so.7")
    hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
    return hip


def _check_frames(oracle_mod, fds, pres, pqs):
    for k, draws in enumerate(fds):
        rc, rd, rpq = oracle_mod.render_legacy(W, H, draws, threads=8, prequant=True)
        got = pres[k]
        assert_color_parity(got, oracle_mod.sdl_present(rc), pqs[k][::-1], rpq[::-1])


@pytest.mark.parametrize("mode", [1, 2], ids=["scan", "bins"])
def test_overflowed_batch_through_present_device_async_copy(oracle_mod, mode):
    import torch
    import shs_gpu
    hip = _hip()
    fds = _frames([301, 302, 303])
    frame = shs_gpu.Frame(W, H, present=True, prequant=True)
    ctx = shs_gpu.Context(0)
    try:
        ctx.set_raster_mode(mode)
        ctx.set_bin_capacity(1)
        ctx.set_overflow_capacities(spill=8, frags=8)
        ctx.render_batch(frame, fds)
        host = torch.empty((len(fds), H, W, 4), dtype=torch.uint8, pin_memory=True)
        for k in range(len(fds)):
            ptr = ctx.present_device(k)     # finishes the batch: the overflowed lists grow, the batch re-runs
            rc = hip.hipMemcpyAsync(ctypes.c_void_p(host[k].data_ptr()), ctypes.c_void_p(ptr), W * H * 4, 2,
                                    ctypes.c_void_p(ctx.stream))
            assert rc == 0
        ctx.synchronize()
        st = ctx.stats()
        # the first pass overflowed: more ghost fragments than the 8-entry list held and, in bin mode,
        # more bin entries than one per 32x32 tile plus an 8-entry spill list (the statistics are the
        # re-issued pass's, whose bin capacity already grew to the fullest tile: nothing spills there)
        assert st["ghost_fragments"] > 8, st
        if mode == 2:
            assert st["bin_entries"] > 3 * ((W + 31) // 32) * ((H + 31) // 32) + 8, st
        pqs = [ctx.resolve_prequant(k) for k in range(len(fds))]
        _check_frames(oracle_mod, fds, host.numpy(), pqs)
    finally:
        ctx.close()


def test_superseded_overflowed_batch_is_finished_first(oracle_mod):
    """Batch A overflows; its staging is handed to an async copy; batch B is enqueued right after
    without a sync (A is superseded).  The copy of A is A's final frame, and B is exact too."""
    import torch
    import shs_gpu
    hip = _hip()
    fa, fb = _frames([311, 312]), _frames([313, 314])
    frame = shs_gpu.Frame(W, H, present=True, prequant=True)
    ctx = shs_gpu.Context(0)
    try:
        ctx.set_raster_mode(2)
        ctx.set_bin_capacity(1)
        ctx.set_overflow_capacities(spill=8, frags=8)
        ctx.render_batch(frame, fa)
        host = torch.empty((len(fa), H, W, 4), dtype=torch.uint8, pin_memory=True)
        for k in range(len(fa)):
            assert hip.hipMemcpyAsync(ctypes.c_void_p(host[k].data_ptr()), ctypes.c_void_p(ctx.present_device(k)),
                                      W * H * 4, 2, ctypes.c_void_p(ctx.stream)) == 0
        ctx.set_bin_capacity(1)             # B starts from a one-entry bin capacity again ...
        ctx.set_overflow_capacities(spill=8, frags=8)   # ... and tiny lists: it overflows as well
        ctx.render_batch(frame, fb)
        ctx.render_batch(frame, fa)         # supersedes B (overflowed, unchecked): B is finished first
        ctx.synchronize()
        torch.cuda.synchronize()
        a_pqs = [ctx.resolve_prequant(k) for k in range(len(fa))]
        _check_frames(oracle_mod, fa, host.numpy(), a_pqs)
        for k, draws in enumerate(fa):
            c, z = ctx.resolve_frame(k)
            rc, rd, rpq = oracle_mod.render_legacy(W, H, draws, threads=8, prequant=True)
            assert_depth_bitexact(z, rd)
            assert_color_parity(c, rc, a_pqs[k], rpq)
    finally:
        ctx.close()
