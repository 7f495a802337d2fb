"""GPU test of the device-side tile-shard gather kernels (shs_tiles_pack / shs_tiles_unpack): one
process plays every rank with its own context; the packed device buffers match the host restatement
of the layout (shard.pack_padded) bit for bit, and unpacking the peers into rank 0 composes the
frame a single unsharded render produces."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _render_lib(ctx, frame, draws):
    ctx.render_pbr_forward(frame, draws)
    return ctx.resolve_lib()


@pytest.mark.parametrize("count", [3, 8])
def test_lib_shards_gather_on_device(count):
    import torch
    import shs_gpu
    from shs_gpu import scene_lib, shard
    frame, draws, _, _, _ = scene_lib.c5_scene(352, 200)
    full = shs_gpu.Context(0)
    fh, fd, fm = _render_lib(full, frame, draws)
    ctxs, bufs = [], []
    for r in range(count):
        c = shs_gpu.Context(0)
        frame.shard_rank, frame.shard_count = r, count
        h, d, m = _render_lib(c, frame, draws)
        words = c.tiles_packed_words(c.TARGET_LIB, count)
        buf = torch.zeros(words, dtype=torch.int32, device="cuda:0")
        c.tiles_pack(c.TARGET_LIB, r, count, buf.data_ptr())
        c.synchronize_lib()
        host = shard.pack_padded(shard.planes_of([(h, False), (d, False), (m, False)]), 352, 200, r, count)
        got = buf.cpu().numpy().view(np.uint32)
        assert np.array_equal(got[:host.size], host)
        ctxs.append(c)
        bufs.append(buf)
    root = ctxs[0]
    for r in range(1, count):
        root.tiles_unpack(root.TARGET_LIB, r, count, bufs[r].data_ptr())
    gh, gd, gm = root.resolve_lib()
    assert np.array_equal(gh.view(np.uint32), fh.view(np.uint32))
    assert np.array_equal(gd.view(np.uint32), fd.view(np.uint32))
    assert np.array_equal(gm.view(np.uint32), fm.view(np.uint32))
    for c in ctxs + [full]:
        c.close()


def test_legacy_shards_gather_on_device():
    import torch
    import shs_gpu
    from shs_gpu import scene
    count = 4
    frame, draws = scene.monkey_scene(640, 480, 3, cam_pos=(0.0, 5.0, -12.0))
    full = shs_gpu.Context(0)
    full.render(frame, draws)
    fc, fd = full.resolve()
    ctxs, bufs = [], []
    for r in range(count):
        c = shs_gpu.Context(0)
        c.render(shs_gpu.Frame(640, 480, shard_rank=r, shard_count=count), draws)
        c.resolve()
        buf = torch.zeros(c.tiles_packed_words(c.TARGET_LEGACY, count), dtype=torch.int32, device="cuda:0")
        c.tiles_pack(c.TARGET_LEGACY, r, count, buf.data_ptr())
        c.synchronize()
        ctxs.append(c)
        bufs.append(buf)
    for r in range(1, count):
        ctxs[0].tiles_unpack(ctxs[0].TARGET_LEGACY, r, count, bufs[r].data_ptr())
    gc, gd = ctxs[0].resolve()
    assert np.array_equal(gc, fc) and np.array_equal(gd.view(np.uint32), fd.view(np.uint32))
    for c in ctxs + [full]:
        c.close()
