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


@pytest.mark.parametrize("W,H,count", [(352, 200, 3), (352, 200, 8), (70, 40, 5), (33, 17, 3), (1, 1, 2)])
def test_lib_shards_gather_on_device(W, H, count):
    """Also frames with fewer 32x32 tiles than ranks (ranks owning no tile pack nothing)."""
    import torch
    import shs_gpu
    from shs_gpu import scene_lib, shard
    frame, draws, _, _, _ = scene_lib.c5_scene(W, H)
    full = shs_gpu.Context(0)
    fh, fd, fm = _render_lib(full, frame, draws)
    ctxs, bufs = [], []
    for r in range(count):
        c = shs_gpu.Context(0)
        frame.shard_rank, frame.shard_count = r, count
        h, d, m = _render_lib(c, frame, draws)
        words = c.tiles_packed_words(c.TARGET_LIB, count)
        buf = torch.zeros(words, dtype=torch.int32, device="cuda:0")
        torch.cuda.synchronize()   # torch's fill runs on its own stream: done before the pack
        c.tiles_pack(c.TARGET_LIB, r, count, buf.data_ptr())
        c.synchronize_lib()
        host = shard.pack_padded(shard.planes_of([(h, False), (d, False), (m, False)]), W, H, r, count)
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
        torch.cuda.synchronize()   # torch's fill runs on its own stream: done before the pack
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


@pytest.mark.parametrize("fused", [False, True])
@pytest.mark.parametrize("count", [2, 8])
def test_lib_present_gather_after_sharded_tonemap(count, fused):
    """The multi-GPU frame as bench C4 / C5 run it: every rank renders its tiles, tonemaps only those
    (k_tonemap_tiles, or fused into the pass's shading kernel as the bench does) into the present
    staging, and ships 4 B/px (SHS_TARGET_LIB_PRESENT); rank 0's composed staging equals the unsharded
    frame's tonemapped staging."""
    import torch
    import shs_gpu
    from shs_gpu import scene_lib, shard
    frame, draws, _, _, _ = scene_lib.c5_scene(352, 200)
    full = shs_gpu.Context(0)
    full.render_pbr_forward(frame, draws)
    full.tonemap(1.0, 2.2, ldr=False, present=True)
    _, want = full.resolve_ldr()
    ctxs, bufs = [], []
    for r in range(count):
        c = shs_gpu.Context(0)
        frame.shard_rank, frame.shard_count = r, count
        if fused:
            c.fuse_tonemap(1.0, 2.2, ldr=False, present=True)
            c.render_pbr_forward(frame, draws)
        else:
            c.render_pbr_forward(frame, draws)
            c.tonemap(1.0, 2.2, ldr=False, present=True)
        buf = torch.zeros(c.tiles_packed_words(c.TARGET_LIB_PRESENT, count), dtype=torch.int32, device="cuda:0")
        torch.cuda.synchronize()   # torch's fill runs on its own stream: done before the pack
        c.tiles_pack(c.TARGET_LIB_PRESENT, r, count, buf.data_ptr())   # finishes the pass chain first
        c.synchronize_lib()
        _, pres = c.resolve_ldr()
        host = shard.pack_padded(shard.planes_of([(pres, True)]), 352, 200, r, count)
        assert np.array_equal(buf.cpu().numpy().view(np.uint32)[:host.size], host)
        ctxs.append(c)
        bufs.append(buf)
    for r in range(1, count):
        ctxs[0].tiles_unpack(ctxs[0].TARGET_LIB_PRESENT, r, count, bufs[r].data_ptr())
    _, got = ctxs[0].resolve_ldr()
    assert np.array_equal(got, want)
    for c in ctxs + [full]:
        c.close()


def test_legacy_present_gather():
    import torch
    import shs_gpu
    from shs_gpu import scene
    count = 3
    frame, draws = scene.monkey_scene(640, 480, 3, cam_pos=(0.0, 5.0, -12.0))
    frame.present = True
    full = shs_gpu.Context(0)
    full.render(frame, draws)
    want = full.resolve_present(0)
    ctxs, bufs = [], []
    for r in range(count):
        c = shs_gpu.Context(0)
        f = shs_gpu.Frame(640, 480, shard_rank=r, shard_count=count)
        f.present = True
        c.render(f, draws)
        buf = torch.zeros(c.tiles_packed_words(c.TARGET_PRESENT, count), dtype=torch.int32, device="cuda:0")
        torch.cuda.synchronize()   # torch's fill runs on its own stream: done before the pack
        c.tiles_pack(c.TARGET_PRESENT, r, count, buf.data_ptr())
        c.synchronize()
        ctxs.append(c)
        bufs.append(buf)
    for r in range(1, count):
        ctxs[0].tiles_unpack(ctxs[0].TARGET_PRESENT, r, count, bufs[r].data_ptr())
    assert np.array_equal(ctxs[0].resolve_present(0), want)
    for c in ctxs + [full]:
        c.close()


def test_legacy_binned_hair_shards_compose():
    """sharded, binned frames with unbounded slivers (k_ghost reads k_setup's records and
    the sliver list and applies the tile ownership): the shards compose to the unsharded frame."""
    import shs_gpu
    from shs_gpu.scene import Mesh
    from test_gpu_parity import _hair_soup, _identity_draw
    W, H, count = 400, 300, 3
    rng = np.random.default_rng(99)
    pos, nrm = _hair_soup(rng, W, H, 3000)
    draw = _identity_draw(Mesh(pos, nrm), 3)
    ctx = shs_gpu.Context(0)
    try:
        ctx.set_raster_mode(2)
        ctx.render(shs_gpu.Frame(W, H), [draw])
        fc, fd = ctx.resolve()
        assert ctx.stats()["ghost_fragments"] > 0
        oc, od = np.zeros_like(fc), np.zeros_like(fd)
        ty, tx = np.mgrid[0:H, 0:W] // 32
        for r in range(count):
            ctx.render(shs_gpu.Frame(W, H, shard_rank=r, shard_count=count), [draw])
            c, d = ctx.resolve()
            own = (ty * ((W + 31) // 32) + tx) % count == r       # screen rows
            od[own] = d[own]
            oc[own[::-1]] = c[own[::-1]]                          # colour in canvas rows
        assert np.array_equal(od.view(np.uint32), fd.view(np.uint32)) and np.array_equal(oc, fc)
    finally:
        ctx.close()


class _RankZeroDist:
    """torch.distributed stand-in for rank 0 of `count` ranks in one process: its point-to-point
    receives take the peers' packed buffers (rendered by other contexts)."""

    def __init__(self, count, peers):
        self.count, self.peers = count, peers

    def get_rank(self):
        return 0

    def get_world_size(self):
        return self.count

    irecv, isend = "irecv", "isend"

    @staticmethod
    def P2POp(op, tensor, peer):
        return (op, tensor, peer)

    def batch_isend_irecv(self, ops):
        for op, t, peer in ops:
            assert op == "irecv" and 1 <= peer < self.count
            t.copy_(self.peers[peer][:t.numel()])
        return []


def test_gather_frame_device_reuses_buffers():
    """shard.gather_frame_device (the bench's N > 1 gather) called twice with the same `out` list, for
    two different frames: rank 0's composed present staging equals the unsharded frame's each time
    (it returns the buffer list; nothing called it in a test)."""
    import torch
    import shs_gpu
    from shs_gpu import scene_lib, shard
    count = 3
    root = shs_gpu.Context(0)
    peers = [shs_gpu.Context(0) for _ in range(count - 1)]
    full = shs_gpu.Context(0)
    out = None
    try:
        root.fuse_tonemap(1.0, 2.2, ldr=False, present=True)
        for yaw in (0.0, 25.0):
            frame, draws, _, _, _ = scene_lib.c5_scene(352, 200, yaw=yaw)
            full.render_pbr_forward(frame, draws)
            full.tonemap(1.0, 2.2, ldr=False, present=True)
            _, want = full.resolve_ldr()
            packed = [None]
            for r, c in enumerate(peers, start=1):
                frame.shard_rank, frame.shard_count = r, count
                c.fuse_tonemap(1.0, 2.2, ldr=False, present=True)
                c.render_pbr_forward(frame, draws)
                b = torch.zeros(c.tiles_packed_words(c.TARGET_LIB_PRESENT, count), dtype=torch.int32, device="cuda:0")
                torch.cuda.synchronize()   # torch's fill runs on its own stream: done before the pack
                c.tiles_pack(c.TARGET_LIB_PRESENT, r, count, b.data_ptr())
                c.synchronize_lib()
                packed.append(b)
            frame.shard_rank, frame.shard_count = 0, count
            root.render_pbr_forward(frame, draws)
            prev = out
            out = shard.gather_frame_device(_RankZeroDist(count, packed), root, root.TARGET_LIB_PRESENT, out=out)
            assert len(out) == count + 1
            if prev is not None:
                assert all(a is b for a, b in zip(prev, out)), "the out buffers were not reused"
            torch.cuda.synchronize()
            _, got = root.resolve_ldr()
            assert np.array_equal(got, want), f"yaw {yaw}: composed frame differs"
    finally:
        for c in [root, full] + peers:
            c.close()


@pytest.mark.parametrize("count", [3, 20])
def test_unpack_ranks_equals_per_rank_unpacks(count):
    """shs_tiles_unpack_ranks (rank 0's side of the gather in one launch; more than 16 peers take a
    launch per 16): the composed frame equals the one shs_tiles_unpack builds rank by rank."""
    import torch
    import shs_gpu
    from shs_gpu import scene_lib
    frame, draws, _, _, _ = scene_lib.c5_scene(400, 260)
    ctxs = [shs_gpu.Context(0) for _ in range(3)]   # peer renderer, per-rank composer, one-launch composer
    try:
        peer, one, many = ctxs
        bufs = [None] * count
        for r in range(count):
            frame.shard_rank, frame.shard_count = r, count
            peer.render_pbr_forward(frame, draws)
            if r == 0:
                continue
            b = torch.zeros(max(peer.tiles_packed_words(peer.TARGET_LIB, count), 1), dtype=torch.int32, device="cuda:0")
            torch.cuda.synchronize()   # torch's fill runs on its own stream: done before the pack
            peer.tiles_pack(peer.TARGET_LIB, r, count, b.data_ptr())
            peer.synchronize_lib()
            bufs[r] = b
        frame.shard_rank, frame.shard_count = 0, count
        for c in (one, many):
            c.render_pbr_forward(frame, draws)
        for r in range(1, count):
            one.tiles_unpack(one.TARGET_LIB, r, count, bufs[r].data_ptr())
        many.tiles_unpack_ranks(many.TARGET_LIB, count, [0] + [bufs[r].data_ptr() for r in range(1, count)])
        for a, b in zip(one.resolve_lib(), many.resolve_lib()):
            assert np.array_equal(a.view(np.uint32), b.view(np.uint32))
    finally:
        frame.shard_rank, frame.shard_count = 0, 1
        for c in ctxs:
            c.close()
