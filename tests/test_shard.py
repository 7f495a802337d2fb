"""CPU tests of the multi-rank tile-shard path: tile ownership, pack/unpack, and the
world_size-2 gloo gather that composes the full frame on rank 0 (the same code runs over RCCL)."""
import os
import socket

import numpy as np
import pytest

from shs_gpu import shard

T = 32


def _frame(w, h, seed=0):
    rng = np.random.default_rng(seed)
    color = rng.integers(0, 256, size=(h, w, 4), dtype=np.uint8)
    depth = rng.normal(size=(h, w)).astype(np.float32)
    depth[rng.random((h, w)) < 0.3] = np.finfo(np.float32).max
    return color, depth


def _keep_owned(color, depth, rank, count):
    """What a shard-rendering rank holds: its own tiles, garbage elsewhere."""
    h, w = depth.shape
    c = np.full_like(color, 77)
    d = np.full_like(depth, -5.0)
    for t in shard.owned_tiles(w, h, T, rank, count):
        y0, y1, x0, x1 = shard._tile_slices(t, w, h, T)
        d[y0:y1, x0:x1] = depth[y0:y1, x0:x1]
        c[h - y1:h - y0, x0:x1] = color[h - y1:h - y0, x0:x1]
    return c, d


@pytest.mark.parametrize("w,h,count", [(333, 241, 2), (1920, 1080, 3), (64, 32, 5)])
def test_pack_unpack_roundtrip(w, h, count):
    color, depth = _frame(w, h)
    full_c = np.zeros_like(color)
    full_d = np.zeros_like(depth)
    owned = np.zeros(((h + T - 1) // T) * ((w + T - 1) // T), np.int64)
    for r in range(count):
        c, d = _keep_owned(color, depth, r, count)
        p = shard.pack_owned(c, d, T, r, count)
        assert p.size == shard.packed_len(w, h, T, r, count)
        shard.unpack_into(full_c, full_d, p, T, r, count)
        owned[shard.owned_tiles(w, h, T, r, count)] += 1
    assert (owned == 1).all()      # every tile owned by exactly one rank
    assert np.array_equal(full_c, color)
    assert np.array_equal(full_d.view(np.uint32), depth.view(np.uint32))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _gloo_worker(rank, world, port, w, h, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        color, depth = _frame(w, h, seed=11)
        c, d = _keep_owned(color, depth, rank, world)
        out = shard.gather_frame(dist, c, d, T)
        if rank == 0:
            ok = np.array_equal(out[0], color) and np.array_equal(out[1].view(np.uint32), depth.view(np.uint32))
            q.put(ok)
        else:
            q.put(out is None)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_gloo_gather_composes_full_frame(world):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gloo_worker, args=(r, world, port, 333, 241, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    assert all(p.exitcode == 0 for p in procs)
    results = [q.get(timeout=5) for _ in range(world)]
    assert all(results)


@pytest.mark.parametrize("w,h,count", [(333, 241, 3), (3840, 2160, 8), (100, 40, 1)])
def test_padded_layout_roundtrip(w, h, count):
    """The device gather's packed layout (shs_tiles.hip), restated on the host: every rank's padded
    tile blocks unpack into exactly the full frame; buffer sizes match shs_tiles_packed_words."""
    rng = np.random.default_rng(4)
    hdr = rng.normal(size=(h, w, 4)).astype(np.float32)
    depth = rng.random((h, w)).astype(np.float32)
    src = shard.planes_of([(hdr, False), (depth, False)])
    dst_hdr, dst_depth = np.zeros_like(hdr), np.zeros_like(depth)
    dst = shard.planes_of([(dst_hdr, False), (dst_depth, False)])
    n_tiles = ((w + 31) // 32) * ((h + 31) // 32)
    for r in range(count):
        p = shard.pack_padded(src, w, h, r, count)
        assert p.size <= ((n_tiles + count - 1) // count) * 1024 * 5
        shard.unpack_padded(dst, p, w, h, r, count)
    assert np.array_equal(dst_hdr.view(np.uint32), hdr.view(np.uint32))
    assert np.array_equal(dst_depth.view(np.uint32), depth.view(np.uint32))


# region layouts of a 333x241 frame (11 x 8 bin tiles) for 2 and 3 ranks, one with an empty rank
_REGIONS = {2: [(0, 0, 3, 7), (4, 0, 10, 7)], 3: [(0, 0, 10, 2), (0, 3, 10, 7), (1, 1, 0, 0)]}


def _gloo_padded_worker(rank, world, port, q, present=False, regions=False):
    """The device gather's protocol over gloo: pack (host restatement), point-to-point sends of each
    rank's exact packed size to rank 0 (shard.send_to_root, what gather_frame_device runs over RCCL),
    unpack.  present: the 4 B/px RGBA8 present staging the sharded bench ships (SHS_TARGET_LIB_PRESENT:
    rows top-down, so the plane is row-flipped into screen order like the device's tile parameters).
    regions: a region layout (ranks of different sizes, possibly empty) instead of interleaved tiles."""
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        w, h = 333, 241
        reg = _REGIONS[world] if regions else None
        rng = np.random.default_rng(12)
        color = rng.integers(0, 2**31, size=(h, w), dtype=np.int64).astype(np.uint32)
        rgba = color.view(np.uint8).reshape(h, w, 4)
        planes = shard.planes_of([(rgba, True)]) if present else [color]
        sizes = [len(shard.owned_tiles(w, h, 32, r, world, reg)) * 1024 for r in range(world)]
        buf = np.zeros(max(sizes) + 7, np.uint32)   # capacity above the payload: only sizes[r] words travel
        mine = shard.pack_padded(planes, w, h, rank, world, regions=reg)
        assert mine.size == sizes[rank]
        buf[:mine.size] = mine
        t = torch.from_numpy(buf.view(np.int32))
        recvs = [torch.zeros_like(t) for _ in range(world)]
        shard.ensure_group_ready(dist)   # what gather_frame_device does before the first batch
        shard.send_to_root(dist, t, recvs, sizes)
        if rank == 0:
            out = np.zeros_like(color)
            out_planes = shard.planes_of([(out.view(np.uint8).reshape(h, w, 4), True)]) if present else [out]
            shard.unpack_padded(out_planes, mine, w, h, 0, world, regions=reg)
            for r in range(1, world):
                shard.unpack_padded(out_planes, recvs[r].numpy().view(np.uint32)[:sizes[r]], w, h, r, world, regions=reg)
            q.put(bool(np.array_equal(out, color)))
        else:
            q.put(True)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("present,regions,world", [(False, False, 2), (True, False, 2), (True, True, 2), (False, True, 3)])
def test_gloo_device_protocol_gather(present, regions, world):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gloo_padded_worker, args=(r, world, port, q, present, regions)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    assert all(p.exitcode == 0 for p in procs)
    assert all(q.get(timeout=5) for _ in range(world))


@pytest.mark.parametrize("w,h,count,regions", [
    (3840, 2160, 8, None), (333, 241, 3, None), (333, 241, 2, _REGIONS[2]), (333, 241, 3, _REGIONS[3]),
    (3840, 2160, 1, None)])
def test_owned_pixels_partition_the_frame(w, h, count, regions):
    """shard.owned_pixels (bench.py's N > 1 roofline: rank 0's camera-pass bytes are its owned pixels x
    32 B, not the whole frame's): the ranks' shares add up to W*H, and rank r's share is the number of
    pixels its tiles cover, edge tiles clipped."""
    shares = [shard.owned_pixels(w, h, T, r, count, regions) for r in range(count)]
    assert sum(shares) == w * h
    for r in range(count):
        m = np.zeros((h, w), bool)
        for t in shard.owned_tiles(w, h, T, r, count, regions):
            y0, y1, x0, x1 = shard._tile_slices(t, w, h, T)
            m[y0:y1, x0:x1] = True
        assert shares[r] == int(m.sum())
    if regions is None and count == 8:
        # 120 x 68 bin tiles, the last row 16 px high: interleaved ranks get 1020 tiles each
        assert shares[0] == 1020 * 1024 - 120 // 8 * 16 * 32


def test_ensure_group_ready_after_reinit():
    """the barrier before a group's first point-to-point batch runs once per group object --
    a re-initialised default group gets its own barrier even where CPython reuses the old one's id."""
    import types
    from shs_gpu import shard
    calls = []

    def fake_dist():
        d = types.SimpleNamespace()
        d.group = types.SimpleNamespace(WORLD=object())
        d.barrier = lambda: calls.append(1)
        return d
    d = fake_dist()
    shard.ensure_group_ready(d)
    shard.ensure_group_ready(d)
    assert len(calls) == 1
    d.group.WORLD = object()          # destroy_process_group + init_process_group
    shard.ensure_group_ready(d)
    assert len(calls) == 2
