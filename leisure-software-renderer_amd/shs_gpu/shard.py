"""Screen-tile sharding of one frame across ranks.

Rank r of N renders only the bin tiles with `tile % N == r` (shs_frame_desc.shard_rank/count; a tile
is shs_gpu_tile_size() px square, row-major), or -- library frames with SHS_OPT_SHARD_LAYOUT regions --
one cost-balanced rectangle of tiles per rank.  The owned tiles of every rank are then gathered into
the full frame on rank 0.  On GPUs the collective runs over RCCL ("nccl" backend) on device tensors;
the same code runs over gloo on CPU tensors (tests/test_shard.py).

Only the owned tiles travel.  The device path (gather_frame_device, what bench.py and the C ABI's
Seam-2 binding use): every rank packs its owned tiles with shs_tiles_pack, sends exactly its packed
size to rank 0 in one batch of point-to-point operations (send_to_root; region ranks differ in size),
and rank 0 unpacks every peer's tiles with one shs_tiles_unpack_ranks launch, all ordered on the
frame's stream.  The host-array path (gather_frame, tests and debugging) packs numpy planes and
exchanges equal-size padded buffers with all_gather.
"""
import numpy as np

try:
    import torch
except ImportError:  # pragma: no cover - torch is present in this image
    torch = None


def owned_tiles(width, height, tile, rank, count, regions=None):
    """Tile indices owned by `rank`: tile % count == rank, or with a region layout (regions[r] =
    (bx0, by0, bx1, by1), inclusive, SHS_OPT_SHARD_LAYOUT) the rank's rectangle row-major -- the order
    of shs_tiles_pack's blocks (shs_shard.hpp shard_tile)."""
    tx = (width + tile - 1) // tile
    ty = (height + tile - 1) // tile
    if regions is not None and count > 1:
        x0, y0, x1, y1 = regions[rank]
        if x1 < x0 or y1 < y0:
            return np.zeros(0, np.int64)
        yy, xx = np.mgrid[y0:y1 + 1, x0:x1 + 1]
        return (yy * tx + xx).reshape(-1).astype(np.int64)
    return np.arange(rank, tx * ty, count, dtype=np.int64)


def owned_pixels(width, height, tile, rank, count, regions=None):
    """Pixels of the frame that `rank` renders (its owned tiles clipped to the frame): the share of a
    sharded camera pass's per-pixel algorithmic bytes that one rank's kernels move (bench.py's N > 1
    roofline)."""
    n = 0
    for t in owned_tiles(width, height, tile, rank, count, regions):
        y0, y1, x0, x1 = _tile_slices(int(t), width, height, tile)
        n += (y1 - y0) * (x1 - x0)
    return n


def _tile_slices(t, width, height, tile):
    tx = (width + tile - 1) // tile
    x0, y0 = (t % tx) * tile, (t // tx) * tile
    return y0, min(y0 + tile, height), x0, min(x0 + tile, width)


def pack_owned(color, depth, tile, rank, count):
    """Pack the owned tiles of (color [H,W,4] uint8 canvas rows, depth [H,W] f32 screen rows) into
    one int32 vector: per tile, its colour words then its depth bits, tiles in index order."""
    height, width = depth.shape
    words = color.view(np.uint32).reshape(height, width)
    dbits = depth.view(np.uint32)
    parts = []
    for t in owned_tiles(width, height, tile, rank, count):
        y0, y1, x0, x1 = _tile_slices(t, width, height, tile)
        # colour lives in canvas rows: screen row y is canvas row H-1-y
        parts.append(words[height - y1:height - y0, x0:x1][::-1].ravel())
        parts.append(dbits[y0:y1, x0:x1].ravel())
    if not parts:
        return np.zeros(0, np.int32)
    return np.concatenate(parts).view(np.int32)


def unpack_into(color, depth, packed, tile, rank, count):
    """Inverse of pack_owned: write rank's tiles into the full frame buffers."""
    height, width = depth.shape
    words = color.view(np.uint32).reshape(height, width)
    dbits = depth.view(np.uint32)
    data = np.asarray(packed).view(np.uint32)
    off = 0
    for t in owned_tiles(width, height, tile, rank, count):
        y0, y1, x0, x1 = _tile_slices(t, width, height, tile)
        n = (y1 - y0) * (x1 - x0)
        words[height - y1:height - y0, x0:x1] = data[off:off + n].reshape(y1 - y0, x1 - x0)[::-1]
        off += n
        dbits[y0:y1, x0:x1] = data[off:off + n].reshape(y1 - y0, x1 - x0)
        off += n
    return off


def packed_len(width, height, tile, rank, count):
    n = 0
    for t in owned_tiles(width, height, tile, rank, count):
        y0, y1, x0, x1 = _tile_slices(t, width, height, tile)
        n += 2 * (y1 - y0) * (x1 - x0)
    return n


# ---- device-resident gather (libshs_gpu shs_tiles_pack / shs_tiles_unpack) -----------------------
# Layout of one rank's packed buffer (shs_tiles.hip): owned tile i = rank + i*count occupies
# TILE*TILE*words int32 words at i*TILE*TILE*words; inside it, plane c (colour words, depth, motion)
# holds the tile's pixels row-major in screen rows, padded to 32x32.

def planes_of(frame_planes):
    """frame_planes: list of (array [H,W,k] or [H,W] of 4-byte words, flip_rows) -> list of
    per-plane uint32 views [H, W] in SCREEN row order."""
    out = []
    for a, flip in frame_planes:
        a = np.ascontiguousarray(a)
        words = a.view(np.uint32)
        words = words.reshape(a.shape[0], a.shape[1], -1)
        for k in range(words.shape[2]):
            p = words[:, :, k]
            out.append(p[::-1] if flip else p)
    return out


def pack_padded(planes, width, height, rank, count, tile=32, regions=None):
    """CPU restatement of shs_tiles_pack for screen-row planes (list of uint32 [H, W])."""
    owned = owned_tiles(width, height, tile, rank, count, regions)
    nw = len(planes)
    out = np.zeros((len(owned), nw, tile, tile), np.uint32)
    for i, t in enumerate(owned):
        y0, y1, x0, x1 = _tile_slices(t, width, height, tile)
        for c, p in enumerate(planes):
            out[i, c, :y1 - y0, :x1 - x0] = p[y0:y1, x0:x1]
    return out.reshape(-1)


def unpack_padded(planes, packed, width, height, rank, count, tile=32, regions=None):
    owned = owned_tiles(width, height, tile, rank, count, regions)
    blk = np.asarray(packed).view(np.uint32).reshape(-1, len(planes), tile, tile)
    for i, t in enumerate(owned):
        y0, y1, x0, x1 = _tile_slices(t, width, height, tile)
        for c, p in enumerate(planes):
            p[y0:y1, x0:x1] = blk[i, c, :y1 - y0, :x1 - x0]


def gather_frame_device(dist, ctx, target, stream=None, out=None):
    """RCCL gather of a tile-sharded frame into rank 0's context buffers (device to device).
    Every rank packs its owned tiles on the GPU (shs_tiles_pack, which first finishes the frame: a
    capacity overflow is re-issued before anything leaves the rank); each peer sends exactly its own
    packed tiles to rank 0 (point-to-point ncclSend / ncclRecv over xGMI, batched: the region layout's
    ranks differ in size) and rank 0 unpacks them in place (shs_tiles_unpack).
    The context runs on the given stream (default torch's current one) so RCCL and the kernels are
    ordered; it is re-pointed only when it is not on that stream already (shs_set_stream synchronises).
    target: ctx.TARGET_PRESENT / TARGET_LIB_PRESENT (RGBA8, 4 B/px: what the SDL present needs) or
    TARGET_LEGACY / TARGET_LIB (colour + depth (+ motion): 8 / 28 B/px).
    out: optional list of preallocated int32 device buffers [count + 1] (send + receive) to reuse;
    returns the list used."""
    rank, count = dist.get_rank(), dist.get_world_size()
    s = stream if stream is not None else torch.cuda.current_stream()
    if ctx.stream != s.cuda_stream:
        ctx.set_stream(s.cuda_stream)
    ensure_group_ready(dist)
    # everything below -- pack, the point-to-point batch (RCCL enqueues on the current stream; the gloo
    # staging copies too) and the unpacks -- is ordered on s, whichever stream the caller has current
    with torch.cuda.stream(s):
        words = ctx.tiles_packed_words(target, count)
        sizes = [ctx.tiles_rank_words(target, r, count) for r in range(count)]
        dev = torch.device("cuda", torch.cuda.current_device())
        if out is None or out[0].numel() < words:
            out = [torch.empty(words, dtype=torch.int32, device=dev) for _ in range(count + 1)]
        buf = out[0]
        ctx.tiles_pack(target, rank, count, buf.data_ptr())
        send_to_root(dist, buf, out[1:], sizes)
        if rank == 0:   # every peer's tiles by one launch
            ctx.tiles_unpack_ranks(target, count, [0] + [out[1 + r].data_ptr() if sizes[r] > 0 else 0
                                                          for r in range(1, count)])
    return out


_READY = []   # the group objects already barriered: weak references (a strong one where the type has none)


def ensure_group_ready(dist):
    """One barrier per process group before its first point-to-point batch.  batch_isend_irecv must be
    joined by every rank when it is the group's first NCCL collective, but a rank whose region is empty
    (or rank 0 with no non-empty peer) posts no operation at all; a barrier first makes the batches
    ordinary point-to-point traffic on an initialised communicator.  The groups are kept by reference,
    not by id(): after destroy_process_group and a re-init, CPython could hand the new default group
    the old one's id while the old object is gone.  Weak references let a destroyed group (and the
    communicator it holds) be collected; an entry is compared by identity while its object lives, so a
    re-created group is still never mistaken for an old one."""
    import weakref
    world = getattr(getattr(dist, "group", None), "WORLD", None)   # the default group (a new one after re-init)
    key = world if world is not None else dist
    _READY[:] = [r for r in _READY if r() is not None]   # drop collected groups
    if any(r() is key for r in _READY):
        return
    barrier = getattr(dist, "barrier", None)
    if barrier is not None:
        barrier()
    try:
        _READY.append(weakref.ref(key))
    except TypeError:   # no weak-reference support: hold it (the previous behaviour)
        _READY.append(lambda k=key: k)


def send_to_root(dist, buf, recvs, sizes):
    """Rank r > 0 sends buf[:sizes[r]] to rank 0, which receives it into recvs[r][:sizes[r]]: one
    batch of point-to-point operations (sizes may differ per rank; empty ranks send nothing).
    Over gloo (bench.py's one-GPU rehearsal; RCCL everywhere else) device tensors are staged through
    host memory: gloo's own device path took ~170 ms per 4 MB against 0.5 ms for host tensors
    (tools/diag_gloo_p2p.py)."""
    rank, count = dist.get_rank(), dist.get_world_size()
    get_backend = getattr(dist, "get_backend", None)
    staged = bool(getattr(buf, "is_cuda", False)) and get_backend is not None and get_backend() == "gloo"
    if rank == 0:
        peers = [r for r in range(1, count) if sizes[r] > 0]
        dst = {r: (recvs[r][:sizes[r]].new_empty(sizes[r], device="cpu") if staged else recvs[r][:sizes[r]]) for r in peers}
        ops = [dist.P2POp(dist.irecv, dst[r], r) for r in peers]
    else:
        src = buf[:sizes[rank]].cpu() if staged and sizes[rank] > 0 else buf[:sizes[rank]]
        ops = [dist.P2POp(dist.isend, src, 0)] if sizes[rank] > 0 else []
    for q in (dist.batch_isend_irecv(ops) if ops else []):
        q.wait()
    if staged and rank == 0:
        for r in peers:
            recvs[r][:sizes[r]].copy_(dst[r])


def gather_frame(dist, color, depth, tile, device=None):
    """Collective: every rank passes its shard-rendered (color, depth) host buffers (only its own
    tiles meaningful); rank 0 returns the composed full frame, other ranks return None.
    `device` selects where the exchange buffers live ("cuda:k" for RCCL, None/cpu for gloo)."""
    rank, count = dist.get_rank(), dist.get_world_size()
    height, width = depth.shape
    mine = pack_owned(color, depth, tile, rank, count)
    longest = max(packed_len(width, height, tile, r, count) for r in range(count))
    buf = np.zeros(longest, np.int32)
    buf[:mine.size] = mine
    t = torch.from_numpy(buf)
    if device is not None:
        t = t.to(device)
    outs = [torch.empty_like(t) for _ in range(count)]
    dist.all_gather(outs, t)
    if rank != 0:
        return None
    full_c = np.zeros_like(color)
    full_d = np.zeros_like(depth)
    for r in range(count):
        unpack_into(full_c, full_d, outs[r].cpu().numpy(), tile, r, count)
    return full_c, full_d
