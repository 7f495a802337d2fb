"""CPU: the region layout's balance (shs_abi_shard.cpp, called through the C ABI's host-only
shs_shard_balance_rects): the rectangles tile the bin grid exactly, follow the predicted cost (pixels,
covered pixels, triangles x covering block bounds), give rank 0 a smaller share when asked, handle more
ranks than tiles, and are a pure function of their input (every rank derives the same layout)."""
import numpy as np
import pytest

T = 32


def _blocks(rects_tris, bounded=1):
    """[(bx0, by0, bx1, by1, triangles)] -> k_lib_setup's per-block records."""
    out = []
    for x0, y0, x1, y1, n in rects_tris:
        out.append((x0 | (x1 << 16), y0 | (y1 << 16), n, bounded))
    return np.array(out, np.uint32).reshape(-1, 4)


def _cover(regions, w, h):
    tx, ty = (w + T - 1) // T, (h + T - 1) // T
    c = np.zeros((ty, tx), np.int32)
    for x0, y0, x1, y1 in regions:
        if x1 >= x0 and y1 >= y0:
            c[y0:y1 + 1, x0:x1 + 1] += 1
    return c


def _cost(regions, w, h, blocks):
    """The balancer's cost model restated: 5 per pixel, +15 per pixel some bounded block covers, + each
    covering bounded block's triangles per tile."""
    tx, ty = (w + T - 1) // T, (h + T - 1) // T
    px = np.array([[min(T, w - T * x) * min(T, h - T * y) for x in range(tx)] for y in range(ty)], np.float64)
    tri = np.zeros((ty, tx))
    cov = np.zeros((ty, tx), bool)
    for bx, by, n, bd in blocks:
        x0, x1, y0, y1 = bx & 0xffff, bx >> 16, by & 0xffff, by >> 16
        if n == 0 or bd == 0 or x1 < x0 or y1 < y0:
            continue
        tri[y0:y1 + 1, x0:x1 + 1] += n
        cov[y0:y1 + 1, x0:x1 + 1] = True
    c = px * (5.0 + 15.0 * cov) + tri
    return [c[y0:y1 + 1, x0:x1 + 1].sum() if x1 >= x0 and y1 >= y0 else 0.0 for x0, y0, x1, y1 in regions]


@pytest.mark.parametrize("count", [1, 2, 3, 5, 8])
def test_pixels_only_split_tiles_the_grid(count):
    import shs_gpu
    regs = shs_gpu.Context.shard_balance(np.zeros((0, 4), np.uint32), 3840, 2160, count)
    assert (_cover(regs, 3840, 2160) == 1).all()
    costs = _cost(regs, 3840, 2160, [])
    assert max(costs) <= 1.15 * (sum(costs) / count)


def test_dense_corner_gets_small_rectangles():
    """A cluster of heavy blocks in one corner: the ranks over it get smaller rectangles and the
    predicted costs even out."""
    import shs_gpu
    rng = np.random.default_rng(3)
    spec = []
    for _ in range(3000):
        x0, y0 = int(rng.integers(0, 30)), int(rng.integers(0, 20))
        spec.append((x0, y0, x0 + int(rng.integers(0, 6)), y0 + int(rng.integers(0, 6)), 256))
    blocks = _blocks(spec)
    regs = shs_gpu.Context.shard_balance(blocks, 3840, 2160, 8)
    assert (_cover(regs, 3840, 2160) == 1).all()
    costs = _cost(regs, 3840, 2160, blocks)
    assert max(costs) <= 1.35 * (sum(costs) / 8), costs
    areas = [(x1 - x0 + 1) * (y1 - y0 + 1) for x0, y0, x1, y1 in regs]
    assert min(areas) * 4 < max(areas)


def test_root_share_and_determinism():
    import shs_gpu
    rng = np.random.default_rng(5)
    spec = [(int(a), int(b), int(a) + 3, int(b) + 3, 256) for a, b in zip(rng.integers(0, 110, 2000), rng.integers(0, 60, 2000))]
    blocks = _blocks(spec)
    full = shs_gpu.Context.shard_balance(blocks, 3840, 2160, 8)
    again = shs_gpu.Context.shard_balance(blocks.copy(), 3840, 2160, 8)
    assert full == again
    small = shs_gpu.Context.shard_balance(blocks, 3840, 2160, 8, root_share=0.6)
    c_full, c_small = _cost(full, 3840, 2160, blocks), _cost(small, 3840, 2160, blocks)
    assert c_small[0] < c_full[0]
    assert (_cover(small, 3840, 2160) == 1).all()


def test_unbounded_and_offscreen_blocks_are_ignored():
    """Blocks without bounds (w = 0) and off-screen blocks (empty bounds) do not change the layout."""
    import shs_gpu
    base = _blocks([(10, 10, 20, 20, 256)] * 50)
    extra = np.concatenate([base, _blocks([(0, 0, 119, 67, 256)] * 40, bounded=0), _blocks([(1, 1, 0, 0, 256)] * 40)])
    assert shs_gpu.Context.shard_balance(base, 3840, 2160, 4) == shs_gpu.Context.shard_balance(extra, 3840, 2160, 4)


def test_more_ranks_than_tiles():
    import shs_gpu
    regs = shs_gpu.Context.shard_balance(np.zeros((0, 4), np.uint32), 40, 20, 5)
    assert (_cover(regs, 40, 20) == 1).all()
    assert sum(1 for x0, y0, x1, y1 in regs if x1 >= x0 and y1 >= y0) == 2
