"""Legacy present staging (Canvas::copy_to_SDLSurface, shs_renderer.hpp:833-848):
the SDL RGBA32 surface rows written by the same k_raster launch as the canvas, vs the oracle's
restatement over the oracle's own canvas (bit-exact wherever the canvas bytes are), with an SDL-style
row pitch, for single frames and batches, clear colour and sharded frames."""
import numpy as np
import pytest

from helpers import assert_color_parity


def test_oracle_present_is_row_flip(oracle_mod):
    rng = np.random.default_rng(1)
    c = rng.integers(0, 256, size=(7, 5, 4), dtype=np.uint8)
    assert np.array_equal(oracle_mod.sdl_present(c), c[::-1])


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", ["c1", "c2"])
def test_present_matches_oracle(gpu_ctx, oracle_mod, cfg):
    from shs_gpu import scene
    frame, draws = scene.config(cfg, yaw=5.0)
    frame.present = True
    frame.prequant = True
    frame.clear_color = (9, 18, 27, 255)
    gpu_ctx.render(frame, draws)
    color, _ = gpu_ctx.resolve()
    pq = gpu_ctx.resolve_prequant(0)
    pres = gpu_ctx.resolve_present(0)
    assert np.array_equal(pres, oracle_mod.sdl_present(color))
    rc, rd, rpq = oracle_mod.render_legacy(frame.width, frame.height, draws, threads=8, prequant=True)
    rc[(rd == np.finfo(np.float32).max)[::-1]] = (9, 18, 27, 255)   # depth: screen rows; colour: canvas rows
    # the staging is the canvas's row flip, and the canvas matches the oracle under the colour rule
    # (a byte may differ by 1 only where both pre-truncation floats agree within 1e-5)
    assert_color_parity(color, rc, pq, rpq)
    assert_color_parity(pres, oracle_mod.sdl_present(rc), pq[::-1], rpq[::-1])


@pytest.mark.gpu
def test_present_pitch_and_batch(gpu_ctx):
    from shs_gpu import scene
    import shs_gpu
    fds = []
    for k in range(3):
        frame, draws = scene.monkey_scene(322, 181, 3, yaw=-10.0 + 9.0 * k)
        fds.append(draws)
    frame.present = True
    gpu_ctx.render_batch(frame, fds)
    for k in range(3):
        c, _ = gpu_ctx.resolve_frame(k)
        p = gpu_ctx.resolve_present(k, pitch=322 * 4 + 24)   # an SDL surface with a padded pitch
        assert p.shape == (181, 322 * 4 + 24)
        assert np.array_equal(p[:, :322 * 4].reshape(181, 322, 4), c[::-1])
    with pytest.raises(shs_gpu.ShsError):
        gpu_ctx.resolve_present(0, pitch=100)


@pytest.mark.gpu
@pytest.mark.parametrize("W,H", [(1, 1), (1, 37), (45, 1), (81, 79)])
def test_present_tiny_frames_batch(gpu_ctx, oracle_mod, W, H):
    """Sub-tile frames, single rows / columns, a batch of two: the staging is each frame's row flip."""
    from shs_gpu import scene
    fds = []
    for k in range(2):
        frame, draws = scene.monkey_scene(W, H, k + 2, yaw=4.0 * k, cam_pos=(0.0, 0.0, -2.0))
        fds.append(draws)
    frame.present = True
    gpu_ctx.render_batch(frame, fds)
    for k in range(2):
        c, _ = gpu_ctx.resolve_frame(k)
        assert np.array_equal(gpu_ctx.resolve_present(k), oracle_mod.sdl_present(c))


@pytest.mark.gpu
def test_present_sharded_owned_tiles(gpu_ctx):
    import shs_gpu
    from shs_gpu import scene
    frame, draws = scene.monkey_scene(640, 480, 3, cam_pos=(0.0, 5.0, -12.0))
    frame.present = True
    gpu_ctx.render(frame, draws)
    full = gpu_ctx.resolve_present(0)
    f = shs_gpu.Frame(640, 480, shard_rank=1, shard_count=3)
    f.present = True
    gpu_ctx.render(f, draws)
    part = gpu_ctx.resolve_present(0)
    ty, tx = np.mgrid[0:480, 0:640] // 32
    owned = (ty * 20 + tx) % 3 == 1      # screen rows: the staging's rows are screen rows
    assert np.array_equal(part[owned], full[owned])
