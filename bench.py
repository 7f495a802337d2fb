#!/usr/bin/env python3
"""bench.py -- Mtri/s + shaded Mpix/s of the shs_renderer legacy hot path on MI355X.

Workload (BASELINE.json configs[1], "C2"): Suzanne (monkey.rawobj, 967 triangles) Blinn-Phong +
z-buffer at 1920x1080, the reference scene of hello_pipeline_blinn_phong_shading.cpp:152-153 and
its Viewer((0,5,-20)) camera.  One step = one full frame through the HIP path: clear, vertex
transform, setup, tile binning, coverage + z resolve, Blinn-Phong shading of the visible pixels and
the colour (RGBA8 canvas rows) + depth (f32 screen rows) write.  Inputs (mesh, per-frame uniform
table) are resident in HBM / pinned host memory before the timed region; the per-frame uniform
upload is inside it.

N > 1 (torchrun, one process per GPU): frame-parallel -- every rank renders its own frame of the
same workload (camera yaw offset per rank), no data-path collective; "scaling": "weak".

Also reported (rank 0, N = 1):
  roofline      dominant kernel (k_raster, which writes every output byte of the frame): SURVEY.md
                8(d) algorithmic bytes per frame (N_tri*72 + W*H*8) / its mean HIP-event duration
                over the timed region, against 8 TB/s (frame_frac: the same bytes over k_setup +
                k_raster); "traffic" = HBM bytes per k_raster dispatch from rocprofv3 PMC counters
                (FETCH_SIZE x2 [gfx950 half-count correction] + WRITE_SIZE, KiB units), collected in
                separate child passes before this process touches the GPU.
  cpu_baseline  the oracle (CPU restatement of the reference's 80x80 tile-job path, gcc -O3) timed
                on this host's cores on a bounded sample of the same frames.
"""
import argparse
import csv
import glob
import json
import os
import platform
import shutil
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "leisure-software-renderer_amd")
for p in (PKG, ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

METRIC = "Mtri/s + shaded Mpix/s at 1920×1080 Blinn-Phong; 1/2/4/8 MI355X scaling"
HBM_PEAK_GBS = 8000.0
WORKLOADS = {
    "c2": "C2: Suzanne monkey.rawobj Blinn-Phong + z-buffer, 1920x1080, a batch of camera poses per step",
    "c1": "C1: Suzanne monkey.rawobj Blinn-Phong + z-buffer, 800x600, a batch of camera poses per step",
    "c3": "C3: 64-instance Suzanne grid, Phong, 1920x1080, a batch of camera poses per step",
    "c5": "C5: Suzanne + floor, PassShadowMap 2048^2 + PassPBRForward (PBR Cook-Torrance, PCF 5x5, motion) "
          "3840x2160 + PassTonemap into the RGBA8 present staging, 1 frame per step",
    "c4": "C4: Forward+ tiled, 1M synthetic triangles, 256 point lights, 3840x2160 (light cull + lit forward pass "
          "+ PassTonemap into the RGBA8 present staging), 1 frame per step",
}
LIB_CONFIGS = {"c5", "c4"}


def algorithmic_bytes(frame, draws):
    """every input read once (fp32 soup: 3 x (pos 12 + normal 12) = 72 B/tri) and
    every output written once (RGBA8 4 B + f32 depth 4 B per pixel), clears fused."""
    n_tri = sum(d.mesh.n_tris for d in draws)
    return n_tri * 72 + frame.width * frame.height * 8, n_tri


def build_workload(name, rank=0):
    from shs_gpu import scene
    # frame-parallel ranks render different frames: the camera yaw advances 3 degrees per rank
    return scene.config(name, yaw=3.0 * rank)


POSE_SETS = 4   # distinct batches of camera poses the timed steps cycle through
LEGACY_FRAMES = {"c1": 128, "c2": 128, "c3": 16}   # default frames per step (one shs_render_legacy_batch)


def batch_poses(name, n_frames, rank=0):
    """POSE_SETS batches of n_frames camera poses of the workload's scene: frame k of set p looks from
    yaw = 3*rank - 12 + 24 * (p * n_frames + k) / (POSE_SETS * n_frames) degrees and a small pitch
    sweep, so every frame of every step is a different image of the same scene (nothing is cached:
    each step re-runs the whole path for its own poses)."""
    from shs_gpu import scene
    total = POSE_SETS * n_frames
    sets = []
    for p in range(POSE_SETS):
        fds = []
        for k in range(n_frames):
            i = p * n_frames + k
            frame, draws = scene.config(name, yaw=3.0 * rank - 12.0 + 24.0 * i / total,
                                        pitch=-3.0 + 6.0 * ((i * 7) % total) / total)
            fds.append(draws)
        sets.append(fds)
    return frame, sets


def run_gpu(args, rank, local_rank, world, dist):
    """One step = one shs_render_legacy_batch of F frames (F = --frames-per-step): one k_setup + one
    k_raster launch render F independent frames, each into its own colour + depth framebuffers.
    F = 1 is the single-frame (latency) path, one shs_render_legacy per step."""
    import shs_gpu
    F = args.frames_per_step
    frame, sets = batch_poses(args.config, F, rank)
    frame.debug_flags = args.debug_flags   # timing experiments only (wrong images; read only by libshs_gpu_exp.so)
    ctx = shs_gpu.Context(local_rank)
    if args.raster_mode:
        ctx.set_raster_mode(args.raster_mode)
    if args.raster_loop >= 0:
        ctx.set_raster_loop(args.raster_loop)
    prepared = [ctx.prepare_batch(frame, fds) for fds in sets]
    render = ctx.render_batch_prepared
    # The auxiliary legs run BEFORE the headline loop: every frame they render is measured for its own
    # figure, and the loop that follows starts on a GPU that has been rendering (clocks up), as a render
    # loop's frames do -- not right after process start-up (tools/diag_short_window.py).
    single = None
    if F > 1 and not args.child and not args.no_single:
        # the single-frame latency figure: one shs_render_legacy per step
        one = ctx.prepare(frame, sets[0][0])
        for _ in range(10):
            ctx.render_prepared(one)
        ctx.synchronize()
        n1 = max(20, min(args.steps * 4, 400))
        ctx.enable_timing(True)
        ctx.timing_reset()
        t1 = time.perf_counter()
        for _ in range(n1):
            ctx.render_prepared(one)
        ctx.synchronize()
        el1 = time.perf_counter() - t1
        _, k1 = ctx.timing_read()
        ctx.enable_timing(False)
        single = {"ms_per_frame": round(el1 / n1 * 1e3, 5), "steps": n1,
                  "kernels_ms": {k: round(v, 5) for k, v in k1.items()}}
    # Clock ramp: the GPU reaches its steady-state clocks only after ~15-20 ms of continuous rendering
    # (tools/diag_short_window.py: consecutive 20-step windows right after 5 warm-up steps run 0.304,
    # 0.294, then 0.285 ms/step, k_raster 0.260 -> 0.242 ms; profiles/r04_c2_short_window.txt).  A render
    # loop runs continuously, so the headline window starts after args.ramp_ms of the same batches
    # (untimed, like the warm-up steps that follow it).
    if args.pipeline:   # SHS_OPT_LEGACY_PIPELINE: a batch's raster in the next batch's launch (k_pipe)
        ctx.set_legacy_pipeline(True)
    t_ramp = time.perf_counter()
    n_ramp = 0
    while args.ramp_ms > 0 and (time.perf_counter() - t_ramp) * 1e3 < args.ramp_ms:
        for _ in range(8):
            render(prepared[n_ramp % POSE_SETS])
            n_ramp += 1
        ctx.synchronize()
    ramp = {"ms": round((time.perf_counter() - t_ramp) * 1e3, 1), "batches": n_ramp}
    for i in range(max(args.warmup, 1)):
        render(prepared[i % POSE_SETS])
    ctx.synchronize()
    # the statistics of a timed-loop batch (the capacity adaptation of the warm-up has settled)
    render(prepared[0])
    stats = ctx.stats()

    def barrier_sync():
        ctx.synchronize()
        if dist is not None:
            import torch
            torch.cuda.synchronize()
            dist.barrier()

    ctx.enable_timing(True)
    ctx.timing_reset()
    barrier_sync()
    t0 = time.perf_counter()
    for i in range(args.steps):
        render(prepared[i % POSE_SETS])
    barrier_sync()
    elapsed = time.perf_counter() - t0
    n_launches, kms = ctx.timing_read()
    ctx.enable_timing(False)
    ctx.close()
    return frame, sets, stats, elapsed, n_launches, kms, single, ramp


def seam1_pcie(args, frame, sets):
    """The end-to-end Seam-1 figure: every frame crosses PCIe into pinned host memory as the SDL
    surface it is presented from (SHS_FRAME_PRESENT staging, 4 B/px, what copy_to_SDLSurface produces),
    D2H overlapped with rendering: two contexts alternate batches, each batch's D2H queued behind its
    render on that context's stream, so one context's copy runs under the other's render.
    It runs LAST in the process: it initialises torch (streams, pinned memory), after which the library
    legs' streams measured 12 % slower in the same process (C4 0.579 -> 0.654 ms per frame,
    profiles/r06_strong_gap.txt), so nothing timed for the line follows it."""
    import ctypes
    import dataclasses
    import shs_gpu
    import torch
    F = args.frames_per_step
    hip = ctypes.CDLL("libamdhip64.so.7")   # the runtime already mapped (shs_gpu._abi.load)
    hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
    pf = dataclasses.replace(frame, present=True)
    nbytes = F * pf.width * pf.height * 4
    ctxs = [shs_gpu.Context(0), shs_gpu.Context(0)]
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    hosts = [torch.empty(nbytes, dtype=torch.uint8, pin_memory=True) for _ in range(2)]
    prepared = []
    for c, st in zip(ctxs, streams):
        c.set_stream(st.cuda_stream)
        prepared.append([c.prepare_batch(pf, fds) for fds in sets])

    def step(i):
        c = i % 2
        ctxs[c].render_batch_prepared(prepared[c][(i // 2) % POSE_SETS])
        rc = hip.hipMemcpyAsync(ctypes.c_void_p(hosts[c].data_ptr()), ctypes.c_void_p(ctxs[c].present_device(0)),
                                nbytes, 2, ctypes.c_void_p(streams[c].cuda_stream))
        assert rc == 0, rc
    for i in range(4):
        step(i)
    torch.cuda.synchronize()
    n = max(8, min(args.steps, 40))
    t0 = time.perf_counter()
    for i in range(n):
        step(i)
    for c in ctxs:
        c.synchronize()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    # the same copies alone: the PCIe ceiling of this figure
    t1 = time.perf_counter()
    for i in range(n):
        hip.hipMemcpyAsync(ctypes.c_void_p(hosts[i % 2].data_ptr()), ctypes.c_void_p(ctxs[i % 2].present_device(0)),
                           nbytes, 2, ctypes.c_void_p(streams[i % 2].cuda_stream))
    torch.cuda.synchronize()
    el_copy = time.perf_counter() - t1
    for c in ctxs:
        c.close()
    n_tri = sum(d.mesh.n_tris for d in sets[0][0])
    return {"frames": n * F, "ms_per_frame": round(el / (n * F) * 1e3, 5),
            "mtri_s": round(n_tri * n * F / el / 1e6, 3), "d2h_gb_s": round(n * nbytes / el / 1e9, 2),
            "d2h_only_gb_s": round(n * nbytes / el_copy / 1e9, 2), "bytes_per_frame": pf.width * pf.height * 4,
            "what": "render + D2H of every frame's RGBA8 SDL staging into pinned host memory, two contexts "
                    "alternating batches (D2H under the other context's render); PCIe-bound"}


def lib_workload(args, rank=0):
    from shs_gpu import scene_lib
    if args.config == "c4":
        return scene_lib.c4_scene(3840, 2160)
    return scene_lib.c5_scene(3840, 2160, 2048)


class LibSlot:
    """One frame in flight: a context with its own stream, workspace and targets (frames k, k + D, ...)."""

    def __init__(self, local_rank, dist, args=None):
        import shs_gpu
        self.ctx = shs_gpu.Context(local_rank)
        if dist is not None and args is not None and args.shard_layout == "regions":
            # one cost-balanced rectangle per rank (SHS_OPT_SHARD_LAYOUT); rank 0 also unpacks the gather
            self.ctx.set_shard_layout(True)
            self.ctx.set_shard_root_share(args.root_share)
        self.stream = None
        if dist is not None:
            # the gather is ordered on the context's own stream (wrapped for torch, not a new torch stream:
            # every extra stream shares the process's 4 hardware queues with the contexts' streams, which
            # cost the library legs 12 % at N = 1, profiles/r06_strong_gap.txt)
            import torch
            self.stream = torch.cuda.ExternalStream(self.ctx.stream, device=torch.device("cuda", local_rank))
        self.gbufs = [None]
        self.prepared = None
        self.gather_events = None   # [(start, end)] HIP events around each gather while timing

    def gather(self, dist):
        """The frame's owned present tiles into rank 0 over RCCL, ordered on this slot's stream."""
        import torch
        from shs_gpu import shard
        with torch.cuda.stream(self.stream):
            ev = None
            if self.gather_events is not None:
                ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                ev[0].record(self.stream)
            self.gbufs[0] = shard.gather_frame_device(dist, self.ctx, self.ctx.TARGET_LIB_PRESENT, stream=self.stream,
                                                      out=self.gbufs[0])
            if ev is not None:
                ev[1].record(self.stream)
                self.gather_events.append(ev)


def camera_phase_bytes(width, height, owned_px, shadow_size=None):
    """Algorithmic bytes of one camera pass's raster phase (k_lib_raster + k_lib_resolve) on one rank:
    per OWNED pixel HDR 16 + depth 4 + motion 8 + the fused tonemap's RGBA8 present 4 = 32 B (SURVEY
    8d); C5 adds the shadow map's PCF reads, 4 B/texel once, apportioned to the rank's pixel share.  At
    N = 1 owned_px = width * height; at N > 1 it is rank 0's share (shard.owned_pixels), the pixels
    rank 0's timed kernels actually produce."""
    b = owned_px * 32
    if shadow_size:
        b += shadow_size * shadow_size * 4 * owned_px // (width * height)
    return b


def rank_owned_pixels(ctx, frame, rank, world, regions_layout):
    """Pixels `rank` renders in the last camera pass of ctx (its region rectangle, or tile % world)."""
    from shs_gpu import shard
    if world <= 1:
        return frame.width * frame.height
    regions = ctx.shard_regions(world) if regions_layout else None
    return shard.owned_pixels(frame.width, frame.height, 32, rank, world, regions)


def shadow_pass_texels(ctx, S):
    """Texels the context's last shadow pass rendered (its footprint's 32x32 tiles, or the whole map)."""
    x0, y0, x1, y1 = ctx.shadow_region()
    if x1 < x0 or y1 < y0:
        return 0
    return (min(S, (x1 + 1) * 32) - x0 * 32) * (min(S, (y1 + 1) * 32) - y0 * 32)


def lib_timed_loop(args, slots, frame_fn, dist, frame=None, rank=0, world=1, on_last=None):
    """Warm-up, then exactly args.steps frames round-robin over the slots (frame i on slot i % D) between
    two barriers; then kernel event times of 20 frames on slot 0 alone (nothing else in flight: the
    roofline's kernel durations).  -> (elapsed s, stats, (n_frames, kms), pixels this rank owned in the
    timed kernels' passes)"""
    D = len(slots)

    def barrier_sync():
        for sl in slots:
            sl.ctx.synchronize_lib()
        if dist is not None:
            import torch
            torch.cuda.synchronize()
            dist.barrier()

    # clock ramp (as the legacy configs): untimed frames for args.ramp_ms of continuous rendering, so the
    # timed window starts at steady-state clocks whatever ran before it (a `--config` run starts on an idle
    # GPU, the strong legs after the C2 loop and their own host set-up)
    # (N > 1: every frame gathers, a collective, so all ranks render the same number of ramp frames -- the
    # loop goes on while any rank's clock says so)
    t_ramp, n_ramp = time.perf_counter(), 0
    more = True
    while more:
        for _ in range(D):
            frame_fn(slots[n_ramp % D])
            n_ramp += 1
        for sl in slots:
            sl.ctx.synchronize_lib()
        more = (time.perf_counter() - t_ramp) * 1e3 < getattr(args, "ramp_ms", 0.0)
        if dist is not None:
            import torch
            t = torch.tensor([1.0 if more else 0.0], dtype=torch.float64, device=args.reduce_device)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            more = bool(t.item() > 0.0)
    for i in range(max(args.warmup, D)):
        frame_fn(slots[i % D])
    barrier_sync()
    args.lib_ramp = {"ms": round((time.perf_counter() - t_ramp) * 1e3, 1), "frames": n_ramp}
    stats = slots[0].ctx.lib_stats()
    t0 = time.perf_counter()
    for i in range(args.steps):
        frame_fn(slots[i % D])
    barrier_sync()
    elapsed = time.perf_counter() - t0
    ctx = slots[0].ctx
    ctx.enable_timing(True)
    ctx.lib_timing_reset()
    if dist is not None:
        slots[0].gather_events = []
    for _ in range(20):
        frame_fn(slots[0])
    barrier_sync()
    n_passes, kms = ctx.lib_timing_read()
    ctx.enable_timing(False)
    if slots[0].gather_events:   # the gather's own time on the slot stream (rank 0: receives + unpack)
        kms = dict(kms, gather=float(np.mean([a.elapsed_time(b) for a, b in slots[0].gather_events])))
        slots[0].gather_events = None
    if on_last is not None:
        on_last(ctx)
    owned = None
    if frame is not None:
        owned = rank_owned_pixels(ctx, frame, rank, world, dist is not None and args.shard_layout == "regions")
    for sl in reversed(slots):   # borrowers first: slots 1.. read slot 0's meshes (shs_mesh_share)
        sl.ctx.close()
    return elapsed, stats, (n_passes["camera"], kms), owned


def share_meshes(args, sl, slots, meshes):
    """Frames in flight read one device copy of each mesh: every slot after the first borrows the first
    slot's buffers (shs_mesh_share) instead of uploading its own (--copy-meshes: one copy per slot)."""
    if slots and not args.copy_meshes:
        for m in meshes:
            sl.ctx.share_lib_mesh(slots[0].ctx, m)


def run_gpu_c4(args, rank, local_rank, world, dist):
    """C4 frame = Forward+ light-list binning (shs_light_cull) + PassPBRForward with the per-pixel
    point-light program over 1M triangles at 3840x2160 + PassTonemap into the RGBA8 present staging.
    N > 1: the frame's 32x32 tiles are sharded (tile % N == rank): every rank culls, renders and
    tonemaps only its tiles, and the owned present tiles (4 B/px) are gathered into rank 0 over RCCL
    every frame (strong scaling: the total work per step is one frame).  args.inflight contexts render
    consecutive frames round-robin (frames in flight, at every N alike)."""
    frame, draws, lights, cull = lib_workload(args, rank)
    if dist is not None:
        frame.shard_rank, frame.shard_count = rank, world
        cull.shard_rank, cull.shard_count = rank, world
    slots = []
    for _ in range(args.inflight):
        sl = LibSlot(local_rank, dist, args)
        share_meshes(args, sl, slots, [d.mesh for d in draws])
        sl.ctx.upload_lights(lights)
        sl.ctx.light_cull(cull)
        sl.prepared = sl.ctx.prepare_lib(frame, draws)
        sl.ctx.fuse_tonemap(1.0, 2.2, ldr=False, present=True)   # PassTonemap inside the pass's shading kernel
        slots.append(sl)

    def one_frame(sl):
        sl.ctx.light_cull(cull)
        sl.ctx.render_pbr_forward_prepared(sl.prepared)
        if dist is not None:
            sl.gather(dist)

    elapsed, stats, (n_cam, kms), owned = lib_timed_loop(args, slots, one_frame, dist, frame, rank, world)
    kms = {k: kms[k] for k in ("setup", "raster", "gather") if k in kms}
    n_tri = sum(d.mesh.n_tris for d in draws)
    # the raster phase writes HDR + depth + motion (28 B/px) and the fused tonemap's RGBA8 present staging
    # (4 B/px) for the pixels this rank owns
    B_cam_raster = camera_phase_bytes(frame.width, frame.height, owned)
    B_frame = n_tri * 72 + frame.width * frame.height * 32 + len(lights) * 160 + cull.n_lists * 4
    return frame, stats, elapsed, n_cam, kms, B_cam_raster, B_frame, n_tri, None, owned


def lib_mesh_bytes(mesh, with_attrs=True):
    """Indexed MeshData bytes read once: 12 B of indices per triangle + per vertex 12 B position
    (+ 12 B normal + 8 B uv for the camera pass)."""
    n_v = mesh.positions.shape[0]
    return mesh.n_tris * 12 + n_v * (32 if with_attrs else 12)


def run_gpu_lib(args, rank, local_rank, world, dist):
    """C5 frame = PassShadowMap + PassPBRForward + PassTonemap (present staging).  N > 1: tile-sharded
    like C4 -- the shadow map (every rank's PCF reads all of it) is rendered on every rank, the camera
    pass and the tonemap only on the rank's tiles, and the present tiles are gathered into rank 0.
    args.inflight contexts render consecutive frames round-robin."""
    import ctypes
    from shs_gpu import scene_lib, _abi
    frame, draws, casters, sun, S = lib_workload(args, 0)
    if dist is not None:
        frame.shard_rank, frame.shard_count = rank, world
    sd = (ctypes.c_float * 3)(*[float(x) for x in sun])
    slots = []
    for _ in range(args.inflight):
        sl = LibSlot(local_rank, dist, args)
        share_meshes(args, sl, slots, [d.mesh for d in draws] + [c.mesh for c in casters])
        ctx = sl.ctx
        # SHS_OPT_SHADOW_FOOTPRINT: the camera pass enqueues the shadow pass over only the shadow-map tiles
        # its pixels' PCF reads (every N alike; the images are the oracle's either way)
        ctx.set_shadow_footprint(not args.shadow_full)
        lvp = ctx.render_shadow_map(S, sun, casters)
        scene_lib.wire_shadow(draws, lvp)
        sl.prepared = ctx.prepare_lib(frame, draws)
        sl.carr = (_abi.ShadowCasterC * len(casters))()
        for i, c in enumerate(casters):
            sl.carr[i].mesh_id = ctx.upload_lib_mesh(c.mesh)
            for k in range(16):
                sl.carr[i].model[k] = float(c.model[k])
        ctx.fuse_tonemap(1.0, 2.2, ldr=False, present=True)   # PassTonemap inside the pass's shading kernel
        slots.append(sl)

    def one_frame(sl):
        sl.ctx._check(sl.ctx._lib.shs_render_shadow_map(sl.ctx._h, S, S, sd, sl.carr, len(casters), None))
        sl.ctx.render_pbr_forward_prepared(sl.prepared)
        if dist is not None:
            sl.gather(dist)

    shadow_texels = []
    elapsed, stats, (n_cam, kms), owned = lib_timed_loop(args, slots, one_frame, dist, frame, rank, world,
                                                         on_last=lambda ctx: shadow_texels.append(shadow_pass_texels(ctx, S)))
    B_cam_raster = camera_phase_bytes(frame.width, frame.height, owned, S)
    # the shadow map written and read once: the whole map, or the texels of the footprint the pass covered
    B_frame = (sum(lib_mesh_bytes(d.mesh) for d in draws) + sum(lib_mesh_bytes(c.mesh, False) for c in casters)
               + 2 * shadow_texels[0] * 4 + frame.width * frame.height * 32)
    n_tri = sum(d.mesh.n_tris for d in draws)
    return frame, stats, elapsed, n_cam, kms, B_cam_raster, B_frame, n_tri, (S, shadow_texels[0]), owned


def strong_roofline(frame_bytes, elapsed_max, frames, rank_cam_bytes, rank_cam_ms):
    """A strong leg's HBM roofline (north_star: the 1/2/4/8 numbers "as absolute numbers and as fraction
    of the HBM roofline"): the whole frame's algorithmic bytes (geometry, lights and lists,
    shadow map, 32 B per output pixel) per ms_per_frame, against N x 8 TB/s; and each rank's camera
    phase (k_lib_raster + k_lib_resolve, its owned pixels' 32 B, HIP events with one frame in flight)
    against one GPU's 8 TB/s."""
    world = len(rank_cam_ms)
    achieved = frame_bytes * frames / elapsed_max / 1e9
    cam = [b / (ms * 1e-3) / 1e9 if ms > 0 else 0.0 for b, ms in zip(rank_cam_bytes, rank_cam_ms)]
    return {"bound": "hbm", "unit": "GB/s", "peak": HBM_PEAK_GBS * world,
            "frame_algorithmic_bytes": int(frame_bytes),
            "achieved": round(achieved, 2), "frac": round(achieved / (HBM_PEAK_GBS * world), 4),
            "rank_camera_phase_frac": [round(c / HBM_PEAK_GBS, 4) for c in cam],
            "rank0_camera_phase_frac": round(cam[0] / HBM_PEAK_GBS, 4),
            "what": "frac: frame bytes x frames / wall time over N x 8 TB/s; camera phase: each rank's owned "
                    "pixels x 32 B (+ its share of the shadow map's PCF reads) / its k_lib_raster + k_lib_resolve "
                    "event time"}


def strong_summary(cfg, n_tri, frames, elapsed_max, rank_kernels_ms, rank_gather_ms, rank_owned, layout, inflight,
                   frame_bytes=None, rank_cam_bytes=None, rank_cam_ms=None, ramp=None):
    """One strong-scaling leg's keys (the 4K tile-sharded frame of north_star's >= 6x target) from the
    per-rank measurements rank 0 collected: frames per second over the whole job between two barriers,
    the worst rank's isolated camera-frame kernels, each rank's gather time and owned pixels, and the
    leg's roofline (strong_roofline)."""
    world = len(rank_kernels_ms)
    worst = int(np.argmax(rank_kernels_ms))
    extra = {}
    if frame_bytes is not None:
        extra["roofline"] = strong_roofline(frame_bytes, elapsed_max, frames, rank_cam_bytes, rank_cam_ms)
    if ramp is not None:
        extra["clock_ramp"] = ramp
    return dict(extra, **{
        "workload": WORKLOADS[cfg],
        "n_gpus": world,
        "frames": frames,
        "ms_per_frame": round(elapsed_max / frames * 1e3, 5),
        "mtri_s": round(n_tri * frames / elapsed_max / 1e6, 3),
        "worst_rank": worst,
        "worst_rank_kernels_ms": round(float(rank_kernels_ms[worst]), 5),
        "rank_kernels_ms": [round(float(x), 5) for x in rank_kernels_ms],
        "gather_ms": [round(float(x), 5) for x in rank_gather_ms],
        "owned_pixels": [int(x) for x in rank_owned],
        "layout": layout if world > 1 else "whole frame",
        "frames_in_flight": inflight,
        "what": "one frame per step split over the ranks (strong scaling): region-sharded camera pass + fused "
                "tonemap, RGBA8 present tiles gathered into rank 0 over RCCL every frame; ms_per_frame = max-over-"
                "ranks wall time between barriers / frames; kernels: each rank's shadow + camera pass kernels, "
                "one frame in flight (HIP events); gather: HIP events around the gather on the frame's stream",
    })


def strong_legs(args, rank, local_rank, world, dist):
    """The bounded C4 / C5 tile-sharded legs run after the headline C2 loop at every N (N = 1 is the
    denominator of the driver's 1 -> 8 curve): -> {"strong_c4": {...}, "strong_c5": {...}} on rank 0."""
    import copy
    out = {}
    for cfg in args.strong:
        a = copy.copy(args)
        a.config, a.steps, a.warmup = cfg, args.strong_frames, 20
        a.shard_layout, a.inflight = "regions", 3
        runner = run_gpu_c4 if cfg == "c4" else run_gpu_lib
        ok, err = 1.0, None
        try:
            frame, stats, elapsed, n_frames, kms, B_k, B_frame, n_tri, _, owned = runner(a, rank, local_rank, world, dist)
            k_ms = sum(v for k, v in kms.items() if k != "gather")
            mine = [elapsed, k_ms, kms.get("gather", 0.0), float(owned), float(B_k), kms.get("raster", 0.0)]
        except Exception as e:  # noqa: BLE001 -- every rank learns of it below, then all raise alike
            ok, err, mine = 0.0, e, [0.0] * 6
        if dist is not None:
            # a common status point before the data reduction: a leg that failed on some rank (after its
            # collectives) fails on every rank, instead of the others waiting in the reduction
            import torch
            st = torch.tensor([ok], dtype=torch.float64, device=args.reduce_device)
            dist.all_reduce(st, op=dist.ReduceOp.MIN)
            ok = float(st.item())
        if ok < 1.0:
            raise RuntimeError(f"strong leg {cfg} failed on " + (f"this rank: {err!r}" if err is not None else "another rank"))
        if dist is not None:
            t = torch.zeros((world, 6), dtype=torch.float64, device=args.reduce_device)
            t[rank] = torch.tensor(mine, dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.SUM)
            rows = t.cpu().numpy()
        else:
            rows = np.asarray([mine])
        out["strong_" + cfg] = strong_summary(cfg, n_tri, a.steps, float(rows[:, 0].max()), rows[:, 1], rows[:, 2],
                                              rows[:, 3], a.shard_layout, a.inflight, frame_bytes=B_frame,
                                              rank_cam_bytes=rows[:, 4], rank_cam_ms=rows[:, 5],
                                              ramp=getattr(a, "lib_ramp", None))
    return out


def strong_legs_guarded(args, rank, local_rank, world, dist):
    """strong_legs, but a failure that every rank hits alike (an error in the sharded legs, not in the
    headline) costs only the strong_* keys: the line then carries strong_error and the C2 value."""
    try:
        return strong_legs(args, rank, local_rank, world, dist)
    except Exception as e:  # noqa: BLE001 -- reported in the line
        print(f"bench: strong legs failed on rank {rank}: {e!r}", file=sys.stderr, flush=True)
        return {"strong_error": repr(e)[:300]}


def collect_pmc(args):
    """rocprofv3 --pmc child passes (one counter per pass: FETCH_SIZE costs 3 TCC slots and
    WRITE_SIZE 2, they do not fit together).  Returns bytes per dominant-phase dispatch (k_raster; for
    the library configs k_lib_raster<false> + k_lib_resolve, summed) or None."""
    exe = shutil.which("rocprofv3")
    if exe is None:
        return None, "rocprofv3 not found"
    out = {}
    kmatch = ("k_lib_raster<false,", "k_lib_resolve<") if args.config in LIB_CONFIGS else ("k_raster<",)
    tmp = tempfile.mkdtemp(prefix="shs_pmc_", dir=os.environ.get("TMPDIR", "/tmp"))
    try:
        for counter in ("FETCH_SIZE", "WRITE_SIZE"):
            d = os.path.join(tmp, counter)
            cmd = [exe, "--pmc", counter, "--output-format", "csv", "-d", d, "-o", "pmc", "--",
                   sys.executable, os.path.abspath(__file__), "--child", "--config", args.config,
                   "--steps", "20", "--warmup", "3", "--frames-per-step", str(args.frames_per_step)]
            r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, timeout=300, text=True)
            if r.returncode != 0:
                return None, f"rocprofv3 {counter} rc={r.returncode}: {r.stdout[-400:]}"
            files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
            if not files:
                return None, f"no counter_collection.csv for {counter}"
            vals = {k: [] for k in kmatch}
            for f in files:
                with open(f) as fh:
                    for row in csv.DictReader(fh):
                        for k in kmatch:
                            if k in row.get("Kernel_Name", "") and row.get("Counter_Name") == counter:
                                vals[k].append(float(row["Counter_Value"]))
            if not all(vals.values()):
                return None, f"no {kmatch} rows for {counter}"
            out[counter] = 0.0
            for v in vals.values():
                v = v[3:] if len(v) > 6 else v   # drop warmup dispatches
                out[counter] += sum(v) / len(v)
    except Exception as e:  # the measurement is optional; never fail the bench line over it
        return None, f"pmc failed: {e!r}"
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    # gfx950: FETCH_SIZE counts half the bytes of a wide coalesced read, WRITE_SIZE all of them (unit
    # KiB): measured with a 1 GiB streaming read / write, FETCH_SIZE 0.500x, WRITE_SIZE 1.000x
    # (tools/pmc_calibrate.py, profiles/r03_pmc_calibration.txt; MI355X_MICROARCH.md HBM section).
    traffic = (2.0 * out["FETCH_SIZE"] + out["WRITE_SIZE"]) * 1024.0
    return {"fetch_kib": out["FETCH_SIZE"], "write_kib": out["WRITE_SIZE"], "bytes": traffic}, None


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def hw_threads():
    """std::thread::hardware_concurrency() (the reference's worker count) and the cores this
    process may run on: its affinity set, capped by the cgroup CPU quota (cpu.max) when there is one --
    a container's share of a many-core host, which neither the affinity nor the core count shows."""
    hc = os.cpu_count() or 1
    try:
        usable = len(os.sched_getaffinity(0))
    except AttributeError:
        usable = hc
    q = cgroup_cpu_quota()
    if q is not None:
        usable = max(1, min(usable, int(q)))
    return hc, usable


def cgroup_cpu_quota():
    """Cores granted by the cgroup v2 CPU quota (cpu.max "quota period"), or None when unlimited."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        if quota == "max":
            return None
        return float(quota) / float(period)
    except (OSError, ValueError):
        return None


def _timed_frames(fn, seconds, max_frames=100000):
    """Run fn() until `seconds` of wall time (at least 2 frames): -> (frames, elapsed s, median ms)."""
    w0 = time.perf_counter()
    while time.perf_counter() - w0 < min(0.5, 0.1 * seconds):   # warm: thread pools, page faults
        fn()
    times = []
    t0 = time.perf_counter()
    while True:
        a = time.perf_counter()
        fn()
        times.append(time.perf_counter() - a)
        el = time.perf_counter() - t0
        if (el >= seconds and len(times) >= 2) or len(times) >= max_frames:
            break
    return len(times), el, 1e3 * float(np.median(times))


def cpu_baseline_lib(args):
    """The library-path oracle (PassShadowMap + PassPBRForward restated) on the box's host.  C5 uses the
    reference's row-parallel split of big bboxes (rasterizer.hpp:424-436) on hardware_concurrency
    threads; C4's 1M small triangles never reach that split's 128x128-pixel threshold, so the reference
    rasterises them on one thread and so does the baseline."""
    from oracle import oracle
    from shs_gpu import scene_lib
    hc, usable = hw_threads()
    if args.config == "c4":
        frame, draws, lights, cull = lib_workload(args, 0)
        n_tri = sum(d.mesh.n_tris for d in draws)

        def one():
            lists = oracle.light_cull(cull, lights)
            return oracle.forward_plus(frame, draws, lights, cull, lists[:2])
        frames, el, med = _timed_frames(one, args.cpu_seconds, 1000)
        return {"value": round(n_tri * frames / el / 1e6, 5), "unit": "Mtri/s", "cores": 1, "kind": "port",
                "median_ms_per_frame": round(med, 2), "cpu_model": cpu_model(),
                "hardware_concurrency": hc, "usable_cores": usable,
                "sample": f"{frames} full frame(s) of the same workload (light cull + Forward+ pass, "
                          f"{frame.width}x{frame.height}, {n_tri} tris, {len(lights)} lights), {el:.1f} s wall, "
                          "1 thread: no bbox reaches rasterize_mesh's row-parallel threshold "
                          "(oracle/shs_oracle_lib.c + shs_oracle_light.c, gcc -O3)"}
    frame, draws, casters, sun, S = lib_workload(args, 0)
    n_tri = sum(d.mesh.n_tris for d in draws)

    def one():
        sm, lvp = oracle.shadow_map(S, sun, casters)
        scene_lib.wire_shadow(draws, lvp)
        return oracle.pbr_forward(frame, draws, sm)
    oracle.set_lib_threads(hc)
    try:
        frames, el, med = _timed_frames(one, args.cpu_seconds, 1000)
    finally:
        oracle.set_lib_threads(1)
    return {"value": round(n_tri * frames / el / 1e6, 5), "unit": "Mtri/s", "cores": hc, "kind": "port",
            "median_ms_per_frame": round(med, 2), "cpu_model": cpu_model(), "hardware_concurrency": hc,
            "usable_cores": usable,
            "sample": f"{frames} frames of the same workload (shadow {S}^2 + {frame.width}x{frame.height} PBR, "
                      f"{n_tri} tris), {el:.1f} s wall, big bboxes row-parallel on {hc} threads as "
                      "rasterize_mesh's job-system split does (oracle/shs_oracle_lib.c, gcc -O3)"}


def cpu_baseline(args):
    """The oracle (CPU restatement of the reference tile-job path) on this host, bounded samples:
    hardware_concurrency workers (the headline), THREAD_COUNT=20 (the reference default,
    blinn_phong_shading.cpp:28) and the cores this process may use; C1 single-threaded."""
    if args.config in LIB_CONFIGS:
        return cpu_baseline_lib(args)
    from oracle import oracle
    hc, usable = hw_threads()
    frame, draws = build_workload(args.config, 0)
    n_tri = sum(d.mesh.n_tris for d in draws)
    _, depth, _ = oracle.render_legacy(frame.width, frame.height, draws, threads=1)
    covered = int((depth.view(np.uint32) != np.float32(np.finfo(np.float32).max).view(np.uint32)).sum())
    legs = [("single_thread", 1)] if args.config == "c1" else [("hardware_concurrency", hc), ("thread_count_20", 20),
                                                                ("usable_cores", usable)]
    # (the tile jobs run on a pool of persistent workers, as the reference's ThreadedPriorityJobSystem;
    # hardware_concurrency threads on a cgroup quota of fewer cores stall frames on descheduled workers)
    out = {}
    for name, threads in legs:
        frames, el, med = _timed_frames(
            lambda: oracle.render_legacy(frame.width, frame.height, draws, threads=threads), args.cpu_seconds / len(legs))
        out[name] = {"threads": threads, "frames": frames, "seconds": round(el, 2), "median_ms_per_frame": round(med, 3),
                     "mean_ms_per_frame": round(el / frames * 1e3, 3),
                     "mtri_s": round(n_tri * frames / el / 1e6, 4), "mpix_s": round(covered * frames / el / 1e6, 3)}
    # the headline is the fastest leg: the baseline the GPU is compared with is the CPU at its best
    # (hardware_concurrency oversubscribes a host whose process share is smaller than its core count)
    head_name = max(out, key=lambda k: out[k]["mtri_s"])
    head = out[head_name]
    quota = cgroup_cpu_quota()
    note = None
    if quota is not None and hc > quota:
        note = (f"hardware_concurrency ({hc}) workers on a cgroup CPU quota of {quota:g} cores: the persistent pool's "
                "frames stall on descheduled workers (median vs mean ms per frame in the legs), so that leg is slower "
                "than the quota-sized ones")
    return {"value": head["mtri_s"], "unit": "Mtri/s", "cores": head["threads"], "kind": "port",
            "median_ms_per_frame": head["median_ms_per_frame"], "mpix_s": head["mpix_s"], "cpu_model": cpu_model(),
            "hardware_concurrency": hc, "usable_cores": usable, "cgroup_cpu_quota": quota, "note": note, "legs": out,
            "sample": f"{head['frames']} frames of the same workload ({frame.width}x{frame.height}, {n_tri} tris, "
                      f"{covered} covered px) in {head['seconds']} s, 80x80 tile jobs on {head['threads']} threads "
                      f"({head_name}; oracle/shs_oracle.c, gcc -O3)"}


def launch_ranks(args):
    """`--gpus N` without a launcher: run this script under torch.distributed.run with N processes on
    this node (rendezvous on 127.0.0.1, a free port), the same command line the driver uses for N > 1.
    The parent never initialises the GPU; its exit status is the launcher's."""
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.run(cmd, env=env).returncode


def launch_dry_run(world, rank, local_rank):
    """The launcher check of tests/test_bench_launch.py: gloo group, no GPU, rank 0 prints one line."""
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo")
    assert dist.get_world_size() == world
    t = torch.tensor([rank, local_rank], dtype=torch.int64)
    outs = [torch.zeros(2, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(outs, t)
    if rank == 0:
        print(json.dumps({"world": world, "ranks": [int(o[0]) for o in outs], "local_ranks": [int(o[1]) for o in outs]}),
              flush=True)
    dist.barrier()
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", default="c2", choices=sorted(WORKLOADS))
    ap.add_argument("--frames-per-step", type=int, default=0,
                    help="legacy configs: frames per shs_render_legacy_batch step (default 128 for c1/c2, 16 for c3; C2 measured 64 / 128 / 256: 230 / 248 / 255 Mtri/s, DESIGN.md 6)")
    ap.add_argument("--inflight", type=int, default=3,
                    help="c4/c5: frames in flight (contexts rendering consecutive frames round-robin)")
    ap.add_argument("--copy-meshes", action="store_true",
                    help="c4/c5: every frame-in-flight context uploads its own mesh copies (default: one copy, shared)")
    ap.add_argument("--shard-layout", default="regions", choices=["regions", "interleaved"],
                    help="c4/c5 at N > 1: tile ownership (one cost-balanced rectangle per rank, or tile %% N)")
    ap.add_argument("--root-share", type=float, default=0.85,
                    help="c4/c5 regions: rank 0's share of the predicted cost (it also unpacks the gather)")
    ap.add_argument("--pipeline", type=int, default=0, choices=[0, 1],
                    help="legacy configs: SHS_OPT_LEGACY_PIPELINE for the timed batches (each batch's raster in the "
                         "next batch's launch; eligible: multi-draw scan-mode batches, i.e. C1 / C2).  Off: measured "
                         "slower (C2 0.328 vs 0.284 ms/step: the fused kernel spills 120 B/lane, DESIGN.md 4)")
    ap.add_argument("--ramp-ms", type=float, default=60.0,
                    help="untimed rendering before the warm-up so the GPU clocks reach steady state (every config and strong leg)")
    ap.add_argument("--shadow-full", action="store_true",
                    help="c5: render the whole shadow map every frame (default: the camera pass's footprint, "
                         "SHS_OPT_SHADOW_FOOTPRINT)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--strong", default="c4,c5", type=lambda x: [c for c in x.split(",") if c],
                    help="legacy configs: the tile-sharded 4K legs run after the headline loop at every N "
                         "(strong_c4 / strong_c5 keys; '' to skip)")
    ap.add_argument("--strong-frames", type=int, default=200, help="timed frames of each strong leg")
    ap.add_argument("--no-pmc", action="store_true")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-single", action="store_true", help="skip the single-frame latency leg (profiling)")
    ap.add_argument("--no-pcie", action="store_true", help="skip the PCIe-inclusive Seam-1 leg")
    ap.add_argument("--child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--debug-flags", type=lambda x: int(x, 0), default=0, help=argparse.SUPPRESS)
    ap.add_argument("--raster-mode", type=int, default=0, help="legacy path: 0 auto, 1 scan, 2 bins")
    ap.add_argument("--raster-loop", type=int, default=-1, help="legacy path: 0 per-pixel, 1 pair tasks (default)")
    ap.add_argument("--launch-dry-run", action="store_true",
                    help="rank launcher check: every rank joins a gloo group and rank 0 prints the ranks (no GPU)")
    args = ap.parse_args()
    if args.frames_per_step <= 0:
        args.frames_per_step = LEGACY_FRAMES.get(args.config, 1)

    if "WORLD_SIZE" not in os.environ and args.gpus > 1 and not args.child:
        # `python bench.py --gpus N` started directly: start the N ranks as child processes (one per
        # GPU) before this process touches the GPU, and exit with their status
        sys.exit(launch_ranks(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal of the N-rank path on a one-GPU box (tests only: every rank on device 0, gloo for the
    # barrier and the max-over-ranks reduction); never used for a reported line
    rehearse = os.environ.get("SHS_BENCH_REHEARSE") == "1"
    if rehearse:
        local_rank = 0
    args.reduce_device = "cpu" if rehearse else f"cuda:{local_rank}"   # where the timing reductions run
    if not args.child and world != args.gpus:
        raise SystemExit(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}; launch with --nproc-per-node equal to --gpus")

    if args.launch_dry_run:
        return launch_dry_run(world, rank, local_rank)

    if args.child:  # profiled child: just render
        {"c4": run_gpu_c4, "c5": run_gpu_lib}.get(args.config, run_gpu)(args, 0, 0, 1, None)
        return

    pmc, pmc_err = (None, "skipped")
    if world == 1 and not args.no_pmc:
        pmc, pmc_err = collect_pmc(args)   # before this process initialises the GPU

    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist_mod
        torch.cuda.set_device(local_rank)
        dist_mod.init_process_group("gloo" if rehearse else "nccl")
        dist = dist_mod

    if args.config in LIB_CONFIGS:
        return main_lib(args, world, rank, local_rank, dist, pmc, pmc_err)
    frame, sets, stats, elapsed, n_launches, kms, single, ramp = run_gpu(args, rank, local_rank, world, dist)
    draws = sets[0][0]
    # the strong-scaling legs ride on the headline configuration's line (the driver's `--gpus N` run)
    strong = strong_legs_guarded(args, rank, local_rank, world, dist) if args.strong and not args.child and args.config == "c2" else {}
    pcie = None   # (last: seam1_pcie)
    if args.frames_per_step > 1 and world == 1 and not args.child and not args.no_pcie:
        pcie = seam1_pcie(args, frame, sets)
    B1, n_tri1 = algorithmic_bytes(frame, draws)
    F = args.frames_per_step
    B, n_tri = B1 * F, n_tri1 * F          # per step (= per k_raster launch)

    el_max = elapsed
    covered = stats["covered_pixels"]       # batch total
    if dist is not None:
        import torch
        t = torch.tensor([elapsed], dtype=torch.float64, device=args.reduce_device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el_max = float(t.item())
        c = torch.tensor([covered], dtype=torch.float64, device=args.reduce_device)
        dist.all_reduce(c, op=dist.ReduceOp.SUM)
        covered_total = float(c.item())
    else:
        covered_total = float(covered)

    if rank != 0:
        if dist is not None:
            dist.barrier()
            dist.destroy_process_group()
        return

    steps = args.steps
    value = world * n_tri * steps / el_max / 1e6     # n_tri = triangles per step (F frames)
    mpix = covered_total * steps / el_max / 1e6
    t_raster_ms = kms["raster"]
    achieved = B / (t_raster_ms * 1e-3) / 1e9 if t_raster_ms > 0 else None
    roofline = {
        "kernel": "k_raster",
        "bound": "hbm",
        "achieved": round(achieved, 2) if achieved else None,
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
        "frac": round(achieved / HBM_PEAK_GBS, 4) if achieved else None,
        "traffic": round(pmc["bytes"]) if pmc else None,
        "traffic_raw_kib": {"fetch_size": round(pmc["fetch_kib"]), "write_size": round(pmc["write_kib"])} if pmc else None,
        "algorithmic_bytes": B,
        "kernel_ms": round(t_raster_ms, 5),
    }
    # the whole step's device time (k_setup + k_raster) against the same bytes, and the driver-timed
    # step (wall clock between the barriers, host enqueue included)
    t_frame_ms = kms.get("setup", 0.0) + t_raster_ms
    if t_frame_ms > 0:
        roofline["frame_kernels_ms"] = round(t_frame_ms, 5)
        roofline["frame_frac"] = round(B / (t_frame_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
    roofline["step_achieved"] = round(world * B * steps / el_max / 1e9, 2)
    roofline["step_frac"] = round(world * B * steps / el_max / 1e9 / HBM_PEAK_GBS / world, 4)
    if pmc is None:
        roofline["traffic_note"] = pmc_err
    line = {
        "metric": METRIC,
        "value": round(value, 3),
        "unit": "Mtri/s",
        "n_gpus": world,
        "steps": steps,
        "warmup": args.warmup,
        "ms_per_step": round(el_max / steps * 1e3, 5),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic: Suzanne soup from the reference's assets/obj/monkey/monkey.rawobj (967 tris), "
                "reference scene constants (camera (0,5,-20) fov60, light, colour)",
        "config": {"workload": WORKLOADS[args.config], "width": frame.width, "height": frame.height,
                   "tris_per_frame": n_tri1, "frames_per_step_per_gpu": F,
                   "pose_sets": POSE_SETS, "legacy_pipeline": bool(args.pipeline),
                   "parallelism": f"frame-parallel x{world}" if world > 1 else "single GPU"},
        "shaded_mpix_s": round(mpix, 3),
        "batch_stats": stats,
        "kernels_ms": {k: round(v, 5) for k, v in kms.items()},
        "timed_launches_with_events": n_launches,
        "roofline": roofline,
    }
    line["clock_ramp"] = dict(ramp, what="untimed batches before the warm-up: steady-state GPU clocks")
    if single:
        line["single_frame"] = single
    if pcie is not None:
        line["seam1_pcie"] = pcie
    line.update(strong)
    if world == 1 and not args.no_cpu:
        line["cpu_baseline"] = cpu_baseline(args)
    print(json.dumps(line), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


def main_lib(args, world, rank, local_rank, dist, pmc, pmc_err):
    runner = run_gpu_c4 if args.config == "c4" else run_gpu_lib
    frame, stats, elapsed, n_frames, kms, B_k, B_frame, n_tri, shadow, owned = runner(args, rank, local_rank, world, dist)
    S, shadow_texels = shadow if shadow else (None, 0)
    world_tri = n_tri              # one frame per step, split over the ranks at N > 1 (strong scaling)
    el_max = elapsed
    covered_total = float(stats["covered_pixels"])
    if dist is not None:
        import torch
        t = torch.tensor([elapsed], dtype=torch.float64, device=args.reduce_device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el_max = float(t.item())
        c = torch.tensor([covered_total], dtype=torch.float64, device=args.reduce_device)
        dist.all_reduce(c, op=dist.ReduceOp.SUM)
        covered_total = float(c.item())
    if rank != 0:
        if dist is not None:
            dist.barrier()
            dist.destroy_process_group()
        return
    steps = args.steps
    t_k = kms["raster"]
    achieved = B_k / (t_k * 1e-3) / 1e9 if t_k > 0 else None
    t_frame = sum(v for k, v in kms.items() if k != "gather")
    # at N > 1 the timed kernels are rank 0's: its frame bytes are the whole frame's minus the 32 B of
    # every pixel another rank renders (geometry and the shadow map are still read whole on every rank)
    B_frame -= (frame.width * frame.height - owned) * 32
    roofline = {"kernel": "k_lib_raster<false> + k_lib_resolve (camera pass raster phase: coverage, then shading + "
                          "fused tonemap)", "bound": "hbm",
                "achieved": round(achieved, 2) if achieved else None, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4) if achieved else None,
                "traffic": round(pmc["bytes"]) if pmc else None,
                "traffic_raw_kib": {"fetch_size": round(pmc["fetch_kib"]), "write_size": round(pmc["write_kib"])} if pmc else None,
                "algorithmic_bytes": B_k,
                "kernel_ms": round(t_k, 5), "frame_kernels_ms": round(t_frame, 5),
                "rank0_owned_pixels": owned,
                "frame_algorithmic_bytes": B_frame,
                "frame_frac": round(B_frame / (t_frame * 1e-3) / 1e9 / HBM_PEAK_GBS, 4) if t_frame > 0 else None}
    if pmc is None:
        roofline["traffic_note"] = pmc_err
    c4 = args.config == "c4"
    if c4:
        data = ("synthetic: 1000 seeded objects x 1000 small triangles (seed 0x5EED), 256 point lights (seed 0x11A7, "
                "range U[2,8], Smooth attenuation), 16-px tiles, max 128 lights per tile")
        parallelism = (f"tile-sharded x{world} ({args.shard_layout}) + RCCL gather of RGBA8 present tiles to rank 0"
                       if world > 1 else "single GPU")
    else:
        data = ("synthetic: Suzanne (indexed from the reference's monkey.rawobj) + make_plane floor, reference "
                "defaults (sun normalize(0.4668,-0.3487,0.8127), intensity 5, PCF 2, bias 0.0008/0.0015)")
        shadow_how = ("the whole shadow map on every rank" if args.shadow_full else
                      "each rank's shadow pass over its own PCF footprint, no shadow-map exchange")
        parallelism = (f"tile-sharded x{world} ({args.shard_layout}; {shadow_how}) + RCCL gather of RGBA8 "
                       "present tiles to rank 0") if world > 1 else "single GPU"
    line = {
        "metric": METRIC, "value": round(world_tri * steps / el_max / 1e6, 3), "unit": "Mtri/s", "n_gpus": world,
        "steps": steps, "warmup": args.warmup, "ms_per_step": round(el_max / steps * 1e3, 5), "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "f32", "data": data,
        "config": {"workload": WORKLOADS[args.config], "width": frame.width, "height": frame.height,
                   "shadow_map": S, "tris_per_frame": n_tri, "frames_per_step_per_gpu": 1,
                   "shadow_pass": None if S is None else (
                       "whole map" if args.shadow_full else
                       f"footprint of the camera pass's PCF reads (SHS_OPT_SHADOW_FOOTPRINT): {shadow_texels} of "
                       f"{S * S} texels on rank 0"),
                   "frames_in_flight": args.inflight, "parallelism": parallelism},
        "shaded_mpix_s": round(covered_total * steps / el_max / 1e6, 3),
        "frame_stats": stats, "kernels_ms": {k: round(v, 5) for k, v in kms.items()},
        "kernel_timing": f"{n_frames} frames on one context alone after the timed loop (HIP events)",
        "roofline": roofline,
        "clock_ramp": dict(getattr(args, "lib_ramp", {}), what="untimed frames before the warm-up: steady-state GPU clocks"),
    }
    if world == 1 and not args.no_cpu:
        line["cpu_baseline"] = cpu_baseline(args)
    print(json.dumps(line), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
