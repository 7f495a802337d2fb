"""Store rates on this GPU (timing tool): torch fill_ of a 2 GiB tensor, and tools/store_probe.hip's
kernels -- a linear 16-B fill and the legacy clear-strip write pattern in isolation (C2's 128 frames of
1920x1080 colour + depth, 2.12 GB) by store kind, strip order, strip height, grid and item dealing --
timed with HIP events over repeats.  The ceiling the legacy raster's clear path is compared with
(DESIGN.md section 4).  usage (GPU box): python tools/store_rate.py  (tools/store_probe.sh builds the
probe library first, on the CPU)"""
import ctypes
import os

import torch

REPS = 10


def timed(fn):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(REPS):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / REPS


def main():
    n = (2 << 30) // 4
    x = torch.empty(n, dtype=torch.float32, device="cuda:0")
    ms = timed(lambda: x.fill_(1.0))
    print(f"torch fill_ 2 GiB: {ms:.3f} ms, {n * 4 / ms / 1e9:.2f} TB/s")
    del x
    lib_path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libstore_probe.so")
    if not os.path.exists(lib_path):
        print("no", lib_path)
        return
    lib = ctypes.CDLL(lib_path)
    F, W, H = 128, 1920, 1080
    plane = F * W * H
    buf = torch.empty(2 * plane, dtype=torch.int32, device="cuda:0")
    color, depth = buf.data_ptr(), buf.data_ptr() + plane * 4
    ticket = torch.zeros(1, dtype=torch.int32, device="cuda:0")
    stream = torch.cuda.current_stream().cuda_stream
    B = 2 * plane * 4
    queues = torch.zeros(16 * 64, dtype=torch.int32, device="cuda:0")
    for nt in (1, 0):
        for kind, grid, c16 in ((0, 1024, 0), (0, 4096, 0), (1, 0, 0), (2, 1024, 1024), (2, 1024, 2048), (2, 1024, 4096),
                                (2, 2048, 1024), (2, 2048, 4096)):
            def go():
                queues.zero_()
                r = lib.probe_fill_var(ctypes.c_void_p(buf.data_ptr()), ctypes.c_size_t(B), kind, grid, c16, nt,
                                       ctypes.c_void_p(queues.data_ptr()), ctypes.c_void_p(stream))
                assert r == 0, r
            ms = timed(go)
            name = ("grid-stride x4", "non-persistent 4x4KB spread", "16 queues")[kind]
            print(f"fill {name} grid {grid} chunk {c16 * 16 // 1024} KB nt {nt}: {ms:.3f} ms {B / ms / 1e9:.2f} TB/s", flush=True)
    for sr in (64, 8):
        for mode in (0, 2):
            for nt in (1, 0):
                def go():
                    r = lib.probe_strips(ctypes.c_void_p(color), ctypes.c_void_p(depth), F, W, H, sr, F * ((H + sr - 1) // sr), nt, mode, 0,
                                         ctypes.c_void_p(ticket.data_ptr()), ctypes.c_void_p(stream))
                    assert r == 0, r
                ms = timed(go)
                print(f"strips non-persistent SR {sr:3d} mode {mode} nt {nt}: {ms:.3f} ms {B / ms / 1e9:.2f} TB/s", flush=True)


if __name__ == "__main__":
    main()
