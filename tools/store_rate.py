"""Reference store rate on this GPU: torch fill_ of a 2 GiB tensor (one streaming write of every byte),
timed with HIP events over 20 repeats -- the ceiling the legacy raster's clear path is compared with
(DESIGN.md section 4).  usage (GPU box): python tools/store_rate.py"""
import torch


def main():
    n = (2 << 30) // 4
    x = torch.empty(n, dtype=torch.float32, device="cuda:0")
    for v in (1.0, 2.0, 3.0):
        x.fill_(v)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for i in range(20):
        x.fill_(float(i))
    b.record()
    torch.cuda.synchronize()
    ms = a.elapsed_time(b) / 20
    print(f"fill_ 2 GiB: {ms:.3f} ms per fill, {x.numel() * 4 / ms / 1e9:.2f} TB/s")


if __name__ == "__main__":
    main()
