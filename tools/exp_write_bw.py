"""Write-only HBM bandwidth of this box (the ceiling of C2's clear-dominated k_raster): torch fill_ and
hipMemsetAsync over 1 GiB, event-timed."""
import ctypes
import json
import sys

sys.path.insert(0, "leisure-software-renderer_amd")


def main():
    from shs_gpu import _abi
    _abi.load()
    import torch
    hip = ctypes.CDLL("libamdhip64.so.7")
    hip.hipMemsetAsync.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p]
    n = 1 << 30
    x = torch.empty(n, dtype=torch.uint8, device="cuda")
    out = {}
    for name, fn in (("torch_fill", lambda: x.fill_(7)),
                     ("hipMemsetAsync", lambda: hip.hipMemsetAsync(ctypes.c_void_p(x.data_ptr()), 0, n,
                                                                   ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)))):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 20
        out[name] = round(n / (ms * 1e-3) / 1e12, 3)
    print(json.dumps({"write_TB_s": out}))


if __name__ == "__main__":
    main()
