"""Time one gloo point-to-point transfer of a CUDA tensor between two ranks on one GPU (what
bench.py's SHS_BENCH_REHEARSE=1 sharded gather does in place of RCCL).
usage (GPU box): python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 tools/diag_gloo_p2p.py [MiB]"""
import sys
import time

import torch
import torch.distributed as dist


def main():
    dist.init_process_group("gloo")
    rank = dist.get_rank()
    n = int(float(sys.argv[1] if len(sys.argv) > 1 else 4) * (1 << 20) / 4)
    for dev in ("cpu", "cuda:0"):
        t = torch.zeros(n, dtype=torch.int32, device=dev)
        times = []
        for _ in range(5):
            dist.barrier()
            t0 = time.perf_counter()
            ops = [dist.P2POp(dist.irecv if rank == 0 else dist.isend, t, 1 - rank)]
            for q in dist.batch_isend_irecv(ops):
                q.wait()
            if dev != "cpu":
                torch.cuda.synchronize()
            times.append((time.perf_counter() - t0) * 1e3)
        if rank == 0:
            print(f"{dev}: {n * 4 / 1e6:.1f} MB gloo p2p ms: " + " ".join(f"{x:.1f}" for x in times), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
