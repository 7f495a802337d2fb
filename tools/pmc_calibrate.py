"""Calibration of the TCC FETCH_SIZE / WRITE_SIZE counters bench.py converts into HBM traffic: a
streaming read (torch sum over a 1 GiB float32 tensor) and a streaming write (fill_ of the same tensor),
each byte touched once, under rocprofv3 --pmc.  Prints counter KiB x 1024 / bytes moved per kernel.
usage (GPU box): python tools/pmc_calibrate.py            (runs the two rocprofv3 passes itself)
                 python tools/pmc_calibrate.py --child   (the profiled workload)"""
import csv
import glob
import os
import subprocess
import sys
import tempfile

NBYTES = 1 << 30


def child():
    import torch
    x = torch.ones(NBYTES // 4, dtype=torch.float32, device="cuda:0")
    torch.cuda.synchronize()
    for _ in range(3):
        x.fill_(2.0)
        s = x.sum()
    torch.cuda.synchronize()
    print(float(s))


def main():
    if "--child" in sys.argv:
        return child()
    tmp = tempfile.mkdtemp(prefix="pmc_cal_", dir=os.environ.get("TMPDIR", "/tmp"))
    for counter in ("FETCH_SIZE", "WRITE_SIZE"):
        d = os.path.join(tmp, counter)
        r = subprocess.run(["rocprofv3", "--pmc", counter, "--output-format", "csv", "-d", d, "-o", "pmc", "--",
                            sys.executable, os.path.abspath(__file__), "--child"], stdout=subprocess.PIPE,
                           stderr=subprocess.STDOUT, text=True, timeout=120)
        if r.returncode != 0:
            print(r.stdout[-2000:])
            return 1
        rows = []
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(f) as fh:
                rows += [row for row in csv.DictReader(fh) if row.get("Counter_Name") == counter]
        by = {}
        for row in rows:
            by.setdefault(row["Kernel_Name"][:80], []).append(float(row["Counter_Value"]))
        for name, v in by.items():
            mean = sum(v[1:]) / max(len(v) - 1, 1) if len(v) > 1 else v[0]
            print(f"{counter:10s} {name:80s} n={len(v)} mean {mean:.0f} KiB = {mean * 1024 / NBYTES:.3f} x {NBYTES} B")
    return 0


if __name__ == "__main__":
    sys.exit(main())
