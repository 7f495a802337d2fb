"""Gaps between consecutive kernels in a rocprofv3 --kernel-trace CSV (run_kernel_trace.csv): where a
step's wall time goes outside the kernels.  usage: python tools/trace_gaps.py <kernel_trace.csv> [skip]"""
import csv
import sys
from collections import defaultdict

import numpy as np


def short(name):
    for k in ("k_setup", "k_ghost", "k_raster", "k_lib_setup", "k_lib_raster", "k_light", "k_tonemap", "k_tiles", "k_occ"):
        if k in name:
            return k
    return name[:24]


def main():
    path = sys.argv[1]
    skip = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    rows = []
    with open(path) as fh:
        for r in csv.DictReader(fh):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])))
    rows.sort()
    rows = rows[skip:]
    dur = defaultdict(list)
    gaps = defaultdict(list)
    for i, (s, e, n) in enumerate(rows):
        dur[n].append((e - s) / 1e3)
        if i:
            gaps[(rows[i - 1][2], n)].append((s - rows[i - 1][1]) / 1e3)
    print(f"{len(rows)} dispatches, span {(rows[-1][1] - rows[0][0]) / 1e3:.1f} us")
    for n, v in dur.items():
        print(f"  {n:14s} n={len(v):5d} mean {np.mean(v):9.2f} us  median {np.median(v):9.2f}  min {np.min(v):9.2f}  max {np.max(v):9.2f}")
    for (a, b), v in gaps.items():
        print(f"  gap {a:>12s} -> {b:12s} n={len(v):5d} mean {np.mean(v):8.2f} us  median {np.median(v):8.2f}  p90 {np.percentile(v, 90):8.2f}")


if __name__ == "__main__":
    main()
