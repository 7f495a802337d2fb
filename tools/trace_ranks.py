"""Per-rank kernel durations of a sharded experiment run under rocprofv3 --kernel-trace (csv): each
kernel's dispatches, in start order, split into N equal consecutive chunks (tools/exp_pipeline.py and
exp_shard_split.py render rank 0's frames, then rank 1's, ...), median us per chunk.
usage: python tools/trace_ranks.py DIR N [name filter]"""
import csv
import glob
import os
import sys

import numpy as np


def main():
    path, n = sys.argv[1], int(sys.argv[2])
    flt = sys.argv[3] if len(sys.argv) > 3 else ""
    rows = []
    for f in glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True):
        with open(f) as fh:
            rows += [(int(r["Start_Timestamp"]), r["Kernel_Name"], int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
                     for r in csv.DictReader(fh)]
    rows.sort()
    by = {}
    for _, name, dur in rows:
        by.setdefault(name, []).append(dur / 1e3)
    for name, v in sorted(by.items(), key=lambda kv: -sum(kv[1])):
        if flt not in name or len(v) < n:
            continue
        k = len(v) // n
        med = [float(np.median(v[i * k:(i + 1) * k])) for i in range(n)]
        print(f"{name[:60]:60s} " + " ".join(f"{m:7.1f}" for m in med))


if __name__ == "__main__":
    main()
