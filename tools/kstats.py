"""Per-kernel dispatch statistics (count, median, mean, max in us) from a rocprofv3 results database
(rocprofv3 --kernel-trace -d DIR -o NAME ...).
usage: python tools/kstats.py DIR_OR_DB [name filter] [--skip-first K] [--last K]
--skip-first K drops each kernel's first K dispatches (the warm-up launches before the timed loop)."""
import csv
import glob
import os
import sqlite3
import sys

import numpy as np


def main():
    path = sys.argv[1]
    args = [a for a in sys.argv[2:]]
    skip = 0
    if "--skip-first" in args:
        i = args.index("--skip-first")
        skip = int(args[i + 1])
        del args[i:i + 2]
    last = 0
    if "--last" in args:   # only each kernel's last K dispatches (bench.py's isolated kernel-timing leg)
        i = args.index("--last")
        last = int(args[i + 1])
        del args[i:i + 2]
    flt = args[0] if args else ""
    dbs = [path] if path.endswith(".db") else glob.glob(os.path.join(path, "**", "*.db"), recursive=True)
    dbs += glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True)
    for db in dbs:
        if db.endswith(".csv"):   # rocprofv3 --output-format csv
            with open(db) as f:
                tr = sorted(csv.DictReader(f), key=lambda r: int(r["Start_Timestamp"]))
            rows = [(r["Kernel_Name"], int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) for r in tr]
        else:
            c = sqlite3.connect(db)
            rows = c.execute("select name, end - start from kernels order by start").fetchall()
        by = {}
        for name, dur in rows:
            by.setdefault(name, []).append(dur / 1e3)
        print(db)
        for name, v in sorted(by.items(), key=lambda kv: -np.sum(kv[1])):
            if flt and flt not in name:
                continue
            v = np.array(v[skip:] if len(v) > skip else v)
            if last and len(v) > last:
                v = v[-last:]
            print(f"  {name[:70]:70s} n={len(v):5d} median={np.median(v):9.2f} mean={v.mean():9.2f} max={v.max():9.2f} us")


if __name__ == "__main__":
    main()
