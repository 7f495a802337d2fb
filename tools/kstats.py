"""Per-kernel dispatch statistics (count, median, mean, max in us) from a rocprofv3 results database
(rocprofv3 --kernel-trace -d DIR -o NAME ...).  usage: python tools/kstats.py DIR_OR_DB [name filter]"""
import glob
import os
import sqlite3
import sys

import numpy as np


def main():
    path = sys.argv[1]
    flt = sys.argv[2] if len(sys.argv) > 2 else ""
    dbs = [path] if path.endswith(".db") else glob.glob(os.path.join(path, "**", "*.db"), recursive=True)
    for db in dbs:
        c = sqlite3.connect(db)
        rows = c.execute("select name, end - start from kernels").fetchall()
        by = {}
        for name, dur in rows:
            by.setdefault(name, []).append(dur / 1e3)
        print(db)
        for name, v in sorted(by.items(), key=lambda kv: -np.sum(kv[1])):
            if flt and flt not in name:
                continue
            v = np.array(v)
            print(f"  {name[:70]:70s} n={len(v):5d} median={np.median(v):9.2f} mean={v.mean():9.2f} max={v.max():9.2f} us")


if __name__ == "__main__":
    main()
