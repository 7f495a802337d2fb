"""Text timeline of a rocprofv3 kernel trace (csv): the last K dispatches, one line each (start offset,
duration, queue, name), and the fraction of the window in which at least one kernel ran.
usage: python tools/trace_timeline.py DIR [K]"""
import csv
import glob
import os
import sys


def main():
    path = sys.argv[1]
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 60
    rows = []
    for f in glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Queue_Id", r.get("Stream_Id", "?")),
                             r["Kernel_Name"]))
    rows.sort()
    rows = rows[-k:]
    t0 = rows[0][0]
    busy, cur_s, cur_e = 0, None, None
    for s, e, q, name in rows:
        print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f} q{q:>3} {name[:70]}")
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    span = max(e for _, e, _, _ in rows) - t0
    print(f"window {span / 1e3:.1f} us, busy {busy / span:.3f}")


if __name__ == "__main__":
    main()
