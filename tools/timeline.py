"""Per-workgroup timeline of one frame (SHS_OPT_TIMELINE): where each kernel's time goes.

usage (GPU box): python tools/timeline.py [c2|c1|c3] [debug_flags]
(debug_flags act only in the experiments build: SHS_GPU_LIB=leisure-software-renderer_amd/shs_gpu/libshs_gpu_exp.so)
Prints, per kernel and block role, start/end offsets (us) relative to the first k_setup workgroup
start, and duration percentiles."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "leisure-software-renderer_amd"), ROOT]
import shs_gpu  # noqa: E402
from shs_gpu import scene  # noqa: E402


def summarize(name, se, t0):
    if len(se) == 0:
        return
    st = (se[:, 0].astype(np.int64) - t0) / 100.0   # 100 MHz ticks -> us
    en = (se[:, 1].astype(np.int64) - t0) / 100.0
    du = en - st
    print(f"  {name:8s} n={len(se):5d} start[min/med/max]={st.min():7.2f}/{np.median(st):7.2f}/{st.max():7.2f}"
          f"  end[med/max]={np.median(en):7.2f}/{en.max():7.2f}  dur[med/p90/max]={np.median(du):6.2f}/"
          f"{np.percentile(du, 90):6.2f}/{du.max():6.2f} us")


def phases(se, names, label):
    """Phase marks (slots 2..) of the slowest workgroup and the median over workgroups that ran them,
    in us after the workgroup start."""
    if len(se) == 0:
        return
    dur = se[:, 1].astype(np.int64) - se[:, 0].astype(np.int64)
    k = int(np.argmax(dur))
    def rel(row):
        return ["%s=%.2f" % (n, (int(row[2 + i]) - int(row[0])) / 100.0) if row[2 + i] else "%s=-" % n
                for i, n in enumerate(names)]
    print(f"  {label} slowest wg {k} ({dur[k] / 100:.2f} us): " + " ".join(rel(se[k])))
    ran = se[se[:, 2 + len(names) - 1] != 0] if len(names) > 1 else se
    if len(ran):
        med = [np.median((ran[:, 2 + i].astype(np.int64) - ran[:, 0].astype(np.int64))[ran[:, 2 + i] != 0]) / 100.0
               if (ran[:, 2 + i] != 0).any() else float("nan") for i in range(len(names))]
        print(f"  {label} median of {len(ran)} wgs: " + " ".join("%s=%.2f" % (n, m) for n, m in zip(names, med)))


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c2"
    flags = int(sys.argv[2], 0) if len(sys.argv) > 2 else 0
    frame, draws = scene.config(cfg)
    frame.debug_flags = flags
    ctx = shs_gpu.Context(0)
    ctx.set_timeline(True)
    prepared = ctx.prepare(frame, draws)
    for _ in range(20):
        ctx.render_prepared(prepared)
    ctx.synchronize()
    for rep in range(3):
        ctx.render_prepared(prepared)
        ctx.synchronize()
        head, s, r = ctx.debug_timeline()
        t0 = int(s[:, 0].min())
        print(f"{cfg} flags={flags:#x} frame {rep}: {head}")
        sb, gb = head["setup_blocks"], head["ghost_blocks"]
        summarize("setup", s[:sb], t0)
        summarize("ghost", s[sb:sb + gb], t0)
        summarize("clear", s[sb + gb:], t0)
        summarize("raster", r, t0)
        phases(s[:sb], ["draw", "setup_tri", "busy", "bins", "make_rec"], "setup")
        phases(r, ["busy_list", "gather", "staged", "rastered", "shaded", "written"], "raster")
        busy = r[r[:, 7] != 0]
        if len(busy):
            k = int(np.argmax(r[:, 1].astype(np.int64) - r[:, 0].astype(np.int64)))
            print(f"  raster first-tile candidates: median {np.median(busy[:, 8]):.0f} max {busy[:, 8].max()} | pair tasks "
                  f"median {np.median(busy[:, 9]):.0f} max {busy[:, 9].max()} | slowest wg: cand {r[k, 8]} hits {r[k, 9]}")
        for nm, arr in (("setup", s), ("raster", r)):
            dt = arr[:, 1].astype(np.int64) - arr[:, 0].astype(np.int64)
            dc = arr[:, 11].astype(np.int64) - arr[:, 10].astype(np.int64)
            ok = dt > 50
            if ok.any():
                f = dc[ok] / dt[ok] * 100.0
                print(f"  {nm} shader clock (s_memtime / realtime): median {np.median(f):.0f} MHz  min {f.min():.0f}  max {f.max():.0f}")
        rd = (r[:, 1].astype(np.int64) - r[:, 0].astype(np.int64)) / 100.0
        print(f"  raster blocks > 2us: {(rd > 2).sum()}  setup kernel span {(s[:, 1].max() - t0) / 100:.2f} us, "
              f"raster span {(r[:, 1].max() - r[:, 0].min()) / 100:.2f} us, gap {(int(r[:, 0].min()) - int(s[:, 1].max())) / 100:.2f} us")
    ctx.close()


if __name__ == "__main__":
    main()
