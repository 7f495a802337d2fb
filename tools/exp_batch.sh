#!/bin/bash
# Phase attribution of the batched C2 raster (debug flags make the images WRONG; timing only).
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/exp_batch.txt; : > $out
run() { timeout -k 10 120 python bench.py --config ${CFG:-c2} --no-pmc --no-cpu --steps 50 --warmup 10 "$@" > gpurun_out/eb.log 2>&1 || { tail -5 gpurun_out/eb.log; exit 1; }
  python - "$*" >> $out <<'PY'
import json,sys
for l in open("gpurun_out/eb.log"):
    if l.startswith("{"):
        d=json.loads(l); r=d["roofline"]
        print(f"{sys.argv[1]:40s} ms/step {d['ms_per_step']:.4f} setup {d['kernels_ms']['setup']*1e3:8.1f}us raster {d['kernels_ms']['raster']*1e3:8.1f}us frac {r['frac']} step_frac {r['step_frac']}")
PY
}
# ARGS_LIST: ';'-separated argument sets
IFS=';' read -ra SETS <<< "${ARGS_LIST:---debug-flags 0;--debug-flags 0x400;--debug-flags 0x4000;--debug-flags 0x200;--debug-flags 0x100;--frames-per-step 1;--frames-per-step 16;--frames-per-step 32;--frames-per-step 128}"
for a in "${SETS[@]}"; do run $a; done
cat $out
