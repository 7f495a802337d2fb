#!/bin/bash
# one extra PMC pass: LDS activity of the raster / resolve / setup kernels (CONFIG, default c4)
set -o pipefail
R=$(pwd); export TMPDIR=/tmp
mkdir -p "$R/gpurun_out"
( cd /tmp && timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES --output-format csv -d "$R/gpurun_out/pmc_lds" -o pmc -- python3 "$R/bench.py" --child --steps 12 --warmup 3 --config ${CONFIG:-c4} ) > "$R/gpurun_out/pmc_lds.log" 2>&1 || { tail -5 gpurun_out/pmc_lds.log; exit 1; }
python3 - <<'PY'
import csv, glob, collections
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob("gpurun_out/pmc_lds/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        agg[r["Kernel_Name"].split("(")[0]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    if "raster" in k or "resolve" in k or "setup" in k or "ghost" in k:
        print(k, {c: round(sum(v[3:]) / max(1, len(v[3:]))) for c, v in d.items()})
PY
