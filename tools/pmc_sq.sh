#!/bin/bash
# SQ counter pass for the bench kernels (own run, --pmc only).  usage: bash tools/pmc_sq.sh <tag> [bench args]
TAG=$1; shift
R=$(pwd); export TMPDIR=/tmp; cd /tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VMEM --output-format csv -d "$R/gpurun_out/pmc_$TAG" -o pmc -- python3 "$R/bench.py" --child --steps 20 --warmup 3 "$@" > "$R/gpurun_out/pmc_$TAG.log" 2>&1 || { echo pmc_failed; tail -5 "$R/gpurun_out/pmc_$TAG.log"; exit 1; }
cd "$R"
python3 - "$TAG" <<'PY'
import csv, glob, sys, collections
tag = sys.argv[1]
rows = []
for f in glob.glob(f"gpurun_out/pmc_{tag}/**/*counter_collection.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in rows:
    k = r["Kernel_Name"].split("(")[0]
    agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    print(k, {c: round(sum(v[3:]) / max(len(v[3:]), 1), 1) for c, v in sorted(d.items())})
PY
