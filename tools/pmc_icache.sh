#!/bin/bash
# Instruction-cache behaviour of the frame kernels (run on the GPU box).
# usage: bash tools/pmc_icache.sh <tag> [bench args]
set -e
TAG=$1; shift
R=$(pwd)
export TMPDIR=/tmp
cd /tmp
timeout -k 10 120 rocprofv3 -L > "$R/gpurun_out/pmc_list_$TAG.txt" 2>&1 || true
grep -o "SQC_ICACHE[A-Z_]*\|SQ_IFETCH[A-Z_]*\|SQ_INSTS_VALU\b\|SQ_WAIT_INST_ANY\|SQ_WAVE_CYCLES\|SQ_BUSY_CYCLES" "$R/gpurun_out/pmc_list_$TAG.txt" | sort -u > "$R/gpurun_out/pmc_avail_$TAG.txt" || true
cat "$R/gpurun_out/pmc_avail_$TAG.txt"
for C in SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_WAIT_INST_ANY SQ_IFETCH; do
  if grep -qx "$C" "$R/gpurun_out/pmc_avail_$TAG.txt"; then
    timeout -k 10 300 rocprofv3 --pmc $C --output-format csv -d "$R/gpurun_out/pmc_$TAG/$C" -o pmc -- python3 "$R/bench.py" --child "$@" > "$R/gpurun_out/pmc_${TAG}_$C.log" 2>&1
  fi
done
cd "$R"
python3 - "$TAG" <<'PY'
import csv, glob, sys, collections
tag = sys.argv[1]
for f in sorted(glob.glob(f"gpurun_out/pmc_{tag}/*/**/*counter_collection.csv", recursive=True)):
    acc = collections.defaultdict(list)
    for row in csv.DictReader(open(f)):
        k = row["Kernel_Name"].split("(")[0].split("::")[-1]
        acc[(k, row["Counter_Name"])].append(float(row["Counter_Value"]))
    for (k, c), v in sorted(acc.items()):
        v = v[3:] if len(v) > 6 else v
        print(f"{c:24s} {k:24s} mean {sum(v)/len(v):14.1f} n={len(v)}")
PY
