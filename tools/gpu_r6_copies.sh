#!/bin/bash
# Round 6: which HIP calls enqueue the per-frame copy / fill kernels of the sharded C4 / C5 frame
# (rocprofv3 HIP API trace, rank 3 of 8, one frame in flight, 20 frames).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for c in c4 c5; do
  rm -rf gpurun_out/cp_$c
  SPLIT_ONLY=3 SPLIT_REGIONS=1 timeout -k 10 200 rocprofv3 --hip-trace --kernel-trace --output-format csv -d gpurun_out/cp_$c -- python3 -u tools/exp_pipeline.py $c 20 8 1 > gpurun_out/cp_$c.log 2>&1 || { tail -20 gpurun_out/cp_$c.log; exit 1; }
  python3 - gpurun_out/cp_$c <<'PY'
import csv, glob, sys, collections
d = sys.argv[1]
cnt = collections.Counter()
for f in glob.glob(d + "/**/*hip_api_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r.get("Function", r.get("Function_Name", ""))
        if "Memcpy" in n or "Memset" in n or "Launch" in n or "Event" in n or "Synchronize" in n:
            cnt[n] += 1
for f in glob.glob(d + "/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "rocclr" in r["Kernel_Name"]:
            cnt["kernel " + r["Kernel_Name"]] += 1
for k, v in cnt.most_common(40):
    print(f"{v:7d} {k}")
PY
  rm -rf gpurun_out/cp_$c
done
