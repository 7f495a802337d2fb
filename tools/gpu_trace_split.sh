#!/bin/bash
# Per-rank kernel durations of the 8-way region-sharded C5 / C4 frames (rank by rank, 3 frames in flight)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for c in c5 c4; do
  rm -rf gpurun_out/tr_$c
  SPLIT_REGIONS=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tr_$c -- python3 -u tools/exp_pipeline.py $c 60 8 ${D:-3} > gpurun_out/tr_$c.log 2>&1 || exit 1
  grep -v amdgpu.ids gpurun_out/tr_$c.log
  python3 tools/trace_ranks.py gpurun_out/tr_$c 8 > gpurun_out/tr_${c}_ranks.txt && cat gpurun_out/tr_${c}_ranks.txt
done
