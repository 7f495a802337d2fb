#!/bin/bash
# Round 6 (after k_lib_hsort): per-rank kernel medians of the 8-way C4 / C5 splits with one frame in flight
# (D=1) and three (D=3), and the host cost of a rank's frame.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for D in 1 3; do
  for c in c4 c5; do
    rm -rf gpurun_out/tr6_${c}_d$D
    SPLIT_REGIONS=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tr6_${c}_d$D -- python3 -u tools/exp_pipeline.py $c 60 8 $D > gpurun_out/tr6_${c}_d$D.log 2>&1 || { tail -20 gpurun_out/tr6_${c}_d$D.log; exit 1; }
    grep per-rank gpurun_out/tr6_${c}_d$D.log
    python3 tools/trace_ranks.py gpurun_out/tr6_${c}_d$D 8 > gpurun_out/tr6_${c}_d${D}_ranks.txt && cat gpurun_out/tr6_${c}_d${D}_ranks.txt
    rm -rf gpurun_out/tr6_${c}_d$D
  done
done
for r in 3 2; do
  SPLIT_REGIONS=1 timeout -k 10 200 python3 -u tools/exp_host.py 8 $r 3 200 2>&1 | grep -v amdgpu.ids
done
