#!/bin/bash
# Round 6: the kernel sequence of the 8-way C5 / C4 rank-3 frame, one frame in flight (what runs per frame,
# the copy / fill kernels' place in it).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for c in c5 c4; do
  rm -rf gpurun_out/seq_$c
  SPLIT_ONLY=3 SPLIT_REGIONS=1 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/seq_$c -- python3 -u tools/exp_pipeline.py $c 20 8 1 > gpurun_out/seq_$c.log 2>&1 || { tail -20 gpurun_out/seq_$c.log; exit 1; }
  python3 tools/trace_timeline.py gpurun_out/seq_$c 30 > gpurun_out/seq_${c}.txt && cat gpurun_out/seq_${c}.txt
  rm -rf gpurun_out/seq_$c
done
