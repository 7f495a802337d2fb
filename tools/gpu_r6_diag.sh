#!/bin/bash
# Round 6 diagnosis: the C4 hot tiles (rank 3 / 1 / 6 of 8 and N = 1), the rank-3 setup timeline, and the
# 8-way C4 / C5 splits at three frames in flight on this code (the baseline of the round's changes).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 240 python -u tools/exp_hot_tiles.py 8 3,1,6 10 > gpurun_out/r6_hot8.log 2>&1 || { tail -30 gpurun_out/r6_hot8.log; exit 1; }
cat gpurun_out/r6_hot8.log
timeout -k 10 240 python -u tools/exp_hot_tiles.py 1 0 6 > gpurun_out/r6_hot1.log 2>&1 || { tail -30 gpurun_out/r6_hot1.log; exit 1; }
cat gpurun_out/r6_hot1.log
SPLIT_REGIONS=1 timeout -k 10 240 python -u tools/exp_setup_timeline.py 8 3 > gpurun_out/r6_setup3.log 2>&1 || { tail -30 gpurun_out/r6_setup3.log; exit 1; }
head -30 gpurun_out/r6_setup3.log
for c in c4 c5; do
  SPLIT_REGIONS=1 timeout -k 10 240 python -u tools/exp_pipeline.py $c 60 1,8 3 > gpurun_out/r6_pipe_$c.log 2>&1 || { tail -30 gpurun_out/r6_pipe_$c.log; exit 1; }
  grep "per-rank" gpurun_out/r6_pipe_$c.log
done
