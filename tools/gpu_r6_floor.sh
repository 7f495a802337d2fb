#!/bin/bash
# Round 6: the per-frame floor of a sharded rank: C4 / C5 at N = 8 (rank 3) against tiny shards (N = 32 and
# 64, rank 0), three frames in flight -- how much of a rank's frame is the fixed chain and host enqueue.
set -o pipefail
mkdir -p gpurun_out
for c in c4 c5; do
  for n in 8 32 64; do
    r=0; [ $n = 8 ] && r=3
    SPLIT_ONLY=$r SPLIT_REGIONS=1 timeout -k 10 300 python -u tools/exp_pipeline.py $c 100 $n 1,3 > gpurun_out/r6fl_${c}_$n.log 2>&1 || { tail -20 gpurun_out/r6fl_${c}_$n.log; exit 1; }
    grep per-rank gpurun_out/r6fl_${c}_$n.log
  done
done
SPLIT_REGIONS=1 timeout -k 10 200 python3 -u tools/exp_host.py 8 3 3 200 2>&1 | grep -v amdgpu.ids
SPLIT_REGIONS=1 timeout -k 10 200 python3 -u tools/exp_host.py 64 0 3 200 2>&1 | grep -v amdgpu.ids
