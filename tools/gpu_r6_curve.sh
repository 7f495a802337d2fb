#!/bin/bash
# Round 6: the 1 / 2 / 4 / 8 strong-scaling curve of C4 and C5 measured rank by rank on one GPU (each rank's
# region shard in turn, three frames in flight), twice.
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
  for c in c4 c5; do
    SPLIT_REGIONS=1 timeout -k 10 400 python -u tools/exp_pipeline.py $c 60 1,2,4,8 3 > gpurun_out/r6c_${c}_$rep.log 2>&1 || { tail -20 gpurun_out/r6c_${c}_$rep.log; exit 1; }
    grep -E "per-rank|regions" gpurun_out/r6c_${c}_$rep.log
  done
done
