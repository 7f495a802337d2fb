#!/bin/bash
# Kernel timeline of one rank's shard of the 8-way region-sharded C4 / C5 frame, 3 frames in flight
# (the steady state's last dispatches: overlap, gaps, queue assignment).  usage: R=3 C=c4 bash tools/gpu_tl_rank.sh
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
C=${C:-c4}; R=${R:-3}
rm -rf gpurun_out/tlr_$C
SPLIT_ONLY=$R SPLIT_REGIONS=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tlr_$C -- python3 -u tools/exp_pipeline.py $C 60 8 3 > gpurun_out/tlr_$C.log 2>&1 || exit 1
grep "frames in flight" gpurun_out/tlr_$C.log
python3 tools/trace_timeline.py gpurun_out/tlr_$C 48 > gpurun_out/tlr_${C}.txt && cat gpurun_out/tlr_${C}.txt
