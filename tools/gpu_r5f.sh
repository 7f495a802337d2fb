#!/bin/bash
# Round 5: kernel timeline of rank 3 of the 8-way C4 region split with 3 frames in flight (overlap of
# the frames' kernels on one GPU).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/r5f_tr
SPLIT_ONLY=3 SPLIT_REGIONS=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r5f_tr -- python3 -u tools/exp_pipeline.py c4 60 8 3 > gpurun_out/r5f.log 2>&1 || exit 1
grep "c4 N" gpurun_out/r5f.log
python3 tools/trace_timeline.py gpurun_out/r5f_tr 90 > gpurun_out/r5f_timeline.txt
tail -95 gpurun_out/r5f_timeline.txt
