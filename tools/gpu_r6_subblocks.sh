#!/bin/bash
# Round 6: setup sub-blocks with the balancer's block bounds unchanged (256-triangle chunk hulls): parity,
# the rank-3 setup timeline, then C4 / C5 at N = 1 and the 8-way splits against HEAD (libshs_base.so).
set -o pipefail
SPLIT_REGIONS=1 timeout -k 10 240 python -u tools/exp_setup_timeline.py 8 3 > gpurun_out/r6s2_setup3.log 2>&1 || { tail -30 gpurun_out/r6s2_setup3.log; exit 1; }
head -3 gpurun_out/r6s2_setup3.log
TAG=r6s2 TESTS="tests/test_regions.py tests/test_shipped_regions.py tests/test_region_balance.py tests/test_shadow_footprint.py tests/test_shard.py tests/test_fullsize.py tests/test_sorted_lists.py" \
  LIBS="base gpu" REPS=3 ENVS="SPLIT_REGIONS=1" bash tools/ab.sh "python -u tools/exp_pipeline.py c4 60 1,8 3" "python -u tools/exp_pipeline.py c5 60 1,8 3"
