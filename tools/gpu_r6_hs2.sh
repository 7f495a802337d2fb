#!/bin/bash
# Round 6: k_lib_hsort as 512-thread workgroups (16 entries per thread), 256 workgroups, against HEAD
# (1024 threads, 512 workgroups): sorted-list parity, then C4 / C5 N = 1 and the 8-way splits.
set -o pipefail
TAG=r6hs2 TESTS="tests/test_sorted_lists.py tests/test_fullsize.py" LIBS="base gpu" REPS=3 ENVS="SPLIT_REGIONS=1" \
  bash tools/ab.sh "python -u tools/exp_pipeline.py c4 60 1,8 3" "python -u tools/exp_pipeline.py c5 60 1,8 3"
