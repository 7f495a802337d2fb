#!/bin/bash
# Round 6: the side stream created on first use (three C4 contexts' streams on hardware queues of their
# own) against HEAD (libshs_base.so: every context creates two streams); library parity first; C4 / C5 at
# N = 1 and the 8-way splits, three and four frames in flight, and the default-config C4 / C5 bench lines.
set -o pipefail
TAG=r6l TESTS="tests/test_lib_parity.py tests/test_regions.py tests/test_shadow_footprint.py tests/test_batch.py tests/test_gpu_parity.py" \
  LIBS="base gpu" REPS=2 ENVS="SPLIT_REGIONS=1" bash tools/ab.sh "python -u tools/exp_pipeline.py c4 60 1,8 3,4" "python -u tools/exp_pipeline.py c5 60 1,8 3" \
  "python -u bench.py --config c4 --no-pmc --no-cpu" "python -u bench.py --config c5 --no-pmc --no-cpu"
