#!/bin/bash
# Round 6: C5's camera pass on the context's one stream (onestream: no side stream beside the shadow pass)
# against the default (gpu): bench --config c5, the strong leg after the C4 leg, the 8-way split.
set -o pipefail
TAG=r6o LIBS="gpu onestream" REPS=2 ENVS="SPLIT_REGIONS=1" GREP='per-rank|ms_per_step' bash tools/ab.sh \
  "python -u bench.py --config c5 --no-pmc --no-cpu" "python -u bench.py --steps 20 --warmup 5 --no-pmc --no-cpu --no-pcie --no-single" \
  "python -u tools/exp_pipeline.py c5 60 1,8 3"
