#!/bin/bash
# Round 6 tuning A/B: k_lib_hsort grid 512 (g512), the deep raster's per-pixel box test up to 32 / 8 px
# (box32 / box8) against the default (gpu: grid 256, 16 px); C4 N = 1 and the 8-way split.
set -o pipefail
TAG=r6t LIBS="gpu g512 box32 box8" REPS=3 ENVS="SPLIT_REGIONS=1" bash tools/ab.sh "python -u tools/exp_pipeline.py c4 60 1,8 3"
