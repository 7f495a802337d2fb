#!/bin/bash
# Round 6: the region balancer's cost weights after k_lib_hsort (per bin tile: REGION_PX x pixels +
# REGION_COVERED_PX x covered pixels + the triangles of the blocks covering it).  Default 5 / 15 (gpu),
# 4 / 12, 3 / 9 and 6.5 / 19.5; the 8-way C4 and C5 splits.
set -o pipefail
TAG=r6w LIBS="gpu w4 w3 w6" REPS=2 ENVS="SPLIT_REGIONS=1" bash tools/ab.sh "python -u tools/exp_pipeline.py c4 60 8 3" "python -u tools/exp_pipeline.py c5 60 8 3"
