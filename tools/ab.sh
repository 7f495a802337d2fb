#!/bin/bash
# One parameterised GPU A/B driver (replaces round 5's per-step tools/gpu_r5*.sh, which are in git history
# up to commit 1dc90d1; DESIGN.md cites them by name).  Runs on the GPU box from the repository root:
#
#   TAG=r6a TESTS="tests/test_regions.py tests/test_fullsize.py" LIBS="base gpu" REPS=2 \
#     bash tools/ab.sh "python tools/exp_pipeline.py c4 60 1,8 3" "python bench.py --config c5 --no-pmc --no-cpu"
#
#   TESTS   -m gpu test files run first with the default library (empty: none); a failure ends the run
#   LIBS    libraries to compare: "gpu" = the default shs_gpu/libshs_gpu.so, NAME = shs_gpu/libshs_NAME.so
#           (tools/build_variant.sh base [REV] | NAME "-DFLAG ...")
#   REPS    interleaved repetitions of every (command, library) pair (default 2)
#   ENVS    extra environment for the timed commands (e.g. "SPLIT_REGIONS=1")
#   GREP    lines of each command's output to echo (default: exp_pipeline / bench result lines)
#   STEP_TIMEOUT  per command, seconds (default 240)
# Logs: gpurun_out/$TAG_*.log.  Every GPU step runs under its own timeout; the first failure ends the run.
set -o pipefail
TAG=${TAG:-ab}
LIBS=${LIBS:-base gpu}
REPS=${REPS:-2}
GREP=${GREP:-per-rank|^\{}
STEP_TIMEOUT=${STEP_TIMEOUT:-240}
mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-600} python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu $TESTS \
    > gpurun_out/${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
  tail -1 gpurun_out/${TAG}_tests.log
fi
i=0
for cmd in "$@"; do
  i=$((i + 1))
  for rep in $(seq 1 "$REPS"); do
    for lib in $LIBS; do
      so=$(pwd)/leisure-software-renderer_amd/shs_gpu/libshs_$lib.so
      log=gpurun_out/${TAG}_c${i}_${lib}_${rep}.log
      env $ENVS SHS_GPU_LIB=$so timeout -k 10 "$STEP_TIMEOUT" $cmd > "$log" 2>&1 || { tail -30 "$log"; exit 1; }
      echo "== [$i] $lib $rep: $cmd"
      grep -E "$GREP" "$log" | cut -c1-600
    done
  done
done
