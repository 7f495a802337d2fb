#!/bin/bash
# Round-end measurement on the GPU box: full bench line (roofline + PMC traffic + CPU baseline) and
# the rocprofv3 kernel-trace summary per config, then the SQ / traffic PMC passes of the library
# configs' kernels.  usage: bash tools/round_profiles.sh <tag> [configs...]
set -o pipefail
TAG=$1; shift
CONFIGS=${@:-c2 c3 c4 c5}
mkdir -p gpurun_out
for c in $CONFIGS; do
  echo "== $c bench"
  timeout -k 10 400 python bench.py --config $c > gpurun_out/${TAG}_bench_$c.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench_$c.log; exit 1; }
  grep '^{' gpurun_out/${TAG}_bench_$c.log | tail -1 > gpurun_out/${TAG}_bench_$c.json
  echo "== $c kernel trace"
  bash tools/profile_kernels.sh ${TAG}_$c --config $c || exit 1
done
for c in $CONFIGS; do
  case $c in c4|c5) echo "== $c PMC"; bash tools/pmc_kernels.sh ${TAG}_$c --config $c || exit 1;; esac
done
