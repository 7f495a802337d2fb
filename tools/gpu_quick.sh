#!/bin/bash
# GPU-box check: selected -m gpu tests, then bench lines (no PMC / CPU legs) for the given configs.
# usage: TESTS="tests/test_batch.py ..." CONFIGS="c2 c3" BENCH_ARGS="..." bash tools/gpu_quick.sh <tag>
set -o pipefail
TAG=${1:-quick}
mkdir -p gpurun_out
if [ -n "${TESTS:-tests}" ] && [ "${TESTS}" != "none" ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu ${TESTS:-tests} \
    > gpurun_out/${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
  tail -2 gpurun_out/${TAG}_tests.log
fi
for c in ${CONFIGS:-c2}; do
  [ "$c" = none ] && continue
  timeout -k 10 300 python bench.py --config $c --no-pmc --no-cpu ${BENCH_ARGS:---steps 50 --warmup 10} \
    > gpurun_out/${TAG}_bench_$c.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench_$c.log; exit 1; }
  grep '^{' gpurun_out/${TAG}_bench_$c.log | tail -1
done
