#!/bin/bash
# Round 5, first GPU pass: the changed tests, the default bench line (C2 headline + the strong C4 / C5
# legs), and the 2-rank rehearsal of the N-rank path on one GPU (gloo; timings not meaningful).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_exp_switches.py tests/test_shadow_footprint.py tests/test_batch.py tests/test_gather_gpu.py \
  > gpurun_out/r5a_tests.log 2>&1 || { tail -40 gpurun_out/r5a_tests.log; exit 1; }
tail -2 gpurun_out/r5a_tests.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-pmc > gpurun_out/r5a_bench.log 2>&1 \
  || { tail -30 gpurun_out/r5a_bench.log; exit 1; }
grep '^{' gpurun_out/r5a_bench.log | tail -1 | cut -c1-600
SHS_BENCH_REHEARSE=1 timeout -k 10 300 python bench.py --gpus 2 --steps 20 --warmup 5 --strong-frames 10 \
  > gpurun_out/r5a_rehearse.log 2>&1 || { tail -30 gpurun_out/r5a_rehearse.log; exit 1; }
grep '^{' gpurun_out/r5a_rehearse.log | tail -1 | cut -c1-300
