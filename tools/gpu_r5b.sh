#!/bin/bash
# Round 5: spatially ordered library meshes -- parity (spatial-order, library, full-size, region tests),
# then the 8-way split of C4 / C5 on one GPU and the single-GPU C4 / C5 bench lines.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_spatial_order.py tests/test_lib_parity.py tests/test_fullsize.py tests/test_shipped_regions.py tests/test_regions.py \
  > gpurun_out/r5b_tests.log 2>&1 || { tail -40 gpurun_out/r5b_tests.log; exit 1; }
tail -2 gpurun_out/r5b_tests.log
for c in c4 c5; do
  SPLIT_REGIONS=1 timeout -k 10 300 python -u tools/exp_pipeline.py $c 60 1,8 3 > gpurun_out/r5b_split_$c.log 2>&1 || exit 1
  grep -v amdgpu.ids gpurun_out/r5b_split_$c.log
  timeout -k 10 300 python bench.py --config $c --no-pmc --no-cpu --steps 200 --warmup 20 > gpurun_out/r5b_bench_$c.log 2>&1 || exit 1
  grep '^{' gpurun_out/r5b_bench_$c.log | tail -1 | cut -c1-400
done
