#!/bin/bash
# Round 5: k_lib_blocks (region-sharded setup blocks listed before k_lib_setup) -- parity, then the
# 8-way C4 / C5 split against libshs_base.so (HEAD), interleaved, and per-rank kernel medians.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_lib_parity.py tests/test_spatial_order.py tests/test_regions.py tests/test_shipped_regions.py \
  tests/test_shadow_footprint.py tests/test_light_parity.py \
  > gpurun_out/r5g_tests.log 2>&1 || { tail -40 gpurun_out/r5g_tests.log; exit 1; }
tail -2 gpurun_out/r5g_tests.log
for v in base default base default; do
  if [ $v = default ]; then L=; else L=$(pwd)/leisure-software-renderer_amd/shs_gpu/libshs_$v.so; fi
  for c in c4 c5; do
    SHS_GPU_LIB=$L SPLIT_REGIONS=1 timeout -k 10 300 python -u tools/exp_pipeline.py $c 60 1,8 3 > gpurun_out/r5g_split_${c}_$v.log 2>&1 || exit 1
    echo "== $v $c"; grep "$c N" gpurun_out/r5g_split_${c}_$v.log
  done
done
rm -rf gpurun_out/r5g_tr
SPLIT_REGIONS=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r5g_tr -- python3 -u tools/exp_pipeline.py c4 60 8 1 > gpurun_out/r5g_tr.log 2>&1 || exit 1
python3 tools/trace_ranks.py gpurun_out/r5g_tr 8 | tee gpurun_out/r5g_tr_ranks.txt
