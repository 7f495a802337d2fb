#!/bin/bash
# rank 0 of the 8-way region frame with the one-launch unpack, for several root shares
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gather_gpu.py tests/test_regions.py > gpurun_out/root_tests.log 2>&1 || { tail -20 gpurun_out/root_tests.log; exit 1; }
tail -1 gpurun_out/root_tests.log
for c in c5 c4; do for sh in 0.55 0.7 0.85; do
  timeout -k 10 300 python -u tools/exp_root.py $c 8 $sh 60 3 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/root_shares.log || exit 1
done; done
