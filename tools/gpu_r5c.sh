#!/bin/bash
# Round 5: A/B of the spatially ordered meshes (default) against libshs_base.so (the commit before) on the
# 8-way C4 split, interleaved twice, then per-rank kernel medians of the default build (rocprofv3).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in base default base default; do
  if [ $v = default ]; then L=; else L=$(pwd)/leisure-software-renderer_amd/shs_gpu/libshs_$v.so; fi
  SHS_GPU_LIB=$L SPLIT_REGIONS=1 timeout -k 10 300 python -u tools/exp_pipeline.py c4 60 1,8 3 > gpurun_out/r5c_split_$v.log 2>&1 || exit 1
  echo "== $v"; grep -v amdgpu.ids gpurun_out/r5c_split_$v.log | grep "c4 N"
done
for v in base default; do
  if [ $v = default ]; then L=; else L=$(pwd)/leisure-software-renderer_amd/shs_gpu/libshs_$v.so; fi
  rm -rf gpurun_out/r5c_tr_$v
  SHS_GPU_LIB=$L SPLIT_REGIONS=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r5c_tr_$v -- python3 -u tools/exp_pipeline.py c4 60 8 1 > gpurun_out/r5c_tr_$v.log 2>&1 || exit 1
  echo "== trace $v (1 frame in flight)"; python3 tools/trace_ranks.py gpurun_out/r5c_tr_$v 8 | tee gpurun_out/r5c_tr_${v}_ranks.txt
done
