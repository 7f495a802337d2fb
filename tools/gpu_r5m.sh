#!/bin/bash
# Round 5: legacy framebuffer stores non-temporal (libshs_gpu_exp.so) vs plain (libshs_plainst.so), C2
# raster and clear-only (DBG_CLEAR_ONLY), interleaved twice.
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
  for v in gpu_exp plainst; do
    for fl in 0 0x400; do
      SHS_GPU_LIB=$(pwd)/leisure-software-renderer_amd/shs_gpu/libshs_$v.so timeout -k 10 200 python bench.py --debug-flags $fl --no-pmc --no-cpu --no-single --no-pcie --strong '' --steps 100 --warmup 10 \
        > gpurun_out/r5m_${v}_$fl.log 2>&1 || { tail -20 gpurun_out/r5m_${v}_$fl.log; exit 1; }
      python3 - gpurun_out/r5m_${v}_$fl.log $v $fl <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print(sys.argv[2], 'flags', sys.argv[3], 'ms/step', d['ms_per_step'], 'kernels', d.get('kernels_ms'))
PY
    done
  done
done
# C3 k_setup traffic with and without its bin appends (DBG_SKIP_BIN, experiments build; wrong images)
export SHS_GPU_LIB=$(pwd)/leisure-software-renderer_amd/shs_gpu/libshs_gpu_exp.so
for fl in 0 0x800; do
  timeout -k 10 500 bash tools/pmc_kernels.sh r5m_c3_$fl --config c3 --debug-flags $fl > /dev/null || exit 1
  python3 -c "
import json; d=json.load(open('gpurun_out/pmc_r5m_c3_$fl.json'))
for k,v in d.items():
    if 'setup' in k or 'raster' in k: print('flags $fl', k[:40], 'fetch MB', round(v.get('fetch_bytes_x2',0)/1e6,1), 'write MB', round(v.get('write_bytes',0)/1e6,1))
"
done
