#!/bin/bash
# Round 5: bin-mode k_setup register bound (SHS_BIN_SETUP_WAVES 8 = 64 VGPRs, the default; 7 / 6 / 5:
# 72 / 80 / 102 VGPRs, fewer spills), C3 A/B interleaved twice, then setup FETCH / WRITE per variant.
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
  for v in gpu sw7 sw6 sw5; do
    SHS_GPU_LIB=$(pwd)/leisure-software-renderer_amd/shs_gpu/libshs_$v.so timeout -k 10 200 python bench.py --config c3 --no-pmc --no-cpu --no-single --no-pcie --strong '' --steps 100 --warmup 10 \
      > gpurun_out/r5z_$v.log 2>&1 || { tail -20 gpurun_out/r5z_$v.log; exit 1; }
    python3 - gpurun_out/r5z_$v.log $v <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print('c3', sys.argv[2], 'ms/step', d['ms_per_step'], 'kernels', d.get('kernels_ms'))
PY
  done
done
for v in gpu sw5; do
  SHS_GPU_LIB=$(pwd)/leisure-software-renderer_amd/shs_gpu/libshs_$v.so timeout -k 10 400 bash tools/pmc_kernels.sh r5z_$v --config c3 > /dev/null || exit 1
  python3 -c "
import json; d=json.load(open('gpurun_out/pmc_r5z_$v.json'))
for k,x in d.items():
    if 'setup' in k or 'raster' in k or 'ghost' in k: print('$v', k[:40], 'fetch MB', round(x.get('fetch_bytes_x2',0)/1e6,1), 'write MB', round(x.get('write_bytes',0)/1e6,1))
"
done
