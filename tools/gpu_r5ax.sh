#!/bin/bash
# Round 5 (after the compile-time specialisations): round profiles of C2 / C3 and the C2 component split.
set -o pipefail
mkdir -p gpurun_out
for fl in 0x1000 0x400; do
  SHS_GPU_LIB=$(pwd)/leisure-software-renderer_amd/shs_gpu/libshs_gpu_exp.so timeout -k 10 200 python bench.py --debug-flags $fl --no-pmc --no-cpu --no-single --no-pcie --strong '' --steps 100 --warmup 10 \
    > gpurun_out/r5ax_$fl.log 2>&1 || { tail -20 gpurun_out/r5ax_$fl.log; exit 1; }
  python3 - gpurun_out/r5ax_$fl.log $fl <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print('flags', sys.argv[2], 'ms/step', d['ms_per_step'], 'kernels', d.get('kernels_ms'))
PY
done
bash tools/round_profiles.sh r05d c2 c3 || exit 1
timeout -k 10 400 bash tools/pmc_kernels.sh r05d_c3 --config c3 > /dev/null || exit 1
