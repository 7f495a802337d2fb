#!/bin/bash
# Round 5: k_raster prefetches the next item (busy entry, bin count) during the current tile (working
# tree) against HEAD (libshs_base.so): the whole -m gpu suite, then C3 / C2 A/B pairs.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/r5cg_tests.log 2>&1 || { tail -30 gpurun_out/r5cg_tests.log; exit 1; }
tail -1 gpurun_out/r5cg_tests.log
run() {  # tag lib config
  SHS_GPU_LIB=$(pwd)/leisure-software-renderer_amd/shs_gpu/libshs_$2.so timeout -k 10 200 python bench.py --config $3 --no-pmc --no-cpu --no-single --no-pcie --strong '' --steps 200 --warmup 10 \
    > gpurun_out/r5cg_$1.log 2>&1 || { tail -20 gpurun_out/r5cg_$1.log; exit 1; }
  python3 - gpurun_out/r5cg_$1.log $1 <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print(sys.argv[2], 'ms/step', d['ms_per_step'], 'kernels', d.get('kernels_ms'), 'frac', d['roofline']['frac'])
PY
}
for rep in 1 2; do
  run c3_base_$rep base c3 || exit 1
  run c3_new_$rep gpu c3 || exit 1
  run c2_base_$rep base c2 || exit 1
  run c2_new_$rep gpu c2 || exit 1
done
