#!/bin/bash
# k_lib_resolve occupancy experiment: library parity tests, then C4 / C5 bench with the default build
# and the SHS_RESOLVE_WAVES=4 build (shs_gpu/libshs_w4.so, built beside the default one).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_lib_parity.py \
  tests/test_light_parity.py tests/test_gather_gpu.py tests/test_fullsize.py > gpurun_out/res_tests.log 2>&1 \
  || { tail -30 gpurun_out/res_tests.log; exit 1; }
tail -2 gpurun_out/res_tests.log
for v in default w5; do
  for c in c4 c5; do
    if [ $v = default ]; then L=; else L=$(pwd)/leisure-software-renderer_amd/shs_gpu/libshs_$v.so; fi
    SHS_GPU_LIB=$L timeout -k 10 200 python bench.py --config $c --no-pmc --no-cpu --no-single --no-pcie --steps 100 --warmup 10 \
      > gpurun_out/res_${v}_$c.log 2>&1 || { tail -20 gpurun_out/res_${v}_$c.log; exit 1; }
    python - gpurun_out/res_${v}_$c.log $v $c <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print(sys.argv[2], sys.argv[3], 'ms/step', d['ms_per_step'], 'kernels', d.get('kernels_ms'))
PY
  done
done
R=$(pwd); export TMPDIR=/tmp
for c in c4 c5; do
  (cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof_res_$c -o run -- \
     python3 $R/bench.py --config $c --no-pmc --no-cpu --no-single --no-pcie --steps 100 --warmup 10 > $R/gpurun_out/prof_res_$c.log 2>&1) \
    || { echo "rocprof $c failed"; exit 1; }
  python3 tools/kstats.py gpurun_out/prof_res_$c "" --skip-first 20
done
