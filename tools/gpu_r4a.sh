#!/bin/bash
# The switches below are read only by the timing-experiments build (make -C leisure-software-renderer_amd exp).
export SHS_GPU_LIB=${SHS_GPU_LIB:-$PWD/leisure-software-renderer_amd/shs_gpu/libshs_gpu_exp.so}
# Round-4 GPU check: the whole -m gpu suite, then the C2 short-window diagnostic, then A/B bench lines
# (C3 record-free binned raster; C4 wave light-list culling on / off via SHS_LIB_EXP=16).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r4a_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r4a_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u tools/diag_short_window.py > gpurun_out/r4a_win.log 2>&1 || exit 1
timeout -k 10 120 python -u tools/diag_short_window.py --pre-legs > gpurun_out/r4a_win_pre.log 2>&1 || exit 1
for c in c3 c4 c5; do
  timeout -k 10 200 python bench.py --config $c --no-pmc --no-cpu --steps 100 --warmup 10 > gpurun_out/r4a_$c.log 2>&1 || exit 1
done
SHS_LIB_EXP=16 timeout -k 10 200 python bench.py --config c4 --no-pmc --no-cpu --steps 100 --warmup 10 > gpurun_out/r4a_c4_nocull.log 2>&1 || exit 1
SHS_LEGACY_NORECS=1 timeout -k 10 200 python bench.py --config c3 --no-pmc --no-cpu --steps 100 --warmup 10 > gpurun_out/r4a_c3_norecs.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-pmc --no-cpu > gpurun_out/r4a_c2_short.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-pmc --no-cpu > gpurun_out/r4a_c2_long.log 2>&1 || exit 1
cat gpurun_out/r4a_win.log gpurun_out/r4a_win_pre.log
for f in c3 c3_norecs c4 c4_nocull c5 c2_short c2_long; do
  python - gpurun_out/r4a_$f.log $f <<'PY'
import json, sys
line = [l for l in open(sys.argv[1]) if l.startswith('{')][-1]
d = json.loads(line)
r = d['roofline']
print(sys.argv[2], d['value'], d['ms_per_step'], d.get('kernels_ms'), r.get('frac'), r.get('step_frac'), r.get('frame_frac'))
PY
done
