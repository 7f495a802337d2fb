#!/bin/bash
# Round-4 GPU check (b): the legacy / batch GPU tests, then C2 bench lines pipelined vs not, short and long windows.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_batch.py tests/test_shipped_frames.py tests/test_gpu_parity.py tests/test_present.py tests/test_gather_gpu.py tests/test_group.py > gpurun_out/r4b_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r4b_tests.log
[ $rc -eq 0 ] || exit $rc
for v in "p1s:--pipeline 1 --steps 20 --warmup 5" "p0s:--pipeline 0 --steps 20 --warmup 5" "p1l:--pipeline 1 --steps 200 --warmup 20" "p0l:--pipeline 0 --steps 200 --warmup 20"; do
  tag=${v%%:*}; a=${v#*:}
  timeout -k 10 200 python bench.py --no-pmc --no-cpu $a > gpurun_out/r4b_c2_$tag.log 2>&1 || exit 1
  python - gpurun_out/r4b_c2_$tag.log $tag <<'PY'
import json, sys
line = [l for l in open(sys.argv[1]) if l.startswith('{')][-1]
d = json.loads(line); r = d['roofline']
print(sys.argv[2], d['value'], d['ms_per_step'], d['kernels_ms'], r['frac'], r['step_frac'])
PY
done
