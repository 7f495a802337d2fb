#!/bin/bash
# GPU-box quick check: legacy parity tests, C2/C3 bench lines, C2 timeline (gpurun_out/).
set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/quick.log
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu ${TESTS:-tests/test_gpu_parity.py} > gpurun_out/par.log 2>&1 || { tail -30 gpurun_out/par.log; exit 1; }
tail -1 gpurun_out/par.log
for c in ${CONFIGS:-c2 c3}; do
  timeout -k 10 120 python bench.py --config $c --no-pmc --no-cpu --steps 400 --warmup 50 $BENCH_ARGS >> gpurun_out/quick.log 2>&1 || exit 1
done
python - <<'PY'
import json
for l in open("gpurun_out/quick.log"):
    if l.startswith("{"):
        d = json.loads(l)
        print(d["config"]["workload"][:3], d["value"], d["ms_per_step"], d.get("kernels_ms"), d["roofline"]["frac"])
PY
timeout -k 10 120 python tools/timeline.py c2 > gpurun_out/tl_c2.log 2>&1 && sed -n 2,11p gpurun_out/tl_c2.log
