#!/bin/bash
# (The trial mode it measures was reverted after this run: profiles/r05_legacy_deferred_raster.txt.)
# Round 5: SHS_OPT_LEGACY_PIPELINE = 2 (each batch's k_raster launched after the next batch's setup was
# queued: no cross-stream wait between two rasters) against the default two-stream pipeline: the
# pipeline parity tests, then C2 / C3 A/B pairs (bench --pipeline 2).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_batch.py -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/r5ch_tests.log 2>&1 || { tail -30 gpurun_out/r5ch_tests.log; exit 1; }
tail -1 gpurun_out/r5ch_tests.log
run() {  # tag pipeline config
  timeout -k 10 200 python bench.py --config $3 --pipeline $2 --no-pmc --no-cpu --no-single --no-pcie --strong '' --steps 200 --warmup 10 \
    > gpurun_out/r5ch_$1.log 2>&1 || { tail -20 gpurun_out/r5ch_$1.log; exit 1; }
  python3 - gpurun_out/r5ch_$1.log $1 <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print(sys.argv[2], 'ms/step', d['ms_per_step'], 'value', d['value'], 'kernels', d.get('kernels_ms'))
PY
}
for rep in 1 2; do
  run c2_p0_$rep 0 c2 || exit 1
  run c2_p2_$rep 2 c2 || exit 1
  run c3_p0_$rep 0 c3 || exit 1
  run c3_p2_$rep 2 c3 || exit 1
done
