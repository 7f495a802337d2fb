#!/bin/bash
# Round 6 evidence, part A: the whole -m gpu suite, smoke(), the default bench line, the 8-rank rehearsal.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/r6f_tests.log 2>&1 || { tail -40 gpurun_out/r6f_tests.log; exit 1; }
tail -1 gpurun_out/r6f_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r6f_smoke.log 2>&1 || { tail -20 gpurun_out/r6f_smoke.log; exit 1; }
tail -1 gpurun_out/r6f_smoke.log
timeout -k 10 600 python -u bench.py > gpurun_out/r6f_default.log 2>&1 || { tail -30 gpurun_out/r6f_default.log; exit 1; }
grep '^{' gpurun_out/r6f_default.log | tail -1 | python3 -c "
import json,sys
d=json.loads(sys.stdin.read())
print('value', d['value'], 'ms/step', d['ms_per_step'], 'frac', d['roofline']['frac'], 'traffic', d['roofline']['traffic'])
for k in ('strong_c4','strong_c5'):
    s=d.get(k); print(k, s['ms_per_frame'], s['roofline']['frac'], s['roofline']['rank0_camera_phase_frac'], s.get('clock_ramp'))
print('cpu', d['cpu_baseline']['value'], 'pcie', d.get('seam1_pcie', {}).get('ms_per_frame'))
"
SHS_BENCH_REHEARSE=1 timeout -k 10 900 python -u bench.py --gpus 8 --steps 20 --warmup 5 --strong-frames 30 --no-cpu > gpurun_out/r6f_rehearse8.log 2>&1 || { tail -30 gpurun_out/r6f_rehearse8.log; exit 1; }
grep '^{' gpurun_out/r6f_rehearse8.log | tail -1 | python3 -c "
import json,sys
d=json.loads(sys.stdin.read())
print('rehearsal n_gpus', d['n_gpus'], 'value', d['value'])
for k in ('strong_c4','strong_c5'):
    s=d.get(k); print(k, s['n_gpus'], s['ms_per_frame'], sum(s['owned_pixels']), 'roofline keys', sorted(s['roofline']))
"
