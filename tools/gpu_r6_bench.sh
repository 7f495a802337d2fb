#!/bin/bash
# Round 6: the default bench line (C2 headline + strong legs with their roofline, PMC, CPU leg) and the
# 8-rank rehearsal of the --gpus 8 path on one GPU (gloo; its timings mean nothing, the keys are checked).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py > gpurun_out/r6b_default.log 2>&1 || { tail -30 gpurun_out/r6b_default.log; exit 1; }
grep '^{' gpurun_out/r6b_default.log | tail -1 | python3 -c "
import json,sys
d=json.loads(sys.stdin.read())
print('value', d['value'], 'ms/step', d['ms_per_step'], 'frac', d['roofline']['frac'], 'traffic', d['roofline']['traffic'])
for k in ('strong_c4','strong_c5'):
    s=d.get(k); print(k, s['ms_per_frame'], s['roofline']['frac'], s['roofline']['rank0_camera_phase_frac'], s.get('clock_ramp'))
print('cpu', d['cpu_baseline']['value'])
"
SHS_BENCH_REHEARSE=1 timeout -k 10 900 python -u bench.py --gpus 8 --steps 20 --warmup 5 --strong-frames 30 --no-cpu > gpurun_out/r6b_rehearse8.log 2>&1 || { tail -30 gpurun_out/r6b_rehearse8.log; exit 1; }
grep '^{' gpurun_out/r6b_rehearse8.log | tail -1 | python3 -c "
import json,sys
d=json.loads(sys.stdin.read())
print('n_gpus', d['n_gpus'], 'value', d['value'])
for k in ('strong_c4','strong_c5'):
    s=d.get(k); print(k, s['n_gpus'], s['ms_per_frame'], sum(s['owned_pixels']), json.dumps(s['roofline'])[:400])
"
