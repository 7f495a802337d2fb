#!/bin/bash
# Round 6: why the N = 1 strong C4 leg reads slower than `bench.py --config c4`: the leg after the C2 loop
# with and without the PCIe leg (the only part of the default run that initialises torch at N = 1), and
# --config c4 alone, twice each.
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
  timeout -k 10 300 python -u bench.py --config c4 --no-pmc --no-cpu > gpurun_out/r6g_cfg_$rep.log 2>&1 || { tail -20 gpurun_out/r6g_cfg_$rep.log; exit 1; }
  grep '^{' gpurun_out/r6g_cfg_$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('config c4', d['ms_per_step'])"
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-pmc --no-cpu --strong c4 > gpurun_out/r6g_leg_$rep.log 2>&1 || { tail -20 gpurun_out/r6g_leg_$rep.log; exit 1; }
  grep '^{' gpurun_out/r6g_leg_$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('leg after C2 (with pcie leg)', d['strong_c4']['ms_per_frame'])"
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-pmc --no-cpu --strong c4 --no-pcie > gpurun_out/r6g_legnp_$rep.log 2>&1 || { tail -20 gpurun_out/r6g_legnp_$rep.log; exit 1; }
  grep '^{' gpurun_out/r6g_legnp_$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('leg after C2 (no pcie leg)', d['strong_c4']['ms_per_frame'])"
done
