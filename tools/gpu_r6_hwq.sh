#!/bin/bash
# Round 6: hardware queues per process (GPU_MAX_HW_QUEUES, default 4) for the library configs with three
# frames in flight (3 contexts x 2 streams), and the PCIe-leg-first order of the previous bench.py.
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
  for q in 4 8; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python -u bench.py --config c4 --no-pmc --no-cpu > gpurun_out/r6q_c4_${q}_$rep.log 2>&1 || { tail -20 gpurun_out/r6q_c4_${q}_$rep.log; exit 1; }
    grep '^{' gpurun_out/r6q_c4_${q}_$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('q$q config c4', d['ms_per_step'])"
    GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python -u bench.py --config c5 --no-pmc --no-cpu > gpurun_out/r6q_c5_${q}_$rep.log 2>&1 || { tail -20 gpurun_out/r6q_c5_${q}_$rep.log; exit 1; }
    grep '^{' gpurun_out/r6q_c5_${q}_$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('q$q config c5', d['ms_per_step'])"
    GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python -u tools/_bench_pcie_first.py --steps 20 --warmup 5 --no-pmc --no-cpu --strong c4 > gpurun_out/r6q_leg_${q}_$rep.log 2>&1 || { tail -20 gpurun_out/r6q_leg_${q}_$rep.log; exit 1; }
    grep '^{' gpurun_out/r6q_leg_${q}_$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('q$q pcie-first leg c4', d['strong_c4']['ms_per_frame'], 'c2', d['value'])"
    GPU_MAX_HW_QUEUES=$q SPLIT_REGIONS=1 timeout -k 10 300 python -u tools/exp_pipeline.py c4 60 8 3 > gpurun_out/r6q_split_${q}_$rep.log 2>&1 || { tail -20 gpurun_out/r6q_split_${q}_$rep.log; exit 1; }
    echo "q$q $(grep per-rank gpurun_out/r6q_split_${q}_$rep.log)"
  done
done
