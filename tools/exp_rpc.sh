#!/bin/bash
# Legacy k_raster resident blocks per CU vs the setup stream's overlap (GPU box, timing only).
set -o pipefail
mkdir -p gpurun_out
for c in ${CFGS:-c2 c3}; do for r in ${RPCS:-4 3 2}; do
  SHS_RASTER_PER_CU=$r timeout -k 10 200 python bench.py --config $c --no-pmc --no-cpu --no-single --no-pcie --steps 20 --warmup 5 \
    > gpurun_out/rpc_${c}_$r.log 2>&1 || { tail -5 gpurun_out/rpc_${c}_$r.log; exit 1; }
  echo "$c per_cu=$r $(grep '^{' gpurun_out/rpc_${c}_$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["kernels_ms"], d["ms_per_step"])')"
done; done
