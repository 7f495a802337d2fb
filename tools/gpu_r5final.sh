#!/bin/bash
# Round 5 end: the whole -m gpu suite, smoke(), and the default bench line (what the driver runs).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/r5final_tests.log 2>&1 || { tail -30 gpurun_out/r5final_tests.log; exit 1; }
tail -1 gpurun_out/r5final_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5final_smoke.log 2>&1 || { tail -20 gpurun_out/r5final_smoke.log; exit 1; }
tail -1 gpurun_out/r5final_smoke.log
timeout -k 10 600 python bench.py > gpurun_out/r5final_bench.log 2>&1 || { tail -20 gpurun_out/r5final_bench.log; exit 1; }
grep '^{' gpurun_out/r5final_bench.log | tail -1 | cut -c1-400
