#!/bin/bash
# Round end, as the driver runs it: the whole -m gpu suite, smoke(), and the default bench line
# (TAG names the logs under gpurun_out/; was tools/gpu_r5final.sh).
set -o pipefail
TAG=${TAG:-final}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.log
timeout -k 10 600 python bench.py > gpurun_out/${TAG}_bench.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench.log; exit 1; }
grep '^{' gpurun_out/${TAG}_bench.log | tail -1 | cut -c1-400
