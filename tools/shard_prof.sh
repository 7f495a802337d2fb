#!/bin/bash
# Per-kernel rocprofv3 stats of one rank's shard of the C4 / C5 frame at shard counts NS (GPU box).
# usage: CFG=c4 NS="1 8" bash tools/shard_prof.sh <tag>
set -o pipefail
TAG=${1:-sp}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for n in ${NS:-1 8}; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_n$n -o k -- python3 tools/exp_shard_split.py ${CFG:-c4} 30 $n \
    > gpurun_out/${TAG}_n$n.log 2>&1 || { tail -20 gpurun_out/${TAG}_n$n.log; exit 1; }
  grep "N=$n" gpurun_out/${TAG}_n$n.log
  python3 tools/kstats.py gpurun_out/${TAG}_n$n || exit 1
done
