#!/bin/bash
# PMC passes over tools/exp_shard_split.py (one rocprofv3 --pmc run per counter set): the per-rank
# kernels of a tile-sharded C4 / C5 frame.  usage (GPU box): bash tools/pmc_split.sh <tag> <cfg> <N>
# (env SPLIT_CULL / SPLIT_PART pass through to exp_shard_split.py)
set -o pipefail
TAG=$1; CFG=${2:-c4}; N=${3:-8}
R=$(pwd); export TMPDIR=/tmp
mkdir -p "$R/gpurun_out"
run_pass() {
  local name=$1; shift
  ( cd /tmp && timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d "$R/gpurun_out/pmcs_${TAG}_$name" -o pmc -- \
      python3 "$R/tools/exp_shard_split.py" $CFG 6 $N ) > "$R/gpurun_out/pmcs_${TAG}_$name.log" 2>&1 \
      || { echo "pass $name failed"; tail -5 "$R/gpurun_out/pmcs_${TAG}_$name.log"; return 1; }
}
run_pass A SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_INSTS_SALU || exit 1
run_pass B FETCH_SIZE GRBM_GUI_ACTIVE || exit 1
run_pass C WRITE_SIZE || exit 1
python3 - "$TAG" <<'PY'
import csv, glob, json, sys, collections
tag = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for p in "ABC":
    for f in glob.glob(f"gpurun_out/pmcs_{tag}_{p}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            agg[r["Kernel_Name"].split("(")[0]][r["Counter_Name"]].append(float(r["Counter_Value"]))
out = {}
for k, d in agg.items():
    m = {c: (sum(v[3:]) / len(v[3:]) if len(v) > 3 else sum(v) / len(v)) for c, v in d.items()}
    if "FETCH_SIZE" in m: m["fetch_bytes_x2"] = 2.0 * m["FETCH_SIZE"] * 1024.0
    if "WRITE_SIZE" in m: m["write_bytes"] = m["WRITE_SIZE"] * 1024.0
    if "SQ_WAIT_ANY" in m and m.get("SQ_WAVE_CYCLES"):
        m["wait_any_frac"] = m["SQ_WAIT_ANY"] / m["SQ_WAVE_CYCLES"]
    out[k] = {c: round(v, 4) for c, v in sorted(m.items())}
json.dump(out, open(f"gpurun_out/pmcs_{tag}.json", "w"), indent=1)
for k, v in out.items():
    print(k, v)
PY
