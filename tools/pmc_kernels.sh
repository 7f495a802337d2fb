#!/bin/bash
# PMC passes (one rocprofv3 --pmc run each, nothing else traced) over a short bench child run:
#   A  SQ: waves, VALU instructions, VALU-active / busy / wave cycles, wait / issue-stall / active buckets
#   B  FETCH_SIZE (3 TCC slots) + GRBM_GUI_ACTIVE      C  WRITE_SIZE
# Per kernel: the mean over the dispatches after the first 3.  FETCH_SIZE is doubled (gfx950 counts
# half of a wide coalesced read, MI355X_MICROARCH.md HBM); KiB -> bytes.
# usage (GPU box): bash tools/pmc_kernels.sh <tag> <bench args...>
set -o pipefail
TAG=$1; shift
R=$(pwd); export TMPDIR=/tmp
mkdir -p "$R/gpurun_out"
run_pass() {
  local name=$1; shift
  ( cd /tmp && timeout -s KILL 150 rocprofv3 --pmc "$@" --output-format csv -d "$R/gpurun_out/pmc_${TAG}_$name" -o pmc -- \
      python3 "$R/bench.py" --child --steps 12 --warmup 3 $BENCH ) > "$R/gpurun_out/pmc_${TAG}_$name.log" 2>&1 \
      || { echo "pass $name failed"; tail -5 "$R/gpurun_out/pmc_${TAG}_$name.log"; return 1; }
}
BENCH="$*"
run_pass A SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY || exit 1
run_pass B FETCH_SIZE GRBM_GUI_ACTIVE || exit 1
run_pass C WRITE_SIZE || exit 1
python3 - "$TAG" <<'PY'
import csv, glob, json, sys, collections
tag = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for p in "ABC":
    for f in glob.glob(f"gpurun_out/pmc_{tag}_{p}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            agg[r["Kernel_Name"].split("(")[0]][r["Counter_Name"]].append(float(r["Counter_Value"]))
out = {}
for k, d in agg.items():
    m = {c: (sum(v[3:]) / len(v[3:]) if len(v) > 3 else sum(v) / len(v)) for c, v in d.items()}
    if "FETCH_SIZE" in m: m["fetch_bytes_x2"] = 2.0 * m["FETCH_SIZE"] * 1024.0
    if "WRITE_SIZE" in m: m["write_bytes"] = m["WRITE_SIZE"] * 1024.0
    if "SQ_ACTIVE_INST_VALU" in m and "SQ_WAVE_CYCLES" in m and m["SQ_WAVE_CYCLES"]:
        m["valu_active_per_wave_cycle"] = m["SQ_ACTIVE_INST_VALU"] / m["SQ_WAVE_CYCLES"]
    if "SQ_WAIT_ANY" in m and "SQ_WAVE_CYCLES" in m and m["SQ_WAVE_CYCLES"]:
        m["wait_any_frac"] = m["SQ_WAIT_ANY"] / m["SQ_WAVE_CYCLES"]
    out[k] = {c: round(v, 4) for c, v in sorted(m.items())}
json.dump(out, open(f"gpurun_out/pmc_{tag}.json", "w"), indent=1)
for k, v in out.items():
    print(k, v)
PY
