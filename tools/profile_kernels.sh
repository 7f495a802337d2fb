#!/bin/bash
# rocprofv3 kernel-trace + stats of a bench run; summary CSV copied to profiles/<tag>_kernel_stats.csv
# Only the timed loop runs (no single-frame / PCIe / PMC / CPU legs, whose different launch shapes
# would mix into the per-kernel means), and the trace's per-dispatch medians / means over the timed
# dispatches (the warm-up launches dropped) go to <tag>_kernel_timed.txt beside the rocprof summary.
# usage (on the GPU box): bash tools/profile_kernels.sh <tag> [bench args...]
set -e
TAG=$1; shift
R=$(pwd)
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_$TAG" -o run -- python3 "$R/bench.py" --no-pmc --no-cpu --no-single --no-pcie --strong '' "$@" > "$R/gpurun_out/prof_$TAG.log" 2>&1
cd "$R"
cp gpurun_out/prof_$TAG/run_kernel_stats.csv gpurun_out/${TAG}_kernel_stats.csv
python3 tools/kstats.py gpurun_out/prof_$TAG "" --skip-first 40 > gpurun_out/${TAG}_kernel_timed.txt
# c4 / c5: the bench's roofline kernel times come from 20 frames on one context alone after the timed
# loop (frames in flight overlap in the loop itself): the same dispatches' medians
case "$*" in *c4*|*c5*) { echo "# the isolated kernel-timing leg (each kernel's last 20 dispatches)";
  python3 tools/kstats.py gpurun_out/prof_$TAG "" --last 20; } >> gpurun_out/${TAG}_kernel_timed.txt;; esac
cut -d, -f1-4 gpurun_out/${TAG}_kernel_stats.csv
cat gpurun_out/${TAG}_kernel_timed.txt
