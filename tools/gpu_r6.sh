#!/bin/bash
# Round 6's GPU measurements that back DESIGN.md / profiles/r06_*, one case each (replaces the round's
# one-off gpu_r6_*.sh steps; the others were instances of tools/ab.sh and are in git history).
#   bash tools/gpu_r6.sh curve      1/2/4/8 strong-scaling curve of C4 / C5, rank by rank on one GPU (r06_scaling_curve.txt)
#   bash tools/gpu_r6.sh floor      a sharded rank's fixed per-frame chain against tiny shards, host cost (r06_rank_floor.txt)
#   bash tools/gpu_r6.sh gap        the N = 1 strong C4 leg after the C2 loop vs --config c4 (r06_strong_gap.txt)
#   bash tools/gpu_r6.sh hwq        GPU_MAX_HW_QUEUES 4 vs 8 for C4 / C5 and the 8-way split (r06_strong_gap.txt)
#   bash tools/gpu_r6.sh c5stream   C5 camera pass on one stream vs a side stream (needs libshs_onestream.so; r06_c5_one_stream_ab.txt)
#   bash tools/gpu_r6.sh lazy       side stream created on first use vs HEAD (needs libshs_base.so; r06_side_stream_ab.txt)
#   bash tools/gpu_r6.sh rehearse   the default line and the 8-rank rehearsal of --gpus 8 on one GPU (r06_rehearse_gpus8.log)
set -o pipefail
mkdir -p gpurun_out
ms() { grep '^{' "$1" | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print($2)"; }
case "$1" in
curve)
  for rep in 1 2; do
    for c in c4 c5; do
      SPLIT_REGIONS=1 timeout -k 10 400 python -u tools/exp_pipeline.py $c 60 1,2,4,8 3 > gpurun_out/r6c_${c}_$rep.log 2>&1 || { tail -20 gpurun_out/r6c_${c}_$rep.log; exit 1; }
      grep -E "per-rank|regions" gpurun_out/r6c_${c}_$rep.log
    done
  done ;;
floor)
  for c in c4 c5; do
    for n in 8 32 64; do
      r=0; [ $n = 8 ] && r=3
      SPLIT_ONLY=$r SPLIT_REGIONS=1 timeout -k 10 300 python -u tools/exp_pipeline.py $c 100 $n 1,3 > gpurun_out/r6fl_${c}_$n.log 2>&1 || { tail -20 gpurun_out/r6fl_${c}_$n.log; exit 1; }
      grep per-rank gpurun_out/r6fl_${c}_$n.log
    done
  done
  SPLIT_REGIONS=1 timeout -k 10 200 python3 -u tools/exp_host.py 8 3 3 200 2>&1 | grep -v amdgpu.ids
  SPLIT_REGIONS=1 timeout -k 10 200 python3 -u tools/exp_host.py 64 0 3 200 2>&1 | grep -v amdgpu.ids ;;
gap)
  for rep in 1 2; do
    timeout -k 10 300 python -u bench.py --config c4 --no-pmc --no-cpu > gpurun_out/r6g_cfg_$rep.log 2>&1 || { tail -20 gpurun_out/r6g_cfg_$rep.log; exit 1; }
    echo "config c4 $(ms gpurun_out/r6g_cfg_$rep.log "d['ms_per_step']")"
    timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-pmc --no-cpu --strong c4 > gpurun_out/r6g_leg_$rep.log 2>&1 || { tail -20 gpurun_out/r6g_leg_$rep.log; exit 1; }
    echo "leg after C2 $(ms gpurun_out/r6g_leg_$rep.log "d['strong_c4']['ms_per_frame']")"
  done ;;
hwq)
  for rep in 1 2; do
    for q in 4 8; do
      for c in c4 c5; do
        GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python -u bench.py --config $c --no-pmc --no-cpu > gpurun_out/r6q_${c}_${q}_$rep.log 2>&1 || { tail -20 gpurun_out/r6q_${c}_${q}_$rep.log; exit 1; }
        echo "q$q config $c $(ms gpurun_out/r6q_${c}_${q}_$rep.log "d['ms_per_step']")"
      done
      GPU_MAX_HW_QUEUES=$q SPLIT_REGIONS=1 timeout -k 10 300 python -u tools/exp_pipeline.py c4 60 8 3 > gpurun_out/r6q_split_${q}_$rep.log 2>&1 || { tail -20 gpurun_out/r6q_split_${q}_$rep.log; exit 1; }
      echo "q$q $(grep per-rank gpurun_out/r6q_split_${q}_$rep.log)"
    done
  done ;;
c5stream)
  TAG=r6o LIBS="gpu onestream" REPS=2 ENVS="SPLIT_REGIONS=1" GREP='per-rank|ms_per_step' bash tools/ab.sh \
    "python -u bench.py --config c5 --no-pmc --no-cpu" "python -u bench.py --steps 20 --warmup 5 --no-pmc --no-cpu --no-pcie --no-single" \
    "python -u tools/exp_pipeline.py c5 60 1,8 3" ;;
lazy)
  TAG=r6l TESTS="tests/test_lib_parity.py tests/test_regions.py tests/test_shadow_footprint.py tests/test_batch.py tests/test_gpu_parity.py" \
    LIBS="base gpu" REPS=2 ENVS="SPLIT_REGIONS=1" bash tools/ab.sh "python -u tools/exp_pipeline.py c4 60 1,8 3,4" \
    "python -u tools/exp_pipeline.py c5 60 1,8 3" "python -u bench.py --config c4 --no-pmc --no-cpu" "python -u bench.py --config c5 --no-pmc --no-cpu" ;;
rehearse)
  timeout -k 10 600 python -u bench.py > gpurun_out/r6b_default.log 2>&1 || { tail -30 gpurun_out/r6b_default.log; exit 1; }
  ms gpurun_out/r6b_default.log "d['value'], d['ms_per_step'], d['roofline']['frac'], {k: (d[k]['ms_per_frame'], d[k]['roofline']['frac']) for k in ('strong_c4', 'strong_c5')}"
  SHS_BENCH_REHEARSE=1 timeout -k 10 900 python -u bench.py --gpus 8 --steps 20 --warmup 5 --strong-frames 30 --no-cpu > gpurun_out/r6b_rehearse8.log 2>&1 || { tail -30 gpurun_out/r6b_rehearse8.log; exit 1; }
  ms gpurun_out/r6b_rehearse8.log "d['n_gpus'], d['value'], {k: (d[k]['n_gpus'], d[k]['ms_per_frame'], sorted(d[k]['roofline'])) for k in ('strong_c4', 'strong_c5')}" ;;
*)
  sed -n '2,12p' "$0"; exit 2 ;;
esac
