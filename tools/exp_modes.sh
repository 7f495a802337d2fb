for m in 1 2; do timeout -k 10 120 python bench.py --no-pmc --no-cpu --raster-mode $m --steps 300 --warmup 30 > gpurun_out/exp_mode$m.log 2>&1 || exit 1; done
timeout -k 10 120 python tools/timeline.py c2 > gpurun_out/exp_tl.log 2>&1
