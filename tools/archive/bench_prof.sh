#!/bin/bash
# GPU box: one bench line (no CPU baseline), then the same run under rocprofv3 kernel stats.
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bp_bench.json 2> gpurun_out/bp_bench.err || exit $?
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/bp_prof -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bp_prof.log 2>&1 || exit $?
find gpurun_out/bp_prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} gpurun_out/bp_kernel_stats.csv
