#!/bin/bash
# GPU box: rocprofv3 kernel stats of a short bench run (no tests).
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/po_prof -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/po_prof.log 2>&1 || exit $?
f=$(find gpurun_out/po_prof -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] && cp "$f" gpurun_out/po_kernel_stats.csv
exit 0
