#!/bin/bash
# GPU box: parity tests, one bench line, then rocprofv3 kernel stats of a short bench run.
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/dev_check.sh || exit $?
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/dp_prof -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/dp_prof.log 2>&1 || exit $?
f=$(find gpurun_out/dp_prof -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] && cp "$f" gpurun_out/dp_kernel_stats.csv
exit 0
