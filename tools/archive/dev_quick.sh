#!/bin/bash
# GPU box: SW/iteration parity tests, one bench line, rocprofv3 kernel stats of a short bench run.
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/q_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/q_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/q_bench.json 2> gpurun_out/q_bench.err || exit $?
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/q_prof -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/q_prof.log 2>&1 || exit $?
f=$(find gpurun_out/q_prof -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] && cp "$f" gpurun_out/q_kernel_stats.csv
exit 0
