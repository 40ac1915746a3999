#!/bin/bash
# GPU box: parity tests, smoke, a full bench line (with the CPU baseline), rocprofv3 kernel stats.
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/rc_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/rc_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/rc_smoke.log 2>&1 || exit $?
timeout -k 10 500 python bench.py > gpurun_out/rc_bench.json 2> gpurun_out/rc_bench.err || exit $?
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/rc_prof -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/rc_prof.log 2>&1 || exit $?
f=$(find gpurun_out/rc_prof -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] && cp "$f" gpurun_out/rc_kernel_stats.csv
exit 0
