#!/bin/bash
# GPU box: the -m gpu suite, smoke, then a bench line (stdout JSON) -- stops at the first failure.
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gt.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gt.log
tail -3 gpurun_out/gt.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke failed; exit 1; }
echo smoke ok
timeout -k 10 600 python bench.py ${BENCH_ARGS} > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench rc=$rc"; exit $rc
