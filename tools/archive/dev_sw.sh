#!/bin/bash
# GPU box: SW + iteration parity tests, then bench lines (normal and backtrack-skipped timing ablation).
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_sw_gpu.py tests/test_iter_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/sw_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/sw_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/sw_bench.json 2> gpurun_out/sw_bench.err || exit $?
PRGPU_SW_DEBUG=1 timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/sw_bench_d1.json 2> gpurun_out/sw_bench_d1.err || exit $?
exit 0
