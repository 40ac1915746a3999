#!/bin/bash
# GPU box: all parity tests, then one bench line (no CPU baseline); stop at the first failure.
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/dev_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/dev_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/dev_bench.json 2> gpurun_out/dev_bench.err
rc=$?; echo "bench rc=$rc" >> gpurun_out/dev_bench.err
exit $rc
