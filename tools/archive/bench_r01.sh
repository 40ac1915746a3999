#!/bin/bash
# round-1 measurement on the GPU box: bench line + rocprofv3 kernel trace of the same command
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python bench.py --steps 5 --warmup 1 > gpurun_out/bench_r01.json 2> gpurun_out/bench_r01.err
rc=$?; echo "bench rc=$rc" >> gpurun_out/bench_r01.err
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r01 -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof_r01.log 2>&1
rc=$?; echo "rocprof rc=$rc" >> gpurun_out/prof_r01.log
exit $rc
