#!/bin/bash
# GPU box: bench lines under PRGPU_SW_DEBUG ablations (timing only; results are not checked).
mkdir -p gpurun_out
for d in 0 1 2; do
  PRGPU_SW_DEBUG=$d timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/ab_$d.json 2> gpurun_out/ab_$d.err || exit $?
done
exit 0
