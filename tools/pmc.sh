#!/bin/bash
# GPU box: HBM traffic of the dominant kernel from PMC counters, one counter per pass
# (MI355X_MICROARCH.md "rocprofv3 PMC slots": FETCH_SIZE and WRITE_SIZE do not fit one pass).
mkdir -p gpurun_out
export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 500 rocprofv3 --pmc $c --kernel-trace -d gpurun_out/pmc_$c -o run --output-format csv -- python3 bench.py --task-only --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_$c.log 2>&1 || exit $?
done
exit 0
