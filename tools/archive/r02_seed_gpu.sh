#!/bin/bash
# GPU: seeding tests, then a short bench with GPU seeding (no CPU baseline)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_seed_gpu.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/seed.log 2>&1
rc=$?; echo "seed tests rc=$rc"; tail -4 gpurun_out/seed.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --steps 2 --no-cpu-baseline --seeds gpu ${BENCH_ARGS} > gpurun_out/bs.json 2> gpurun_out/bs.err
rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/bs.err; exit $rc
