#!/bin/bash
# GPU: consensus goldens, then one short bench line (no CPU baseline)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_cns_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/cns.log 2>&1
rc=$?; echo "cns rc=$rc"; tail -2 gpurun_out/cns.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --steps 2 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/bq.json 2> gpurun_out/bq.err
rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/bq.err; exit $rc
