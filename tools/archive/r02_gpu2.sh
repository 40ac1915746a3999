#!/bin/bash
# GPU pass: the whole -m gpu suite (stop at the first failure), then one bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r02_gputest2.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/r02_gputest2.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 400 python -u bench.py > gpurun_out/r02_bench2.json 2> gpurun_out/r02_bench2.err
echo "bench rc=$?"; cat gpurun_out/r02_bench2.json
