#!/bin/bash
# GPU pass: consensus tests first (new kernel), then the whole suite, the bench and a kernel profile
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_cns_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r02_cns3.log 2>&1
rc=$?; echo "cns rc=$rc"; tail -3 gpurun_out/r02_cns3.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r02_gputest3.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r02_gputest3.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 400 python -u bench.py > gpurun_out/r02_bench3.json 2> gpurun_out/r02_bench3.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/r02_bench3.json
[ $rc -eq 0 ] || exit $rc
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof3" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 3 --no-cpu-baseline > "$GRAFT_REPO_ROOT/gpurun_out/r02_bench3_prof.json" 2>&1
echo "prof rc=$?"
