#!/bin/bash
# GPU pass on HEAD: whole -m gpu suite (verbose, one process), smoke, a full bench line
# (CPU baseline included), then the same bench under rocprofv3 kernel stats.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r02_4}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/${T}_gputest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/${T}_gputest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/${T}_smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/${T}_bench.json
[ $rc -eq 0 ] || exit $rc
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/${T}_prof" -o run --output-format csv \
  -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 3 --no-cpu-baseline > "$GRAFT_REPO_ROOT/gpurun_out/${T}_bench_prof.json" 2>&1
echo "prof rc=$?"
