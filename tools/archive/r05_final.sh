#!/bin/bash
# Round-5 evidence on the current build: the whole -m gpu suite, smoke, the bench with both
# CPU baselines, rocprofv3 kernel stats of the bench, FETCH_SIZE / WRITE_SIZE passes and one
# SQ pass (each PMC counter set in its own run, MI355X_MICROARCH.md)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r05_final}
if [ -z "$NOTEST" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/${T}_gputest.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/${T}_gputest.log; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1
  rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/${T}_smoke.log; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 600 python -u bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/${T}_bench.json | cut -c1-400; [ $rc -eq 0 ] || exit $rc
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/${T}_prof" -o run --output-format csv \
  -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 3 --no-cpu-baseline > "$GRAFT_REPO_ROOT/gpurun_out/${T}_bench_prof.json" 2>&1)
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
for c in FETCH_SIZE WRITE_SIZE; do
  rm -rf "$GRAFT_REPO_ROOT/gpurun_out/pmc_$c"
  (cd /tmp && timeout -s KILL 420 rocprofv3 --pmc $c --kernel-trace -d "$GRAFT_REPO_ROOT/gpurun_out/pmc_$c" -o run \
     --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 1 --warmup 1 --no-cpu-baseline \
     > "$GRAFT_REPO_ROOT/gpurun_out/pmc_$c.log" 2>&1) || { echo "pass $c rc=$?"; exit 1; }
  echo "pass $c ok"
done
TAG=sq_${T} bash tools/pmc_sq.sh || exit 1
# the traffic the bench line reports: this build's PMC passes, then the bench once more
PMC_BUILD="${BUILD:-unknown}" python3 tools/pmc_summary.py pmc_traffic.json > /dev/null && cp pmc_traffic.json gpurun_out/pmc_traffic.json || exit 1
timeout -k 10 600 python -u bench.py > gpurun_out/${T}_bench_traffic.json 2> gpurun_out/${T}_bench_traffic.err
rc=$?; echo "bench (traffic) rc=$rc"; cut -c1-300 gpurun_out/${T}_bench_traffic.json; exit $rc
