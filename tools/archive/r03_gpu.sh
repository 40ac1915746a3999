#!/bin/bash
# Round-3 GPU pass: the -m gpu tests (TESTS, default the whole suite), a bench line (CPU baseline
# unless NOCPU), optionally the bench under rocprofv3 kernel stats (PROF=1) and the FETCH_SIZE /
# WRITE_SIZE PMC passes (PMC=1, separate runs as MI355X_MICROARCH.md prescribes).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r03}
TESTS=${TESTS:-tests}
if [ -z "$NOTEST" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest $TESTS -m gpu -x -v --timeout 300 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/${T}_gputest.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/${T}_gputest.log
  [ $rc -eq 0 ] || exit $rc
fi
if [ -n "$SMOKE" ]; then
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1
  rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/${T}_smoke.log
  [ $rc -eq 0 ] || exit $rc
fi
[ -n "$NOBENCH" ] && exit 0
CPU=""; [ -n "$NOCPU" ] && CPU="--no-cpu-baseline"
timeout -k 10 600 python -u bench.py $CPU $BENCH_ARGS > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/${T}_bench.json
[ $rc -eq 0 ] || exit $rc
[ -z "$PROF" ] && exit 0
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/${T}_prof" -o run --output-format csv \
  -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 3 --no-cpu-baseline $BENCH_ARGS > "$GRAFT_REPO_ROOT/gpurun_out/${T}_bench_prof.json" 2>&1)
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
[ -z "$PMC" ] && exit 0
for c in FETCH_SIZE WRITE_SIZE; do
  rm -rf "$GRAFT_REPO_ROOT/gpurun_out/pmc_$c"
  (cd /tmp && timeout -s KILL 420 rocprofv3 --pmc $c --kernel-trace -d "$GRAFT_REPO_ROOT/gpurun_out/pmc_$c" -o run \
     --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 1 --warmup 1 --no-cpu-baseline $BENCH_ARGS \
     > "$GRAFT_REPO_ROOT/gpurun_out/pmc_$c.log" 2>&1) || { echo "pass $c rc=$?"; exit 1; }
  echo "pass $c ok"
done
