#!/bin/bash
# GPU pass after a kernel change: the consensus / bwa-mode / iteration parity tests, a bench line
# (no CPU baseline), the bench under rocprofv3 kernel stats, then FETCH_SIZE and WRITE_SIZE in
# separate PMC passes (MI355X_MICROARCH.md: they do not fit one pass).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r02_5}
TESTS=${TESTS:-"tests/test_cns_gpu.py tests/test_aln_gpu.py tests/test_iter_gpu.py"}
timeout -k 10 600 python -u -m pytest $TESTS -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/${T}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/${T}_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/${T}_bench.json
[ $rc -eq 0 ] || exit $rc
[ -n "$NOPROF" ] && exit 0
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/${T}_prof" -o run --output-format csv \
  -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 3 --no-cpu-baseline > "$GRAFT_REPO_ROOT/gpurun_out/${T}_bench_prof.json" 2>&1)
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
[ -n "$NOPMC" ] && exit 0
for c in FETCH_SIZE WRITE_SIZE; do
  rm -rf "$GRAFT_REPO_ROOT/gpurun_out/pmc_$c"
  (cd /tmp && timeout -s KILL 420 rocprofv3 --pmc $c --kernel-trace -d "$GRAFT_REPO_ROOT/gpurun_out/pmc_$c" -o run \
     --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 1 --warmup 1 --no-cpu-baseline \
     > "$GRAFT_REPO_ROOT/gpurun_out/pmc_$c.log" 2>&1) || { echo "pass $c rc=$?"; exit 1; }
  echo "pass $c ok"
done
