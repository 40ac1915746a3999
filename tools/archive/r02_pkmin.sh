#!/bin/bash
# bwa-mode round sizes and the small-list routing threshold (PRGPU_PK_MIN_TASKS) under kernel trace
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_aln_gpu.py tests/test_iter_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pkmin_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/pkmin_tests.log; [ $rc -eq 0 ] || exit $rc
for k in ${KS:-0 65536 300000}; do
  (cd /tmp && PRGPU_BWA_DEBUG=1 PRGPU_PK_MIN_TASKS=$k timeout -k 10 300 rocprofv3 --kernel-trace -d "$GRAFT_REPO_ROOT/gpurun_out/pkmin_$k" -o run --output-format csv \
    -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline > "$GRAFT_REPO_ROOT/gpurun_out/pkmin_$k.json" 2> "$GRAFT_REPO_ROOT/gpurun_out/pkmin_$k.err") || { echo "k=$k failed"; exit 1; }
  echo "k=$k ok"
done
