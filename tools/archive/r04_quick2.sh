# quick GPU check of the hand-off path (bin filter) + bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${TAG:-r04_k}
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_iter_gpu.py tests/test_xchg_gpu.py tests/test_file_chain_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_test.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/${T}_test.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err
rc=$?; echo "bench rc=$rc"; cut -c1-300 gpurun_out/${T}_bench.json; [ $rc -eq 0 ] || exit $rc
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/${T}_prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 3 --no-cpu-baseline > "$GRAFT_REPO_ROOT/gpurun_out/${T}_bench_prof.json" 2>&1)
echo "prof rc=$?"
