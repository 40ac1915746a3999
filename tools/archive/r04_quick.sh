set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${TAG:-r04_d}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_sw_gpu.py tests/test_sw_edge_gpu.py tests/test_aln_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/${T:-r04_d}_test.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/${T:-r04_d}_test.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/${T:-r04_d}_bench.json 2> gpurun_out/${T:-r04_d}_bench.err
rc=$?; echo "bench rc=$rc"; cut -c1-300 gpurun_out/${T:-r04_d}_bench.json; [ $rc -eq 0 ] || exit $rc
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/${T:-r04_d}_prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 3 --no-cpu-baseline > "$GRAFT_REPO_ROOT/gpurun_out/${T:-r04_d}_bench_prof.json" 2>&1)
echo "prof rc=$?"
# optional extra bench runs, one per "VAR=value" word in $SWEEP (tuning hooks)
for kv in $SWEEP; do
  env "$kv" timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 3 > gpurun_out/${T}_sweep_${kv}.json 2>&1
  rc=$?; echo "sweep $kv rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
