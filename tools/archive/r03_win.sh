# fused CIGAR kernel with an 8-row backtrack window (half the unrolled walk code) vs 16, and the
# kernel trace of the default build (what the step's memsets cost)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_sw_gpu.py tests/test_sw_edge_gpu.py -m gpu -x -q --timeout 300 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/win_test.log 2>&1
rc=$?; tail -2 gpurun_out/win_test.log; [ $rc -eq 0 ] || exit $rc
PRGPU_PK_WIN=8 timeout -k 10 600 python -u -m pytest tests/test_sw_gpu.py tests/test_sw_edge_gpu.py -m gpu -x -q --timeout 300 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/win8_test.log 2>&1
rc=$?; tail -2 gpurun_out/win8_test.log; [ $rc -eq 0 ] || exit $rc
for v in "w16:" "w8:PRGPU_PK_WIN=8"; do
  n=${v%%:*}; e=${v#*:}
  env $e timeout -k 10 400 python -u bench.py --no-cpu-baseline --steps 3 > gpurun_out/win_$n.json 2> gpurun_out/win_$n.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/win_$n.json'));print('$n',d['value'],d['stage_ms'],d['roofline']['launch_ms'],d['cigar_kernel_phase_share'])"
done
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/win_prof" -o run --output-format csv \
  -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 2 --no-cpu-baseline > "$GRAFT_REPO_ROOT/gpurun_out/win_prof.json" 2>&1) || exit 1
echo prof ok
