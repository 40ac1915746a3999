# backtrack: one-select state step, one-perm D4 bytes, unsigned store index, one-compare op cap: SW / bwa-mode GPU parity, bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_sw_gpu.py tests/test_sw_edge_gpu.py tests/test_aln_gpu.py -m gpu -x -q \
  --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/bt5_test.log 2>&1
rc=$?; tail -1 gpurun_out/bt5_test.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --no-cpu-baseline --steps 5 > gpurun_out/bt5_bench.json 2> gpurun_out/bt5_bench.err || exit 1
python -c "import json;d=json.load(open('gpurun_out/bt5_bench.json'));print(d['value'],d['stage_ms'],d['roofline']['launch_ms'],d['cigar_kernel_phase_share'])"
