# chain-head links after round 0's left DP launch, 12-byte SMEM intervals: bwa-mode + seeding tests, bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=${TAG:-heads}
timeout -k 10 600 python -u -m pytest tests/test_aln_gpu.py tests/test_seed_gpu.py tests/test_iter_gpu.py -m gpu -x -q --timeout 300 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_test.log 2>&1
rc=$?; tail -2 gpurun_out/${T}_test.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/seed_time.py > gpurun_out/${T}_seed.log 2>&1 || exit 1
cat gpurun_out/${T}_seed.log
timeout -k 10 400 python -u bench.py --no-cpu-baseline --steps 3 > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || exit 1
python -c "import json;d=json.load(open('gpurun_out/${T}_bench.json'));print(d['value'],d['stage_ms'],d['seeding']['kernel_ms'],d['seeding']['parity_vs_host'],d['iteration_end_to_end_ms'])"
