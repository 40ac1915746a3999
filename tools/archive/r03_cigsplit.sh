# packed CIGAR pass split into DP + backtrack kernels, seeding chains in per-range lists:
# parity tests, seeding timings, then the bench (backtrack window 8 / 16, fused for comparison)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_sw_gpu.py tests/test_sw_edge_gpu.py tests/test_iter_gpu.py tests/test_aln_gpu.py \
  tests/test_seed_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/cs_test.log 2>&1
rc=$?; tail -3 gpurun_out/cs_test.log; [ $rc -eq 0 ] || exit $rc
for c in 4096,64,256,512,256 4096,64,512,512,384; do
  PRGPU_SEED_SMALL=$c timeout -k 10 300 python -u tools/seed_time.py >> gpurun_out/cs_seed.log 2>&1 || exit 1
done
cat gpurun_out/cs_seed.log
for v in "win8:PRGPU_PK_SPLIT=1" "win16:PRGPU_PK_SPLIT=1 PRGPU_PK_BT_WIN=16" "fused:"; do
  n=${v%%:*}; e=${v#*:}
  env $e timeout -k 10 400 python -u bench.py --no-cpu-baseline --steps 3 > gpurun_out/cs_bench_$n.json 2> gpurun_out/cs_bench_$n.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/cs_bench_$n.json'));print('$n',d['value'],d['stage_ms'],d['roofline']['launch_ms'],d['cigar_kernel_phase_share'],d['seeding']['kernel_ms'],d['iteration_end_to_end_ms'])"
done
