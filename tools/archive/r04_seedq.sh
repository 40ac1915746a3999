# seeding GPU tests + bench (seeding kernel time, host-path parity) + rocprof of the bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${TAG:-r04_l}
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_seed_gpu.py tests/test_aln_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_test.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/${T}_test.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/${T}_bench.err; exit $rc; }
python -c "import json; d=json.loads(open('gpurun_out/${T}_bench.json').read().strip().splitlines()[-1]); s=d['seeding']; print(d['value'], d['ms_per_step'], s['kernel_ms'], s['parity_vs_host'], d['iteration_end_to_end_ms'], s['kernel_phase_ms_summed_over_waves'])"
PRGPU_SEED_LPT=0 timeout -k 10 400 python -u bench.py --no-cpu-baseline --steps 1 > gpurun_out/${T}_bench_nolpt.json 2> gpurun_out/${T}_bench_nolpt.err
rc=$?; echo "bench nolpt rc=$rc"; [ $rc -eq 0 ] || exit $rc
python -c "import json; d=json.loads(open('gpurun_out/${T}_bench_nolpt.json').read().strip().splitlines()[-1]); s=d['seeding']; print('nolpt', s['kernel_ms'], s['parity_vs_host'], d['iteration_end_to_end_ms'])"
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/${T}_prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 3 --no-cpu-baseline > "$GRAFT_REPO_ROOT/gpurun_out/${T}_bench_prof.json" 2>&1)
echo "prof rc=$?"
