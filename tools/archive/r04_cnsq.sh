# consensus GPU tests (goldens, fantasticus, scale fixtures vs Perl outputs, product path) + bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${TAG:-r04_m}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_cns_gpu.py tests/test_fantasticus_cns.py tests/test_scale_cns.py tests/test_iter_gpu.py tests/test_product_configs_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_test.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/${T}_test.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/${T}_bench.err; exit $rc; }
python -c "import json; d=json.loads(open('gpurun_out/${T}_bench.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['stage_ms'], d['roofline_consensus']['frac'], d['consensus_phase_ms_summed_over_workgroups'])"
PRGPU_CNS_PREP=0 timeout -k 10 400 python -u bench.py --no-cpu-baseline --steps 3 > gpurun_out/${T}_bench_noprep.json 2> gpurun_out/${T}_bench_noprep.err
rc=$?; echo "bench noprep rc=$rc"; [ $rc -eq 0 ] || exit $rc
python -c "import json; d=json.loads(open('gpurun_out/${T}_bench_noprep.json').read().strip().splitlines()[-1]); print('noprep', d['value'], d['ms_per_step'], d['stage_ms'], d['roofline_consensus']['frac'])"
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/${T}_prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 3 --no-cpu-baseline > "$GRAFT_REPO_ROOT/gpurun_out/${T}_bench_prof.json" 2>&1)
echo "prof rc=$?"
