# seed/scale GPU tests in the order that exposed the big-index leftover, then an
# interleaved A/B (base,new,base,new) printing step and seeding times
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest ${TESTS:-tests/test_seed_gpu.py tests/test_seed_big_gpu.py tests/test_scale_configs_gpu.py} -m gpu -x -q --timeout 400 --timeout-method thread -p no:cacheprovider > gpurun_out/r05j_tests.log 2>&1
rc=$?
echo "tests rc=$rc"; tail -3 gpurun_out/r05j_tests.log
[ $rc -le 1 ] || exit $rc
for it in "$@"; do
  tag=$(basename $it .so)
  PRGPU_LIB=$it timeout -k 10 200 python -u bench.py --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/abj_$tag.json 2> gpurun_out/abj_$tag.err || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/abj_$tag.json').read());s=d['stage_event_ms'];print('$tag', d['ms_per_step'], s.get('seeding'), d.get('seeding_phase_ms_summed_over_waves'))" | tee -a gpurun_out/abj.txt
done
