# A/B of pass 1's chaining by the wave (PRGPU_SEED_WCHAIN) on MI355X: seeding parity tests, then
# the configs[1] correction loop both ways
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
PRGPU_SEED_WCHAIN=1 timeout -k 10 400 python -u -m pytest tests/test_seed_gpu.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/ab_seedtests.log 2>&1
for wc in 0 1 0 1; do
  PRGPU_SEED_WCHAIN=$wc timeout -k 10 200 python bench.py --loop-only --steps 3 --warmup 1 > gpurun_out/ab_loop_wc$wc.json 2> gpurun_out/ab_loop_wc$wc.err
  python -c "
import json;d=json.load(open('gpurun_out/ab_loop_wc$wc.json'))
print('wc=$wc', d['value'], d['ms_per_step'], [ (t['task'], t['stage_event_ms']['seeding']) for t in d['loop']['tasks']], d['loop'].get('final_reads_sha256'))"
done
