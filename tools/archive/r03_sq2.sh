# extension chunk statistics, then one SQ counter pass (where the backtrack kernel's waves spend their cycles)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
PRGPU_SW_DEBUG=4 timeout -k 10 400 python -u bench.py --no-cpu-baseline --steps 1 > gpurun_out/sq2_bench.json 2> gpurun_out/sq2_bench.err || exit 1
grep "\[sw\]" gpurun_out/sq2_bench.err | tail -2
python -c "import json;d=json.load(open('gpurun_out/sq2_bench.json'));print(d['value'],d['stage_ms'],d['roofline']['launch_ms'],d['seeding']['kernel_ms'],d['iteration_end_to_end_ms'])"
TAG=sq2 bash tools/pmc_sq.sh && python tools/sq_summary.py gpurun_out/pmc_sq2 gpurun_out/sq2.json > /dev/null && python -c "
import json; d=json.load(open('gpurun_out/sq2.json'))
for k,v in d.items():
    if 'pk' in k or 'seed_batch' in k: print(k, v)"
