# seeding (balanced grid, larger pass-1 caps) and the CIGAR backtrack walk statistics
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/seed_time.py > gpurun_out/bt_seed.log 2>&1 || exit 1
PRGPU_SEED_NO_BALANCE=1 timeout -k 10 300 python -u tools/seed_time.py >> gpurun_out/bt_seed.log 2>&1 || exit 1
cat gpurun_out/bt_seed.log
PRGPU_SW_DEBUG=4 timeout -k 10 400 python -u bench.py --no-cpu-baseline --steps 1 > gpurun_out/bt_bench.json 2> gpurun_out/bt_bench.err || exit 1
grep "\[sw\]" gpurun_out/bt_bench.err | tail -2
python -c "import json;d=json.load(open('gpurun_out/bt_bench.json'));print(d['value'],d['stage_ms'],d['roofline']['launch_ms'],d['seeding']['kernel_ms'],d['iteration_end_to_end_ms'])"
