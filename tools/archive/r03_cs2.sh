# CIGAR pass variants (split backtrack window 8 / 4, fused) on the current build
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for v in "win8:PRGPU_PK_SPLIT=1" "win4:PRGPU_PK_SPLIT=1 PRGPU_PK_BT_WIN=4" "fused:"; do
  n=${v%%:*}; e=${v#*:}
  env $e timeout -k 10 400 python -u bench.py --no-cpu-baseline --steps 3 > gpurun_out/cs2_bench_$n.json 2> gpurun_out/cs2_bench_$n.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/cs2_bench_$n.json'));print('$n',d['value'],d['stage_ms'],d['roofline']['launch_ms'],d['roofline_extension']['summed_launch_ms'],d['seeding']['kernel_ms'])"
done
