# fused vs split CIGAR pass after the backtrack rewrite: bench (3 steps) and kernel stats
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in "fused:PRGPU_PK_WIN=8" "split8:PRGPU_PK_SPLIT=1" "split4:PRGPU_PK_SPLIT=1 PRGPU_PK_BT_WIN=4"; do
  n=${v%%:*}; e=${v#*:}
  env $e timeout -k 10 400 python -u bench.py --no-cpu-baseline --steps 3 > gpurun_out/splitb_$n.json 2> gpurun_out/splitb_$n.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/splitb_$n.json'));print('$n',d['value'],d['stage_ms'])"
done
(cd /tmp && PRGPU_PK_SPLIT=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/splitb_prof" -o run --output-format csv \
  -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 2 --no-cpu-baseline > "$GRAFT_REPO_ROOT/gpurun_out/splitb_prof.json" 2>&1) || exit 1
echo prof ok
