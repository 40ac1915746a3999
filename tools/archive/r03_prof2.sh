# kernel stats of the bench for the current build (split CIGAR pass) and the fused CIGAR kernel
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in "split:PRGPU_PK_SPLIT=1" "fused:"; do
  n=${v%%:*}; e=${v#*:}
  (cd /tmp && env $e timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/p2_$n" -o run --output-format csv \
    -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 2 --no-cpu-baseline > "$GRAFT_REPO_ROOT/gpurun_out/p2_$n.json" 2> "$GRAFT_REPO_ROOT/gpurun_out/p2_$n.err") || exit 1
  f=$(find "$GRAFT_REPO_ROOT/gpurun_out/p2_$n" -name "*kernel_stats.csv" | head -1)
  cp "$f" "$GRAFT_REPO_ROOT/gpurun_out/p2_${n}_kernel_stats.csv"
  head -14 "$GRAFT_REPO_ROOT/gpurun_out/p2_${n}_kernel_stats.csv" | cut -c1-150
done
