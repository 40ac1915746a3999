# the non-default CIGAR paths after the backtrack rewrite: fused window 16, and the split
# DP / backtrack kernels (windows 8 and 4), SW + bwa-mode GPU parity each
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in "w16:PRGPU_PK_WIN=16" "split8:PRGPU_PK_SPLIT=1" "split4:PRGPU_PK_SPLIT=1 PRGPU_PK_BT_WIN=4"; do
  n=${v%%:*}; e=${v#*:}
  env $e timeout -k 10 600 python -u -m pytest tests/test_sw_gpu.py tests/test_sw_edge_gpu.py tests/test_aln_gpu.py -m gpu -x -q \
    --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/btmodes_$n.log 2>&1
  rc=$?; echo "$n: $(tail -1 gpurun_out/btmodes_$n.log)"; [ $rc -eq 0 ] || exit $rc
done
