#!/bin/bash
# occupancy sweep of the bwa-mode one-lane-per-read kernels (PRGPU_ALN_*_WG): bench under kernel trace
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for k in ${KS:-0 1 2 3 4}; do
  (cd /tmp && PRGPU_ALN_FINAL_WG=$k PRGPU_ALN_WALK_WG=$k timeout -k 10 300 rocprofv3 --kernel-trace -d "$GRAFT_REPO_ROOT/gpurun_out/alnwg_$k" -o run --output-format csv \
    -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline > "$GRAFT_REPO_ROOT/gpurun_out/alnwg_$k.json" 2>&1) || { echo "k=$k failed"; exit 1; }
  echo "k=$k ok"
done
