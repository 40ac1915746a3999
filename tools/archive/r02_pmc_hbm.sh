#!/bin/bash
# GPU box: HBM bytes per launch of every kernel of the bench step (SW, hand-off, consensus),
# FETCH_SIZE and WRITE_SIZE in separate rocprofv3 passes (they do not fit one pass).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for c in FETCH_SIZE WRITE_SIZE; do
  (cd /tmp && timeout -s KILL 420 rocprofv3 --pmc $c --kernel-trace -d "$GRAFT_REPO_ROOT/gpurun_out/pmc_$c" -o run \
     --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 1 --warmup 1 --no-cpu-baseline \
     > "$GRAFT_REPO_ROOT/gpurun_out/pmc_$c.log" 2>&1) || { echo "pass $c rc=$?"; exit 1; }
  echo "pass $c ok"
done
