#!/bin/bash
# One SQ counter pass (<= 8 SQ counters) over a 1-step bench run: where the waves of every
# kernel spend their cycles (MI355X_MICROARCH.md: WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY ~
# WAVE_CYCLES, quad-cycle units) and how many VALU instructions they issue.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-sq}
C=${SQ_COUNTERS:-"SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES"}
rm -rf "$GRAFT_REPO_ROOT/gpurun_out/pmc_$T"
(cd /tmp && timeout -s KILL 420 rocprofv3 --pmc $C --kernel-trace -d "$GRAFT_REPO_ROOT/gpurun_out/pmc_$T" -o run \
   --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 1 --warmup 1 --no-cpu-baseline $BENCH_ARGS \
   > "$GRAFT_REPO_ROOT/gpurun_out/pmc_$T.log" 2>&1) || { echo "pass $T rc=$?"; exit 1; }
echo "pass $T ok"
