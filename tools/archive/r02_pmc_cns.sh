#!/bin/bash
# PMC pass over the consensus kernel (instruction mix, LDS, waits); one rocprofv3 pass
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
cd /tmp && timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY --kernel-trace -d "$GRAFT_REPO_ROOT/gpurun_out/pmc_cns" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --scale 0.3 --steps 1 --warmup 0 --no-cpu-baseline > "$GRAFT_REPO_ROOT/gpurun_out/pmc_cns.log" 2>&1
echo "pmc rc=$?"
