#!/bin/bash
# consensus walk timing ablations (outputs invalid under PRGPU_CNS_DEBUG; timing only)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for dbg in 0 1 2 3; do
  PRGPU_CNS_DEBUG=$dbg timeout -k 10 200 python -u bench.py --scale 0.3 --steps 1 --no-cpu-baseline > gpurun_out/abl_$dbg.json 2> gpurun_out/abl_$dbg.err
  rc=$?; echo "dbg=$dbg rc=$rc"; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
done
