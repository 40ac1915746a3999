#!/bin/bash
# GPU box: the -m gpu suite (or the files given as arguments), one process, per-test timeout.
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${*:-tests}
timeout -k 10 900 python -u -m pytest $T -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gt.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gt.log
tail -5 gpurun_out/gt.log
exit $rc
