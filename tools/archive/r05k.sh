# kernel statistics of the configs[3] rank task (the scale test) under rocprofv3
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3 -o c3 -- python3 -u -m pytest tests/test_scale_configs_gpu.py -k configs3 -m gpu -x -q --timeout 500 --timeout-method thread -p no:cacheprovider > gpurun_out/r05k.log 2>&1
rc=$?; echo "rc=$rc"; tail -2 gpurun_out/r05k.log
f=$(find gpurun_out/prof_c3 -name '*kernel_stats.csv' | head -1); echo "$f"
[ -n "$f" ] && cp "$f" gpurun_out/c3_kernel_stats.csv
find gpurun_out/prof_c3 -name '*kernel_trace.csv' -delete
exit $rc
