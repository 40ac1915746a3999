# seeding changes: GPU = oracle tests, then the seeding time at configs[1]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=${TAG:-seed}
timeout -k 10 600 python -u -m pytest tests/test_seed_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/${T}_test.log 2>&1
rc=$?; tail -2 gpurun_out/${T}_test.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/seed_time.py > gpurun_out/${T}_seed.log 2>&1 || exit 1
cat gpurun_out/${T}_seed.log
