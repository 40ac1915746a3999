set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_seed_gpu.py tests/test_cns_gpu.py tests/test_iter_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r05h_tests.log 2>&1
rc=$?
echo "tests rc=$rc"; tail -2 gpurun_out/r05h_tests.log
[ $rc -le 1 ] || exit $rc
bash tools/r05_abv.sh "$@"
