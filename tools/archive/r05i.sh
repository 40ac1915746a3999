set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_seed_gpu.py tests/test_sw_gpu.py tests/test_sw_edge_gpu.py tests/test_aln_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r05i_tests.log 2>&1
rc=$?
echo "tests rc=$rc"; tail -2 gpurun_out/r05i_tests.log
[ $rc -le 1 ] || exit $rc
if [ -n "$TW2TEST" ]; then
  PRGPU_LIB=tools/probe/libext_tw2.so timeout -k 10 600 python -u -m pytest tests/test_sw_gpu.py tests/test_aln_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r05i_tw2.log 2>&1
  echo "tw2 tests rc=$?"; tail -1 gpurun_out/r05i_tw2.log
fi
bash tools/r05_abv.sh "$@"
