set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_cns_gpu.py tests/test_iter_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/cnstests.log 2>&1
rc=$?
echo "cns tests rc=$rc"; tail -3 gpurun_out/cnstests.log
[ $rc -le 1 ] || exit $rc
bash tools/r05_ab.sh "$@"
if [ -n "$IV12" ]; then
  PRGPU_LIB=tools/probe/libprgpu_iv12.so timeout -k 10 300 python -u tools/probe/iv12_probe.py > gpurun_out/iv12_r05.log 2>&1
  echo "iv12 rc=$?"
fi
