set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T="python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread"
timeout -k 10 300 $T tests/test_correct_loop.py > gpurun_out/k_alone.log 2>&1 || echo "alone failed"
PRGPU_INDEX_KEXT_BYTES=1 timeout -k 10 400 $T tests/test_seed_big_gpu.py tests/test_correct_loop.py > gpurun_out/k_bytes.log 2>&1 || echo "bytes-order failed"
timeout -k 10 400 $T tests/test_seed_big_gpu.py tests/test_correct_loop.py > gpurun_out/k_nib.log 2>&1 || echo "nibble-order failed"
tail -1 gpurun_out/k_alone.log gpurun_out/k_bytes.log gpurun_out/k_nib.log
