set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_sw_gpu.py tests/test_sw_edge_gpu.py tests/test_aln_gpu.py tests/test_product_configs_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/swtests.log 2>&1
rc=$?
echo "sw tests rc=$rc"; tail -3 gpurun_out/swtests.log
[ $rc -le 1 ] || exit $rc
bash tools/r05_ab.sh base new new2 base new new2
