# seeding / loop GPU tests on the default build, then the correction-loop profile
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_seed_gpu.py tests/test_iter_gpu.py tests/test_file_chain_gpu.py tests/test_product_configs_gpu.py tests/test_configs4_gpu.py -m gpu -x -q --timeout 400 --timeout-method thread -p no:cacheprovider > gpurun_out/r05m_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r05m_tests.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 400 python -u tools/loop_profile.py 1.0 gpurun_out/loop_r05b.json > gpurun_out/loop_r05b.log 2>&1
rc=$?; echo "loop rc=$rc"; tail -3 gpurun_out/loop_r05b.log; exit $rc
