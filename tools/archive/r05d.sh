set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_seed_gpu.py tests/test_seed_big_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/seedt.log 2>&1
echo "seed tests rc=$?"
timeout -k 10 900 python -u -m pytest tests/test_scale_configs_gpu.py -x -q -s --timeout 800 --timeout-method thread > gpurun_out/scale_d.log 2>&1
echo "scale rc=$?"
