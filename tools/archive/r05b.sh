set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_seed_gpu.py tests/test_seed_big_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/seedt.log 2>&1
echo "seed tests rc=$?"
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 > gpurun_out/bench_b.json 2> gpurun_out/bench_b.err
echo "bench rc=$?"
