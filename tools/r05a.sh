set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 > gpurun_out/bench_a.json 2> gpurun_out/bench_a.err && \
timeout -k 10 900 python -u -m pytest tests/test_scale_configs_gpu.py -x -v -s --timeout 800 --timeout-method thread > gpurun_out/scale1.log 2>&1
