set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 > gpurun_out/bench_a.json 2> gpurun_out/bench_a.err
echo "bench rc=$?"
timeout -k 10 300 python -u -m pytest tests/test_local_group_gpu.py -x -v --timeout 200 --timeout-method thread > gpurun_out/lg.log 2>&1
echo "lg rc=$?"
timeout -k 10 900 python -u -m pytest tests/test_scale_configs_gpu.py -x -v -s --timeout 800 --timeout-method thread > gpurun_out/scale1.log 2>&1
