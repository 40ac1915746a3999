# consensus geometry experiment: correctness on the iteration tests, then the bench stage times
mkdir -p gpurun_out
PRGPU_CNS_GEO=M timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_iter_gpu.py tests/test_cns_gpu.py > gpurun_out/geo.log 2>&1 || exit 1
PRGPU_CNS_GEO=M timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 2 > gpurun_out/bench_geoM.json 2>> gpurun_out/geo.log || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 2 > gpurun_out/bench_geoS.json 2>> gpurun_out/geo.log
