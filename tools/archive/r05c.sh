set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c.json 2> gpurun_out/bench_c.err
echo "bench rc=$?"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c_prof.json 2> gpurun_out/bench_c_prof.err
echo "prof rc=$?"
timeout -k 10 600 python -u -m pytest "tests/test_scale_configs_gpu.py::test_one_rank_share_on_one_gpu[configs3]" -x -q -s --timeout 500 --timeout-method thread > gpurun_out/scale_c.log 2>&1
echo "scale rc=$?"
