# seeding parity tests, then the loop; prefix $1
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
P=${1:-z}
timeout -k 10 700 python -u -m pytest tests/test_seed_gpu.py tests/test_seed_big_gpu.py tests/test_correct_loop.py tests/test_bwa_mem_gpu_path.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/${P}_tests.log 2>&1
timeout -k 10 200 python bench.py --loop-only --steps 5 --warmup 1 > gpurun_out/${P}_loop.json 2> gpurun_out/${P}_loop.err
