# consensus parity tests, then the loop with the finish task's consensus phase clocks; prefix $1
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
P=${1:-n}
timeout -k 10 600 python -u -m pytest tests/test_cns_gpu.py tests/test_scale_cns.py tests/test_fantasticus_cns.py tests/test_correct_loop.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/${P}_tests.log 2>&1
timeout -k 10 200 python bench.py --loop-only --steps 5 --warmup 1 > gpurun_out/${P}_loop.json 2> gpurun_out/${P}_loop.err
PRGPU_CNS_PROF=1 timeout -k 10 200 python bench.py --loop-only --steps 2 --warmup 1 > gpurun_out/${P}_loopprof.json 2> gpurun_out/${P}_loopprof.err
