set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/h_tests.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/h_smoke.log 2>&1
timeout -k 10 300 python bench.py --gpus 1 --steps 10 --warmup 3 > gpurun_out/h_bench.json 2> gpurun_out/h_bench.err
