# GPU suite, smoke and the driver's bench command; prefix $1
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
P=${1:-f}
timeout -k 10 900 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/${P}_tests.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${P}_smoke.log 2>&1
timeout -k 10 500 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${P}_bench.json 2> gpurun_out/${P}_bench.err
