# GPU suite + smoke + bench of the current tree (outputs under gpurun_out/, prefix $1)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
P=${1:-c}
timeout -k 10 900 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/${P}_tests.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${P}_smoke.log 2>&1
timeout -k 10 400 python bench.py --gpus 1 --steps 10 --warmup 3 > gpurun_out/${P}_bench.json 2> gpurun_out/${P}_bench.err
