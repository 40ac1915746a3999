# rocprofv3 kernel trace of the correction loop; prefix $1
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
P=${1:-t}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${P}_loop -o run --output-format csv -- python3 bench.py --loop-only --steps 2 --warmup 1 > gpurun_out/${P}_loop.json 2> gpurun_out/${P}_loop.err
