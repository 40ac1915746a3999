# Round profiles (GPU box): rocprofv3 kernel stats of the bwa-sr-1 task phase (the rooflines'
# kernels) and of the correction loop, then the PMC FETCH_SIZE / WRITE_SIZE passes of the task
# phase; outputs under gpurun_out/, prefix $1
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
P=${1:-p}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${P}_task -o run --output-format csv -- python3 bench.py --task-only --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${P}_task.json 2> gpurun_out/${P}_task.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${P}_loop -o run --output-format csv -- python3 bench.py --loop-only --steps 2 --warmup 1 > gpurun_out/${P}_loop.json 2> gpurun_out/${P}_loop.err
bash tools/pmc.sh
