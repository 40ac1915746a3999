set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpuall.log 2>&1
rc=$?
echo "gpu tests rc=$rc"
if [ $rc -le 1 ]; then
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/bench_e.json 2> gpurun_out/bench_e.err
echo "bench rc=$?"
fi
