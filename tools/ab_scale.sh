# A/B of library variants (tools/probe/lib<name>.so, "base" = the in-tree build) on the dense
# configs' scale test and the configs[1] loop: bash tools/ab_scale.sh <name>...
set -e
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
for n in "$@"; do
  if [ "$n" = base ]; then unset PRGPU_LIB; else export PRGPU_LIB=$PWD/tools/probe/lib$n.so; fi
  timeout -k 10 200 python -u -m pytest tests/test_scale_configs_gpu.py -x -q -m gpu --timeout 190 --timeout-method thread > gpurun_out/ab_$n.log 2>&1
  for k in 2 3; do cp gpurun_out/scale_configs$k.json gpurun_out/ab_${n}_scale_configs$k.json; done
  timeout -k 10 200 python bench.py --loop-only --steps 3 --warmup 1 > gpurun_out/ab_${n}_loop.json 2> gpurun_out/ab_${n}_loop.err
  echo done $n
done
