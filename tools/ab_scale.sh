# A/B of library variants (tools/probe/lib<name>.so, "base" = the in-tree build) on the dense
# configs' scale test and the configs[1] loop: bash tools/ab_scale.sh <name>[:VAR=value]...
# (e.g. p5:PRGPU_SEED_WAVES_PER_CU=20 loads tools/probe/libp5.so with that variable set)
set -e
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
for spec in "$@"; do
  n=${spec%%:*}
  ev=""
  [ "$spec" != "$n" ] && ev=${spec#*:}
  if [ "$n" = base ]; then unset PRGPU_LIB; else export PRGPU_LIB=$PWD/tools/probe/lib$n.so; fi
  tag=$n${ev:+_$(echo $ev | tr '=' '_')}
  env $ev timeout -k 10 200 python -u -m pytest tests/test_scale_configs_gpu.py -x -q -m gpu --timeout 190 --timeout-method thread > gpurun_out/ab_$tag.log 2>&1
  for k in 2 3; do cp gpurun_out/scale_configs$k.json gpurun_out/ab_${tag}_scale_configs$k.json; done
  env $ev timeout -k 10 200 python bench.py --loop-only --steps 3 --warmup 1 > gpurun_out/ab_${tag}_loop.json 2> gpurun_out/ab_${tag}_loop.err
  echo done $tag
done
