set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
run() {  # name, env...
  n=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 1 --warmup 1 > gpurun_out/sv_$n.json 2> gpurun_out/sv_$n.err
  rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/sv_$n.err; exit $rc; }
  python -c "import json; d=json.loads(open('gpurun_out/sv_$n.json').read().strip().splitlines()[-1]); s=d['seeding']; print('$n', s['kernel_ms'], s['parity_vs_host'], d['iteration_end_to_end_ms'])"
}
run base PRGPU_SEED_WAVES_PER_CU=16
run m8 PRGPU_LIB=tools/probe/libm8.so PRGPU_SEED_WAVES_PER_CU=32
run m6 PRGPU_LIB=tools/probe/libm6.so PRGPU_SEED_WAVES_PER_CU=24
