# A/B of library variants on one box: PRGPU_LIB=proovread_amd/libprgpu_<v>.so bench.py, alternating
set -o pipefail
mkdir -p gpurun_out
for v in "$@"; do
  PRGPU_LIB=proovread_amd/libprgpu_$v.so timeout -k 10 200 python -u bench.py --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err || exit 1
  python3 -c "import json,sys;d=json.loads(open('gpurun_out/ab_$v.json').read());print('$v', d['ms_per_step'], d['stage_event_ms'], d['value'])" | tee -a gpurun_out/ab.txt
done
