# A/B of library variants on one box, each item lib[:ENV=VAL]: lib = a path under the repo
set -o pipefail
mkdir -p gpurun_out
for it in "$@"; do
  lib=${it%%:*}; env=""; [ "$lib" != "$it" ] && env=${it#*:}
  tag=$(basename $lib .so)${env:+_${env//=/}}
  env PRGPU_LIB=$lib $env timeout -k 10 200 python -u bench.py --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/abv_$tag.json 2> gpurun_out/abv_$tag.err || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/abv_$tag.json').read());c=d['consensus_phase_ms_summed_over_workgroups'];print('$tag', d['ms_per_step'], d['stage_event_ms']['consensus'], {k:round(c[k]) for k in ('prep','binning','state_table','scatter','argmax_write')})" | tee -a gpurun_out/abv.txt
done
