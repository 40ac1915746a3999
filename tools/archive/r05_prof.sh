set -o pipefail
export TMPDIR=/tmp
T=${TAG:-r05_p}
mkdir -p gpurun_out
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/${T}_prof" -o run --output-format csv \
  -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 3 --no-cpu-baseline > "$GRAFT_REPO_ROOT/gpurun_out/${T}_bench_prof.json" 2>&1)
rc=$?; echo "prof rc=$rc"
f=$(find gpurun_out/${T}_prof -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/${T}_kernel_stats.csv
python3 -c "
import csv
rows=list(csv.DictReader(open('gpurun_out/${T}_kernel_stats.csv')))
for r in rows[:25]: print(r['Name'][:70], r['Calls'], round(float(r['AverageNs'])/1e6,3))
"
