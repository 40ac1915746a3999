# SW / CIGAR GPU tests, an interleaved A/B (base,new,base,new: step and stage times), then the
# CIGAR kernel's FETCH_SIZE / WRITE_SIZE passes on the new build (each counter set its own run)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_sw_gpu.py tests/test_sw_edge_gpu.py tests/test_aln_gpu.py tests/test_iter_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r05l_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r05l_tests.log; [ $rc -le 1 ] || exit $rc
for it in proovread_amd/libprgpu_base.so proovread_amd/libprgpu.so proovread_amd/libprgpu_base.so proovread_amd/libprgpu.so; do
  tag=$(basename $it .so)
  PRGPU_LIB=$it timeout -k 10 200 python -u bench.py --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/abl_$tag.json 2> gpurun_out/abl_$tag.err || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/abl_$tag.json').read());print('$tag', d['ms_per_step'], d['stage_event_ms'], d.get('parity'))" | tee -a gpurun_out/abl.txt
done
for c in FETCH_SIZE WRITE_SIZE; do
  rm -rf "$GRAFT_REPO_ROOT/gpurun_out/pmcl_$c"
  (cd /tmp && timeout -s KILL 420 rocprofv3 --pmc $c --kernel-trace -d "$GRAFT_REPO_ROOT/gpurun_out/pmcl_$c" -o run \
     --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 1 --warmup 1 --no-cpu-baseline \
     > "$GRAFT_REPO_ROOT/gpurun_out/pmcl_$c.log" 2>&1) || { echo "pass $c rc=$?"; exit 1; }
  echo "pass $c ok"
done
