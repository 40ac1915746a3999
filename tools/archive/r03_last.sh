# last check of the round's final build: the whole -m gpu suite and smoke
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/r03_last_gputest.log 2>&1
rc=$?; tail -1 gpurun_out/r03_last_gputest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03_last_smoke.log 2>&1 || exit 1
tail -1 gpurun_out/r03_last_smoke.log
