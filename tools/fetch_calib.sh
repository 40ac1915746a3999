#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration passes (tools/fetch_calib.hip), one counter per run
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
# (built on the box: a bare executable does not travel with the snapshot)
timeout -k 10 120 /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -o /tmp/fetch_calib tools/fetch_calib.hip || exit 1
for c in FETCH_SIZE WRITE_SIZE; do
  rm -rf "$GRAFT_REPO_ROOT/gpurun_out/calib_$c"
  (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace -d "$GRAFT_REPO_ROOT/gpurun_out/calib_$c" -o run \
     --output-format csv -- /tmp/fetch_calib > "$GRAFT_REPO_ROOT/gpurun_out/calib_$c.log" 2>&1) \
     || { echo "calib $c rc=$?"; exit 1; }
  echo "calib $c ok"
done
