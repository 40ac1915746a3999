#!/bin/bash
# round-2 first GPU pass: GPU tests (the known CIGAR-capacity case deselected), then the bench and its kernel profile
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  --deselect "tests/test_sw_edge_gpu.py::test_sw_gpu_ragged_lengths_and_ns" > gpurun_out/r02_gputest1.log 2>&1
echo "pytest rc=$?"
timeout -k 10 400 python -u bench.py > gpurun_out/r02_bench1.json 2> gpurun_out/r02_bench1.err || { echo "bench rc=$?"; exit 1; }
cat gpurun_out/r02_bench1.json
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof1" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 3 --no-cpu-baseline > "$GRAFT_REPO_ROOT/gpurun_out/r02_bench1_prof.json" 2>&1
echo "prof rc=$?"
