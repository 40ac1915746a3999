# seeding kernel occupancy: 4 (default), 3 and 2 workgroups of 4 waves per CU (VGPR budget
# 128 / 168 / 256: fewer spills, fewer lanes' scratch in flight); GPU seeding tests + seed time each
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
cp proovread_amd/libprgpu.so gpurun_out/libprgpu_minb4.so
for b in 4 3 2; do
  cp gpurun_out/libprgpu_minb4.so proovread_amd/libprgpu.so
  [ $b -ne 4 ] && cp proovread_amd/libprgpu_minb$b.so proovread_amd/libprgpu.so
  timeout -k 10 600 python -u -m pytest tests/test_seed_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/seedocc_${b}_test.log 2>&1
  rc=$?; echo "minb $b"; tail -1 gpurun_out/seedocc_${b}_test.log; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python -u tools/seed_time.py > gpurun_out/seedocc_${b}.log 2>&1 || exit 1
  tail -4 gpurun_out/seedocc_${b}.log
done
cp gpurun_out/libprgpu_minb4.so proovread_amd/libprgpu.so
rm -f gpurun_out/libprgpu_minb4.so
