# Block inverse: barrier per pair (GELIM_GJ_FLAG=0) vs a publication counter (1): numerics tests under the
# counter form, the inverse alone, hip-rbt solves and the DistributedRBT replay, alternating
set -o pipefail
GELIM_GJ_FLAG=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_mixed.py tests/test_gpu_dist_rbt.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gjflag.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_gjflag.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/pytest_gjflag.log | head -20; exit $rc; }
for r in 1 2; do for v in 0 1; do
  echo "== GELIM_GJ_FLAG=$v"
  GELIM_GJ_FLAG=$v timeout -k 10 120 python -u scripts/gj_probe_check.py 2>&1 | grep -v amdgpu.ids | head -4 || exit 1
  GELIM_GJ_FLAG=$v timeout -k 10 150 python -u scripts/time_rbt.py 2048 8192 16384 2>&1 | grep -v amdgpu.ids || exit 1
done; done
