# hip-rbt with the chain's 128-wide products as 16 x 16 tiles: numerics tests, then timings + a trace
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_gpu_mixed.py tests/test_gpu_dist_rbt.py tests/test_gpu_rccl.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_rbt.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_rbt.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/pytest_rbt.log | head -20; exit $rc; }
for r in 1 2; do timeout -k 10 120 python -u scripts/time_rbt.py 2048 4096 8192 16384 2>&1 | grep -v amdgpu.ids; done
bash scripts/trace_rbt.sh
