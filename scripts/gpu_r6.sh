set -o pipefail
timeout -k 10 120 python -u scripts/gj_probe_check.py > gpurun_out/gj_probe.txt 2>&1 || { tail -20 gpurun_out/gj_probe.txt; exit 1; }
cat gpurun_out/gj_probe.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_mixed.py tests/test_gpu_dist_rbt.py tests/test_gpu_rccl.py -q --timeout 120 --timeout-method thread > gpurun_out/t_mixed.log 2>&1; tail -4 gpurun_out/t_mixed.log
timeout -k 10 120 python -u scripts/time_rbt.py 2048 8192 16384 > gpurun_out/time_rbt.txt 2>&1 || { tail -20 gpurun_out/time_rbt.txt; exit 1; }
cat gpurun_out/time_rbt.txt
