set -o pipefail
timeout -k 10 120 python -u scripts/gj_probe_check.py > gpurun_out/gj_probe.txt 2>&1 || { tail -20 gpurun_out/gj_probe.txt; exit 1; }
cat gpurun_out/gj_probe.txt
timeout -k 10 300 python -u scripts/gj_tol_sweep.py 8192 > gpurun_out/gj_tol_sweep.txt 2>&1 || { tail -20 gpurun_out/gj_tol_sweep.txt; exit 1; }
cat gpurun_out/gj_tol_sweep.txt
