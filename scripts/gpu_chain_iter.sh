set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_dist_rbt.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_drbt.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_drbt.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/pytest_drbt.log | head -20; exit $rc; }
timeout -k 10 120 python -u scripts/one_rank_of_p.py --n 8192 --P 8 --rank 1 --json gpurun_out/orp_8192_p8.json > gpurun_out/orp_8192_p8.log 2>&1 || { tail -20 gpurun_out/orp_8192_p8.log; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/orp_8192_p8.json'))
print('factor', round(d['factor_min_ms'],3), 'per block', round(d['factor_per_block_us'],1), 'total', round(d['measured_total_ms'],3))"
bash scripts/gpu_orp_prof.sh
