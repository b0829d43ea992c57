# DistributedRBT one-rank-of-P replay: tests, then several runs for variance, then a trace
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_dist_rbt.py tests/test_gpu_rccl.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_drbt.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_drbt.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/pytest_drbt.log | head -20; exit $rc; }
for P in ${PS:-8 8 8 4 2}; do
  timeout -k 10 120 python -u scripts/one_rank_of_p.py --n 8192 --P $P --rank 1 --json gpurun_out/orp.json > gpurun_out/orp.log 2>&1 || { tail -20 gpurun_out/orp.log; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/orp.json'))
print('P=$P factor', d['factor_ms'], 'apply', round(d['apply_min_ms'],3), 'resid', round(d['residual_min_ms'],3), 'total', round(d['measured_total_ms'],3), 'models', [round(m['total_ms'], 2) for m in d['models']])"
done
bash scripts/gpu_orp_prof.sh
