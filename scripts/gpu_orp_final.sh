# DistributedRBT one-rank-of-P replays for profiles/dist_rbt_replay_r6.md:
# the replay / executor tests, then 8192 at P = 8 (three processes), 4, 2; 16384 at P = 8
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_dist_rbt.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_orp.log 2>&1; rc=$?; tail -1 gpurun_out/pytest_orp.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/pytest_orp.log | head -20; exit $rc; }
run() {  # n P tag
  timeout -k 10 150 python -u scripts/one_rank_of_p.py --n $1 --P $2 --rank 1 --json gpurun_out/orp_$3.json > gpurun_out/orp_$3.log 2>&1 || { tail -20 gpurun_out/orp_$3.log; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/orp_$3.json'))
print('n=$1 P=$2 factor', d['factor_ms'], 'per block us', round(d['factor_per_block_us'],1), 'apply', round(d['apply_min_ms'],3), 'resid', round(d['residual_min_ms'],3), 'total', round(d['measured_total_ms'],3), 'models', [(m['lat_us'], m['bw_GBs'], round(m['total_ms'], 2)) for m in d['models']])"
}
run 8192 8 p8a && run 8192 8 p8b && run 8192 8 p8c && run 8192 4 p4 && run 8192 2 p2 && run 16384 8 n16k_p8
