# DistributedRBT replay at P = 8: side cap 0 vs 224 vs 240, four alternating rounds
set -o pipefail
for r in ${ROUNDS:-1 2 3 4}; do for c in ${CAPS:-0 224 240}; do
  timeout -k 10 150 python -u scripts/one_rank_of_p.py --n 8192 --P 8 --rank 1 --side-cap $c --json gpurun_out/orp_cp.json > gpurun_out/orp_cp.log 2>&1 || { tail -5 gpurun_out/orp_cp.log; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/orp_cp.json'))
print('cap $c factor', round(d['factor_min_ms'],3), 'total', round(d['measured_total_ms'],3))"
done; done
