# DistributedRBT replay: side cap 0 (uncapped) vs the default (CUs - 32) at P = 2, 4, 8, alternating processes
set -o pipefail
for r in 1 2; do for P in 2 4 8; do for c in 0 224; do
  timeout -k 10 150 python -u scripts/one_rank_of_p.py --n 8192 --P $P --rank 1 --side-cap $c --json gpurun_out/orp_cp.json > gpurun_out/orp_cp.log 2>&1 || { tail -5 gpurun_out/orp_cp.log; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/orp_cp.json'))
print('P=$P cap $c factor', round(d['factor_min_ms'],3), [round(x,2) for x in d['factor_ms']], 'total', round(d['measured_total_ms'],3))"
done; done; done
