# same-box A/B of an executor variant (GELIM_AB=0/1), alternating, P=8 replay
set -o pipefail
for r in 1 2 3; do for v in 0 1; do
  GELIM_AB=$v timeout -k 10 120 python -u scripts/one_rank_of_p.py --n 8192 --P ${P:-8} --rank 1 --json gpurun_out/orp_ab.json > gpurun_out/orp_ab.log 2>&1 || { tail -20 gpurun_out/orp_ab.log; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/orp_ab.json'))
print('AB=$v factor', round(d['factor_min_ms'],3), 'total', round(d['measured_total_ms'],3))"
done; done
