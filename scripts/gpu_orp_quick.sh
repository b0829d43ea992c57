set -o pipefail
for c in ${CAPS:-0 224}; do
  timeout -k 10 120 python -u scripts/one_rank_of_p.py --n 8192 --P ${P:-8} --rank 1 --side-cap $c --json gpurun_out/orp_cap$c.json > gpurun_out/orp_cap$c.log 2>&1 || { tail -20 gpurun_out/orp_cap$c.log; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/orp_cap$c.json'))
print('P=${P:-8} cap $c factor', round(d['factor_min_ms'],3), d['factor_ms'], 'per block', round(d['factor_per_block_us'],1), 'total', round(d['measured_total_ms'],3))"
done
bash scripts/gpu_orp_prof.sh
