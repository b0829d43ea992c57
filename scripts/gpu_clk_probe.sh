set -o pipefail
for r in 1 2 3 4; do
  ( for i in $(seq 1 12); do timeout 5 rocm-smi --showclocks 2>/dev/null | grep -E "sclk|mclk|fclk" | tr -s ' ' | tr '\n' ' '; echo; sleep 1; done ) > gpurun_out/clk_$r.txt 2>&1 &
  sp=$!
  timeout -k 10 150 python -u scripts/one_rank_of_p.py --n 8192 --P 8 --rank 1 --reps 10 --json gpurun_out/orp_clk.json > gpurun_out/orp_clk.log 2>&1 || { kill $sp; exit 1; }
  wait $sp
  python3 -c "
import json; d=json.load(open('gpurun_out/orp_clk.json')); print('run $r factor', [round(x,2) for x in d['factor_ms']])"
  sort gpurun_out/clk_$r.txt | uniq -c | sort -rn | head -3
done
