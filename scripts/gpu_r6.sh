# replay: graph vs eager issue (scripts/one_rank_of_p.py)
set -o pipefail
timeout -k 10 120 python -u scripts/one_rank_of_p.py --n 8192 --P 8 --rank 1 --no-graph --json gpurun_out/orp_8192_p8_eager.json > gpurun_out/orp_eager.log 2>&1 || { tail -20 gpurun_out/orp_eager.log; exit 1; }
python - <<'PY'
import json
for f in ("orp_8192_p8", "orp_8192_p8_cap192", "orp_8192_p8_eager", "orp_8192_p2"):
    try:
        d = json.load(open(f"gpurun_out/{f}.json"))
    except FileNotFoundError:
        continue
    print(f, "factor", d["factor_min_ms"], "apply", d["apply_min_ms"], "resid", d["residual_min_ms"], "total", round(d["measured_total_ms"], 3))
PY
