set -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -4 gpurun_out/pytest_gpu.log
case $rc in 0|1) ;; *) echo "pytest rc=$rc: stopping"; exit $rc ;; esac
for P in 8 4 2; do
  timeout -k 10 120 python -u scripts/one_rank_of_p.py --n 8192 --P $P --rank 1 --json gpurun_out/orp_8192_p$P.json > gpurun_out/orp_8192_p$P.log 2>&1 || { echo "orp P=$P failed"; tail -20 gpurun_out/orp_8192_p$P.log; exit 1; }
done
timeout -k 10 120 python -u scripts/one_rank_of_p.py --n 16384 --P 8 --rank 1 --json gpurun_out/orp_16384_p8.json > gpurun_out/orp_16384.log 2>&1 || { tail -20 gpurun_out/orp_16384.log; exit 1; }
python - <<'PY'
import json
for f in ("orp_8192_p8", "orp_8192_p4", "orp_8192_p2", "orp_16384_p8"):
    d = json.load(open(f"gpurun_out/{f}.json"))
    print(f, d.get("schedule"), "issue", round(d.get("issue_ms", 0), 2), "factor", round(d["factor_min_ms"], 3), "per block us", round(d["factor_per_block_us"], 1), "apply", round(d["apply_min_ms"], 3), "resid", round(d["residual_min_ms"], 3), "total", round(d["measured_total_ms"], 3), "models", [round(m["total_ms"], 2) for m in d["models"]])
PY
