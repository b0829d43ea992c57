#!/usr/bin/env bash
# (GELIM_GJ_SCALED was removed after this A/B: profiles/rbt_engine_round3.txt has the result)
# Gauss-Jordan diagonal-inverse change check: the randomised engines' tests,
# the hip-rbt breakdown, one PMC pass over the factor kernels
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/gj
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_mixed.py -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|Error" "$OUT/pytest.log" | tail -5
[ $rc -ne 0 ] && exit $rc
for SC in 1 0; do
  echo "== GELIM_GJ_SCALED=$SC"
  GELIM_GJ_SCALED=$SC timeout -k 10 200 python -u scripts/mixed_breakdown.py --backend hip-rbt 2048 4096 8192 > "$OUT/rbt_$SC.txt" 2>&1 || exit $?
  grep "n=" "$OUT/rbt_$SC.txt"
done
ARGS="8192 2" bash scripts/pmc_rbt.sh
