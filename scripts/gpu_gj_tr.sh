#!/usr/bin/env bash
# Gauss-Jordan tile shape A/B (GELIM_GJ_TR = 2: 1024 threads, 4: 512 (default),
# 8: 256) after the diag-inverse tests of every shape
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/gjtr
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_mixed.py -x -q -k "diag_inverses or rbt_random" --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 "$OUT/pytest.log"
[ $rc -ne 0 ] && exit $rc
for TR in ${TRS:-4 2 8}; do
  echo "== GELIM_GJ_TR=$TR"
  GELIM_GJ_TR=$TR timeout -k 10 200 python -u scripts/mixed_breakdown.py --backend hip-rbt 2048 4096 8192 > "$OUT/rbt_$TR.txt" 2>&1 || exit $?
  grep "n=" "$OUT/rbt_$TR.txt" | sed 's/, apply.*solve / solve /; s/ (\([0-9]*\) corrections.*/ (\1 corrections)/'
done
