#!/usr/bin/env bash
# Gauss-Jordan tile shape A/B after the LDS padding (GELIM_GJ_TR = 8: 256 threads,
# 4: 512 threads), then rocprofv3 kernel stats of hip-rbt at 2048
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/gjtr
mkdir -p "$OUT"
for TR in 8 4; do
  echo "== GELIM_GJ_TR=$TR"
  GELIM_GJ_TR=$TR timeout -k 10 200 python -u scripts/mixed_breakdown.py --backend hip-rbt 2048 8192 > "$OUT/rbt_$TR.txt" 2>&1 || exit $?
  grep "n=" "$OUT/rbt_$TR.txt" | sed 's/, apply.*solve / solve /; s/ (\([0-9]*\) corrections.*/ (\1 corrections)/'
done
SIZES=2048 bash scripts/prof_rbt.sh
