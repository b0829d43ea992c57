#!/usr/bin/env bash
# hip-rbt timing under the GEMM-tile and triangular-solve grid knobs
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/rbtknobs
mkdir -p "$OUT"
i=0
for cfg in "GELIM_DGEMM_TILE=0" "GELIM_DGEMM_TILE=128" "GELIM_DGEMM_TILE=64" "GELIM_TRSV_PACK=0"; do
  i=$((i + 1))
  echo "== $cfg"
  env $cfg timeout -k 10 200 python -u scripts/mixed_breakdown.py --backend hip-rbt 2048 4096 8192 > "$OUT/r$i.txt" 2>&1 || exit $?
  grep "n=" "$OUT/r$i.txt" | sed 's/, matvec.*solve / solve /; s/ (\([0-9]*\) corrections.*/ (\1 corrections)/'
done
