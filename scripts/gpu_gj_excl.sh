#!/usr/bin/env bash
# Gauss-Jordan inverse alone on its CU (GELIM_GJ_EXCL KiB of reserved LDS) x tile shape
# (GELIM_GJ_TR), under the default schedules and with lookahead forced at 2048.
# Record of the round-3 run in profiles/rbt_engine_round3.txt: the LDS reservation changed
# nothing measurable and GELIM_GJ_EXCL was removed afterwards (it is ignored now).
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/gjexcl
mkdir -p "$OUT"
i=0
for cfg in "GELIM_GJ_TR=8" "GELIM_GJ_TR=4" "GELIM_GJ_TR=8 GELIM_GJ_EXCL=150" "GELIM_GJ_TR=4 GELIM_GJ_EXCL=150" \
           "GELIM_GJ_TR=4 GELIM_GJ_EXCL=150 GELIM_RBT_AUX=1" "GELIM_GJ_TR=8 GELIM_GJ_EXCL=150 GELIM_RBT_AUX=1"; do
  i=$((i + 1))
  echo "== $cfg"
  env $cfg timeout -k 10 200 python -u scripts/mixed_breakdown.py --backend hip-rbt 2048 4096 8192 > "$OUT/r$i.txt" 2>&1 || exit $?
  env $cfg GELIM_RBT_LOOKAHEAD=1 timeout -k 10 100 python -u scripts/mixed_breakdown.py --backend hip-rbt 2048 > "$OUT/l$i.txt" 2>&1 || exit $?
  cat "$OUT/r$i.txt" "$OUT/l$i.txt" | grep "n=" | sed 's/, apply.*solve / solve /; s/ (\([0-9]*\) corrections.*/ (\1 corrections)/'
done
