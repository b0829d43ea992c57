#!/usr/bin/env bash
# three-stream hip-rbt schedule: tests, then timings with / without it and
# with lookahead forced at 2048
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/la3
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_mixed.py -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|Error|assert" "$OUT/pytest.log" | tail -8
[ $rc -ne 0 ] && exit $rc
for cfg in "GELIM_RBT_AUX=1" "GELIM_RBT_AUX=0" "GELIM_RBT_AUX=1 GELIM_RBT_LOOKAHEAD=1" "GELIM_RBT_AUX=0 GELIM_RBT_LOOKAHEAD=1"; do
  echo "== $cfg"
  env $cfg timeout -k 10 200 python -u scripts/mixed_breakdown.py --backend hip-rbt 2048 4096 8192 16384 > "$OUT/rbt.txt" 2>&1 || exit $?
  grep "n=" "$OUT/rbt.txt" | sed 's/, apply.*solve / solve /; s/ (.*error/ error/; s/| fp64.*//'
done
