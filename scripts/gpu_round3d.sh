#!/usr/bin/env bash
# round-3 session D: randomised no-pivoting engines (hip-mixed fp32 / hip-rbt fp64) tests + timing, then the GPU suite + bench
set -u
OUT="${GRAFT_REPO_ROOT:-.}/gpurun_out"
mkdir -p "$OUT"
run() { local t=$1; shift; timeout -k 10 "$t" "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*"; exit $rc; fi; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_mixed.py -v --timeout 120 --timeout-method thread > "$OUT/mixed_d.log" 2>&1; prc=$?; echo "pytest rc=$prc"; [ $prc -gt 1 ] && exit $prc; grep -E "PASS|FAIL|Error|assert" "$OUT/mixed_d.log" | head -60
tail -3 "$OUT/mixed_d.log"
run 200 python -u scripts/mixed_breakdown.py --backend hip-rbt 2048 4096 8192 16384
run 200 python -u scripts/mixed_breakdown.py --backend hip-mixed 2048 4096 8192
if [ "${FULL:-0}" = 1 ]; then
  run 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
  tail -2 "$OUT/pytest_gpu.log"
  run 500 python bench.py --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err"
  cat "$OUT/bench.json"
fi
run 300 bash scripts/prof_rbt.sh
