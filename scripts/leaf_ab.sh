#!/usr/bin/env bash
# A/B of the leaf's waves per participant (GELIM_LEAF_WAVES = 1 | 4): the
# wide-panel GPU tests under both, the lone leaf at several m, whole solves.
set -u
OUT="${GRAFT_REPO_ROOT:-.}/gpurun_out"
mkdir -p "$OUT"
for W in 4 1; do
  GELIM_LEAF_WAVES=$W timeout -k 10 300 python -u -m pytest tests/test_gpu_biglu.py -x -q --timeout 200 --timeout-method thread \
    > "$OUT/biglu_w$W.log" 2>&1 || { echo "biglu tests failed (W=$W)"; tail -30 "$OUT/biglu_w$W.log"; exit 1; }
  tail -2 "$OUT/biglu_w$W.log"
done
for W in 4 1; do
  for m in 2048 4096 8192 16384 32768; do
    GELIM_LEAF_WAVES=$W timeout -k 10 120 python scripts/leaf_bench.py $m --time-only || exit 1
  done
done
for W in 4 1; do
  echo "== solves, GELIM_LEAF_WAVES=$W"
  GELIM_LEAF_WAVES=$W timeout -k 10 200 python scripts/time_solver.py 3072 4096 8192 16384 || exit 1
done
GELIM_LEAF_WAVES=4 timeout -k 10 120 python scripts/leaf_bench.py 8192 > "$OUT/leaf_stamps_w4.txt" 2>&1 || exit 1
cat "$OUT/leaf_stamps_w4.txt"
