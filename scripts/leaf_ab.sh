#!/usr/bin/env bash
# A/B of the leaf participant shape (GELIM_LEAF_SHAPE = 1x4 | 2x2 | 4x1 | 4x4; SHAPES lists them): the
# wide-panel GPU tests under both, the lone leaf at several m, whole solves.
set -u
OUT="${GRAFT_REPO_ROOT:-.}/gpurun_out"
mkdir -p "$OUT"
for W in ${SHAPES:-2x2 1x4}; do
  GELIM_LEAF_SHAPE=$W timeout -k 10 300 python -u -m pytest tests/test_gpu_biglu.py -x -q --timeout 200 --timeout-method thread \
    > "$OUT/biglu_w$W.log" 2>&1 || { echo "biglu tests failed ($W)"; tail -30 "$OUT/biglu_w$W.log"; exit 1; }
  tail -2 "$OUT/biglu_w$W.log"
done
for W in ${SHAPES:-2x2 1x4}; do
  for m in 2048 4096 8192 16384 32768; do
    GELIM_LEAF_SHAPE=$W timeout -k 10 120 python scripts/leaf_bench.py $m --time-only || exit 1
  done
done
for W in ${SHAPES:-2x2 1x4}; do
  echo "== solves, GELIM_LEAF_SHAPE=$W"
  GELIM_LEAF_SHAPE=$W timeout -k 10 200 python scripts/time_solver.py 3072 4096 8192 16384 || exit 1
done
for W in ${SHAPES:-2x2}; do
  GELIM_LEAF_SHAPE=$W timeout -k 10 120 python scripts/leaf_bench.py 8192 > "$OUT/leaf_stamps_w$W.txt" 2>&1 || exit 1
  cat "$OUT/leaf_stamps_w$W.txt"
done
