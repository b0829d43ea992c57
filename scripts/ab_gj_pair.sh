#!/usr/bin/env bash
# A/B of the paired Gauss-Jordan inverse (GELIM_GJ_PAIR=1: two steps per
# barrier, bit-identical) against one step per barrier: inverse tests, the
# lone inverse (dist_rbt_prof.py --micro) and hip-rbt solves, alternated.
set -u
OUT="${GRAFT_REPO_ROOT:-.}/gpurun_out"
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_mixed.py -x -q --timeout 200 --timeout-method thread \
  > "$OUT/gj_pair_tests.log" 2>&1 || { tail -40 "$OUT/gj_pair_tests.log"; exit 1; }
tail -2 "$OUT/gj_pair_tests.log"
for rep in 1 2; do
  for f in 1 0; do
    echo "== GELIM_GJ_PAIR=$f"
    GELIM_GJ_PAIR=$f timeout -k 10 120 python scripts/dist_rbt_prof.py --micro 2>&1 | grep -i "inverse" || exit 1
    GELIM_GJ_PAIR=$f timeout -k 10 150 python scripts/time_rbt.py 2048 4096 8192 || exit 1
  done
done
