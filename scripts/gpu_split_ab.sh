#!/bin/bash
# A/B of the per-leaf split (GELIM_BIG_SPLIT=1: only the next leaf's columns on
# the critical stream, the rest of the leaf's update on a second stream):
# the wide-panel GPU tests with the split, then solves with and without it.
set -e
O=${GRAFT_REPO_ROOT:-.}/gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_biglu.py tests/test_gpu_dist.py -x -q --timeout 200 --timeout-method thread > $O/split_tests.log 2>&1
tail -2 $O/split_tests.log
for S in 1 0 1; do
  echo "== GELIM_BIG_SPLIT=$S"
  GELIM_BIG_SPLIT=$S timeout -k 10 200 python scripts/time_solver.py 3072 4096 8192 16384
done
