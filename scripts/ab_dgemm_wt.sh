#!/usr/bin/env bash
# fp64 GEMM C tiles stored write-through (GELIM_DGEMM_WT=1: no dirty L2 left
# for the launch boundaries of the critical stream) against plain stores:
# partial-pivoting solves (wide-panel engine) and hip-rbt, alternated.
set -u
for rep in 1 2; do
  for f in 1 0; do
    echo "== GELIM_DGEMM_WT=$f"
    GELIM_DGEMM_WT=$f timeout -k 10 200 python scripts/time_solver.py 4096 8192 16384 || exit 1
    GELIM_DGEMM_WT=$f timeout -k 10 150 python scripts/time_rbt.py 2048 8192 || exit 1
  done
done
