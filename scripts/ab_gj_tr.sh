#!/usr/bin/env bash
# Gauss-Jordan inverse: tile rows per thread (GELIM_GJ_TR = 4: 512 threads, 2
# waves per SIMD; 2: 1024 threads, 4 waves per SIMD) x pairs on / off.
set -u
for tr in 4 2; do
  for pr in 1 0; do
    echo -n "GELIM_GJ_TR=$tr GELIM_GJ_PAIR=$pr: "
    GELIM_GJ_TR=$tr GELIM_GJ_PAIR=$pr timeout -k 10 120 python scripts/dist_rbt_prof.py --micro 2>&1 | grep -i "inverse" || exit 1
  done
done
GELIM_GJ_TR=2 timeout -k 10 150 python scripts/time_rbt.py 2048 8192 || exit 1
GELIM_GJ_TR=4 timeout -k 10 150 python scripts/time_rbt.py 2048 8192 || exit 1
