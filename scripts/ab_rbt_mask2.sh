#!/usr/bin/env bash
# hip-rbt with the CUs partitioned: side GEMMs off k CUs and the chain ON
# those k alone (GELIM_RBT_MASK=k GELIM_RBT_MASK_CRIT=1), against the default.
set -u
for cfg in "" "GELIM_RBT_MASK=32 GELIM_RBT_MASK_CRIT=1" "GELIM_RBT_MASK=64 GELIM_RBT_MASK_CRIT=1" "GELIM_RBT_MASK=96 GELIM_RBT_MASK_CRIT=1"; do
  echo "== ${cfg:-default}"
  env $cfg timeout -k 10 150 python scripts/time_rbt.py 2048 4096 8192 16384 || exit 1
done
