#!/usr/bin/env bash
# hip-rbt with the side stream's GEMMs kept off k CUs (GELIM_RBT_MASK=k,
# CU-masked queue; the chain on a stream of its own), spread over the XCDs or
# the lowest-numbered CUs, against the default.
set -u
for cfg in "" "GELIM_RBT_MASK=16" "GELIM_RBT_MASK=32" "GELIM_RBT_MASK=64" "GELIM_RBT_MASK=32 GELIM_RBT_MASK_SPREAD=0" ""; do
  echo "== ${cfg:-default}"
  env $cfg timeout -k 10 150 python scripts/time_rbt.py 4096 8192 16384 || exit 1
done
