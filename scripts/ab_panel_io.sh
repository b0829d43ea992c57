#!/usr/bin/env bash
# fused-step panel IO mode (GELIM_PANEL_IO = 2 default: coalesced loads all in
# flight + LDS transpose; 1 direct 16-byte register loads; 0 LDS-staged one
# slot at a time): the 2048 headline, alternated.
set -u
for r in 1 2; do
  for m in 2 1 0; do
    echo -n "GELIM_PANEL_IO=$m: "
    GELIM_PANEL_IO=$m timeout -k 10 120 python bench.py --headline-only --no-matmul --steps 50 --warmup 5 2>/dev/null \
      | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['max_error'])" || exit 1
  done
done
