#!/usr/bin/env bash
# copy-in of the system stored write-through (GELIM_COPY_WT=1) vs plain: the
# 2048 headline (bench.py), alternated.
set -u
for r in 1 2 3; do
  for f in 1 0; do
    echo -n "GELIM_COPY_WT=$f: "
    GELIM_COPY_WT=$f timeout -k 10 120 python bench.py --headline-only --no-matmul --steps 50 --warmup 5 2>/dev/null \
      | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['max_error'])" || exit 1
  done
done
