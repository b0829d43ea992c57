#!/usr/bin/env bash
# A/B of the 3-rows-per-lane step kernel for 1024 < m <= 1536 (GELIM_STEP_R3=1,
# default) against 4 rows per lane up to 2048 (=0): solver GPU tests, then the
# 2048 headline (bench.py) under both, alternated.
set -u
OUT="${GRAFT_REPO_ROOT:-.}/gpurun_out"
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_solver.py -x -q --timeout 200 \
  --timeout-method thread > "$OUT/step_r3_tests.log" 2>&1 || { tail -40 "$OUT/step_r3_tests.log"; exit 1; }
tail -2 "$OUT/step_r3_tests.log"
for rep in 1 2; do
  for f in 1 0; do
    echo -n "GELIM_STEP_R3=$f: "
    GELIM_STEP_R3=$f timeout -k 10 120 python bench.py --headline-only --no-matmul --steps 50 --warmup 5 \
      2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(f\"{d['ms_per_step']:.3f} ms, err {d['max_error']:.2e}\")" || exit 1
  done
done
