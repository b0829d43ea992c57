#!/usr/bin/env bash
# A/B of the fused narrow update (GELIM_NARROW_FUSED=1, default: the step
# launch's trailing workgroups update the next panel's strip) against the
# separate narrow launch (=0): solver GPU tests under the fused form, then the
# 2048 headline (bench.py, graph replay) under both, alternated.
set -u
OUT="${GRAFT_REPO_ROOT:-.}/gpurun_out"
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_solver.py tests/test_gpu_kernels.py -x -q --timeout 200 \
  --timeout-method thread > "$OUT/narrow_fused_tests.log" 2>&1 || { tail -40 "$OUT/narrow_fused_tests.log"; exit 1; }
tail -2 "$OUT/narrow_fused_tests.log"
for rep in 1 2; do
  for f in 1 0; do
    echo -n "GELIM_NARROW_FUSED=$f: "
    GELIM_NARROW_FUSED=$f timeout -k 10 120 python bench.py --headline-only --no-matmul --steps 50 --warmup 5 \
      2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(f\"{d['ms_per_step']:.3f} ms, err {d['max_error']:.2e}\")" || exit 1
  done
done
