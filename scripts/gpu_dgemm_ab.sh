#!/usr/bin/env bash
# (GELIM_DGEMM_STAGGER was removed after this A/B: profiles/dgemm_r3_lds.txt has the result)
# dgemm change check: its numerics tests, then the f64 GEMM shapes and the
# solvers that use it under each C schedule (GELIM_DGEMM_STAGGER)
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/dgemm_ab
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_biglu.py -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" "$OUT/pytest.log" | tail -3
[ $rc -ne 0 ] && exit $rc
for S in ${STAGGERS:-0 1 2}; do
  export GELIM_DGEMM_STAGGER=$S
  echo "== GELIM_DGEMM_STAGGER=$S"
  timeout -k 10 200 python -u scripts/gemm_bench.py f64 > "$OUT/gemm_$S.txt" 2>&1 || exit $?
  grep dgemm "$OUT/gemm_$S.txt"
  timeout -k 10 200 python -u scripts/time_solver.py 4096 8192 16384 > "$OUT/solver_$S.txt" 2>&1 || exit $?
  grep "n=" "$OUT/solver_$S.txt"
  timeout -k 10 200 python -u scripts/mixed_breakdown.py --backend hip-rbt 2048 8192 > "$OUT/rbt_$S.txt" 2>&1 || exit $?
  grep "n=" "$OUT/rbt_$S.txt"
done
