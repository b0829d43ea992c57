#!/usr/bin/env bash
# round-3 session B: distributed GPU tests + timings, then n = 70000 (own residual, no rocSOLVER)
set -u
OUT="${GRAFT_REPO_ROOT:-.}/gpurun_out"
mkdir -p "$OUT"
run() { local t=$1; shift; timeout -k 10 "$t" "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*"; exit $rc; fi; }
run 300 python -u -m pytest tests/test_gpu_dist_emulated.py tests/test_gpu_dist.py -x -q \
  --timeout 250 --timeout-method thread > "$OUT/pytest_b.log" 2>&1 || { grep -v amdgpu.ids "$OUT/pytest_b.log" | tail -40; exit 1; }
tail -2 "$OUT/pytest_b.log"
run 120 python -u scripts/time_dist.py 1 8192
run 120 python -u scripts/time_solver.py 8192
run 200 python -u scripts/time_dist.py 2 8192
run 300 python -u scripts/big_n_check.py 70000
