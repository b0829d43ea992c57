#!/usr/bin/env bash
# round-3 session A: wide-panel + distributed GPU tests, big-n solves,
# distributed timings at 1 (real code path) and 2/8 emulated ranks
set -u
OUT="${GRAFT_REPO_ROOT:-.}/gpurun_out"
mkdir -p "$OUT"
run() { local t=$1; shift; timeout -k 10 "$t" "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*"; exit $rc; fi; }
run 400 python -u -m pytest tests/test_gpu_biglu.py tests/test_gpu_dist_emulated.py tests/test_gpu_dist.py -x -q \
  --timeout 250 --timeout-method thread > "$OUT/pytest_a.log" 2>&1 || { tail -40 "$OUT/pytest_a.log"; exit 1; }
tail -3 "$OUT/pytest_a.log"
run 120 python -u scripts/time_dist.py 1 8192
run 120 python -u scripts/time_dist.py 1 8192 --no-lookahead
run 120 python -u scripts/time_solver.py 8192
run 200 python -u scripts/time_dist.py 2 8192
run 200 python -u scripts/time_dist.py 8 8192
run 400 python -u scripts/big_n_check.py 40000 70000
