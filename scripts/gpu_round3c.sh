#!/usr/bin/env bash
# round-3 session C: dgemm thin tiles (A/B by GELIM_DGEMM_TILE), wide-panel tests, solves, bench
set -u
OUT="${GRAFT_REPO_ROOT:-.}/gpurun_out"
mkdir -p "$OUT"
run() { local t=$1; shift; timeout -k 10 "$t" "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*"; exit $rc; fi; }
run 300 python -u -m pytest tests/test_gpu_biglu.py -x -q --timeout 250 --timeout-method thread > "$OUT/biglu_c.log" 2>&1 || { grep -v amdgpu.ids "$OUT/biglu_c.log" | tail -30; exit 1; }
tail -1 "$OUT/biglu_c.log"
echo "== dgemm default (64-tiles for thin shapes)"; run 120 python -u scripts/gemm_bench.py f64
echo "== dgemm forced 128-tiles"; GELIM_DGEMM_TILE=128 run 120 python -u scripts/gemm_bench.py f64
echo "== solves default"; run 200 python -u scripts/time_solver.py 4096 8192 16384
echo "== solves forced 128-tiles"; GELIM_DGEMM_TILE=128 run 200 python -u scripts/time_solver.py 4096 8192 16384
run 120 python -u scripts/time_dist.py 1 8192
run 500 python bench.py --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err"
cat "$OUT/bench.json"
