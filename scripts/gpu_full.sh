#!/usr/bin/env bash
# full GPU test suite + bench (one JSON line) + rocprofv3 kernel stats of the headline
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -v amdgpu.ids "$OUT/pytest_gpu.log" | tail -15
[ $rc -gt 1 ] && exit $rc
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err"
brc=$?; echo "bench rc=$brc"; cat "$OUT/bench.json"; grep -v amdgpu.ids "$OUT/bench.err" | tail -5
[ $brc -gt 1 ] && exit $brc
timeout -k 10 200 python -u scripts/mixed_breakdown.py --backend hip-rbt 2048 8192
exit $(( rc > brc ? rc : brc ))
