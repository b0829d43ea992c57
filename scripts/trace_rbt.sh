#!/usr/bin/env bash
# kernel trace of the hip-rbt factorisation (scripts/rbt_factor_only.py) + per-kernel / per-queue summary
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d "$OUT/trace_rbt" -o run -- \
  python3 "$ROOT/scripts/rbt_factor_only.py" ${N:-8192} 3 > "$OUT/trace_rbt.log" 2>&1
rc=$?; echo "rocprof rc=$rc"
f=$(find "$OUT/trace_rbt" -name "*kernel_trace.csv" | head -1)
[ -n "$f" ] && python3 "$ROOT/scripts/rbt_trace_summary.py" "$f"
exit $rc
