#!/usr/bin/env bash
# kernel stats of the randomised no-pivoting engine: rocprofv3 over scripts/mixed_breakdown.py
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_rbt" -o run -- \
  python3 "$ROOT/scripts/mixed_breakdown.py" --backend "${BACKEND:-hip-rbt}" ${SIZES:-8192} > "$OUT/prof_rbt.log" 2>&1
rc=$?; echo "rocprof rc=$rc"; grep -v amdgpu.ids "$OUT/prof_rbt.log" | tail -3
f=$(find "$OUT/prof_rbt" -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] && python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:14]:
    print(f'{float(r["TotalDurationNs"])/1e6:9.2f} ms {int(r["Calls"]):6d} calls {float(r["AverageNs"])/1e3:9.1f} us  {r["Name"][:110]}')
PY
exit $rc
