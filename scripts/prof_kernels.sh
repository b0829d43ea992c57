#!/usr/bin/env bash
# rocprofv3 kernel stats of scripts/time_solver.py for one order n, summary
# printed grouped by kernel name (and by grid size for the top kernels).
#   bash scripts/prof_kernels.sh 8192 [tag]
set -u
N=${1:-8192}; TAG=${2:-n$N}
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/prof_$TAG"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o run -- \
  python3 "$ROOT/scripts/time_solver.py" "$N" --reps 2 > "$OUT/log.txt" 2>&1
rc=$?
grep "n=" "$OUT/log.txt"
python3 "$ROOT/scripts/kernel_summary.py" "$OUT/run_kernel_trace.csv" 4
exit $rc
