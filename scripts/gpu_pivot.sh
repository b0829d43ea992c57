#!/usr/bin/env bash
# hip-pivot timing + its kernel stats + the pivot-related GPU tests
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p gpurun_out
timeout -k 10 120 python scripts/time_pivot.py 1024 2048 > gpurun_out/tp.txt 2>&1 || exit $?
timeout -k 10 300 python -m pytest tests -m gpu -q -x --timeout=300 -k "pivot or zero or internal or refine or golden" \
  > gpurun_out/pytest_gpu.log 2>&1 || exit $?
export TMPDIR=/tmp
R="$PWD"
cd /tmp && timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/profpiv" -o run \
  -- python3 "$R/scripts/time_pivot.py" 2048 --reps 2 > "$R/gpurun_out/profpiv.log" 2>&1 || exit $?
echo done
