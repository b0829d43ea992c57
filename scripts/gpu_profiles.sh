#!/usr/bin/env bash
# Refresh the committed profiles: 2048 kernel stats + trace summary, 8192 lookahead trace summary
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p "$R/gpurun_out"
export TMPDIR=/tmp
( cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof2048" -o run \
    -- python3 "$R/bench.py" --steps 10 --warmup 2 --no-matmul --headline-only > "$R/gpurun_out/prof.log" 2>&1 ) || exit $?
python3 "$R/scripts/trace_summary.py" "$R/gpurun_out/prof2048/run_kernel_trace.csv" > "$R/gpurun_out/gauss2048_trace_summary.txt" 2>&1 || true
bash "$R/scripts/prof_big.sh" "la:GELIM_BIG_LOOKAHEAD=1" || exit $?
echo done
