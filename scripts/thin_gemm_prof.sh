#!/bin/bash
# Kernel durations (rocprofv3 --kernel-trace --stats) of the thin fp64 GEMM
# shapes, one run per shape: dgemm.hip's LDS-tiled kernel vs dgemm_thin.hip.
# Output: gpurun_out/thinprof/<shape>/..._kernel_stats.csv
set -e
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p "$R/gpurun_out/thinprof"
for s in 0 1 3 8; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/thinprof/s$s" -o run -- \
    python3 "$R/scripts/thin_gemm_bench.py" --shape $s > "$R/gpurun_out/thinprof/s$s.txt" 2>&1
done
