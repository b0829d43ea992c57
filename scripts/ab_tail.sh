#!/usr/bin/env bash
# 2048^2 solve vs the hybrid schedule's resident-tail size (GELIM_HYBRID)
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p gpurun_out
for t in 1024 768 896 1152 1280 1536; do
  echo "## GELIM_HYBRID=$t"
  GELIM_HYBRID=$t timeout -k 10 60 python scripts/time_solver.py 2048 --reps 20 || exit $?
done > gpurun_out/ab_tail.txt 2>&1
