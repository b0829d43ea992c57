#!/usr/bin/env bash
# A/B of the lookahead side-grid reserve (GELIM_BIG_RESERVE) at the default outer width, and of
# lookahead vs serial at 3072 / 4096
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p gpurun_out
{
for rs in 64 32 96 128; do
  echo "## GELIM_BIG_RESERVE=$rs"
  GELIM_BIG_RESERVE=$rs timeout -k 10 120 python scripts/time_solver.py 8192 --reps 5 || exit $?
done
echo "## serial (GELIM_BIG_LOOKAHEAD=0)"
GELIM_BIG_LOOKAHEAD=0 timeout -k 10 120 python scripts/time_solver.py 3072 4096 5120 --reps 5 || exit $?
echo "## lookahead (GELIM_BIG_LOOKAHEAD=1)"
GELIM_BIG_LOOKAHEAD=1 timeout -k 10 120 python scripts/time_solver.py 3072 4096 5120 --reps 5 || exit $?
} > gpurun_out/ab_bigla.txt 2>&1
echo done
