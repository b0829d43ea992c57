#!/usr/bin/env bash
# A/B of the wide-panel outer width under the default (lookahead) schedule at 8192
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p gpurun_out
for nb in 256 512 128; do
  echo "## GELIM_BIG_NB=$nb"
  GELIM_BIG_NB=$nb timeout -k 10 120 python scripts/time_solver.py 6144 8192 --reps 5 || exit $?
done > gpurun_out/ab_bignb.txt 2>&1
echo done
