#!/usr/bin/env bash
# Kernel traces of the 8192 wide-panel solve under the schedules given as
# NAME=ENV pairs, e.g.  scripts/prof_big.sh la32:GELIM_BIG_RESERVE=32 serial:GELIM_BIG_LOOKAHEAD=0
# Each run: rocprofv3 --kernel-trace --stats, then scripts/big_trace.py.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
N="${N:-8192}"
export TMPDIR=/tmp
for spec in "$@"; do
  name="${spec%%:*}"; envs="${spec#*:}"
  out="$ROOT/gpurun_out/pbig_$name"
  rm -rf "$out"
  ( cd /tmp && export $envs && timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$out" -o run \
      -- python3 "$ROOT/scripts/time_solver.py" "$N" --reps 2 > "$out.log" 2>&1 )
  rc=$?
  echo "== $name ($envs) rc=$rc"; grep "n=" "$out.log"
  if [ $rc -ne 0 ]; then tail -5 "$out.log"; exit $rc; fi
  python3 "$ROOT/scripts/big_trace.py" "$out/run_kernel_trace.csv" | tee "$out.summary"
done
