#!/usr/bin/env bash
# A/B of HIP stream priorities for the lookahead schedules: side streams at
# low priority (GELIM_SIDE_PRIO=1) and/or hip-rbt's factor chain on a
# high-priority stream (GELIM_CRIT_PRIO=-1); hip-rbt and partial-pivoting
# solves at 4096 / 8192 / 16384.
set -u
R="${GRAFT_REPO_ROOT:-.}"
python -c "
import sys; sys.path.insert(0, '$R')
import ctypes, gelim, torch
from gelim import _native
torch.zeros(1, device='cuda')
a = (ctypes.c_int32 * 2)()
_native.lib().gelim_gpu_stream_priority_range(a)
print('stream priority range: least', a[0], 'greatest', a[1])
" || exit 1
for cfg in "" "GELIM_SIDE_PRIO=1" "GELIM_CRIT_PRIO=-1" "GELIM_SIDE_PRIO=1 GELIM_CRIT_PRIO=-1"; do
  echo "== ${cfg:-default}"
  env $cfg timeout -k 10 150 python scripts/time_rbt.py 2048 4096 8192 16384 || exit 1
  env $cfg timeout -k 10 150 python scripts/time_solver.py 4096 8192 16384 || exit 1
done
