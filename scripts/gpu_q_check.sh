#!/bin/bash
# lookahead side streams vs hardware queues: the dist 2048 (tail=0) solve and
# the single-GPU 8192 solve after the bench's earlier sections, with the
# box's 4 hardware queues and with 8, side streams probed (default).  (The
# round-4 record in profiles/hw_queues_r4.txt ran while gelim still raised the
# queue count itself; GELIM_KEEP_HW_QUEUES=1 then kept the exported 4.)
set -o pipefail
out=gpurun_out/qcheck.txt
: > $out
run() { timeout -k 10 240 python scripts/bench_order_check2.py "$@" >> $out 2>/dev/null; }
FINAL=t0 run || exit 1
FINAL=t0 run head mm d8 rbt || exit 1
FINAL=t0 GPU_MAX_HW_QUEUES=8 run head mm d8 rbt || exit 1
run mm d8 rbt t0 || exit 1
run head mm d8 rbt t0 te || exit 1
GPU_MAX_HW_QUEUES=8 run head mm d8 rbt t0 te || exit 1
