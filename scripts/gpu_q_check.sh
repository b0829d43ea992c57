#!/bin/bash
# lookahead side streams vs hardware queues: the dist 2048 (tail=0) solve and
# the single-GPU 8192 solve after the bench's earlier sections, with HIP's 4
# queues (GELIM_KEEP_HW_QUEUES=1) and gelim's 8, side streams probed (default)
set -o pipefail
out=gpurun_out/qcheck.txt
: > $out
run() { timeout -k 10 240 python scripts/bench_order_check2.py "$@" >> $out 2>/dev/null; }
FINAL=t0 GELIM_KEEP_HW_QUEUES=1 run || exit 1
FINAL=t0 GELIM_KEEP_HW_QUEUES=1 run head mm d8 rbt || exit 1
FINAL=t0 run head mm d8 rbt || exit 1
GELIM_KEEP_HW_QUEUES=1 run mm d8 rbt t0 || exit 1
GELIM_KEEP_HW_QUEUES=1 run head mm d8 rbt t0 te || exit 1
run head mm d8 rbt t0 te || exit 1
