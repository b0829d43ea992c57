#!/bin/bash
# back-substitution session: GPU suite, headline timing, kernel trace of the headline
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
export MASTER_ADDR=127.0.0.1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 300 python bench.py --headline-only --no-matmul > $O/bench_h.json 2> $O/bench_h.err
timeout -k 10 300 python scripts/time_rbt.py 8192 > $O/rbt8192.txt 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/bs_prof -o run -- python3 $R/bench.py --headline-only --no-matmul --steps 10 --warmup 2 > $O/bs_prof.txt 2>&1
