#!/bin/bash
# split-TRSV iteration: correctness of the hip-rbt / distributed-rbt paths, 2048/8192 timing, kernel stats
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_mixed.py tests/test_gpu_dist_rbt.py -x -q --timeout 240 --timeout-method thread > $O/pytest_mixed.log 2>&1
timeout -k 10 300 python -u scripts/time_rbt.py 2048 8192 > $O/trsv_quick.txt 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/trsv_prof -o run -- python3 $R/scripts/time_rbt.py 8192 > $O/trsv_prof.txt 2>&1
