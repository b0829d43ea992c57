#!/bin/bash
# Round 5 GPU session b: RCCL one-rank tests (graph-replayed DistributedRBT),
# the distributed-RBT GPU tests, and the host-issue measurements.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
export MASTER_ADDR=127.0.0.1
timeout -k 10 400 python -u -m pytest tests/test_gpu_rccl.py tests/test_gpu_dist_rbt.py tests/test_gpu_streams.py -x -v --timeout 320 --timeout-method thread > $O/pytest_rccl.log 2>&1
timeout -k 10 300 python -u scripts/dist_issue.py > $O/dist_issue_none.json 2> $O/dist_issue_none.err
timeout -k 10 300 python -u scripts/dist_issue.py --pg > $O/dist_issue_pg.json 2> $O/dist_issue_pg.err
