#!/bin/bash
# Round 5 GPU session a: the RCCL one-rank tests, the full GPU suite, and
# host-issue vs GPU-only times of the distributed schedules (one rank, with
# and without a one-rank RCCL group).  Each step has its own limit; the chain
# stops at the first failure.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
export MASTER_ADDR=127.0.0.1
timeout -k 10 400 python -u -m pytest tests/test_gpu_rccl.py -x -v --timeout 320 --timeout-method thread > $O/pytest_rccl.log 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 300 python -u scripts/dist_issue.py > $O/dist_issue_none.json 2> $O/dist_issue_none.err
timeout -k 10 300 python -u scripts/dist_issue.py --pg > $O/dist_issue_pg.json 2> $O/dist_issue_pg.err
