#!/bin/bash
# Round-5 GPU sessions (run through gpurun): each stage has its own time
# limit and the chain stops at the first failure.
#   rccl    the one-rank RCCL suite + host-issue measurements (profiles/dist_issue_r5.md)
#   rbt     hip-rbt tests + 2048/8192/16384 timing + 8192 kernel trace (profiles/trsv_split_r5.txt)
#   full    the whole GPU suite + hip-rbt timing + the bench line
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
export MASTER_ADDR=127.0.0.1
case "${1:-full}" in
  rccl)
    timeout -k 10 400 python -u -m pytest tests/test_gpu_rccl.py tests/test_gpu_dist_rbt.py tests/test_gpu_streams.py -x -v --timeout 320 --timeout-method thread > $O/pytest_rccl.log 2>&1
    timeout -k 10 300 python -u scripts/dist_issue.py --out $O/dist_issue_none.json > $O/dist_issue_none.txt 2>&1
    timeout -k 10 300 python -u scripts/dist_issue.py --pg --out $O/dist_issue_pg.json > $O/dist_issue_pg.txt 2>&1
    ;;
  rbt)
    timeout -k 10 600 python -u -m pytest tests/test_gpu_mixed.py tests/test_gpu_dist_rbt.py -x -q --timeout 240 --timeout-method thread > $O/pytest_mixed.log 2>&1
    timeout -k 10 300 python -u scripts/time_rbt.py 2048 8192 16384 > $O/rbt_times.txt 2>&1
    cd /tmp && export TMPDIR=/tmp
    timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/rbt_prof -o run -- python3 $R/scripts/time_rbt.py 8192 > $O/rbt_prof.txt 2>&1
    ;;
  full)
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1
    timeout -k 10 300 python -u scripts/time_rbt.py 2048 8192 16384 > $O/rbt_times.txt 2>&1
    timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err
    ;;
esac
