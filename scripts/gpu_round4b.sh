#!/bin/bash
# Round 4 GPU session b: full GPU suite, the bench line, the distributed
# randomised solver's uncontended kernel times and a kernel trace of its
# one-rank schedule (critical-path inputs).  Each step has its own limit;
# the chain stops at the first failure.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err
timeout -k 10 120 python scripts/dist_rbt_prof.py --micro > $O/drbt_micro.txt 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace -d $O/drbt -o run -- python3 $R/scripts/dist_rbt_prof.py 8192 > $O/drbt.txt 2>&1
