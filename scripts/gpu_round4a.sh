#!/bin/bash
# Round 4 GPU session: full GPU suite, the bench line, and rocprofv3 kernel
# traces of the new engines (distributed randomised solver on one rank, the
# persistent hip-pivot, the thin GEMM variants).  Every step has its own
# time limit; the chain stops at the first failure.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace -d $O/drbt -o run -- python3 $R/scripts/dist_rbt_prof.py 8192 > $O/drbt.txt 2>&1
timeout -k 10 240 rocprofv3 --kernel-trace -d $O/pivot -o run -- python3 $R/scripts/time_pivot.py 2048 --reps 3 > $O/pivot.txt 2>&1
bash $R/scripts/thin_gemm_prof.sh
