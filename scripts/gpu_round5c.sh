#!/bin/bash
# Round 5 GPU session c: split block triangular solves (blk_trsv_split_kernel)
# -- hip-rbt / hip-mixed tests, whole-solve A/B against the one-workgroup-per-
# row kernel, and a kernel trace of the 8192 solve.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_mixed.py tests/test_gpu_dist_rbt.py -x -q --timeout 240 --timeout-method thread > $O/pytest_mixed.log 2>&1
for v in 0 1; do
  echo "== GELIM_TRSV_SPLIT=$v" >> $O/trsv_ab.txt
  GELIM_TRSV_SPLIT=$v timeout -k 10 300 python -u scripts/time_rbt.py 2048 8192 16384 >> $O/trsv_ab.txt 2>&1
  GELIM_TRSV_SPLIT=$v timeout -k 10 300 python -u scripts/time_mixed.py 8192 16384 >> $O/trsv_ab.txt 2>&1
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/trsv_prof -o run -- python3 $R/scripts/time_rbt.py 8192 > $O/trsv_prof.txt 2>&1
