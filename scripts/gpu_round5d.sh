#!/bin/bash
# Round 5 GPU session d: full GPU suite after the knob pruning, hip-rbt
# timing (split triangular solves), and the 1-GPU bench line.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
export MASTER_ADDR=127.0.0.1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 300 python -u scripts/time_rbt.py 2048 8192 16384 > $O/rbt_times.txt 2>&1
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err
