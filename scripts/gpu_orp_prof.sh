set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/orp_prof -o run -- python3 scripts/one_rank_of_p.py --n 8192 --P 8 --rank 1 --factor-only --reps 3 > gpurun_out/orp_prof.log 2>&1 || { tail -20 gpurun_out/orp_prof.log; exit 1; }
f=$(find gpurun_out/orp_prof -name '*kernel_trace.csv' | head -1)
python3 scripts/orp_trace_summary.py "$f" 30 3
