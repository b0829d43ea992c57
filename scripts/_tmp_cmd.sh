set -e
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/p8 -o run --output-format csv -- python3 $R/scripts/time_solver.py 8192 --reps 2 > $R/gpurun_out/p8.txt 2>&1
