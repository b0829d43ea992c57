# rocprofv3 kernel statistics of the 2048^2 headline solve (bench.py --headline-only), then one PMC pass
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof2048_r6 -o run -- python3 bench.py --steps 10 --warmup 2 --no-matmul --headline-only > gpurun_out/prof2048_r6.log 2>&1 || { tail -5 gpurun_out/prof2048_r6.log; exit 1; }
f=$(find gpurun_out/prof2048_r6 -name '*kernel_stats.csv' | head -1); cut -c1-160 "$f" | head -12
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS --output-format csv -d gpurun_out/pmc2048_r6 -o run -- python3 bench.py --steps 3 --warmup 1 --no-matmul --headline-only > gpurun_out/pmc2048_r6.log 2>&1 || { tail -5 gpurun_out/pmc2048_r6.log; exit 1; }
echo pmc done
