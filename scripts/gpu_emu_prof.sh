set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python scripts/extras_emulated.py 8 > gpurun_out/emu8.txt 2>&1 || exit $?
timeout -k 10 300 python scripts/extras_emulated.py 4 > gpurun_out/emu4.txt 2>&1 || exit $?
timeout -k 10 200 python scripts/time_solver.py 2048 4096 8192 > gpurun_out/ts.txt 2>&1 || exit $?
export TMPDIR=/tmp
cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof2048" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 10 --warmup 2 --no-matmul --headline-only > "$GRAFT_REPO_ROOT/gpurun_out/prof.log" 2>&1 || exit $?
echo done
