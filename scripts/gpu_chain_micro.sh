set -o pipefail
timeout -k 10 200 python -u -m pytest tests/test_gpu_dist_rbt.py -m gpu -x -q --timeout 120 --timeout-method thread -k "chain_products or native_executor" > gpurun_out/pytest_cp.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_cp.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/pytest_cp.log | head -20; exit $rc; }
timeout -k 10 120 python -u scripts/chain_products_bench.py
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/cp_prof -o run -- python3 scripts/chain_products_bench.py > /dev/null 2>&1 && cat $(find gpurun_out/cp_prof -name '*kernel_stats.csv') | cut -c1-200
