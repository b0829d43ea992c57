# Round-6 closing run on one MI355X: the whole GPU suite, the chain-product
# micro-benchmark, then bench.py (the driver's contract) -- each step bounded
set -o pipefail
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_r6.txt 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu_r6.txt
case $rc in 0|1) ;; *) echo "pytest rc=$rc: stopping"; exit $rc ;; esac
timeout -k 10 120 python -u scripts/chain_products_bench.py > gpurun_out/chain_products_r6.txt 2>&1 || exit 1
cat gpurun_out/chain_products_r6.txt
timeout -k 10 600 python -u bench.py > gpurun_out/bench_r6.json 2> gpurun_out/bench_r6.err || { tail -20 gpurun_out/bench_r6.err; exit 1; }
tail -c 3000 gpurun_out/bench_r6.json
