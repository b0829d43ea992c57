set -e
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
timeout -k 10 300 python bench.py --headline-only --no-matmul > gpurun_out/bench_h.json 2> gpurun_out/bench_h.err
