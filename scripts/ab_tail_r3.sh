set -u
for t in 1024 1152 1280 1408 1536 1792; do
  echo "tail $t"; GELIM_HYBRID=$t timeout -k 10 60 python -u scripts/time_solver.py 2048 --reps 20 || exit 1
done
GELIM_SCHEDULE=resident timeout -k 10 60 python -u scripts/time_solver.py 2048 --reps 20 || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_solver.py -q -k "hybrid or resident" --timeout 120 --timeout-method thread
