# A/B of two builds of libgelim.so (tools/ablib/libgelim_{A,B}.so), alternating processes:
# hip-rbt solves (scripts/time_rbt.py) and the DistributedRBT P = 8 replay
set -o pipefail
L=gaussian_elimination-cuda-openmp-mpi-pthreads_amd/lib/libgelim.so
for r in 1 2; do for v in ${VARIANTS:-noprio prio}; do
  cp tools/ablib/libgelim_$v.so $L
  echo -n "$v: "; timeout -k 10 150 python -u scripts/time_rbt.py 2048 8192 16384 2>&1 | grep -v amdgpu.ids | tr '\n' ' '
  timeout -k 10 150 python -u scripts/one_rank_of_p.py --n 8192 --P 8 --rank 1 --json gpurun_out/orp_ab.json > gpurun_out/orp_ab.log 2>&1 || { tail -5 gpurun_out/orp_ab.log; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/orp_ab.json'))
print('| replay P=8 factor', round(d['factor_min_ms'],3), 'total', round(d['measured_total_ms'],3))"
done; done
