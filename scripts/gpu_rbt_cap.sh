# hip-rbt 8192 / 2048: the lookahead side GEMM's grid cap (GELIM_RBT_SIDE_CAP), alternating processes
set -o pipefail
for r in 1 2; do for c in 0 248 240 224; do
  echo -n "cap $c: "; GELIM_RBT_SIDE_CAP=$c timeout -k 10 120 python -u scripts/time_rbt.py 8192 2048 2>&1 | grep -v amdgpu.ids | tr '\n' ' '; echo
done; done
