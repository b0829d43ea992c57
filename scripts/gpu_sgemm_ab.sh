# fp32 GEMM tile shapes at 2048^2 and 4096^2 (GELIM_SGEMM_AB: 0 default, 1 64x64x32, 2 64x128x16, 3 128x128x16, 4 128x64x16)
set -o pipefail
for r in 1 2; do for v in 0 1 2 3 4; do
  echo -n "shape $v: "; GELIM_SGEMM_AB=$v timeout -k 10 120 python -u scripts/gemm_bench.py f32 2>&1 | grep -E "n=(2048|4096):" | tr '\n' ' '; echo
done; done
