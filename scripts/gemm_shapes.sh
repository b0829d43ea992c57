#!/usr/bin/env bash
# A/B of the fp32 GEMM tile shapes (GELIM_SGEMM_SHAPE), scripts/gemm_bench.py f32
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p gpurun_out
for sh in default 64x64x32 128x64x16 128x64x32 64x128x16; do
  if [ "$sh" = default ]; then unset GELIM_SGEMM_SHAPE; else export GELIM_SGEMM_SHAPE=$sh; fi
  echo "## $sh"
  timeout -k 10 120 python scripts/gemm_bench.py f32 || exit $?
done > gpurun_out/gemm_shapes.txt 2>&1
echo done
