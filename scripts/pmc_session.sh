#!/usr/bin/env bash
# PMC counter passes (rocprofv3 --pmc, one pass per run, no tracing domains)
# over the 2048^2 fp32 MFMA matmul and the 2048^2 fp64 Gauss solve.
# Every pass has its own hard time limit; the first failure ends the session.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/pmc"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp

PASSES=(
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_WAIT_ANY SQ_WAIT_INST_ANY"
  "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_MFMA"
  "FETCH_SIZE"
  "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"
)
WORKLOADS=(
  "matmul|$ROOT/bin/hip_matmul 2048 --no-seq --no-omp"
  "gauss|python3 $ROOT/bench.py --steps 2 --warmup 1 --no-matmul --headline-only"
)
for wl in "${WORKLOADS[@]}"; do
  name="${wl%%|*}"
  cmd="${wl#*|}"
  i=0
  for p in "${PASSES[@]}"; do
    i=$((i + 1))
    timeout -s KILL "${PASS_TIMEOUT:-90}" rocprofv3 --pmc $p --output-format csv \
      -d "$OUT/${name}_p$i" -o run -- $cmd > "$OUT/${name}_p$i.log" 2>&1
    rc=$?
    echo "$name pass $i rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 "$OUT/${name}_p$i.log"; exit $rc; fi
  done
done
echo "pmc session done"
