#!/usr/bin/env bash
# PMC passes over the Gauss-Jordan block inverse (scripts/gj_only.py), one
# pass per run, each under its own hard limit.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/pmcgj"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
PASSES=(
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS"
  "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU"
)
i=0
for p in "${PASSES[@]}"; do
  i=$((i + 1))
  timeout -s KILL 90 rocprofv3 --pmc $p --output-format csv -d "$OUT/p$i" -o run -- python3 "$ROOT/scripts/gj_only.py" \
    > "$OUT/p$i.log" 2>&1
  rc=$?
  echo "pass $i rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/p$i.log"; exit $rc; fi
done
