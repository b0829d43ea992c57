#!/usr/bin/env bash
# PMC passes over the randomised engine's factor kernels (one pass per run)
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/pmc_rbt"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
PASSES=(
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_BRANCH"
  "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM"
)
i=0
for p in "${PASSES[@]}"; do
  i=$((i + 1))
  timeout -s KILL 90 rocprofv3 --pmc $p --output-format csv -d "$OUT/p$i" -o run -- \
    python3 "$ROOT/scripts/rbt_factor_only.py" ${ARGS:-2048 2} > "$OUT/p$i.log" 2>&1
  rc=$?
  echo "pass $i rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.Counter()
for f in sorted(glob.glob(out + "/p*/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"][:70]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, d in agg.items():
    if "diag" in k or "trsv" in k or "dgemm" in k:
        print(k)
        print("   " + ", ".join(f"{c}={v:.4g}" for c, v in sorted(d.items())))
PY
