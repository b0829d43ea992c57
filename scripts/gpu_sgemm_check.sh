#!/usr/bin/env bash
# fp32 GEMM change check: matmul tests, square-size timings, LDS conflict counters
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out/sgemm"
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_matmul.py -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" "$OUT/pytest.log" | tail -3
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u scripts/gemm_bench.py f32 > "$OUT/gemm.txt" 2>&1 || exit $?
cat "$OUT/gemm.txt" | grep sgemm
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 60 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_INST_ANY --output-format csv -d "$OUT/pmc" -o run -- "$ROOT/bin/hip_matmul" 2048 --no-seq --no-omp > "$OUT/pmc.log" 2>&1 || exit $?
python3 - "$OUT/pmc" <<'PY'
import csv, glob, sys, collections
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        agg[r["Kernel_Name"][:60]][r["Counter_Name"]] += float(r["Counter_Value"])
for k, d in agg.items():
    if "mfma" in k:
        print(k, ", ".join(f"{c}={v:.4g}" for c, v in sorted(d.items())))
PY
