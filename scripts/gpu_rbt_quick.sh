#!/usr/bin/env bash
# quick loop for the randomised engines: their GPU tests + timing breakdown
set -u
OUT="${GRAFT_REPO_ROOT:-.}/gpurun_out"
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_mixed.py -q --timeout 120 --timeout-method thread > "$OUT/mixed_q.log" 2>&1
prc=$?; echo "pytest rc=$prc"; grep -v amdgpu.ids "$OUT/mixed_q.log" | grep -E "passed|failed|Error|assert" | head -20
[ $prc -gt 1 ] && exit $prc
timeout -k 10 200 python -u scripts/mixed_breakdown.py --backend hip-rbt ${SIZES:-2048 8192}
