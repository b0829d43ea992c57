#!/usr/bin/env bash
# One GPU-box session: GPU tests, bench, rocprofv3 kernel stats.
# Every GPU step has its own time limit; a crash-type exit (fault, abort,
# segfault, timeout) ends the session immediately (no further GPU work).
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
cd "$ROOT"
STEPS="${STEPS:-tests,bench,prof}"

fatal() { # exit codes that mean "do not touch the GPU again in this call"
  case "$1" in 0|1) return 1;; *) return 0;; esac
}

if [[ ",$STEPS," == *",tests,"* ]]; then
  timeout -k 10 "${TEST_TIMEOUT:-600}" python -m pytest tests -m gpu -q -x --timeout=300 ${PYTEST_ARGS:-} \
    > "$OUT/pytest_gpu.log" 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -25 "$OUT/pytest_gpu.log"
  if fatal $rc; then echo "FATAL after pytest ($rc)"; exit $rc; fi
fi

if [[ ",$STEPS," == *",bench,"* ]]; then
  timeout -k 10 "${BENCH_TIMEOUT:-300}" python bench.py --steps 20 --warmup 5 ${BENCH_ARGS:-} \
    > "$OUT/bench.json" 2> "$OUT/bench.err"
  rc=$?; echo "bench rc=$rc"; cat "$OUT/bench.json"; tail -5 "$OUT/bench.err"
  if [ $rc -ne 0 ]; then echo "FATAL after bench ($rc)"; exit $rc; fi
fi

if [[ ",$STEPS," == *",prof,"* ]]; then
  export TMPDIR=/tmp
  ( cd /tmp && timeout -k 10 "${PROF_TIMEOUT:-240}" rocprofv3 --kernel-trace --stats --output-format csv \
      -d "$OUT/prof" -o run -- python3 "$ROOT/bench.py" --steps 5 --warmup 2 --no-matmul ${PROF_BENCH_ARGS:-} > "$OUT/prof.log" 2>&1 )
  rc=$?; echo "rocprof rc=$rc"; tail -3 "$OUT/prof.log"
  find "$OUT/prof" -name "*kernel_stats.csv" | head -3
  if [ $rc -ne 0 ]; then exit $rc; fi
fi

if [[ ",$STEPS," == *",cli,"* ]]; then
  timeout -k 10 "${CLI_TIMEOUT:-300}" ./bin/hip_matmul 2048 --json > "$OUT/hip_matmul_2048.txt" 2>&1
  rc=$?; echo "hip_matmul rc=$rc"; cat "$OUT/hip_matmul_2048.txt"
  if [ $rc -ne 0 ]; then exit $rc; fi
  timeout -k 10 120 ./bin/gauss_internal_input -s 2048 --json > "$OUT/gauss_internal_2048.txt" 2>&1
  rc=$?; echo "gauss_internal rc=$rc"; cat "$OUT/gauss_internal_2048.txt"
  if [ $rc -ne 0 ]; then exit $rc; fi
  timeout -k 10 120 ./bin/gauss_internal_input -s 2048 --backend=seq --json > "$OUT/gauss_internal_2048_seq.txt" 2>&1
  echo "seq rc=$?"; cat "$OUT/gauss_internal_2048_seq.txt"
fi
echo "session done"
