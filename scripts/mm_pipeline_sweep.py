"""End-to-end 2048^2 fp32 matmul: serial (reference copy pattern) vs the
chunked H2D / GEMM / D2H pipeline at several chunk counts (median of 9)."""
import statistics
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

import gelim  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
dev = torch.device("cuda:0")
A, B = gelim.ops.matmul.reference_inputs(n)
A, B = A.pin_memory(), B.pin_memory()
Ch = torch.empty_like(A).pin_memory()
m = gelim.MatMul("mfma", dev)
runs = {"serial": lambda: m.run_reference_style(A, B, Ch)}
for c in (1, 2, 4, 8, 16):
    runs[f"pipe{c}"] = (lambda c=c: m.run_pipelined(A, B, Ch, chunks=c))
res = {k: [] for k in runs}
for _ in range(3):
    for f in runs.values():
        f()
for _ in range(9):
    for k, f in runs.items():
        res[k].append(f().end_to_end_s * 1e3)
for k, v in res.items():
    print(f"{k:>8}: median {statistics.median(v):.3f} ms  min {min(v):.3f} ms", flush=True)
