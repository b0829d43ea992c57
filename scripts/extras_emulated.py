"""Rehearse bench.py's multi-GPU extras (8192^2 distributed Gauss, 16384^2
ring matmul) on ONE GPU with P emulated ranks (threads sharing the card):
checks the full-size distributed code paths end to end; the times are NOT
multi-GPU numbers (the ranks share one device).

  python scripts/extras_emulated.py [P] [n_gauss] [n_mm]
"""
import importlib.util
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import torch  # noqa: E402

import gelim  # noqa: E402
from gelim.parallel import run_emulated  # noqa: E402

P = int(sys.argv[1]) if len(sys.argv) > 1 else 8
ng = int(sys.argv[2]) if len(sys.argv) > 2 else 8192
nm = int(sys.argv[3]) if len(sys.argv) > 3 else 16384
spec = importlib.util.spec_from_file_location("bench_mod", ROOT / "bench.py")
bench = importlib.util.module_from_spec(spec)
spec.loader.exec_module(bench)
dev = "cuda:0" if torch.cuda.is_available() else "cpu"
res = run_emulated(P, lambda c: {f"dist_gauss_{ng}": bench.bench_dist_gauss(c, gelim, torch, ng),
                                  f"dist_matmul_{nm}": bench.bench_dist_matmul(c, gelim, torch, nm)},
                   device=dev, timeout_s=600)
print(json.dumps({"emulated_ranks": P, "device": dev, "rank0": res[0]}), flush=True)
