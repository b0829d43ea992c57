"""One rank of the distributed randomised solver (parallel/dist_rbt.py) on the
distributed SCHEDULE (single_fast_path=False): wall time per solve and, under
rocprofv3 --kernel-trace, the per-kernel durations the 8-rank critical-path
estimate is built from (scripts/dist_rbt_critical_path.py).

  rocprofv3 --kernel-trace -d gpurun_out/drbt -o run -- python3 scripts/dist_rbt_prof.py 8192
"""
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import gelim  # noqa: E402
from gelim.parallel import DistributedRBT  # noqa: E402
from gelim.parallel.comm import Communicator  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
    dev = torch.device("cuda:0")
    c = Communicator(0, 1, dev, "none")
    for fast in (True, False):
        d = DistributedRBT(c, n, single_fast_path=fast)
        ts = []
        for _ in range(3):
            loc = d.generate_random(seed=99)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            x = d.solve_(loc)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        print(f"n={n} fast_path={fast}: solve {min(ts) * 1e3:.2f} ms (best of 3), error "
              f"{gelim.ops.gauss.error_metric(x):.2e}, corrections {d.last_steps}, fallback {d.last_fallback}",
              flush=True)
        d.close()


if __name__ == "__main__":
    main()
