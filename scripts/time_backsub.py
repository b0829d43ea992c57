"""Back substitution alone (csrc/hip/backsub.hip, gelim_gpu_backsub) on a
random well-conditioned upper-triangular system: time per call for a range of
n, so the prologue (n = 64: one block) and the per-block chain step (slope)
separate.  python scripts/time_backsub.py [n ...]"""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import gelim  # noqa: E402,F401
from gelim import _native  # noqa: E402
from gelim.utils.tensors import ptr, stream_handle  # noqa: E402


def main():
    ns = [int(a) for a in sys.argv[1:]] or [64, 128, 256, 512, 1024, 2048, 4096, 8192]
    lib = _native.lib()
    dev = torch.device("cuda:0")
    for n in ns:
        g = torch.Generator(device=dev).manual_seed(n)
        U = torch.rand(n, n, dtype=torch.float64, device=dev, generator=g) - 0.5
        U = torch.triu(U, 1) / n ** 0.5 + torch.diag(1.0 + torch.rand(n, dtype=torch.float64, device=dev, generator=g))
        xt = torch.rand(n, dtype=torch.float64, device=dev, generator=g)
        y = U @ xt
        x = torch.empty(n, dtype=torch.float64, device=dev)
        sh = stream_handle()

        def run():
            _native.check(lib.gelim_gpu_backsub(ptr(U), n, ptr(y), 1, ptr(x), None, n, 0, sh), "backsub")

        run()
        torch.cuda.synchronize()
        err = ((x - xt).abs().max() / xt.abs().max()).item()
        ts = []
        for _ in range(7):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                run()
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3 / 20)
        t = sorted(ts)[len(ts) // 2]
        print(f"n={n:6d} blocks={(n + 63) // 64:4d}  {t:8.1f} us/call  err {err:.2e}", flush=True)


if __name__ == "__main__":
    main()
