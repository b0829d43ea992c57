"""laswp+TRSM kernel variants for rocprofv3 (told apart by their grid):
random pivot rows / rows 0..63 / TRSM only / empty pair list.

  rocprofv3 --kernel-trace -- python3 scripts/laswp_bench.py
"""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import gelim  # noqa: E402
from gelim import _native  # noqa: E402
from gelim.utils.tensors import ptr, stream_handle  # noqa: E402


def main() -> None:
    m = 8192
    dev = torch.device("cuda:0")
    lib = _native.lib()
    sh = stream_handle(dev)
    lda = m + 8
    A = torch.rand(m, lda, dtype=torch.float64, device=dev)
    g = torch.Generator().manual_seed(0)

    def pairs_of(rows):
        rows = rows.tolist()
        p = torch.zeros(256, dtype=torch.int32)
        p[0] = len(rows)
        for e, r in enumerate(rows):  # a cyclic permutation of the rows
            p[1 + 2 * e], p[2 + 2 * e] = r, rows[(e + 1) % len(rows)]
        return p.to(dev)

    rnd = pairs_of(torch.randperm(m, generator=g)[:64])
    low = pairs_of(torch.arange(64))
    empty = torch.zeros(256, dtype=torch.int32, device=dev)
    for _ in range(20):
        lib.gelim_gpu_laswp_trsm(ptr(A), lda, 0, 0, 32, m + 1, 32, m, ptr(rnd), sh)        # 8161 cols
        lib.gelim_gpu_laswp_trsm(ptr(A), lda, 0, 0, 32, m - 63, 32, m, ptr(low), sh)       # 8097 cols
        lib.gelim_gpu_laswp_trsm(ptr(A), lda, 0, 0, 32, m - 127, m - 127, m, None, sh)     # 8033 cols: TRSM
        lib.gelim_gpu_laswp_trsm(ptr(A), lda, 0, 0, 32, m - 191, 32, m, ptr(empty), sh)    # 7969 cols: nothing
    torch.cuda.synchronize()
    print("done")


if __name__ == "__main__":
    main()
