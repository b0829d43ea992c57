"""Diagnostic: per-block timing of the randomised engine's persistent lower
block solve (realtime stamps per workgroup: start, last block's values in
hand, published).

  python scripts/trsv_stamps.py 8192
"""
import ctypes as C
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import gelim  # noqa: E402
from gelim.utils.tensors import ptr, stream_handle  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
dev = torch.device("cuda:0")
lib = gelim._native.lib()
lib.gelim_debug_trsv_stamps.argtypes = [C.c_void_p]
lib.gelim_debug_trsv_stamps.restype = None
aug = gelim.random_system(n, seed=n, device=dev)
s = gelim.GaussSolver(n, backend="hip-rbt", device=dev)
sh = stream_handle(dev)
gelim._native.check(lib.gelim_mixed_factor(s._mixed, ptr(aug), aug.stride(0), sh), "factor")
nblk = int(lib.gelim_mixed_plan_np(s._mixed)) // 128
st = torch.zeros(3 * nblk, dtype=torch.int64, device=dev)
r = aug[:, n].contiguous()
d = torch.empty(n, dtype=torch.float64, device=dev)
for _ in range(3):
    lib.gelim_debug_trsv_stamps(st.data_ptr())
    gelim._native.check(lib.gelim_mixed_apply(s._mixed, ptr(r), 1, ptr(d), sh), "apply")
    torch.cuda.synchronize()
lib.gelim_debug_trsv_stamps(None)
t = st.view(nblk, 3).cpu().double() * 10e-3  # 100 MHz ticks -> us
t -= t[:, 0].min()
print(f"n={n}: {nblk} blocks, lower solve span {t[:, 2].max():.1f} us")
print(" blk   start   ready   pub  | chain(pub_w - pub_w-1)  wait(ready_w - pub_w-1)  finish(pub_w - ready_w)")
for w in list(range(0, 6)) + list(range(nblk // 2, nblk // 2 + 3)) + list(range(nblk - 4, nblk)):
    if w >= nblk:
        continue
    prev = t[w - 1, 2] if w > 0 else t[w, 0]
    print(f"{w:4d} {t[w,0]:7.1f} {t[w,1]:7.1f} {t[w,2]:7.1f} | {t[w,2]-prev:8.2f} {t[w,1]-prev:8.2f} {t[w,2]-t[w,1]:8.2f}")
s.close()
