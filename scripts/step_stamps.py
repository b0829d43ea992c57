"""Diagnostic: realtime (10 ns) phase timings of one fused LU step kernel:
workgroup 0 (prologue = previous step on its strip, panel factorisation) vs
the wide workgroups (previous step on the trailing strips)."""
import ctypes as C
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import gelim  # noqa: E402

lib = gelim._native.lib()
f = lib.gelim_debug_step_stamps
f.argtypes = [C.c_int64, C.c_int64, C.POINTER(C.c_double)]
f.restype = C.c_int
n = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
print("step m | wg0: prologue_us panel_us total_us | wide: max_end_us median_end_us count")
for j in (1, 2, 8, 32, 64, 65, 96, 97, 120):
    if 16 * j >= n:
        continue
    for rep in range(2):
        out = (C.c_double * 24)()
        gelim._native.check(f(n, j, out))
    print(f"{j:4d} {n - 16 * j:5d} | {out[0] / 100:8.2f} {out[1] / 100:8.2f} {out[2] / 100:8.2f} | "
          f"{out[3] / 100:8.2f} {out[4] / 100:8.2f} {int(out[5])} | prologue phases us: "
          + " ".join(f"{v / 100:6.2f}" for v in out[6:12])
          + f" | panel load/steps/store us: {out[12] / 100:6.2f} {out[13] / 100:6.2f} {out[14] / 100:6.2f}"
          + f" | store = recon+drain {out[15] / 100:5.2f} barrier {out[16] / 100:5.2f} dest {out[17] / 100:5.2f}"
          + f" fixup+end {out[18] / 100:5.2f} (recon alone {out[19] / 100:5.2f})")
