"""Diagnostic: in-kernel phase timings of the resident LU (rlu.hip) for one
n x n solve: per engine step F (panel factorisation), publish, wait for the
next strip, drain + flag, TRSM, strip update; and how early the updaters
finish the strip the engine needs next.  Units: microseconds."""
import ctypes as C
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import gelim  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
np_ = (n + 15) // 16
need = 8 * np_ + 2 * (np_ + 1) * np_ + 8
buf = (C.c_ulonglong * need)()
lib = gelim._native.lib()
lib.gelim_debug_rlu_stamps.argtypes = [C.c_int64, C.POINTER(C.c_ulonglong), C.c_int64]
gelim._native.check(lib.gelim_debug_rlu_stamps(n, buf, need), "debug_rlu_stamps")
e = [[buf[j * 8 + k] for k in range(8)] for j in range(np_)]
base = e[0][0]
us = lambda a, b: (b - a) / 100.0  # noqa: E731
names = ["F+poll", "loads+pub", "-", "trsm", "update", "drain+flag"]
tot = [0.0] * 6
print(f"n={n} steps={np_}; engine phases (us) per step")
print("step   " + " ".join(f"{x:>8s}" for x in names) + "    step_total  strip_ready_before_need")
for j in range(np_):
    ph = [us(e[j][k], e[j][k + 1]) if e[j][k + 1] else 0.0 for k in range(6)]
    for k in range(6):
        tot[k] += ph[k]
    nxt = e[j + 1][0] if j + 1 < np_ else e[j][6] or e[j][4]
    st = us(e[j][0], nxt)
    # updater j+1 applied its last step (j-1): its end stamp vs the engine's need (end of publish)
    slack = ""
    if 1 <= j and j + 1 < np_:
        s = j + 1
        end = buf[8 * np_ + 2 * (s * np_ + (j - 1)) + 1]
        if end:
            slack = f"{us(end, e[j][2]):8.2f}"
    if j < 4 or j % 16 == 0 or j >= np_ - 3:
        print(f"{j:4d}   " + " ".join(f"{v:8.2f}" for v in ph) + f"    {st:8.2f}    {slack}")
print("sum    " + " ".join(f"{v:8.1f}" for v in tot) + f"    total {us(base, e[-1][4] or e[-1][2]):.1f}")
cs = [buf[8 * np_ + 2 * (np_ + 1) * np_ + k] for k in range(7)]
if cs[0]:
    d = [cs[k + 1] - cs[k] for k in range(6)]
    print("column 4 of step 10 (shader cycles): candidate+rcp %d | wave argmax+publish %d | barrier %d | "
          "merge %d | pivot row+mults+col J+1 %d | rest of update %d | total %d" % (*d, cs[6] - cs[0]))
