"""Diagnostic: in-kernel s_memtime phase timings of the panel kernel."""
import ctypes as C
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import gelim  # noqa: E402

lib = gelim._native.lib()
f = lib.gelim_debug_panel_stamps
f.argtypes = [C.c_int64, C.c_int64, C.POINTER(C.c_ulonglong)]
f.restype = C.c_int
print("m w load_cyc steps_cyc store_cyc total_cyc steps_per_col")
for m in [int(x) for x in sys.argv[1:]] or (200, 1000, 2048):
    for w in (1, 2, 4, 8, 16):
        out = (C.c_ulonglong * 9)()
        gelim._native.check(f(m, w, out))
        print(m, w, out[0], out[1], out[2], out[3], out[1] / w, "step4:", list(out[4:9]))
