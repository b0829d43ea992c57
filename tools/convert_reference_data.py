"""Convert the reference's `.dat` matrices into compact `data/<name>.coo.npz`
fixtures (int32 1-based rows/cols + float64 values, numpy.savez_compressed).

The reference tree is not present on the GPU box, so tests there read these
fixtures; on a host with /root/reference the tests also cross-check the
native `.dat` reader against them.  Usage:
    python tools/convert_reference_data.py [/root/reference/Pthreads/Version-1/matrices_dense]
"""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import gelim  # noqa: E402
from gelim.utils import io  # noqa: E402

NAMES = ["matrix_10", "jpwh_991", "orsreg_1", "sherman5", "saylr4", "sherman3", "memplus"]


def main(src: str) -> None:
    out = Path(__file__).resolve().parents[1] / "data"
    out.mkdir(exist_ok=True)
    for name in NAMES:
        p = Path(src) / f"{name}.dat"
        if not p.exists():
            print(f"skip {name}: {p} missing")
            continue
        n, r, c, v = io.dat_to_coo(p)
        io.save_coo_npz(out / f"{name}.coo.npz", n, r, c, v)
        print(f"{name}: n={n} nnz={len(v)}")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "/root/reference/Pthreads/Version-1/matrices_dense")
