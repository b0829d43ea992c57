"""L1 data / IO: the reference `.dat` coordinate format, matrix_gen output and
the compact `.coo.npz` fixtures shipped in `data/`.

`.dat` (Pthreads/Version-1/gauss_external_input.c:34-86): header "n n nnz",
then "row col value" 1-based, terminated by a row-0 line.  Parsing is done by
the native reader (`gelim_dat_read`); the `.coo.npz` fixtures hold the same
coordinates as int32 rows/cols + float64 values (loaded with
numpy.load(allow_pickle=False)).
"""
from __future__ import annotations

import os
from pathlib import Path

import numpy as np
import torch

from .. import _native

DATA_DIR = Path(__file__).resolve().parents[2] / "data"


def dat_size(path: str | os.PathLike) -> int:
    return _native.check(_native.lib().gelim_dat_size(os.fsencode(path)), f"dat_size({path})")


def read_dat(path: str | os.PathLike, ld: int | None = None, dtype=torch.float64) -> torch.Tensor:
    """Dense (n, ld) float64 CPU tensor of a `.dat` file (columns >= n zero)."""
    n = dat_size(path)
    ld = n if ld is None else ld
    out = torch.zeros((n, ld), dtype=torch.float64)
    _native.check(_native.lib().gelim_dat_read(os.fsencode(path), out.data_ptr(), n, ld), "dat_read")
    return out if dtype == torch.float64 else out.to(dtype)


def write_dat(path: str | os.PathLike, rows: np.ndarray, cols: np.ndarray, vals: np.ndarray, n: int) -> None:
    """Write 1-based coordinates in the reference format (values as %.17g)."""
    with open(path, "w") as f:
        f.write(f"{n} {n} {len(vals)}\n")
        for r, c, v in zip(rows, cols, vals):
            f.write(f"{int(r)} {int(c)} {float(v)!r}\n")
        f.write("0 0 0\n")


def dat_to_coo(path: str | os.PathLike) -> tuple[int, np.ndarray, np.ndarray, np.ndarray]:
    """Parse a `.dat` file into (n, rows, cols, vals) 1-based, in file order."""
    rows, cols, vals = [], [], []
    with open(path) as f:
        n = int(f.readline().split()[0])
        for line in f:
            parts = line.split()
            if not parts:
                continue
            r = int(parts[0])
            if r == 0:
                break
            rows.append(r)
            cols.append(int(parts[1]))
            vals.append(float(parts[2]))
    return n, np.asarray(rows, np.int32), np.asarray(cols, np.int32), np.asarray(vals, np.float64)


def save_coo_npz(path: str | os.PathLike, n: int, rows, cols, vals) -> None:
    np.savez_compressed(path, n=np.int64(n), rows=rows, cols=cols, vals=vals)


def load_coo_npz(path: str | os.PathLike) -> tuple[int, np.ndarray, np.ndarray, np.ndarray]:
    z = np.load(path, allow_pickle=False)
    return int(z["n"]), z["rows"], z["cols"], z["vals"]


def coo_to_dense(n: int, rows, cols, vals, ld: int | None = None) -> torch.Tensor:
    """Densify 1-based coordinates; later duplicates overwrite earlier ones,
    like the reference's `matrix[l1-1][l2-1] = d`."""
    ld = n if ld is None else ld
    out = np.zeros((n, ld), np.float64)
    out[np.asarray(rows, np.int64) - 1, np.asarray(cols, np.int64) - 1] = vals
    return torch.from_numpy(out)


def fixture_path(name: str) -> Path:
    """data/<name>.coo.npz (name without extension, e.g. 'jpwh_991')."""
    return DATA_DIR / f"{name}.coo.npz"


def load_fixture(name: str, ld: int | None = None) -> torch.Tensor:
    n, r, c, v = load_coo_npz(fixture_path(name))
    return coo_to_dense(n, r, c, v, ld)


def matrix_gen(n: int, path: str | os.PathLike = "-") -> None:
    """matrix_gen-compatible output (Pthreads/Version-1/matrices_dense/matrix_gen.cc)."""
    _native.check(_native.lib().gelim_matrix_gen(n, os.fsencode(path)), "matrix_gen")
