"""GaussSolver — the framework's Gaussian-elimination "model": one n x n
system A x = b, solved by a selectable backend with reference semantics
(forward elimination + back substitution).

Backends
  hip / hip-blocked : blocked right-looking LU with partial (or zero) pivoting,
                      register-resident panel + fp64 MFMA trailing GEMM,
                      the whole solve replayed from a captured hipGraph (fp64)
  hip-pivot         : the reference per-pivot algorithm on the GPU
                      (unit-diagonal elimination, fp64 or fp32)
  hip-rbt           : random butterfly transform + NO-pivoting blocked LU with
                      fp64 factors (fp64 MFMA GEMMs, no per-column global
                      arg-max) + classic fp64 iterative refinement on the
                      original system, falling back to `hip` (fp64, partial
                      pivoting) whenever it does not reach the fp64 error
                      class (csrc/hip/lu_mixed.hip)

fp32 elimination + fp64 refinement is `hip-pivot` with
dtype=float32 and `solve_refined` (stored fp32 factors, O(n^2) per
correction).  It is NOT a fast path: the per-pivot loop is latency-bound, so
fp32 saves no time (2048: 11.9 vs 11.4 ms); it serves the reference's fp32
programs and fp32 inputs.  The fast paths are fp64 (`hip`, `hip-rbt`).  The
round-3/4 "hip-mixed" engine (fp32 trailing products + GMRES-IR) was removed
in round 5: slower than hip-rbt at every n and not convergent at 16384
(profiles/trsv_split_r5.txt).
  seq / omp / pthreads-v1 / pthreads-v2 / pthreads-v3 : the reference CPU
                      strategies (csrc/cpu/gauss_cpu.cpp), fp64

Input is an augmented system `aug` (n rows, >= n+1 columns, b in column n),
as produced by `ops.init.*_system`.  `solve` never modifies `aug`.
"""
from __future__ import annotations

import sys as _sys

import torch

from .. import _native
from ..ops import gauss as cpu_ops
from ..ops import lu
from ..utils.tensors import ptr, row_major_ld, stream_handle

GPU_BACKENDS = {"hip": _native.GPU_BLOCKED, "hip-blocked": _native.GPU_BLOCKED, "hip-pivot": _native.GPU_PIVOT}
RBT_BACKEND = "hip-rbt"
RBT_BACKENDS = {RBT_BACKEND: 1}  # factor precision: fp64
CPU_BACKENDS = tuple(cpu_ops.CPU_BACKENDS)
RESOLVE_LDS_BYTES = 160 * 1024  # lower_resolve_kernel (csrc/hip/gauss_pivot.hip)
BACKENDS = tuple(GPU_BACKENDS) + tuple(RBT_BACKENDS) + CPU_BACKENDS


class GaussSolver:
    def __init__(self, n: int, backend: str = "hip", pivot: str = "partial", dtype=torch.float64,
                 device=None, use_graph: bool = True, threads: int = 0, affinity: bool = True):
        if backend not in BACKENDS:
            raise ValueError(f"unknown backend {backend!r}; choose from {BACKENDS}")
        if pivot not in ("partial", "zero"):
            raise ValueError("pivot must be 'partial' or 'zero'")
        self.n, self.backend, self.pivot, self.dtype = n, backend, pivot, dtype
        self.threads, self.affinity = threads, affinity
        self._plan = None
        self._mixed = None
        self._fp64 = None
        self.last_steps = 0
        self.last_fallback = None
        self.last_berr = None
        if backend in ("hip", "hip-blocked") and dtype == torch.float32:
            raise ValueError("the blocked LU is fp64 (partial-pivoting accuracy on the reference matrices); "
                             "for fp32 elimination choose backend='hip-pivot' (the reference loop in fp32, "
                             "solve_refined for fp64 accuracy); the fastest fp64-class solver is "
                             "backend='hip-rbt'")
        self.gpu = backend in GPU_BACKENDS or backend in RBT_BACKENDS
        if backend in RBT_BACKENDS:
            self._init_mixed(device, seed=0x5eed, fp64=RBT_BACKENDS[backend])
        elif self.gpu:
            self.device = torch.device(device if device is not None else "cuda")
            if dtype == torch.float32 and backend != "hip-pivot":
                raise ValueError("fp32 elimination is only offered by hip-pivot (fp64 is required for "
                                 "partial-pivoting accuracy on the reference matrices)")
            eb = 8 if dtype == torch.float64 else 4
            with torch.cuda.device(self.device):
                plan = _native.lib().gelim_gauss_plan_create(n, GPU_BACKENDS[backend], lu._pivot_code(pivot), eb,
                                                             int(use_graph))
            if not plan:
                raise _native.GelimError(_native.E_ARG, _native.last_error())
            self._plan = plan
        else:
            if dtype != torch.float64:
                raise ValueError("CPU backends are fp64 (reference precision)")
            self.device = torch.device("cpu")

    # -- randomised no-pivoting engines (RBT + no-pivot LU + fp64 refinement) --
    def _init_mixed(self, device, seed: int, fp64: int = 0) -> None:
        import numpy as np

        self.device = torch.device(device if device is not None else "cuda")
        # the factorisation's precision; x is fp64
        self.dtype = torch.float64 if fp64 else torch.float32
        lib = _native.lib()
        n = self.n
        npad = int(lib.gelim_mixed_padded(n))
        if npad > int(lib.gelim_mixed_max_n()):
            self._mixed_unavailable = f"n = {n} beyond the mixed engine's {int(lib.gelim_mixed_max_n())}"
            return
        self._mixed_unavailable = None
        rng = np.random.default_rng(seed)
        # butterfly diagonals exp(r / 10), r uniform in [-1/2, 1/2] (8 arrays of npad/4 each, for U and V)
        self._ud = np.exp((rng.random(2 * npad) - 0.5) / 10.0)
        self._vd = np.exp((rng.random(2 * npad) - 0.5) / 10.0)
        with torch.cuda.device(self.device):
            plan = lib.gelim_mixed_plan_create2(n, self._ud.ctypes.data, self._vd.ctypes.data, int(fp64))
        if not plan:
            raise _native.GelimError(_native.E_ARG, _native.last_error())
        self._mixed = plan

    def _fallback(self, aug64: torch.Tensor, reason: str, check: bool) -> torch.Tensor:
        self.last_fallback = reason
        if self._fp64 is None:
            self._fp64 = GaussSolver(self.n, backend="hip", pivot=self.pivot, device=self.device)
        return self._fp64.solve(aug64, check=check)

    def _solve_mixed(self, aug: torch.Tensor, max_steps: int = 6, check: bool = False) -> torch.Tensor:
        """x of the augmented system: RBT + no-pivot LU, then x <- x + d
        until the componentwise backward error max_i |r_i| / (|b| + |A||x|)_i
        is <= 4 eps64 (or <= sqrt(n) eps64 once refinement stagnates), at most
        max_steps outer corrections (last_berr holds the final value), d =
        (LU)^-1 r with the fp64 factors; the residual is always fp64 on the
        ORIGINAL system.  A stall, a zero pivot or too many steps hand the
        system to the fp64 partial-pivoting engine (last_fallback says why;
        last_steps counts outer corrections)."""
        n, dev = self.n, self.device
        lib = _native.lib()
        aug64 = aug.to(dev, torch.float64)
        if aug64.shape[0] != n or aug64.shape[1] < n + 1 or aug64.stride(1) != 1:
            aug64 = aug64[:, :n + 1].contiguous()
        self.last_steps, self.last_fallback = 0, None
        if self._mixed is None:
            return self._fallback(aug64, self._mixed_unavailable or "no mixed plan", check)
        ld = aug64.stride(0)
        sh = stream_handle(dev)
        # the whole solve + classic refinement in native code (csrc/hip/
        # lu_mixed.hip gelim_mixed_solve: one 8-byte read-back per correction)
        import ctypes

        x = torch.empty(n, dtype=torch.float64, device=dev)
        st, be = ctypes.c_int(0), ctypes.c_double(0.0)
        rc = lib.gelim_mixed_solve(self._mixed, ptr(aug64), ld, ptr(x), max_steps, ctypes.byref(st),
                                   ctypes.byref(be), sh)
        _native.check(rc, "mixed_solve")
        self.last_steps, self.last_berr = st.value, be.value
        if rc == 1:
            return self._fallback(aug64, f"no-pivot LU: zero pivot or refinement stalled after {st.value} "
                                         f"corrections (componentwise backward error {be.value:.3e})", check)
        return x

    # -- GPU ---------------------------------------------------------------
    def _solve_gpu(self, aug: torch.Tensor, want_bnorm: bool):
        n = self.n
        if aug.device != self.device or aug.dtype != self.dtype:
            aug = aug.to(self.device, self.dtype)
        if aug.shape[0] != n or aug.shape[1] < n + 1 or aug.stride(1) != 1:
            raise ValueError(f"aug must be a row-major (n, >=n+1) tensor, got {tuple(aug.shape)}")
        x = torch.empty(n, dtype=torch.float64, device=self.device)
        bn = torch.empty(n, dtype=torch.float64, device=self.device) if want_bnorm else None
        rc = _native.lib().gelim_gauss_plan_solve(self._plan, ptr(aug), row_major_ld(aug), ptr(x), ptr(bn),
                                                  stream_handle(self.device))
        _native.check(rc, "gauss_plan_solve")
        return x, bn

    def info(self) -> int:
        """0 if the last solve was non-singular, else 1 + first zero-pivot column."""
        if self.backend in RBT_BACKENDS:
            return self._fp64.info() if (self.last_fallback and self._fp64 is not None) else 0
        if not self.gpu:
            return 0
        return _native.check(_native.lib().gelim_gauss_plan_info(self._plan, stream_handle(self.device)),
                             "plan_info")

    # -- CPU ---------------------------------------------------------------
    def _solve_cpu(self, aug: torch.Tensor, want_bnorm: bool):
        n = self.n
        A = aug[:, :n].to("cpu", torch.float64).contiguous().clone()
        b = aug[:, n].to("cpu", torch.float64).contiguous().clone()
        cpu_ops.cpu_gauss_(A, b, self.backend, self.pivot, self.threads, self.affinity)
        x = cpu_ops.cpu_backsub_unit(A, b)
        return x, (b if want_bnorm else None)

    def solve(self, aug: torch.Tensor, return_bnorm: bool = False, check: bool = False):
        """Solve the augmented system; returns x (and the reference's
        transformed b when return_bnorm).  check=True synchronises and raises
        SingularMatrixError on a zero pivot."""
        if self.backend in RBT_BACKENDS:
            if return_bnorm:
                raise ValueError(f"{self.backend} solves a transformed system: no reference-style B")
            return self._solve_mixed(aug, check=check)
        if self.gpu:
            x, bn = self._solve_gpu(aug, return_bnorm)
            if check and self.info() != 0:
                raise _native.SingularMatrixError(_native.E_SINGULAR,
                                                  f"The matrix is singular (column {self.info() - 1})")
        else:
            x, bn = self._solve_cpu(aug, return_bnorm)
        return (x, bn) if return_bnorm else x

    __call__ = solve

    def resolve(self, c: torch.Tensor) -> torch.Tensor:
        """hip-pivot only: solve A x = c with the factors of the LAST solve
        (O(n^2): permutation, lower and unit-upper triangular solves on the
        GPU; c fp64 on the device)."""
        if self.backend != "hip-pivot":
            raise ValueError("only the hip-pivot plan keeps its factors")
        c = c.to(self.device, torch.float64).contiguous()
        x = torch.empty(self.n, dtype=torch.float64, device=self.device)
        _native.check(_native.lib().gelim_gauss_plan_resolve(self._plan, ptr(c), ptr(x), stream_handle(self.device)),
                      "plan_resolve")
        return x

    def solve_refined(self, aug: torch.Tensor, max_steps: int = 5, tol: float | None = None,
                      check: bool = False):
        """Mixed-precision iterative refinement.

        The elimination runs ONCE in the solver's dtype (fp32 on `hip-pivot`,
        or fp64); the residual r = b - A x (native fp64 kernel) and the
        accumulated x are fp64.  Each step solves A d = r / s with the STORED
        factors (`resolve`, O(n^2): s = ||r||_inf keeps r inside fp32's
        exponent range) and adds s·d to x -- so the refinement costs one
        factorisation plus O(n^2) per step.  Backends whose plans keep no
        factors (the blocked LU) re-solve instead.  Stops after `max_steps`
        corrections, once ||s·d||_inf <= tol·||x||_inf (tol defaults to
        4·eps64), or when a correction fails to shrink ||r||_inf (refinement
        diverges once cond(A)·eps of the factor dtype reaches 1; x is then
        never worse than the plain solve).  Returns (x, accepted_steps).

        The reference has no refinement (its fp64 loops are one-shot,
        `OpenMP_and_MPI/gauss_openmp/gauss_external_input.c:150-200`); this is
        the path that lets the fp32 elimination reach fp64-level error on
        the `.dat` matrices.
        """
        if self.backend in RBT_BACKENDS:
            x = self._solve_mixed(aug, max_steps=max(max_steps, 1), check=check)
            return x, self.last_steps
        n = self.n
        dev = self.device
        aug64 = aug[:, :n + 1].to(dev, torch.float64).contiguous()
        work = aug[:, :n + 1].to(dev, self.dtype).contiguous()
        tol = 4 * torch.finfo(torch.float64).eps if tol is None else tol
        # the stored-factor re-solve is one workgroup with y and the row map
        # in LDS (12 bytes per row of 160 KiB); larger systems re-solve
        stored = self.gpu and self.backend == "hip-pivot" and n * 12 <= RESOLVE_LDS_BYTES

        def residual(xv: torch.Tensor) -> torch.Tensor:
            if self.gpu:
                r = torch.empty(n, dtype=torch.float64, device=dev)
                _native.check(_native.lib().gelim_gpu_residual(ptr(aug64), aug64.stride(0), n, ptr(xv), ptr(r),
                                                               stream_handle(dev)), "residual")
                return r
            return aug64[:, n] - aug64[:, :n] @ xv

        def correction(rs: torch.Tensor) -> torch.Tensor:
            if stored:
                return self.resolve(rs)
            work[:, n] = rs.to(self.dtype)
            return self.solve(work, check=check).to(torch.float64)

        x = self.solve(work, check=check).to(torch.float64)
        r = residual(x)
        s = float(r.abs().max())
        steps = 0
        while steps < max_steps and s > 0.0 and s == s:
            d = correction(r / s) * s
            xn = x + d
            rn = residual(xn)
            sn = float(rn.abs().max())
            if not sn < s:  # diverging (cond(A)·eps of the factor dtype >= 1): keep the better x
                break
            x, r, s = xn, rn, sn
            steps += 1
            if float(d.abs().max()) <= tol * float(x.abs().max()):
                break
        return x, steps

    def close(self) -> None:
        if self._plan:
            _native.lib().gelim_gauss_plan_destroy(self._plan)
            self._plan = None
        if self._mixed:
            _native.lib().gelim_mixed_plan_destroy(self._mixed)
            self._mixed = None
        if self._fp64 is not None:
            self._fp64.close()
            self._fp64 = None

    def __del__(self):
        # never tear down HIP objects during interpreter shutdown (the HIP
        # runtime may already be gone); explicit close() is the normal path
        if _sys is None or _sys.is_finalizing():
            return
        try:
            self.close()
        except Exception:
            pass

    def __repr__(self):
        return f"GaussSolver(n={self.n}, backend={self.backend!r}, pivot={self.pivot!r}, dtype={self.dtype})"


def solve(aug: torch.Tensor, backend: str | None = None, pivot: str = "partial", **kw) -> torch.Tensor:
    """One-shot solve of an augmented system (backend defaults to the GPU
    blocked LU for CUDA tensors, the sequential reference loop otherwise)."""
    if backend is None:
        backend = "hip" if aug.device.type == "cuda" else "seq"
    s = GaussSolver(aug.shape[0], backend=backend, pivot=pivot,
                    device=aug.device if aug.device.type == "cuda" else None, **kw)
    try:
        return s.solve(aug, check=True)
    finally:
        s.close()


def blocked_solve_(aug: torch.Tensor, pivot: str = "partial", width: int | None = None) -> torch.Tensor:
    """The blocked LU of `plan.hip`, composed from `ops.lu` building blocks
    (works on CPU and GPU tensors; used by tests and the distributed driver).
    Destroys `aug`; returns x."""
    n = aug.shape[0]
    piv = torch.zeros(n + 64, dtype=torch.int32, device=aug.device)
    info = torch.zeros(4, dtype=torch.int32, device=aug.device)
    k = 0
    while k < n:
        m = n - k
        w = width or _default_width(m)
        w = min(w, m)
        lu.panel_factor(aug[k:, k:k + w], piv[k:k + w], info, row0=k, pivot=pivot)
        lu.swap_trsm(aug[k:, k + w:n + 1], aug[k:k + w, k:k + w], piv[k:k + w])
        if m > w:
            lu.gemm_update(aug[k + w:, k + w:n + 1], aug[k + w:, k:k + w], aug[k:k + w, k + w:n + 1])
        k += w
    if int(info[0].item()) != 0:
        raise _native.SingularMatrixError(_native.E_SINGULAR, "The matrix is singular")
    return lu.backsub(aug[:, :n], aug[:, n])


def _default_width(m: int) -> int:
    for w, rows in ((16, 2048), (8, 4096), (4, 8192), (2, 16384)):
        if m <= rows:
            return w
    raise ValueError("panel too tall")
