"""GPU building blocks vs their CPU/fp64 references (numerics of each HIP
kernel against a plain reference of the same op)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("m,w", [(5, 2), (40, 8), (1000, 16), (1024, 16), (1500, 16), (2048, 16),
                                 (3000, 8), (4096, 8), (5000, 4), (8192, 4), (9000, 2)])
def test_panel_factor_matches_cpu(gelim, cuda, m, w):
    torch.manual_seed(m + w)
    P = torch.randn(m, w + 3, dtype=torch.float64)  # padded row pitch
    Pc = P.clone()
    Pg = P.to(cuda)
    piv_c = torch.zeros(w, dtype=torch.int32)
    piv_g = torch.zeros(w, dtype=torch.int32, device=cuda)
    info_c = torch.zeros(4, dtype=torch.int32)
    info_g = torch.zeros(4, dtype=torch.int32, device=cuda)
    gelim.ops.lu.panel_factor(Pc[:, :w], piv_c, info_c)
    gelim.ops.lu.panel_factor(Pg[:, :w], piv_g, info_g)
    torch.cuda.synchronize()
    assert torch.equal(piv_g.cpu(), piv_c)
    assert torch.allclose(Pg.cpu()[:, :w], Pc[:, :w], rtol=1e-11, atol=1e-11)
    assert torch.equal(Pg.cpu()[:, w:], P[:, w:])  # columns outside untouched
    # and against LAPACK
    lu_, ipiv = torch.linalg.lu_factor(P[:, :w])
    assert torch.equal(piv_c.long() + 1, ipiv.long())


def test_panel_factor_ties_and_zero_rule(gelim, cuda):
    # ties -> lowest row (reference strict '>')
    P = torch.tensor([[1.0, 2.0], [-3.0, 1.0], [3.0, 5.0], [2.0, 0.0]], dtype=torch.float64)
    piv = torch.zeros(2, dtype=torch.int32, device=cuda)
    info = torch.zeros(4, dtype=torch.int32, device=cuda)
    Pg = P.to(cuda)
    gelim.ops.lu.panel_factor(Pg, piv, info, pivot="partial")
    assert piv.cpu().tolist()[0] == 1
    # ZERO rule: non-zero diagonal stays
    Pg = P.to(cuda)
    gelim.ops.lu.panel_factor(Pg, piv, info, pivot="zero")
    assert piv.cpu().tolist()[0] == 0
    # zero column -> info
    Z = torch.zeros(6, 2, dtype=torch.float64, device=cuda)
    info.zero_()
    gelim.ops.lu.panel_factor(Z, piv, info, row0=10)
    assert info.cpu()[0].item() == 11


@pytest.mark.parametrize("w", [2, 4, 8, 16])
@pytest.mark.parametrize("ncols", [1, 77, 300])
def test_swap_trsm_matches_cpu(gelim, cuda, w, ncols):
    torch.manual_seed(w * 1000 + ncols)
    m = 3 * w + 5
    C = torch.randn(m, ncols + 2, dtype=torch.float64)
    L = torch.randn(w, w, dtype=torch.float64)
    # sequential-interchange pivots with repeats and in-panel targets
    piv = torch.tensor([min(m - 1, j + (j * 7) % (m - j)) for j in range(w)], dtype=torch.int32)
    piv[w // 2] = piv[0] if piv[0] >= w // 2 else piv[w // 2]
    Cc = C.clone()
    gelim.ops.lu.swap_trsm(Cc[:, :ncols], L, piv)
    Cg = C.to(cuda)
    gelim.ops.lu.swap_trsm(Cg[:, :ncols], L.to(cuda), piv.to(cuda))
    torch.cuda.synchronize()
    assert torch.allclose(Cg.cpu(), Cc, rtol=1e-12, atol=1e-12)


@pytest.mark.parametrize("M,N,K", [(1, 1, 1), (64, 64, 4), (100, 37, 16), (513, 1025, 32), (7, 300, 3),
                                   (2000, 1, 64)])
def test_gemm_update_f64_mfma(gelim, cuda, M, N, K):
    torch.manual_seed(M + N + K)
    C = torch.randn(M, N + 5, dtype=torch.float64, device=cuda)
    L = torch.randn(M, K, dtype=torch.float64, device=cuda)
    U = torch.randn(K, N, dtype=torch.float64, device=cuda)
    ref = C[:, :N] - L @ U
    C0 = C.clone()
    gelim.ops.lu.gemm_update(C[:, :N], L, U)
    torch.cuda.synchronize()
    assert torch.allclose(C[:, :N], ref, rtol=1e-12, atol=1e-12)
    assert torch.equal(C[:, N:], C0[:, N:])


def test_gemm_update_asymmetric_exact(gelim, cuda):
    # integer-valued asymmetric operands: exact result, catches a transposed C/D map
    M, N, K = 48, 40, 12
    L = torch.arange(M * K, dtype=torch.float64, device=cuda).view(M, K) % 7
    U = (torch.arange(K * N, dtype=torch.float64, device=cuda).view(K, N) * 3) % 11
    C = torch.zeros(M, N, dtype=torch.float64, device=cuda)
    gelim.ops.lu.gemm_update(C, L, U)
    assert torch.equal(C, -(L @ U))


@pytest.mark.parametrize("n", [1, 5, 64, 65, 300, 2048])
@pytest.mark.parametrize("unit", [False, True])
def test_backsub(gelim, cuda, n, unit):
    torch.manual_seed(n)
    U = torch.triu(torch.randn(n, n, dtype=torch.float64)) + 4 * torch.eye(n, dtype=torch.float64)
    if unit:
        U.fill_diagonal_(1.0)
    y = torch.randn(n, dtype=torch.float64)
    ref = torch.linalg.solve_triangular(U, y[:, None], upper=True, unitriangular=unit)[:, 0]
    x = gelim.ops.lu.backsub(U.to(cuda), y.to(cuda), unit=unit)
    torch.cuda.synchronize()
    assert torch.allclose(x.cpu(), ref, rtol=1e-10, atol=1e-10)


@pytest.mark.parametrize("n", [130, 4200, 8192])
def test_backsub_block_inverse_form(gelim, cuda, n, monkeypatch):
    """The persistent back substitution (backsub.hip, round 5) reads only the
    upper triangle of a full matrix (LU storage: multipliers below), inverts
    its 64 x 64 diagonal blocks and chains x_b = v - W x_{b+1}; it must agree
    with torch's triangular solve and with the one-launch-per-block fallback
    (forced with GELIM_FORCE_NONPERSISTENT=1) to fp64 rounding."""
    g = torch.Generator(device=cuda).manual_seed(n)
    A = torch.randn(n, n, dtype=torch.float64, device=cuda, generator=g)
    A += (2.0 + torch.rand(n, dtype=torch.float64, device=cuda, generator=g)).diag() * n ** 0.5
    y = torch.randn(n, dtype=torch.float64, device=cuda, generator=g)
    ref = torch.linalg.solve_triangular(torch.triu(A), y[:, None], upper=True)[:, 0]
    x = gelim.ops.lu.backsub(A, y)
    torch.cuda.synchronize()
    scale = ref.abs().max().item()
    assert (x - ref).abs().max().item() <= 1e-12 * scale
    monkeypatch.setenv("GELIM_FORCE_NONPERSISTENT", "1")
    x2 = gelim.ops.lu.backsub(A, y)
    torch.cuda.synchronize()
    assert (x - x2).abs().max().item() <= 1e-12 * scale


def test_device_random_matches_host(gelim, cuda):
    h = gelim.random_system(130, seed=42)
    d = gelim.random_system(130, seed=42, device=cuda)
    assert torch.equal(d.cpu()[:, :130], h[:, :130])
    assert torch.allclose(d.cpu()[:, 130], h[:, 130], rtol=1e-12)
    s = gelim.synthetic_system(50, device=cuda)
    assert torch.equal(s.cpu(), gelim.synthetic_system(50))


@pytest.mark.parametrize("m,w", [(40, 8), (1000, 16), (2048, 16)])
def test_panel_zero_rule_positions(gelim, cuda, m, w):
    """ZERO rule in the register panel: after step 0 moves row 0 to position 5,
    step 1's zero diagonal must be replaced by the first non-zero row in
    POSITION order (row 3), not the lowest physical row (row 0) -- the same
    interchanges as the CPU panel (physical swaps, the reference's loop)."""
    torch.manual_seed(m)
    P = torch.rand(m, w, dtype=torch.float64) + 0.5
    P[:, 0] = 0.0
    P[5, 0] = 1.0
    P[:, 1] = 0.0
    P[3, 1] = 2.0
    P[0, 1] = 7.0
    Pc, Pg = P.clone(), P.to(cuda)
    piv_c = torch.zeros(w, dtype=torch.int32)
    piv_g = torch.zeros(w, dtype=torch.int32, device=cuda)
    info_c = torch.zeros(4, dtype=torch.int32)
    info_g = torch.zeros(4, dtype=torch.int32, device=cuda)
    gelim.ops.lu.panel_factor(Pc, piv_c, info_c, pivot="zero")
    gelim.ops.lu.panel_factor(Pg, piv_g, info_g, pivot="zero")
    torch.cuda.synchronize()
    assert piv_c.tolist()[:2] == [5, 3]
    assert torch.equal(piv_g.cpu(), piv_c)
    assert torch.allclose(Pg.cpu(), Pc, rtol=1e-11, atol=1e-11)
