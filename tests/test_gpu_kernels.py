"""-m gpu: the dense fp64 kernels against a NumPy fp64 reference of the same op.

Tolerances: fp64 sums of k products in a different order -> |err| <= 64 eps * sum|a*b|.
"""
import numpy as np
import pytest

from gpu_util import colmajor_lower, dev, handle, host, potrf, potrs, syrk

pytestmark = pytest.mark.gpu
EPS = np.finfo(np.float64).eps


@pytest.mark.parametrize("k,n", [(4, 16), (1, 1), (16, 128), (37, 130), (300, 257), (512, 1024), (0, 5),
                                 (2050, 700), (64, 1000), (2048, 8192), (2050, 8100), (600, 10000),
                                 (4608, 4096), (1024, 4096), (520, 4096), (300, 4096)])
def test_syrk_weighted_matches_numpy(k, n):
    """Includes grids whose tail runs as split K halves (k_mfma_gemm_split: n = 1000 and 1024 on
    64-tiles -- every tile split, ragged edge tiles included) and as stream-K pieces
    (k_mfma_gemm_streamk on 128-tiles, default IPM_STREAMK=2, pieces last: n = 8192, K = 2048 -> 32
    tail tiles x 16 pieces; n = 8100, K = 2050 -> ragged edge tiles and 15 pieces, the run-time
    piece count of the fixup; n = 10000, K = 600 -> 3160 tiles, 88 tail tiles: too many for the 256
    partial slots, so the K-halves split runs).  n = 4096 (528 tiles on 512 slots, config 5's grid):
    K = 4608 / 1024 -> 16 pieces, K = 520 -> 7 (run-time count), K = 300 -> 4: each compile-time
    piece count of the fixup and the fallback."""
    rng = np.random.default_rng(k * 1000 + n)
    X = rng.uniform(-2, 2, (k, n))
    w = rng.uniform(0.1, 3, k)
    H = syrk(X, w, n)
    ref = X.T @ (w[:, None] * X)
    bound = 64 * EPS * (np.abs(X).T @ (w[:, None] * np.abs(X))) + 1e-300
    got = colmajor_lower(H, n)
    assert np.all(np.abs(np.tril(got - ref)) <= np.tril(bound) + 1e-14 * (k == 0))


def test_syrk_fragment_layout_asymmetric():
    """A = I-style check with an asymmetric operand (cdna_hip_programming.md §3 warning)."""
    n, k = 64, 64
    X = np.zeros((k, n))
    for i in range(k):
        X[i, i] = 1.0
    X[3, 17] = 5.0   # makes H[3][17] = H[17][3] = 5 and H[17][17] = 26
    H = colmajor_lower(syrk(X, None, n), n)
    ref = np.tril(X.T @ X)
    np.testing.assert_array_equal(H, ref)


def test_syrk_odd_ld_and_beta():
    rng = np.random.default_rng(3)
    n, k, ldh = 75, 33, 79
    X = rng.normal(size=(k, n))
    H0 = rng.normal(size=(n, ldh))
    H = syrk(X, None, n, ldh=ldh, beta=1.0, H0=H0, alpha=-1.0)
    M0 = H0.T[:n, :n]
    ref = np.tril(M0 - X.T @ X)
    got = colmajor_lower(H, n)
    np.testing.assert_allclose(got, ref, rtol=0, atol=1e-12 * (1 + np.abs(X).max() ** 2 * k))


@pytest.mark.parametrize("ncols,extra", [(128, 1), (129, 1), (200, 1), (200, 70), (255, 1), (256, 1), (257, 1),
                                         (300, 1), (320, 64), (1000, 1), (2049, 1), (2048, 130)])
def test_potrf_partial_bordered(ncols, extra):
    """The bordered factorization of the Newton step: the first ncols columns are factored and
    the rows below them (e.g. the -g row) get L21 = A21 L11^-T -- every block-size remainder,
    including a next-panel diagonal block that ends inside a row chunk."""
    n = ncols + extra
    rng = np.random.default_rng(ncols * 7 + extra)
    M = rng.normal(size=(n + 5, n))
    A = M.T @ M + n * np.eye(n)
    Hm = dev(A.T.copy())
    rc, info = potrf(Hm, n, n, ncols=ncols)
    assert rc == 0 and info == 0
    got = host(Hm).T                       # row-major view of the column-major buffer
    L11 = np.linalg.cholesky(A[:ncols, :ncols])
    L21 = np.linalg.solve(L11, A[ncols:, :ncols].T).T
    np.testing.assert_allclose(np.tril(got[:ncols, :ncols]), L11, rtol=1e-10, atol=1e-10 * np.abs(L11).max())
    np.testing.assert_allclose(got[ncols:, :ncols], L21, rtol=1e-10, atol=1e-10 * np.abs(L21).max())


@pytest.mark.parametrize("n", [1, 7, 64, 65, 200, 300, 513, 640, 1030, 2100])
def test_potrf_potrs_match_numpy(n):
    rng = np.random.default_rng(n)
    M = rng.normal(size=(n + 5, n))
    A = M.T @ M + n * np.eye(n)
    Hm = dev(A.T.copy())  # column-major A == row-major A^T (symmetric anyway)
    rc, info = potrf(Hm, n, n)
    assert rc == 0 and info == 0
    L = colmajor_lower(Hm, n)
    Lr = np.linalg.cholesky(A)
    np.testing.assert_allclose(L, Lr, rtol=1e-10, atol=1e-10 * np.abs(Lr).max())
    b = rng.normal(size=(n, 3))
    x = potrs(Hm, n, n, b.copy())
    np.testing.assert_allclose(x, np.linalg.solve(A, b), rtol=1e-9, atol=1e-12)


# the failing column in the first panel, in a later block's first and second panels (the
# failure must stop every later launch and come back as LAPACK's info)
@pytest.mark.parametrize("n,bad", [(150, 97), (1030, 300), (1030, 450), (1030, 1029)])
def test_potrf_reports_lapack_info(n, bad):
    rng = np.random.default_rng(0)
    M = rng.normal(size=(n, n))
    A = M @ M.T + np.eye(n)
    A[bad, bad] = -1e6 * n   # leading minor bad+1 is not PD
    Hm = dev(A)
    rc, info = potrf(Hm, n, n)
    assert rc == 1
    import scipy.linalg
    with pytest.raises(np.linalg.LinAlgError) as e:
        scipy.linalg.cho_factor(A)
    assert f"{info}-th leading minor" in str(e.value)


@pytest.mark.parametrize("n", [1, 5, 64, 65, 127, 128, 200, 1000, 2049])
def test_potrs_single_rhs_persistent_solve(n):
    """nrhs = 1 runs the persistent ticketed solve kernels (k_trsv_chain); partial last block,
    one block, many blocks."""
    rng = np.random.default_rng(n + 17)
    M = rng.normal(size=(n + 3, n))
    A = M.T @ M + n * np.eye(n)
    Hm = dev(A)
    rc, info = potrf(Hm, n, n)
    assert rc == 0 and info == 0
    b = rng.normal(size=n)
    x = potrs(Hm, n, n, b.copy()).ravel()
    ref = np.linalg.solve(A, b)
    np.testing.assert_allclose(x, ref, rtol=1e-10, atol=1e-12 * np.abs(ref).max())
    # repeated calls reuse the control words (reset per call)
    x2 = potrs(Hm, n, n, b.copy()).ravel()
    np.testing.assert_array_equal(x, x2)


@pytest.mark.parametrize("n,ncols", [(8194, 8193), (1030, 1030), (2690, 2689)])
def test_potrf_ragged_rows(n, ncols, monkeypatch):
    """The 1-8 trailing rows past a multiple of 128 (the bordered Newton system) are updated by
    row workgroups (IPM_RAG=1; the default above 5120 rows) instead of a row of 128-tiles: same factor to fp64 rounding
    as the tile path, and torch's Cholesky / triangular solve to 1e-10."""
    import torch
    from gpu_util import potrf as P
    g = torch.Generator(device="cuda").manual_seed(n)
    M = torch.rand((n + 5, n), dtype=torch.float64, device="cuda", generator=g) - 0.5
    A = M.T @ M + n * torch.eye(n, dtype=torch.float64, device="cuda")
    out = {}
    for mode in ("0", "1"):
        monkeypatch.setenv("IPM_RAG", mode)
        H = A.clone()   # symmetric: the column-major buffer is A itself
        rc, info = P(H, n, n, ncols=ncols)
        assert rc == 0 and info == 0
        out[mode] = torch.tril(H.T)[:, :ncols]
    scale = out["0"].abs().max()
    assert ((out["1"] - out["0"]).abs().max() / scale).item() < 1e-12
    L11 = torch.linalg.cholesky(A[:ncols, :ncols])
    got = out["1"]
    assert ((got[:ncols] - L11).abs().max() / L11.abs().max()).item() < 1e-10
    if ncols < n:
        L21 = torch.linalg.solve_triangular(L11, A[ncols:, :ncols].T, upper=False).T
        assert ((got[ncols:] - L21).abs().max() / L21.abs().max()).item() < 1e-10


@pytest.mark.parametrize("n,ncols", [(8194, 8193), (2050, 2049), (266, 264), (272, 264), (520, 520)])
def test_potrf_tail_block(n, ncols, monkeypatch):
    """A last block of <= 8 columns with <= 16 rows from its origin (the bordered phase-1 system:
    1 column + the right-hand-side row) is finished by a tail workgroup inside the launch before it
    (IPM_TAIL, default on) instead of a launch of its own: the factor agrees with the own-launch
    path to fp64 rounding and with torch's Cholesky / triangular solve to 1e-10; a non-positive
    pivot in the tail columns reports its 1-based column like the diagonal role."""
    import torch
    from gpu_util import potrf as P
    g = torch.Generator(device="cuda").manual_seed(n + 7)
    M = torch.rand((n + 5, n), dtype=torch.float64, device="cuda", generator=g) - 0.5
    A = M.T @ M + n * torch.eye(n, dtype=torch.float64, device="cuda")
    out = {}
    for mode in ("0", "1"):
        monkeypatch.setenv("IPM_TAIL", mode)
        H = A.clone()
        rc, info = P(H, n, n, ncols=ncols)
        assert rc == 0 and info == 0
        out[mode] = torch.tril(H.T)[:, :ncols]
    scale = out["0"].abs().max()
    assert ((out["1"] - out["0"]).abs().max() / scale).item() < 1e-12
    L11 = torch.linalg.cholesky(A[:ncols, :ncols])
    assert ((out["1"][:ncols] - L11).abs().max() / L11.abs().max()).item() < 1e-10
    if ncols < n:
        L21 = torch.linalg.solve_triangular(L11, A[ncols:, :ncols].T, upper=False).T
        assert ((out["1"][ncols:] - L21).abs().max() / L21.abs().max()).item() < 1e-10
    # the last factored column made indefinite: info = ncols with and without the tail
    B = A.clone()
    B[ncols - 1, ncols - 1] = -1.0
    for mode in ("0", "1"):
        monkeypatch.setenv("IPM_TAIL", mode)
        H = B.clone()
        rc, info = P(H, n, n, ncols=ncols)
        assert rc == 1 and info == ncols, (mode, rc, info)


@pytest.mark.parametrize("n,ncols", [(8194, 8193), (4100, 4100)])
def test_potrf_split_trailing_tiles(n, ncols, monkeypatch):
    """Trailing tiles of a launch's last round split in two K halves (IPM_SPLIT, default on; the
    upper half's partial tile handed over through the workspace), on the C-burst tile loop
    (IPM_LAZYC=0: the default keeps lazy-eligible launches whole), the lazy-C loop for K = 256
    tiles only (IPM_LAZYC=1), and the library default (IPM_LAZYC unset: K = 512 pair tiles lazy
    too): the factors agree with the unsplit one to fp64 rounding and with
    torch's Cholesky to 1e-10."""
    import torch
    from gpu_util import potrf as P
    g = torch.Generator(device="cuda").manual_seed(n + 1)
    M = torch.rand((n + 5, n), dtype=torch.float64, device="cuda", generator=g) - 0.5
    A = M.T @ M + n * torch.eye(n, dtype=torch.float64, device="cuda")
    out = {}
    for mode, lazy in (("0", "0"), ("1", "0"), ("1", "1"), ("1", "default")):
        monkeypatch.setenv("IPM_SPLIT", mode)
        if lazy == "default":
            monkeypatch.delenv("IPM_LAZYC", raising=False)
        else:
            monkeypatch.setenv("IPM_LAZYC", lazy)
        H = A.clone()
        rc, info = P(H, n, n, ncols=ncols)
        assert rc == 0 and info == 0
        out[mode + lazy] = torch.tril(H.T)[:, :ncols]
    scale = out["00"].abs().max()
    L11 = torch.linalg.cholesky(A[:ncols, :ncols])
    for k in ("10", "11", "1default"):
        d = ((out[k] - out["00"]).abs().max() / scale).item()
        print(f"n={n}: split {k[0]} lazy {k[1]} vs unsplit max rel {d:.2e}")
        assert d < 1e-12
        assert ((out[k][:ncols] - L11).abs().max() / L11.abs().max()).item() < 1e-10


@pytest.mark.parametrize("n", [1, 7, 64, 65, 200, 1030, 2100])
def test_getrf_getrs_match_numpy(n):
    """Blocked LU with partial pivoting (64-column panels, MFMA trailing update) vs np.linalg.solve;
    the pivots are LAPACK's (first index of the largest |a|) -- identical to scipy's getrf."""
    import ctypes
    import scipy.linalg
    import torch
    from gpu_util import handle
    from ipm355 import _lib as L
    h = handle()
    rng = np.random.default_rng(n)
    A = rng.normal(size=(n, n))
    Ad = torch.as_tensor(A.T.copy(), device="cuda")        # column-major
    piv = torch.empty(n, dtype=torch.int64, device="cuda")
    info = ctypes.c_int(0)
    assert h.lib.ipm_getrf(h.ptr, n, L.dptr(Ad), n, L.dptr(piv), ctypes.byref(info)) == 0
    lu_ref, piv_ref = scipy.linalg.lu_factor(A)
    np.testing.assert_array_equal(piv.cpu().numpy(), piv_ref)
    LU = Ad.cpu().numpy().T
    np.testing.assert_allclose(LU, lu_ref, rtol=1e-9, atol=1e-9 * np.abs(lu_ref).max())
    b = rng.normal(size=(n, 2))
    Bd = torch.as_tensor(b.copy(), device="cuda")
    assert h.lib.ipm_getrs(h.ptr, n, 2, L.dptr(Ad), n, L.dptr(piv), L.dptr(Bd), 2) == 0
    ref = np.linalg.solve(A, b)
    np.testing.assert_allclose(Bd.cpu().numpy(), ref, rtol=1e-8, atol=1e-10 * np.abs(ref).max())


@pytest.mark.parametrize("n,rank,nrhs,indef", [(50, 50, 1, False), (200, 120, 3, False), (300, 90, 1, True),
                                               (301, 90, 1, False), (1024, 700, 1, False), (1025, 1025, 1, False),
                                               (1025, 700, 2, False), (257, 257, 1, False),
                                               (1000, 1000, 16, True), (2048, 1500, 64, False)])
def test_lstsq_sym_matches_numpy(n, rank, nrhs, indef):
    """Minimum-norm least squares (ipm_lstsq_sym: eigenvectors, gelsd's rcond = eps*n cut) vs
    np.linalg.lstsq(H, B, rcond=None) -- the np_lstsq method and the Cholesky-failure backup
    (NewtonSolver.py:212-227, 334-341).  Rank-deficient H (PSD, or indefinite) is where it differs
    from an LU solve; B row-major n x nrhs.  n <= 256: the one-workgroup Jacobi; above, the blocked
    Jacobi (32-index blocks, odd block counts padded: n = 257, 301, 1025); nrhs >= 8 applies the
    pseudo-inverse through the MFMA GEMM."""
    import ctypes
    import torch
    from gpu_util import handle
    from ipm355 import _lib as L
    h = handle()
    rng = np.random.default_rng(n + rank)
    G = rng.normal(size=(rank, n))
    D = rng.uniform(0.5, 3.0, rank) * (np.where(rng.random(rank) < 0.5, -1.0, 1.0) if indef else 1.0)
    H = G.T @ (D[:, None] * G)
    H = 0.5 * (H + H.T)
    B = rng.normal(size=(n, nrhs))
    ref = np.linalg.lstsq(H, B, rcond=None)[0]
    Ad = torch.as_tensor(H.copy(), device="cuda")              # symmetric: either layout
    Bd = torch.as_tensor(B.copy(), device="cuda")
    info = ctypes.c_int(-1)
    assert h.lib.ipm_lstsq_sym(h.ptr, n, nrhs, L.dptr(Ad), n, L.dptr(Bd), nrhs, ctypes.byref(info)) == 0
    assert info.value == 0
    X = Bd.cpu().numpy()
    # same minimum-norm vector: the error is the conditioning of the kept part times eps
    err = np.linalg.norm(X - ref) / np.linalg.norm(ref)
    print(f"[lstsq n={n} rank={rank}] rel {err:.1e}")
    assert err <= 1e-8, err
    if rank < n:
        # no component in the null space of H (an LU solve of a singular H has no such property)
        _, V = np.linalg.eigh(H)
        null = V[:, :n - rank] if not indef else V[:, np.argsort(np.abs(np.linalg.eigvalsh(H)))[:n - rank]]
        assert np.linalg.norm(null.T @ X) <= 1e-8 * np.linalg.norm(X)


@pytest.mark.parametrize("n,nrhs", [(130, 40), (1030, 300), (2100, 64), (4097, 4097)])
def test_potrs_many_rhs_blocked(n, nrhs):
    """L L^T X = B with many right-hand sides (128-row blocks on MFMA GEMMs, the Lasso's Q = M^-1)
    against torch's Cholesky solve."""
    import torch
    from gpu_util import potrf as P
    from gpu_util import handle
    from ipm355 import _lib as L
    g = torch.Generator(device="cuda").manual_seed(n)
    M = torch.rand((n + 5, n), dtype=torch.float64, device="cuda", generator=g) - 0.5
    A = M.T @ M + n * torch.eye(n, dtype=torch.float64, device="cuda")
    H = A.clone()
    rc, info = P(H, n, n)
    assert rc == 0 and info == 0
    B = torch.rand((n, nrhs), dtype=torch.float64, device="cuda", generator=g) - 0.5
    X = B.clone()
    h = handle()
    assert h.lib.ipm_potrs(h.ptr, n, nrhs, L.dptr(H), n, L.dptr(X), nrhs) == 0
    ref = torch.cholesky_solve(B, torch.linalg.cholesky(A))
    err = ((X - ref).abs().max() / ref.abs().max()).item()
    print(f"n={n} nrhs={nrhs}: max rel {err:.2e}")
    assert err < 1e-10


def test_trsv_backward_solve_fails_loudly():
    """The persistent backward solve (k_trsv_bwd128) polls x_{B+1} with a bounded spin.  With the
    bound shrunk to 1 us and chain ticket 1 storing its x block ~7 ms late (debug knobs), ticket 2's
    poll runs out on every solve: the device error word must surface as IPMBackendError, never as a
    silently wrong step.  (The bound alone is checked every 16 polls, so without
    the late store a run may finish without tripping it.)"""
    from ipm355 import _lib as L
    h = handle()
    n = 8192
    rng = np.random.default_rng(5)
    M = rng.normal(size=(n + 8, n)) * 2.0 ** -4
    A = M.T @ M + n * np.eye(n)
    Hm = dev(A)
    rc, info = potrf(Hm, n, n)
    assert rc == 0 and info == 0
    b = rng.normal(size=n)
    ref = np.linalg.solve(A, b)
    tripped = 0
    try:
        h.lib.ipm_debug_set_trsv_spin_limit(1)
        h.lib.ipm_debug_set_trsv_publish_delay(-2 - 1)
        for _ in range(4):
            try:
                potrs(Hm, n, n, b.copy())
            except L.IPMBackendError as e:
                assert "spin bound" in str(e)
                tripped += 1
    finally:
        h.lib.ipm_debug_set_trsv_publish_delay(-1)
        h.lib.ipm_debug_set_trsv_spin_limit(0)
    assert tripped == 4
    x = potrs(Hm, n, n, b.copy()).ravel()    # default bound again: correct, and no sticky error left
    np.testing.assert_allclose(x, ref, rtol=1e-10, atol=1e-12 * np.abs(ref).max())


@pytest.mark.parametrize("ticket", [0, 1, 5])
def test_trsv_backward_solve_late_publisher(ticket):
    """A backward-solve workgroup that publishes its progress word late (debug knob: ~7 ms sleep
    before the store) is overtaken by the next tickets, which read its x block straight from y.
    The progress word is published with an atomic max, so it never moves backwards and the
    waiting workgroups still drain.  Result identical to the undelayed solve."""
    h = handle()
    n = 4096
    rng = np.random.default_rng(11)
    M = rng.normal(size=(n + 8, n)) * 2.0 ** -4
    A = M.T @ M + n * np.eye(n)
    Hm = dev(A)
    rc, info = potrf(Hm, n, n)
    assert rc == 0 and info == 0
    b = rng.normal(size=n)
    x0 = potrs(Hm, n, n, b.copy()).ravel()
    try:
        h.lib.ipm_debug_set_trsv_publish_delay(ticket)
        x1 = potrs(Hm, n, n, b.copy()).ravel()
    finally:
        h.lib.ipm_debug_set_trsv_publish_delay(-1)
    np.testing.assert_array_equal(x0, x1)


def test_potrf_wait_bound_fails_loudly():
    """every wait inside the ticketed Cholesky (k_potrf_block) has a wall-clock bound.
    Shrunk to 1 us (debug knob) the waits run out: ipm_potrf must report IPM_HIP_ERROR with
    info = -1000 (never a LAPACK column, never a silently wrong factor), the failure must drain
    every later launch (the call returns), and with the default bound the same matrix factors
    correctly again (nothing sticky left in the workspace)."""
    from ipm355 import _lib as L
    h = handle()
    n = 4096
    rng = np.random.default_rng(17)
    M = rng.normal(size=(n + 8, n)) * 2.0 ** -4
    A = M.T @ M + n * np.eye(n)
    tripped = 0
    try:
        h.lib.ipm_debug_set_potrf_spin_limit(1)
        for _ in range(3):
            rc, info = potrf(dev(A), n, n)
            if rc == L.IPM_HIP_ERROR:
                assert info == -1000, info
                tripped += 1
            else:
                assert rc == 0 and info == 0, (rc, info)
    finally:
        h.lib.ipm_debug_set_potrf_spin_limit(0)
    assert tripped >= 1
    Hm = dev(A)
    rc, info = potrf(Hm, n, n)
    assert rc == 0 and info == 0
    got = np.tril(host(Hm).T)
    ref = np.linalg.cholesky(A)
    np.testing.assert_allclose(got, ref, rtol=1e-10, atol=1e-10 * np.abs(ref).max())


@pytest.mark.parametrize("n,ncols", [(130, 129), (200, 200), (1030, 1030), (2049, 2048), (4097, 4096), (8193, 8192)])
def test_potrf_partial_and_bordered(n, ncols):
    """The fused Cholesky on full and partial last panels and on the bordered Newton layout
    (ncols = n - 1): the factor against NumPy's, the rows below it against L21 = A21 L11^-T."""
    rng = np.random.default_rng(n + 3 * ncols)
    M = rng.normal(size=(n + 5, n))
    A = M.T @ M + n * np.eye(n)
    Hm = dev(A.T.copy())
    rc, info = potrf(Hm, n, n, ncols=ncols)
    assert rc == 0 and info == 0
    got = host(Hm).T
    L11 = np.linalg.cholesky(A[:ncols, :ncols])
    np.testing.assert_allclose(np.tril(got[:ncols, :ncols]), L11, rtol=1e-10, atol=1e-10 * np.abs(L11).max())
    if ncols < n:
        L21 = np.linalg.solve(L11, A[ncols:, :ncols].T).T
        np.testing.assert_allclose(got[ncols:, :ncols], L21, rtol=1e-10, atol=1e-10 * np.abs(L21).max())


def test_potrf_not_pd_info_matches_lapack():
    """A non-positive pivot inside a diagonal role: LAPACK's info (first failing column, 1-based),
    and the factorization ends (every later launch sees the failure word)."""
    import scipy.linalg
    n = 1030
    rng = np.random.default_rng(21)
    M = rng.normal(size=(n + 5, n))
    A = M.T @ M + n * np.eye(n)
    k = 300                      # make the leading (k+1) x (k+1) minor indefinite
    A[k, k] = -abs(A[k, k])
    rc, info = potrf(dev(A.T.copy()), n, n)
    try:
        scipy.linalg.cholesky(A, lower=True)
        ref = 0
    except np.linalg.LinAlgError as e:
        ref = int(str(e).split("-th")[0].split()[-1])
    assert info == ref == k + 1, (info, ref)
    assert rc != 0


@pytest.mark.parametrize("n,ncols,lda", [(2049, 2048, 2050), (4097, 4096, 4098), (1030, 1030, 1031)])
def test_potrf_unaligned_ld_is_deterministic(n, ncols, lda):
    """ipm_potrf_partial with a leading dimension that is not a whole number of 128-byte lines is
    factored in an aligned copy (the fused kernel's in-launch hand-offs need line-aligned columns,
    r6): repeated factorizations are bitwise equal to each other and to the aligned layout's."""
    import torch
    rng = np.random.default_rng(n)
    M = rng.uniform(-0.5, 0.5, size=(n, n))
    A = M @ M.T + n * np.eye(n)
    outs = []
    for ld in (lda, lda, lda, (n + 15) // 16 * 16):
        buf = torch.zeros(n, ld, dtype=torch.float64, device="cuda")
        buf[:, :n] = dev(A)
        rc, info = potrf(buf, n, ld, ncols)
        assert rc == 0 and info == 0
        outs.append(np.tril(host(buf).T[:n, :ncols]))
    for o in outs[1:]:
        np.testing.assert_array_equal(o, outs[0])
    Lr = np.linalg.cholesky(A[:ncols, :ncols])
    assert np.linalg.norm(outs[0][:ncols] - Lr) <= 1e-12 * np.linalg.norm(Lr)


@pytest.mark.parametrize("n,ncols,lda", [(8193, 8192, 8208), (8194, 8193, 8208)])
def test_potrf_repeat_is_bitwise(n, ncols, lda):
    """The fused factorization is deterministic by construction (fixed reduction orders, ticketed
    roles): 40 factorizations of one matrix are bitwise equal.  The diagonal-role race fixed in r6
    (wave 1 reading LDS rows wave 0 had already overwritten; scripts/race_check.py) showed here as
    1-8 differing runs in 250 at these shapes."""
    import torch
    torch.manual_seed(0)
    M = torch.rand(n, n, dtype=torch.float64, device="cuda") - 0.5
    A = M @ M.T + n * torch.eye(n, dtype=torch.float64, device="cuda")
    buf0 = torch.zeros(n, lda, dtype=torch.float64, device="cuda")
    buf0[:, :n] = A
    ref = None
    for r in range(40):
        H = buf0.clone()
        rc, info = potrf(H, n, lda, ncols)
        assert rc == 0 and info == 0
        Lf = torch.tril(H[:, :n].T)[:, :ncols]
        if ref is None:
            ref = Lf.clone()
        else:
            assert torch.equal(Lf, ref), f"run {r} differs"


_STREAMK_CHILD = r"""
import sys, numpy as np
sys.path[:0] = [sys.argv[1], sys.argv[2]]
from gpu_util import colmajor_lower, syrk
EPS = np.finfo(np.float64).eps
worst = 0.0
for k, n in [(2048, 4096), (520, 4096), (300, 4096)]:
    rng = np.random.default_rng(k + n)
    X = rng.uniform(-2, 2, (k, n))
    w = rng.uniform(0.1, 3, k)
    got = colmajor_lower(syrk(X, w, n), n)
    ref = X.T @ (w[:, None] * X)
    bound = 64 * EPS * (np.abs(X).T @ (w[:, None] * np.abs(X))) + 1e-300
    worst = max(worst, float(np.max(np.tril(np.abs(got - ref) / bound))))
print("worst", worst)
"""


@pytest.mark.parametrize("mode", ["0", "1", "2", "3", "4"])
def test_syrk_streamk_modes(mode):
    """Every IPM_STREAMK tail (0 K-halves, 1 / 2 pieces first / last, 3 / 4 the same with at most
    8 pieces) on config 5's 528-tile grid at three K (16, 7 and 4 pieces in the default plan), each
    in its own process (the knob is read once per process), within the 64 eps bound."""
    import os
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    pkg = os.path.join(here, "..", "interiorpoint-gpu_amd")
    env = dict(os.environ, IPM_STREAMK=mode)
    out = subprocess.run([sys.executable, "-c", _STREAMK_CHILD, here, pkg], env=env, capture_output=True,
                         text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-2000:]
    worst = float(out.stdout.split("worst")[-1])
    assert worst <= 1.0, worst
