"""Assembled ILU(k) preconditioner (gls_ilu_attach; the reference's ILU-preconditioned GMRES,
setup_ILU gls_navier_stokes.cc:1161-1176): the CSR matrix it probes from the device operator equals
the oracle's assembled, constraint-eliminated system matrix (assemble_matrix_and_rhs, the matrix
Trilinos factors in the reference), and ILU-preconditioned GMRES reaches the Jacobi-preconditioned
Newton solution in far fewer iterations."""
import os

import numpy as np
import pytest
import scipy.sparse as sp

from oracle.oracle import Oracle, StructuredProblem, ilu_factor, iluk_levels
from tests.gpu_util import context_for, cuda

SEED = 20200200


def _cavity(dim, n, k, kp, scheme="steady", nu=1.0):
    p = StructuredProblem(dim, n, k=k, kp=kp, viscosity=nu, scheme=scheme, time_steps=(0.01,) * 4, colorize=True)
    lid = 3 if dim == 3 else 3
    walls = [b for b in range(2 * dim) if b != lid]
    p.set_dirichlet([("noslip", b, None) for b in walls] +
                    [("function", lid, lambda X: np.stack([np.ones(len(X))] + [0 * X[:, 0]] * (dim - 1), 1))])
    return p


@pytest.mark.gpu
@pytest.mark.parametrize("dim,n,k,kp,scheme", [(2, 4, 1, 1, "steady"), (2, 3, 2, 1, "bdf2"), (3, 2, 2, 2, "bdf1"),
                                               (3, 2, 1, 1, "steady"), (2, 3, 3, 3, "steady")])
def test_probed_matrix_equals_oracle_csr(dim, n, k, kp, scheme):
    p = _cavity(dim, n, k, kp, scheme, 0.05)
    rng = np.random.default_rng(SEED)
    u, u1, u2 = (p.apply_nonzero_constraints(rng.uniform(-1, 1, p.n_dofs)) for _ in range(3))
    A, _ = Oracle(p).matrix_and_rhs(u, u1, u2)
    ctx = context_for(p)
    ctx.set_state(cuda(u), cuda(u1), cuda(u2))
    nnz, nprobe = ctx.attach_ilu()
    M = ctx.ilu_matrix()
    A = A.tocsr()
    assert nnz >= A.nnz
    d = (M - A).tocsr()
    scale = np.abs(A.data).max()
    assert np.abs(d.data).max() <= 1e-12 * scale if d.nnz else True


@pytest.mark.gpu
@pytest.mark.parametrize("dim,n,k,kp", [(2, 16, 1, 1), (2, 8, 2, 1)])
def test_ilu_gmres_newton(dim, n, k, kp):
    """Steady cavity (nu = 1): Newton with ILU-GMRES == Newton with Jacobi-GMRES; far fewer GMRES its."""
    out = {}
    for pre in ("jacobi", "ilu"):
        p = _cavity(dim, n, k, kp, "steady", 1.0)
        ctx = context_for(p)
        if pre == "ilu":
            ctx.attach_ilu(1e-12, 1.0)
        x = cuda(p.apply_nonzero_constraints(np.zeros(p.n_dofs)))
        st = ctx.newton(x, tolerance=1e-10, max_iterations=10, lin_max_iterations=20000, restart=100,
                        relative_residual=1e-9, minimum_residual=1e-13)
        out[pre] = (x.cpu().numpy(), st)
    assert out["ilu"][1]["final_residual"] < 1e-10, out["ilu"][1]
    nv = dim * p.n_vnodes
    assert np.abs(out["ilu"][0][:nv] - out["jacobi"][0][:nv]).max() < 1e-7
    assert out["ilu"][1]["linear_iterations"] * 4 < out["jacobi"][1]["linear_iterations"], (out["ilu"][1], out["jacobi"][1])


@pytest.mark.gpu
@pytest.mark.parametrize("dim,n,k,kp,fill,rthresh,order,blk", [
    (2, 4, 1, 1, 0, 1.0, "cm", 0), (2, 4, 1, 1, 1, 1.0, "cm", 0), (2, 4, 1, 1, 4, 1.02, "cm", 0),
    (2, 3, 2, 1, 1, 1.0, "cm", 0), (3, 2, 1, 1, 1, 1.0, "cm", 0), (3, 2, 2, 2, 2, 1.0, "cm", 0),
    (2, 4, 2, 1, 0, 1.0, "multicolor", 0), (3, 2, 2, 2, 0, 1.0, "multicolor", 200), (2, 6, 1, 1, 1, 1.0, "cm", 40),
    (3, 2, 2, 1, 0, 1.02, "multicolor", 0), (2, 4, 1, 1, 1, 1.0, "multicolor", 0)])
def test_iluk_factors_match_oracle(dim, n, k, kp, fill, rthresh, order, blk):
    """ILU(fill) factors computed on the device (probe -> level-of-fill pattern -> Ifpack diagonal
    perturbation -> rocSPARSE csrilu0, or in multicolor order the color-by-color factorization
    kernel) equal the oracle's Ifpack restatement (ilu_factor) of the
    oracle's assembled matrix in the factorization's numbering, on the device's pattern; that pattern
    holds the oracle's ILU(fill) graph of the matrix."""
    p = _cavity(dim, n, k, kp, "bdf1", 0.05)
    rng = np.random.default_rng(SEED)
    u, u1 = (p.apply_nonzero_constraints(rng.uniform(-1, 1, p.n_dofs)) for _ in range(2))
    A, _ = Oracle(p).matrix_and_rhs(u, u1)
    ctx = context_for(p)
    ctx.set_time("bdf1", p.time_steps)
    ctx.set_state(cuda(u), cuda(u1))
    athresh = 1e-5
    ctx.attach_ilu(athresh, rthresh, fill=fill, ordering=order, block_dofs=blk)
    perm, F = ctx.ilu_factors()
    A = A.tocoo()
    B = sp.csr_matrix((A.data, (perm[A.row], perm[A.col])), shape=A.shape)
    B.eliminate_zeros()
    F = F.tocsr()
    pattern = [(i, int(j)) for i in range(F.shape[0]) for j in F.indices[F.indptr[i]:F.indptr[i + 1]]]
    if blk:  # block-Jacobi: the couplings between subdomains are dropped before the factorisation
        S = set(pattern)
        B = B.tocoo()
        keep = np.array([(int(i), int(j)) in S for i, j in zip(B.row, B.col)], dtype=bool)
        assert (~keep).any()
        B = sp.csr_matrix((B.data[keep], (B.row[keep], B.col[keep])), shape=B.shape)
    assert set(iluk_levels(B, fill)) <= set(pattern)
    ref = ilu_factor(B, pattern, athresh=athresh, rthresh=rthresh)
    got = {(i, int(j)): v for i in range(F.shape[0]) for j, v in zip(F.indices[F.indptr[i]:F.indptr[i + 1]],
                                                                       F.data[F.indptr[i]:F.indptr[i + 1]])}
    scale = max(abs(v) for v in ref.values())
    err = max(abs(got[key] - ref[key]) for key in ref)
    assert err <= 1e-10 * scale, (err, scale)


@pytest.mark.gpu
def test_ilu1_needs_fewer_gmres_iterations_than_ilu0():
    """Steady 2D cavity, Q2-Q1: the same Newton solution with ILU(0) and ILU(1); ILU(1) is the
    stronger preconditioner (fewer GMRES iterations)."""
    out = {}
    for fill in (0, 1):
        p = _cavity(2, 8, 2, 1, "steady", 0.1)
        ctx = context_for(p)
        ctx.attach_ilu(1e-12, 1.0, fill=fill)
        x = cuda(p.apply_nonzero_constraints(np.zeros(p.n_dofs)))
        st = ctx.newton(x, tolerance=1e-10, max_iterations=10, lin_max_iterations=5000, restart=30,
                        relative_residual=1e-9, minimum_residual=1e-13)
        out[fill] = (x.cpu().numpy(), st)
    assert out[1][1]["final_residual"] < 1e-10
    nv = 2 * p.n_vnodes  # enclosed flow: the pressure is defined up to a constant
    assert np.abs(out[1][0][:nv] - out[0][0][:nv]).max() < 1e-7
    assert out[1][1]["linear_iterations"] < out[0][1]["linear_iterations"], (out[0][1], out[1][1])


@pytest.mark.gpu
def test_ilu_fill_out_of_range_fails_loudly():
    p = _cavity(2, 4, 1, 1)
    ctx = context_for(p)
    for bad in (-1, 11):
        with pytest.raises(Exception, match="fill"):
            ctx.attach_ilu(1e-8, 1.0, fill=bad)


@pytest.mark.gpu
@pytest.mark.parametrize("dim,n,k,kp,order,blk", [(2, 6, 2, 1, "multicolor", 0), (3, 3, 2, 2, "multicolor", 0),
                                                  (3, 3, 2, 1, "multicolor", 500), (2, 6, 1, 1, "cm", 100)])
def test_ilu_apply_is_the_factored_solve(dim, n, k, kp, order, blk):
    """gls_apply_preconditioner with the ILU attached (multicolor: the color-by-color solves of
    gls_ilu_kernels.hip; Cuthill-McKee: rocSPARSE csrsv) equals P^T U^-1 L^-1 P v computed from the
    returned factors by scipy's triangular solves."""
    import scipy.sparse.linalg as spla
    p = _cavity(dim, n, k, kp, "bdf1", 0.05)
    rng = np.random.default_rng(SEED + 3)
    u, u1 = (p.apply_nonzero_constraints(rng.uniform(-1, 1, p.n_dofs)) for _ in range(2))
    ctx = context_for(p)
    ctx.set_time("bdf1", p.time_steps)
    ctx.set_state(cuda(u), cuda(u1))
    ctx.attach_ilu(1e-5, 1.0, fill=0, ordering=order, block_dofs=blk)
    v = rng.uniform(-1, 1, p.n_dofs)
    z = ctx.apply_preconditioner(cuda(v)).cpu().numpy()
    perm, F = ctx.ilu_factors()
    F = F.tocsr()
    L = (sp.tril(F, -1) + sp.identity(F.shape[0])).tocsr()
    U = sp.triu(F).tocsr()
    pv = np.zeros_like(v)
    pv[perm] = v
    y = spla.spsolve_triangular(L, pv, lower=True)
    x = spla.spsolve_triangular(U, y, lower=False)
    zref = x[perm]
    assert np.abs(z - zref).max() <= 1e-10 * np.abs(zref).max(), np.abs(z - zref).max()


@pytest.mark.gpu
@pytest.mark.parametrize("dim,n,k,kp", [(3, 3, 2, 1), (2, 8, 2, 2)])
def test_multicolor_factorization_equals_rocsparse(dim, n, k, kp):
    """The multicolor order's color-by-color factorization (k_mc_ilu0: rows of earlier colors in
    parallel, the node's own rows in order) and rocSPARSE csrilu0 on the same pattern and values
    (GLS_ILU_ROCSPARSE_FACTOR=1) give the same factors; the kernel with the precomputed row-position
    map (default) and with column searches (GLS_ILU_FACTOR_MAP=0) give bitwise the same factors."""
    p = _cavity(dim, n, k, kp, "bdf1", 0.05)
    rng = np.random.default_rng(SEED + 3)
    u, u1 = (p.apply_nonzero_constraints(rng.uniform(-1, 1, p.n_dofs)) for _ in range(2))
    out = []
    for env in ({"GLS_ILU_ROCSPARSE_FACTOR": "1"}, {"GLS_ILU_FACTOR_MAP": "0"}, {}):
        os.environ.update(env)
        try:
            ctx = context_for(p)
            ctx.set_time("bdf1", p.time_steps)
            ctx.set_state(cuda(u), cuda(u1))
            ctx.attach_ilu(1e-5, 1.0, fill=0, ordering="multicolor")
            out.append(ctx.ilu_factors())
        finally:
            for key in env:
                os.environ.pop(key, None)
    (p0, F0), (p1, F1), (p2, F2) = out
    assert np.array_equal(p0, p1) and np.array_equal(p0, p2)
    F0, F1, F2 = F0.tocsr(), F1.tocsr(), F2.tocsr()
    assert np.array_equal(F0.indptr, F1.indptr) and np.array_equal(F0.indices, F1.indices)
    assert np.abs(F0.data - F1.data).max() <= 1e-12 * np.abs(F0.data).max()
    assert np.array_equal(F1.indices, F2.indices) and np.array_equal(F1.data, F2.data)


@pytest.mark.gpu
def test_batched_probing_equals_probe_loop_with_hanging_and_slip_lines():
    """The batched probe launches (per-cell path) give the same probed matrix as one
    gls_jacobian_apply per probe (GLS_ILU_PROBE_LOOP=1) on an adapted mapped shell with hanging-node
    and curved-slip constraint lines."""
    from oracle.oracle import MappedProblem
    from tests.test_dist_plan import _adapted_space
    from tests.test_gpu_uforest import dof_lines
    sp_ = _adapted_space(3, 2, 1)
    lines = dof_lines(sp_)
    p = MappedProblem(sp_, viscosity=1.0, scheme="steady")
    p.set_hanging(*lines)
    p.hang_lines = lines
    rot = lambda X: np.stack([-X[:, 1], X[:, 0], 0 * X[:, 0]], 1)
    p.set_dirichlet([("function", 0, rot), ("noslip", 1, None), ("slip", 2, None), ("slip", 3, None)])
    rng = np.random.default_rng(SEED + 5)
    x0 = p.apply_nonzero_constraints(0.1 * rng.standard_normal(p.n_dofs))
    out = []
    for env in (None, "1"):
        if env:
            os.environ["GLS_ILU_PROBE_LOOP"] = env
        try:
            g = context_for(p)
            g.attach_ilu(1e-12, 1.0)
            g.set_state(cuda(x0))
            out.append(g.ilu_matrix().tocsr())
        finally:
            os.environ.pop("GLS_ILU_PROBE_LOOP", None)
    a, b = out
    assert np.array_equal(a.indptr, b.indptr) and np.array_equal(a.indices, b.indices)
    assert np.abs(a.data - b.data).max() <= 1e-14 * np.abs(b.data).max()


@pytest.mark.gpu
def test_recorded_probe_activity_gives_the_same_matrix():
    """Batched probing records which (probe, cell batch) pairs are active at its first run and launches only those
    afterwards (from the cached linearization where the state has one): at a second state the probed matrix equals the
    one of a context that tests every pair (GLS_ILU_PROBE_LIST=0), in chunks of 7 probes, on the adapted mapped shell
    with hanging and slip lines."""
    from oracle.oracle import MappedProblem
    from tests.test_dist_plan import _adapted_space
    from tests.test_gpu_uforest import dof_lines
    sp_ = _adapted_space(3, 2, 1)
    lines = dof_lines(sp_)
    p = MappedProblem(sp_, viscosity=1.0, scheme="steady")
    p.set_hanging(*lines)
    p.hang_lines = lines
    rot = lambda X: np.stack([-X[:, 1], X[:, 0], 0 * X[:, 0]], 1)  # noqa: E731
    p.set_dirichlet([("function", 0, rot), ("noslip", 1, None), ("slip", 2, None), ("slip", 3, None)])
    rng = np.random.default_rng(SEED + 6)
    x0 = p.apply_nonzero_constraints(0.1 * rng.standard_normal(p.n_dofs))
    x1 = p.apply_nonzero_constraints(0.1 * rng.standard_normal(p.n_dofs))
    os.environ["GLS_ILU_PROBE_BATCH"] = "7"
    try:
        g = context_for(p)
        g.attach_ilu(1e-12, 1.0)
        g.set_state(cuda(x0))
        g.ilu_matrix()  # first probing: records the activity
        g.set_state(cuda(x1))
        listed = g.ilu_matrix().tocsr()
        os.environ["GLS_ILU_PROBE_LIST"] = "0"
        h = context_for(p)
        h.attach_ilu(1e-12, 1.0)
        h.set_state(cuda(x1))
        tested = h.ilu_matrix().tocsr()
    finally:
        os.environ.pop("GLS_ILU_PROBE_BATCH", None)
        os.environ.pop("GLS_ILU_PROBE_LIST", None)
    assert np.array_equal(listed.indptr, tested.indptr) and np.array_equal(listed.indices, tested.indices)
    # the listed blocks read the linearization the diagonal pass cached (its own FMA contraction): rounding only
    assert np.abs(listed.data - tested.data).max() <= 1e-14 * np.abs(tested.data).max()
