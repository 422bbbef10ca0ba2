"""Assembled ILU(0) preconditioner (gls_ilu_attach; the reference's ILU-preconditioned GMRES,
setup_ILU gls_navier_stokes.cc:1161-1176): the CSR matrix it probes from the device operator equals
the oracle's assembled, constraint-eliminated system matrix (assemble_matrix_and_rhs, the matrix
Trilinos factors in the reference), and ILU-preconditioned GMRES reaches the Jacobi-preconditioned
Newton solution in far fewer iterations."""
import numpy as np
import pytest

from oracle.oracle import Oracle, StructuredProblem
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
