"""The CPU baseline's complete Newton iteration (oracle gls_oracle_newton_csr: CSR assembly, ILU(0),
GMRES(30) right-preconditioned, line search -- the reference's solve_system_GMRES path,
gls_navier_stokes.cc:1161-1176, 1242-1289) takes the same Newton step as the oracle's exact-solve
Newton when its GMRES is converged, on one thread and on several."""
import numpy as np
import pytest

from oracle.oracle import StructuredProblem, newton_csr, newton_solve


def _cavity(dim, n, k, nu, scheme="steady"):
    p = StructuredProblem(dim, n, k=k, kp=k, viscosity=nu, scheme=scheme, time_steps=(0.05,) * 4, colorize=True)
    p.set_dirichlet([("noslip", b, None) for b in range(2 * dim) if b != 3] +
                    [("function", 3, lambda X: np.stack([np.ones(len(X))] + [0 * X[:, 0]] * (dim - 1), 1))])
    return p


@pytest.mark.parametrize("dim,n,k,nu,threads", [(2, 8, 1, 1.0, 1), (2, 6, 2, 0.1, 4), (3, 4, 1, 1.0, 2)])
def test_cpu_newton_iteration_matches_exact_newton_step(dim, n, k, nu, threads):
    p = _cavity(dim, n, k, nu)
    x0 = p.apply_nonzero_constraints(np.zeros(p.n_dofs))
    ref, _, _ = newton_solve(p, x0.copy(), tol=1e-30, max_it=1)
    x = x0.copy()
    st = newton_csr(p, x, threads=threads, rel=1e-13, minres=1e-16)
    assert st["gmres_its"] > 0 and st["res1"] < 0.9 * st["res0"], st
    nv = dim * p.n_vnodes  # enclosed flow: pressure up to a constant (the exact solve pins one DoF)
    assert np.abs(x[:nv] - ref[:nv]).max() <= 1e-8 * max(np.abs(ref[:nv]).max(), 1.0), np.abs(x[:nv] - ref[:nv]).max()
