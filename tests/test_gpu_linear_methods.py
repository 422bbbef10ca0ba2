"""The linear-solver switch of the reference (parameters.cc:519-532; solve_linear_system,
gls_navier_stokes.cc:1140-1157): GMRES (solve_system_GMRES :1242-1289) with either orthogonalisation
and BiCGStab (solve_system_BiCGStab :1293-1340), each checked against the TRUE residual ||b - A x||
recomputed here from the device operator, not against the solver's own estimate. The GMRES repair
branches of the Gram-corrected orthogonalisation are forced with their test knobs
(GLS_GMRES_REPAIR_TOL=0: every column repaired; GLS_GMRES_REPAIR_MEASURED=1: the measured-norm
normalisation) so that they run in this suite."""
import os

import numpy as np
import pytest

from oracle.oracle import StructuredProblem
from tests.gpu_util import context_for, cuda


def _problem(nu=0.002, n=5, k=2):
    """A 3D Q2 cavity at a high cell Reynolds number: a nonsymmetric, badly conditioned Jacobian."""
    p = StructuredProblem(3, n, k=k, viscosity=nu, scheme="bdf1", time_steps=(0.05,) * 4, colorize=True)
    p.set_dirichlet([("noslip", b, None) for b in (0, 1, 2, 4, 5)] +
                    [("function", 3, lambda X: np.stack([np.ones(len(X)), 0 * X[:, 0], 0 * X[:, 0]], 1))])
    rng = np.random.default_rng(11)
    u = p.apply_nonzero_constraints(rng.uniform(-1, 1, p.n_dofs))
    return p, u


def _true_residual(ctx, b, x):
    ax = ctx.jacobian_apply(x)
    return float((b - ax).norm())


@pytest.fixture
def env():
    saved = {k: os.environ.get(k) for k in ("GLS_GMRES_REPAIR_TOL", "GLS_GMRES_REPAIR_MEASURED", "GLS_GMRES_VERBOSE")}
    yield os.environ
    for k, v in saved.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v


@pytest.mark.gpu
@pytest.mark.parametrize("method,ortho,knob", [
    ("gmres", "gram", None), ("gmres", "cgs2", None), ("gmres", "gram", "repair_all"),
    ("gmres", "gram", "repair_measured"), ("bicgstab", "gram", None)])
def test_linear_solve_true_residual(env, capfd, method, ortho, knob):
    """Jacobi-preconditioned solve with a large restart (loss of orthogonality accumulates): the
    reported residual agrees with ||b - A x|| within 10x and the true residual meets the tolerance."""
    p, u = _problem()
    ctx = context_for(p)
    U = cuda(u)
    ctx.set_state(U, U, U)
    b = ctx.residual()
    if knob == "repair_all":
        env["GLS_GMRES_REPAIR_TOL"] = "0"
    if knob == "repair_measured":
        env["GLS_GMRES_REPAIR_TOL"] = "0"
        env["GLS_GMRES_REPAIR_MEASURED"] = "1"
    env["GLS_GMRES_VERBOSE"] = "1"
    rel = 1e-9
    x, its, res, ok = ctx.solve_linear(b, max_iterations=4000, restart=150, relative_residual=rel,
                                       minimum_residual=1e-30, method=method, orthogonalization=ortho)
    out = capfd.readouterr().out
    assert ok, (its, res)
    tol = rel * float(b.norm())
    tr = _true_residual(ctx, b, x)
    assert tr <= 10 * tol, (tr, tol, res, its)
    assert res <= tol and tr <= 10 * max(res, 1e-3 * tol), (tr, res)
    if knob is not None:
        assert "orthogonality repair passes" in out, out[-2000:]
    # true_residual=1 reports ||b - A x|| itself
    _, _, res_t, ok = ctx.solve_linear(b, max_iterations=4000, restart=150, relative_residual=rel,
                                       minimum_residual=1e-30, method=method, orthogonalization=ortho,
                                       true_residual=True)
    assert ok and res_t == pytest.approx(tr, rel=0.5, abs=1e-3 * tol), (res_t, tr)


@pytest.mark.gpu
@pytest.mark.parametrize("prec", ["jacobi", "ilu"])
def test_bicgstab_solution_equals_gmres(prec):
    """Both Krylov methods reach the same solution of J x = r to the solve tolerance, with the
    Jacobi preconditioner and with the assembled ILU(0) (setup_ILU) the reference pairs with both."""
    p, u = _problem(nu=0.02, n=4)
    ctx = context_for(p)
    if prec == "ilu":
        ctx.attach_ilu(1e-8, 1.0, fill=0)
    U = cuda(u)
    ctx.set_state(U, U, U)
    b = ctx.residual()
    xs = {}
    for m in ("gmres", "bicgstab"):
        x, its, res, ok = ctx.solve_linear(b, max_iterations=3000, restart=100, relative_residual=1e-12,
                                           minimum_residual=1e-30, method=m)
        assert ok, (m, its, res)
        xs[m] = (x.cpu().numpy(), its)
    d = np.abs(xs["gmres"][0] - xs["bicgstab"][0]).max() / np.abs(xs["gmres"][0]).max()
    assert d < 1e-8, (d, xs["gmres"][1], xs["bicgstab"][1])
    if prec == "ilu":  # the preconditioner acts: far fewer iterations than Jacobi would need
        assert xs["bicgstab"][1] < 200, xs["bicgstab"][1]


@pytest.mark.gpu
def test_newton_with_bicgstab_matches_gmres():
    """NewtonNonLinearSolver with method = bicgstab converges to GMRES's solution (BDF1 step)."""
    p, u = _problem(nu=0.05, n=4)
    sols = {}
    for m in ("gmres", "bicgstab"):
        ctx = context_for(p)
        m1 = cuda(p.apply_nonzero_constraints(0.1 * u))
        x = m1.clone()
        st = ctx.newton(x, m1, m1, tolerance=1e-10, max_iterations=12, lin_max_iterations=3000, restart=100,
                        relative_residual=1e-8, minimum_residual=1e-14, lin_method=m)
        assert st["final_residual"] < 1e-10 and st["linear_failures"] == 0, (m, st)
        sols[m] = x.cpu().numpy()
    nv = 3 * p.n_vnodes
    assert np.abs(sols["gmres"][:nv] - sols["bicgstab"][:nv]).max() < 1e-8
