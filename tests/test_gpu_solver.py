"""End-to-end GPU solver parity: the device Newton + GMRES on the matrix-free HIP operator
reproduces the reference's own golden L2 errors (mms3d_gls, mms2d_gls) and the oracle's
direct-solve solution."""
import json
import os

import numpy as np
import pytest

from oracle.oracle import Oracle, StructuredProblem, muparser_to_numpy, newton_solve
from tests.gpu_util import context_for, cuda

G = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "reference_goldens.json")))


def printed(x, digits):
    return 0.5 * 10.0 ** (1 - digits) * abs(x) * 1.0000001


@pytest.mark.gpu
@pytest.mark.parametrize("dim,i", [(3, 0), (3, 1), (2, 1)])
def test_mms_goldens_on_gpu(dim, i):
    g = G["mms3d_gls" if dim == 3 else "mms2d_gls"]
    F = muparser_to_numpy(g["force"])
    E = muparser_to_numpy(g["exact"])
    p = StructuredProblem(dim, g["cells_per_dir"][i], k=1)
    p.set_dirichlet([("noslip", 0, None)])
    p.set_force(lambda X: F(X)[:, :dim])
    ctx = context_for(p)
    x = cuda(p.apply_nonzero_constraints(np.zeros(p.n_dofs)))
    st = ctx.newton(x, tolerance=1e-8, max_iterations=10, lin_max_iterations=5000, restart=100,
                    relative_residual=1e-4, minimum_residual=1e-9)
    assert st["final_residual"] < 1e-8, st
    eu, ep = Oracle(p).l2_error(x.cpu().numpy(), E)
    assert abs(eu - g["error_velocity"][i]) <= printed(g["error_velocity"][i], 5)
    assert abs(ep - g["error_pressure"][i]) <= printed(g["error_pressure"][i], 5)


@pytest.mark.gpu
def test_cavity_q2_bdf2_step_matches_oracle():
    """One BDF2 step of a small 3D Q2 cavity: GPU Newton/GMRES vs the oracle's direct Newton."""
    p = StructuredProblem(3, 3, k=2, viscosity=0.05, scheme="bdf2", time_steps=(0.01, 0.01, 0.01, 0.01),
                          colorize=True)
    p.set_dirichlet([("noslip", b, None) for b in (0, 1, 2, 4, 5)] +
                    [("function", 3, lambda X: np.stack([np.ones(len(X)), 0 * X[:, 0], 0 * X[:, 0]], 1))])
    rng = np.random.default_rng(5)
    m1 = p.apply_nonzero_constraints(0.1 * rng.uniform(-1, 1, p.n_dofs))
    m2 = p.apply_nonzero_constraints(0.1 * rng.uniform(-1, 1, p.n_dofs))
    x_ref, _, _ = newton_solve(p, x0=m1, u1=m1, u2=m2, tol=1e-10)
    ctx = context_for(p)
    x = cuda(m1)
    st = ctx.newton(x, cuda(m1), cuda(m2), tolerance=1e-10, max_iterations=10, lin_max_iterations=2000,
                    restart=60, relative_residual=1e-8, minimum_residual=1e-13)
    xs = x.cpu().numpy()
    nu_ = p.dim * p.n_vnodes
    assert np.abs(xs[:nu_] - x_ref[:nu_]).max() < 1e-7, st
    pg, pr = xs[nu_:] - xs[nu_:].mean(), x_ref[nu_:] - x_ref[nu_:].mean()
    assert np.abs(pg - pr).max() < 1e-6 * max(1.0, np.abs(pr).max())


@pytest.mark.gpu
@pytest.mark.parametrize("k", [1, 2])
def test_multigrid_preconditioner(k):
    """GMRES + geometric multigrid V-cycle (gls_mg_attach) reaches the same Newton solution as
    GMRES + Jacobi, in far fewer iterations (mesh-independent)."""
    import torch
    import bench
    from softx_2020_200_amd.problem import CavityProblem
    n = 16
    out = {}
    for mg in (False, True):
        prob = CavityProblem(dim=3, n=n, k=k, viscosity=0.01, multigrid=mg)
        ctx = prob.ctx
        ctx.set_time("bdf2", (0.01,) * 4)
        m1 = torch.from_numpy(bench.smooth_state(prob.mesh, n, 3, prob.dir_dofs, prob.dir_vals, 0.0)).cuda()
        m2 = torch.from_numpy(bench.smooth_state(prob.mesh, n, 3, prob.dir_dofs, prob.dir_vals, 0.3)).cuda()
        x = m1.clone()
        st = ctx.newton(x, m1, m2, tolerance=1e-9, max_iterations=8, lin_max_iterations=3000, restart=100,
                        relative_residual=1e-6, minimum_residual=1e-14)
        out[mg] = (x.cpu().numpy(), st)
    assert out[True][1]["final_residual"] < 1e-9 and out[False][1]["final_residual"] < 1e-9
    assert out[True][1]["linear_iterations"] * 5 < out[False][1]["linear_iterations"], (out[True][1], out[False][1])
    nv = 3 * (k * n + 1) ** 3
    assert np.abs(out[True][0][:nv] - out[False][0][:nv]).max() < 1e-7


@pytest.mark.gpu
@pytest.mark.parametrize("k", [1, 2])
def test_multigrid_steady_two_levels(k):
    """Steady Stokes-like regime (nu = 1) on 8^3 with one coarse level (4^3): the V-cycle
    preconditioned Newton matches the Jacobi one."""
    import torch
    import bench
    from softx_2020_200_amd.problem import CavityProblem
    n = 8
    out = {}
    for mg in (False, True):
        prob = CavityProblem(dim=3, n=n, k=k, viscosity=1.0, multigrid=mg, pre_smooth=1, post_smooth=1,
                             omega=0.9, coarse_sweeps=100, coarse_omega=0.7, mg_coarsest=2)
        ctx = prob.ctx
        ctx.set_time("steady")
        u = torch.from_numpy(bench.smooth_state(prob.mesh, n, 3, prob.dir_dofs, prob.dir_vals, 0.0)).cuda()
        x = u.clone()
        st = ctx.newton(x, tolerance=1e-10, max_iterations=8, lin_max_iterations=2000, restart=60,
                        relative_residual=1e-8, minimum_residual=1e-14)
        out[mg] = (x.cpu().numpy(), st)
        assert np.isfinite(out[mg][0]).all(), (mg, st)
    assert out[True][1]["final_residual"] < 1e-10, out[True][1]
    nv = 3 * (k * n + 1) ** 3
    assert np.abs(out[True][0][:nv] - out[False][0][:nv]).max() < 1e-7


@pytest.mark.gpu
def test_multigrid_mixed_precision():
    """FP32 smoothing inside the V-cycle (gls_mg_params.mixed_precision) leaves the outer FP64
    GMRES/Newton untouched: same converged solution, GMRES iteration count within one of FP64."""
    import torch
    import bench
    from softx_2020_200_amd.problem import CavityProblem
    n = 16
    out = {}
    for mp in (0, 1):
        prob = CavityProblem(dim=3, n=n, k=2, viscosity=0.01, multigrid=True, pre_smooth=1, post_smooth=1,
                             omega=0.9, coarse_sweeps=100, coarse_omega=0.7, mixed_precision=mp)
        ctx = prob.ctx
        ctx.set_time("bdf2", (0.01,) * 4)
        m1 = torch.from_numpy(bench.smooth_state(prob.mesh, n, 3, prob.dir_dofs, prob.dir_vals, 0.0)).cuda()
        m2 = torch.from_numpy(bench.smooth_state(prob.mesh, n, 3, prob.dir_dofs, prob.dir_vals, 0.3)).cuda()
        x = m1.clone()
        st = ctx.newton(x, m1, m2, tolerance=1e-9, max_iterations=8, lin_max_iterations=500, restart=60,
                        relative_residual=1e-6, minimum_residual=1e-14)
        out[mp] = (x.cpu().numpy(), st)
    assert out[1][1]["final_residual"] < 1e-9, out[1][1]
    assert out[1][1]["linear_iterations"] <= out[0][1]["linear_iterations"] + out[0][1]["newton_iterations"], (
        out[0][1], out[1][1])
    nv = 3 * (2 * n + 1) ** 3
    assert np.abs(out[1][0][:nv] - out[0][0][:nv]).max() < 1e-7
