"""End-to-end GPU solver parity: the device Newton + GMRES on the matrix-free HIP operator
reproduces the reference's own golden L2 errors (mms3d_gls, mms2d_gls) and the oracle's
direct-solve solution."""
import json
import os

import numpy as np
import pytest

from oracle.oracle import Oracle, StructuredProblem, muparser_to_numpy, newton_solve
from tests.gpu_util import context_for, cuda, relerr

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
@pytest.mark.parametrize("k,variant", [(1, "default"), (2, "default"), (2, "bench")])
def test_multigrid_preconditioner(k, variant):
    """GMRES + geometric multigrid V-cycle (gls_mg_attach) reaches the same Newton solution as
    GMRES + Jacobi, in far fewer iterations (mesh-independent). "bench": bench.py's hierarchy --
    FP32 smoothing, 2+2 sweeps on the level above an exact LU solve of the 2^3-cell coarsest level
    (gls_mg_params.level_sweeps)."""
    import torch
    import bench
    from softx_2020_200_amd.problem import CavityProblem
    n = 16
    out = {}
    opts = {}
    if variant == "bench":
        opts = dict(mg_coarsest=2, pre_smooth=1, post_smooth=1, omega=0.9, mixed_precision=True,
                    level_sweeps={-2: (2, 2)})
    for mg in (False, True):
        prob = CavityProblem(dim=3, n=n, k=k, viscosity=0.01, multigrid=mg, **(opts if mg else {}))
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


@pytest.mark.gpu
def test_multigrid_oseen_smoother_operator():
    """The V-cycle's FP32 smoothing J.v with the Oseen (Picard) linearization (gls_mg_params.smoother_operator =
    1: no (grad u) v terms, no SUPG tau (v . grad phi) R_s term). (a) The operator: at a state with grad u = 0 and
    R_s = 0 (constant velocity, constant pressure, steady, no force) it is the FP32 Newton operator to FP32
    rounding; at the bench's state it differs by far more (the dropped terms act). (b) The outer FP64 GMRES /
    Newton is untouched: the same converged solution as with the Newton smoothing operator, GMRES iterations
    within one per Newton iteration."""
    import torch
    import bench
    from softx_2020_200_amd.problem import CavityProblem
    n = 16
    probs = {}
    for so in (0, 1):
        probs[so] = CavityProblem(dim=3, n=n, k=2, viscosity=0.01, multigrid=True, pre_smooth=1, post_smooth=1,
                                  omega=0.9, coarse_sweeps=100, coarse_omega=0.7, mixed_precision=1,
                                  smoother_operator=so)
    mesh = probs[0].mesh
    nv = mesh["n_vnodes"]
    v = torch.from_numpy(np.random.default_rng(7).uniform(-1, 1, probs[0].ctx.n_dofs)).cuda()
    const = np.zeros(probs[0].ctx.n_dofs)
    const[:3 * nv] = np.tile([0.3, -0.2, 0.1], nv)
    const[3 * nv:] = 0.7
    smooth = bench.smooth_state(mesh, n, 3, probs[0].dir_dofs, probs[0].dir_vals, 0.0)
    res = {}
    for tag, state, scheme in (("const", const, "steady"), ("bench", smooth, "bdf2")):
        ys = []
        for so in (0, 1):
            ctx = probs[so].ctx
            ctx.set_time(scheme, (0.01,) * 4)
            u = torch.from_numpy(state).cuda()
            ctx.set_state(u, u, u)
            ys.append(ctx.mg_smoother_apply(v).cpu().numpy())
        res[tag] = np.abs(ys[1] - ys[0]).max() / np.abs(ys[0]).max()
    print("Oseen vs Newton smoothing operator: constant state %.2e, bench state %.2e" % (res["const"], res["bench"]))
    assert res["const"] < 2e-6 and res["bench"] > 1e-4, res
    out = {}
    for so in (0, 1):
        ctx = probs[so].ctx
        ctx.set_time("bdf2", (0.01,) * 4)
        m1 = torch.from_numpy(smooth).cuda()
        m2 = torch.from_numpy(bench.smooth_state(mesh, n, 3, probs[so].dir_dofs, probs[so].dir_vals, 0.3)).cuda()
        x = m1.clone()
        st = ctx.newton(x, m1, m2, tolerance=1e-9, max_iterations=8, lin_max_iterations=500, restart=60,
                        relative_residual=1e-6, minimum_residual=1e-14)
        out[so] = (x.cpu().numpy(), st)
    assert out[1][1]["final_residual"] < 1e-9, out[1][1]
    assert out[1][1]["linear_iterations"] <= out[0][1]["linear_iterations"] + out[0][1]["newton_iterations"], (
        out[0][1], out[1][1])
    assert np.abs(out[1][0][:3 * nv] - out[0][0][:3 * nv]).max() < 1e-7


def _interp_1d(nf, nc, k):
    """Qk interpolation on nested equidistant node lattices (numpy, independent of the C++ tap
    tables): fine lattice node i sits at x = i / (2k) coarse cells."""
    P = np.zeros((nf, nc))
    ncc = (nc - 1) // k
    for i in range(nf):
        x = i / (2.0 * k)
        cc = min(int(np.floor(x)), ncc - 1)
        xi = x - cc
        for q in range(k + 1):
            L = 1.0
            for b in range(k + 1):
                if b != q:
                    L *= (xi * k - b) / (q - b)
            P[i, cc * k + q] = L
    return P


@pytest.mark.gpu
@pytest.mark.parametrize("k,n", [(1, 16), (2, 16), (2, 24)])
def test_multigrid_transfers_exact(k, n):
    """gls_mg_transfer: prolongation == tensor-product Qk interpolation (numpy, 1e-13) on every level
    pair, restriction == its transpose (<R f, c> == <f, P c>), for velocity and pressure."""
    import torch
    from softx_2020_200_amd.problem import CavityProblem
    prob = CavityProblem(dim=3, n=n, k=k, viscosity=0.01, multigrid=True, mg_coarsest=2 if n % 3 else 3)
    ctx = prob.ctx
    levels = ctx._mg_levels
    rng = np.random.default_rng(20200200)
    for l in range(len(levels) - 1):
        nf = round(levels[l].n_vnodes ** (1 / 3))
        nc = round(levels[l + 1].n_vnodes ** (1 / 3))
        P1 = _interp_1d(nf, nc, k)
        c = rng.uniform(-1, 1, levels[l + 1].n_dofs)
        f = rng.uniform(-1, 1, levels[l].n_dofs)
        out_f = torch.zeros(levels[l].n_dofs, dtype=torch.float64, device="cuda")
        out_c = torch.zeros(levels[l + 1].n_dofs, dtype=torch.float64, device="cuda")
        ctx.mg_transfer(l, 1, torch.from_numpy(c).cuda(), out_f)
        ctx.mg_transfer(l, 0, torch.from_numpy(f).cuda(), out_c)
        pf, rc = out_f.cpu().numpy(), out_c.cpu().numpy()
        ncn, nfn = nc ** 3, nf ** 3
        fields_c = [c[3 * np.arange(ncn) + a] for a in range(3)] + [c[3 * ncn:]]
        fields_f = [pf[3 * np.arange(nfn) + a] for a in range(3)] + [pf[3 * nfn:]]
        for fc, ff in zip(fields_c, fields_f):
            ref = np.einsum("zc,yb,xa,cba->zyx", P1, P1, P1, fc.reshape(nc, nc, nc), optimize=True).reshape(-1)
            assert np.abs(ff - ref).max() < 1e-13 * max(1.0, np.abs(ref).max()), (l, np.abs(ff - ref).max())
        lhs, rhs = np.dot(rc, c), np.dot(f, pf)
        assert abs(lhs - rhs) < 1e-12 * np.abs(f).sum(), (l, lhs, rhs)


@pytest.mark.gpu
@pytest.mark.parametrize("mp", [0, 1])
def test_fused_jacobi_sweeps_match_unfused(mp, monkeypatch):
    """The V-cycle's damped-Jacobi sweeps fused into the brick J.v + slab sum (single rank) give the
    same preconditioner application as J.v followed by the separate update (FP64 smoother: to
    rounding; FP32 smoother with FP32 slabs vs FP64 slabs: to FP32 rounding)."""
    import torch
    import bench
    from softx_2020_200_amd.problem import CavityProblem
    n = 16
    prob = CavityProblem(dim=3, n=n, k=2, viscosity=0.01, multigrid=True, pre_smooth=2, post_smooth=2,
                         omega=0.9, coarse_sweeps=20, coarse_omega=0.7, mixed_precision=mp)
    ctx = prob.ctx
    ctx.set_time("bdf2", (0.01,) * 4)
    m1 = torch.from_numpy(bench.smooth_state(prob.mesh, n, 3, prob.dir_dofs, prob.dir_vals, 0.0)).cuda()
    m2 = torch.from_numpy(bench.smooth_state(prob.mesh, n, 3, prob.dir_dofs, prob.dir_vals, 0.3)).cuda()
    ctx.set_state(m1, m1, m2)
    v = torch.from_numpy(np.random.default_rng(20200200).uniform(-1, 1, ctx.n_dofs)).cuda()
    z_fused = ctx.apply_preconditioner(v).cpu().numpy()
    monkeypatch.setenv("GLS_MG_NO_FUSE", "1")
    monkeypatch.setenv("GLS_SLAB_F64", "1")
    z_ref = ctx.apply_preconditioner(v).cpu().numpy()
    rel = np.abs(z_fused - z_ref).max() / np.abs(z_ref).max()
    assert rel < (1e-5 if mp else 1e-12), rel
    assert np.abs(z_ref).max() > 0


@pytest.mark.gpu
@pytest.mark.parametrize("mp", [0, 1])
def test_coarse_graph_matches_plain_launches(mp, monkeypatch):
    """The coarsest level's Jacobi sweeps replayed as one captured HIP graph give bit-identical
    preconditioner applications to the plain launches, also after a state change (the graph is
    re-captured per state, never replayed with a stale linearization)."""
    import torch
    import bench
    from softx_2020_200_amd.problem import CavityProblem
    n = 16
    prob = CavityProblem(dim=3, n=n, k=2, viscosity=0.01, multigrid=True, pre_smooth=1, post_smooth=1,
                         omega=0.9, coarse_sweeps=30, coarse_omega=0.7, mixed_precision=mp)
    ctx = prob.ctx
    ctx.set_time("bdf2", (0.01,) * 4)
    v = torch.from_numpy(np.random.default_rng(20200200).uniform(-1, 1, ctx.n_dofs)).cuda()
    for shift in (0.0, 0.45):
        m1 = torch.from_numpy(bench.smooth_state(prob.mesh, n, 3, prob.dir_dofs, prob.dir_vals, shift)).cuda()
        m2 = torch.from_numpy(bench.smooth_state(prob.mesh, n, 3, prob.dir_dofs, prob.dir_vals, shift + 0.3)).cuda()
        ctx.set_state(m1, m1, m2)
        monkeypatch.setenv("GLS_MG_GRAPH", "1")
        z_graph = ctx.apply_preconditioner(v).cpu().numpy()
        z_graph2 = ctx.apply_preconditioner(v).cpu().numpy()  # replay of the captured graph
        monkeypatch.delenv("GLS_MG_GRAPH")
        z_plain = ctx.apply_preconditioner(v).cpu().numpy()
        assert np.abs(z_plain).max() > 0
        assert np.array_equal(z_graph, z_plain), (shift, np.abs(z_graph - z_plain).max())
        assert np.array_equal(z_graph2, z_plain), shift


@pytest.mark.gpu
@pytest.mark.parametrize("k", [1, 2])
def test_frozen_jacobian_operators(k):
    """gls_freeze_jacobian (skip_newton matrix reuse): after freezing at state a and moving the state
    to b, J.v and the diagonal stay those of a (bitwise), the residual is that of b; releasing the
    freeze re-derives J at b. Brick path (k = 1, 2 in 3D) and per-cell path (2D)."""
    import torch
    for dim in (3, 2):
        p = StructuredProblem(dim, 4, k=k, viscosity=0.02, scheme="bdf2", time_steps=(0.01, 0.012, 0.01, 0.01))
        p.set_dirichlet([("noslip", 0, None)])
        rng = np.random.default_rng(11)
        a, b, h1, h2, v = (cuda(rng.uniform(-1, 1, p.n_dofs)) for _ in range(5))
        ctx = context_for(p)
        ctx.set_state(a, h1, h2)
        ja, da, ra = ctx.jacobian_apply(v).clone(), ctx.jacobian_diagonal().clone(), ctx.residual().clone()
        ctx.freeze_jacobian(True)
        ctx.set_time("bdf1", (0.02, 0.01, 0.01, 0.01))  # the residual's scheme moves, J keeps bdf2
        ctx.set_state(b, h1)
        rb_frozen = ctx.residual().clone()
        # (the Q1 wave kernel sums its brick in LDS atomics: equal up to summation order)
        same = lambda x, y: relerr(x.cpu().numpy(), y.cpu().numpy()) < 1e-13  # noqa: E731
        assert same(ctx.jacobian_apply(v), ja)
        assert same(ctx.jacobian_diagonal(), da)
        ctx.freeze_jacobian(False)
        jb = ctx.jacobian_apply(v).clone()
        rb = ctx.residual().clone()
        assert same(rb_frozen, rb) and not same(rb, ra) and not same(jb, ja)
        ref = context_for(p)
        ref.set_time("bdf1", (0.02, 0.01, 0.01, 0.01))
        ref.set_state(b, h1)
        assert same(jb, ref.jacobian_apply(v))


@pytest.mark.gpu
def test_skip_newton_reaches_newton_solution():
    """SkipNewtonNonLinearSolver (skip_newton_non_linear_solver.h:54-131) on the 3D Q2 cavity BDF2
    step: the chord iterations (Jacobian of the first iteration reused) converge to the Newton
    solution; more Newton iterations, one assembly."""
    p = StructuredProblem(3, 4, k=2, viscosity=0.05, scheme="bdf2", time_steps=(0.01, 0.01, 0.01, 0.01),
                          colorize=True)
    p.set_dirichlet([("noslip", b, None) for b in (0, 1, 2, 4, 5)] +
                    [("function", 3, lambda X: np.stack([np.ones(len(X)), 0 * X[:, 0], 0 * X[:, 0]], 1))])
    rng = np.random.default_rng(5)
    m1 = p.apply_nonzero_constraints(0.1 * rng.uniform(-1, 1, p.n_dofs))
    m2 = p.apply_nonzero_constraints(0.1 * rng.uniform(-1, 1, p.n_dofs))
    out = {}
    for solver in ("newton", "skip_newton"):
        ctx = context_for(p)
        x = cuda(m1)
        st = ctx.newton(x, cuda(m1), cuda(m2), tolerance=1e-10, max_iterations=30, lin_max_iterations=2000,
                        restart=60, relative_residual=1e-10, minimum_residual=1e-14, solver=solver,
                        skip_iterations=3, is_initial_step=False, force_matrix_renewal=True)
        assert st["final_residual"] < 1e-10, (solver, st)
        out[solver] = (x.cpu().numpy(), st)
    (xn, sn), (xs, ss) = out["newton"], out["skip_newton"]
    assert ss["newton_iterations"] > sn["newton_iterations"]
    nu_ = p.dim * p.n_vnodes
    assert np.abs(xs[:nu_] - xn[:nu_]).max() < 1e-8


@pytest.mark.gpu
@pytest.mark.parametrize("n", [8, 16])
def test_fused_first_sweep_is_bitwise(n, monkeypatch):
    """V(1,1) with the FP32 smoother: the first pre-sweep from x = 0 formed inside the residual's pencil
    J.v (x = omega D^-1 b in the gather, stored by the J.v and the slab sum; no separate mg_jacobi_update)
    gives the BITWISE same preconditioner application as the separate update + residual (the default;
    the fusion is opt-in, GLS_MG_FIRST_FUSE=1, measured slower), and GMRES the same iterations and solution."""
    import torch
    import bench
    from softx_2020_200_amd.problem import CavityProblem
    prob = CavityProblem(dim=3, n=n, k=2, viscosity=0.01, multigrid=True, pre_smooth=1, post_smooth=1,
                         omega=0.9, coarse_sweeps=20, coarse_omega=0.7, mixed_precision=1)
    ctx = prob.ctx
    ctx.set_time("bdf2", (0.01,) * 4)
    m1 = torch.from_numpy(bench.smooth_state(prob.mesh, n, 3, prob.dir_dofs, prob.dir_vals, 0.0)).cuda()
    m2 = torch.from_numpy(bench.smooth_state(prob.mesh, n, 3, prob.dir_dofs, prob.dir_vals, 0.3)).cuda()
    ctx.set_state(m1, m1, m2)
    v = torch.from_numpy(np.random.default_rng(4).uniform(-1, 1, ctx.n_dofs)).cuda()
    b = ctx.residual()
    out = {}
    for tag, env in (("fused", "1"), ("plain", "0")):
        monkeypatch.setenv("GLS_MG_FIRST_FUSE", env)
        z = ctx.apply_preconditioner(v).cpu().numpy()
        x, its, _, ok = ctx.solve_linear(b, max_iterations=200, relative_residual=1e-8)
        assert ok
        out[tag] = (z, x.cpu().numpy(), its)
    assert np.array_equal(out["fused"][0], out["plain"][0])
    assert np.array_equal(out["fused"][1], out["plain"][1])
    assert out["fused"][2] == out["plain"][2]
    assert np.abs(out["plain"][0]).max() > 0


@pytest.mark.gpu
def test_coarse_lu_unpivoted_default_matches_pivoted(monkeypatch):
    """The coarsest-level LU defaults to rocSOLVER's unpivoted factorization (a pivoted retry when a pivot
    vanishes): bench.py's hierarchy gives the same Newton / GMRES iteration counts and the same solution
    to 1e-10 as the pivoted LU (GLS_MG_COARSE_SOLVER=lu)."""
    import torch
    import bench
    from softx_2020_200_amd.problem import CavityProblem
    n = 16
    out = {}
    for env in (None, "lu"):
        if env:
            monkeypatch.setenv("GLS_MG_COARSE_SOLVER", env)
        prob = CavityProblem(dim=3, n=n, k=2, viscosity=0.01, multigrid=True, mg_coarsest=2, pre_smooth=1,
                             post_smooth=1, omega=0.9, mixed_precision=True, level_sweeps={-2: (2, 2)})
        ctx = prob.ctx
        ctx.set_time("bdf2", (0.01,) * 4)
        m1 = torch.from_numpy(bench.smooth_state(prob.mesh, n, 3, prob.dir_dofs, prob.dir_vals, 0.0)).cuda()
        m2 = torch.from_numpy(bench.smooth_state(prob.mesh, n, 3, prob.dir_dofs, prob.dir_vals, 0.3)).cuda()
        x = m1.clone()
        st = ctx.newton(x, m1, m2, tolerance=1e-9, max_iterations=8, lin_max_iterations=500, restart=30,
                        relative_residual=1e-6, minimum_residual=1e-14)
        out[env] = (x.cpu().numpy(), st)
    a, b = out[None], out["lu"]
    assert a[1]["final_residual"] < 1e-9 and b[1]["final_residual"] < 1e-9
    assert a[1]["linear_iterations"] == b[1]["linear_iterations"], (a[1], b[1])
    assert np.abs(a[0] - b[0]).max() < 1e-10 * max(1.0, np.abs(b[0]).max())
