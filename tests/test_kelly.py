"""Kelly-driven refinement (first adaptation of a uniform mesh): refine_mesh_kelly,
navier_stokes_base.cc:612-733 — KellyErrorEstimator<dim>::estimate (deal.II, not vendored; its
published algorithm restated in oracle.kelly_estimate), GridRefinement::refine_and_coarsen_fixed_number
(refinement part) and SolutionTransfer::interpolate onto the refined mesh.

CPU: the oracle's indicator on fields with known face jumps (|x|, |z|) and on Qk polynomials (0);
the product's fixed-number flagging against numpy; the product's solution transfer against the
oracle's evaluation of the coarse field (and exactly for Qk polynomials).
GPU: gls_kelly_estimate == the oracle (1e-12) on 2D/3D, Q1/Q2, Q2-Q1, velocity and pressure,
Morton-ordered and periodic meshes; the adaptive mms2d pipeline (solve -> Kelly -> flag -> refine
with hanging nodes -> transfer -> solve) equals the oracle's pipeline. Parity unpinned beyond
the oracle: the reference holds no Kelly golden for these meshes."""
import json
import os

import numpy as np
import pytest

from oracle.oracle import (Oracle, StructuredProblem, evaluate_field, kelly_estimate, muparser_to_numpy, newton_solve, refine_mark,
                           pd_refine_fixed)
import softx_2020_200_amd as sx

SEED = 20200200
G = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "reference_goldens.json")))


def test_oracle_kelly_known_jumps():
    p = StructuredProblem(2, 2, k=1)
    X = p.vnode_coords()
    sol = np.zeros(p.n_dofs)
    sol[0:2 * p.n_vnodes:2] = np.abs(X[:, 0])  # [du/dx] = 2 across x = 0, face length 1
    assert np.allclose(kelly_estimate(p, sol, 0), np.sqrt(np.sqrt(2) / 24 * 4), rtol=1e-13)
    p = StructuredProblem(3, 2, k=2)
    X = p.vnode_coords()
    sol = np.zeros(p.n_dofs)
    sol[2:3 * p.n_vnodes:3] = np.abs(X[:, 2])  # [dw/dz] = 2 across z = 0, face area 1
    assert np.allclose(kelly_estimate(p, sol, 0), np.sqrt(np.sqrt(3) / 24 * 4), rtol=1e-13)
    sol[3 * p.n_vnodes:] = X[:, 0] * X[:, 1] ** 2  # a Q2 pressure: continuous gradient, no jump
    assert np.abs(kelly_estimate(p, sol, 1)).max() < 1e-13


def test_refine_fixed_number_matches_numpy():
    rng = np.random.default_rng(SEED)
    for n, frac in ((100, 0.3), (64, 0.125), (37, 0.5), (10, 0.0)):
        c = rng.uniform(0, 1, n).astype(np.float32)
        c[: n // 5] = c[n // 5]  # ties
        f = sx.refine_fixed_number(c, frac)
        nr = int(frac * n)
        exp = np.zeros(n, dtype=np.int32)
        if nr:
            thr = np.sort(c)[::-1][nr - 1]
            exp = (c >= thr).astype(np.int32)
        assert np.array_equal(f, exp)


def test_pd_refine_known_answers():
    """parallel::distributed fixed-number / fixed-fraction thresholds on hand-checkable inputs."""
    c = np.arange(1, 11, dtype=np.float32)
    for impl in (lambda *a, **k: sx.refine_pd(*a, **k), pd_refine_fixed):
        f, thr = impl(c, 2, 0.3)  # target int(0.3 * 10) = 3 cells strictly above the bisection value
        assert f.tolist() == [0] * 7 + [1] * 3 and 7 < thr <= 8
        f, _ = impl(np.array([1, 1, 1, 1, 6], np.float32), 2, 0.5, "fraction")  # 6 of 10 >= half
        assert f.tolist() == [0, 0, 0, 0, 1]
        # max number elements: 100 + 30 * 3 > 130 -> alpha = 30 / 90 -> 10 cells
        f, _ = impl(np.linspace(0.1, 1, 100).astype(np.float32), 2, 0.3, "number", 130)
        assert f.sum() == 10 and f[-10:].all()
        f, _ = impl(c, 3, 0.3, "number", 10)  # already at the cap: nothing refines
        assert f.sum() == 0
        f, _ = impl(np.zeros(8, np.float32), 3, 0.5)  # all-zero indicators: GridRefinement::refine
        assert f.sum() == 0                             # returns before marking anything


def test_refine_zero_threshold_rules():
    """dealii::GridRefinement::refine's zero rules through the fixed-number path, whose threshold is
    0 when fewer cells than requested have a positive indicator."""
    assert sx.refine_fixed_number(np.zeros(8, np.float32), 0.5).sum() == 0  # all zero: no flags
    # the zero threshold becomes the smallest positive indicator: zero cells stay unflagged
    z = np.array([0.5, 0, 0, 0.25, 0, 1.0, 0, 0], np.float32)
    assert sx.refine_fixed_number(z, 0.75).tolist() == [1, 0, 0, 1, 0, 1, 0, 0]
    assert refine_mark(z, 0.0)[0].tolist() == [1, 0, 0, 1, 0, 1, 0, 0]
    # deal.II's scan starts from criteria[0]: with a leading zero the threshold stays 0
    lead = np.array([0, 0.5, 0.25, 1.0, 0], np.float32)
    assert sx.refine_fixed_number(lead, 1.0).sum() == 5
    assert refine_mark(lead, 0.0)[0].sum() == 5


@pytest.mark.parametrize("ftype", ["number", "fraction"])
def test_pd_refine_matches_oracle(ftype):
    rng = np.random.default_rng(SEED)
    for n, frac, dim, cap in ((100, 0.3, 2, 10 ** 8), (512, 0.1, 3, 10 ** 8), (37, 0.5, 2, 60), (64, 0.0, 3, 10 ** 8),
                              (200, 0.25, 3, 500), (1000, 0.05, 2, 10 ** 8)):
        c = (10.0 ** rng.uniform(-6, 0, n)).astype(np.float32)  # Kelly-like spread over decades
        c[: n // 7] = c[n // 7]  # ties
        f, thr = sx.refine_pd(c, dim, frac, ftype, cap)
        fo, thro = pd_refine_fixed(c, dim, frac, ftype, cap)
        assert thr == thro and np.array_equal(f, fo), (n, frac, dim, cap)
        if ftype == "number" and cap == 10 ** 8 and frac > 0:  # bisection lands near int(frac * n) cells
            assert abs(int(f.sum()) - int(frac * n)) <= n // 7 + 1


@pytest.mark.parametrize("dim,n,k,kp", [(2, 3, 1, 1), (2, 3, 2, 1), (3, 2, 2, 2), (3, 3, 1, 1)])
def test_solution_transfer_matches_oracle(dim, n, k, kp):
    rng = np.random.default_rng(SEED)
    flags = (rng.uniform(0, 1, n ** dim) < 0.4).astype(np.int32)
    flags[0] = 1
    p = StructuredProblem(dim, n, k=k, kp=kp)
    coarse = rng.uniform(-1, 1, p.n_dofs)
    fine = sx.refined_interpolate(dim, n, k, kp, flags, coarse)
    m = sx.refined_cube(dim, n, k, kp, flags)
    vel, _ = evaluate_field(p, coarse, m["vnode_x"])
    _, pre = evaluate_field(p, coarse, m["pnode_x"])
    nv = m["n_vnodes"]
    assert np.abs(fine[:dim * nv] - vel.reshape(-1)).max() < 1e-13
    assert np.abs(fine[dim * nv:] - pre).max() < 1e-13


def _uniform(dim, n, k, kp, periodic=()):
    p = StructuredProblem(dim, n, k=k, kp=kp, periodic=periodic)
    if not periodic:
        p.set_dirichlet([("noslip", 0, None)])
    return p


@pytest.mark.gpu
@pytest.mark.parametrize("case", [(2, 4, 2, 1, ()), (2, 5, 1, 1, (0,)), (3, 3, 1, 1, ()), (3, 4, 2, 2, ()),
                                  (3, 4, 2, 2, "morton")], ids=lambda c: "d%d_n%d_Q%dQ%d_%s" % (c[0], c[1], c[2], c[3], c[4]))
def test_kelly_gpu_vs_oracle(case):
    from tests.gpu_util import context_for, cuda, relerr
    dim, n, k, kp, extra = case
    p = _uniform(dim, n, k, kp, periodic=extra if extra != "morton" else ())
    if extra == "morton":  # the product's Morton-ordered hyper_cube (brick layout)
        m = sx.hyper_cube(3, n, k, k, -1.0, 1.0)
        for key in ("cell_vnodes", "cell_pnodes", "cell_x0", "cell_h"):
            setattr(p, key, np.ascontiguousarray(m[key]))
    rng = np.random.default_rng(SEED)
    sol = rng.uniform(-1, 1, p.n_dofs)
    ctx = context_for(p)
    for var in (0, 1):
        eta = ctx.kelly_estimate(cuda(sol), var).cpu().numpy()
        ref = kelly_estimate(p, sol, var)
        assert relerr(eta, ref) < 1e-12, (var, relerr(eta, ref))
        assert (ref > 0).all()


@pytest.mark.gpu
def test_kelly_adaptive_mms2d_pipeline():
    """mms2d_gls (applications_tests/gls_navier_stokes_2d/mms2d_gls.prm) on 8^2 Q1-Q1: device Newton,
    Kelly on the velocity, refine the top 30 % once (hanging nodes), transfer the solution, device
    Newton again; every stage equals the oracle's, and the refined mesh lowers the L2 error."""
    from tests.gpu_util import context_for, cuda
    g = G["mms2d_gls"]
    F, E = muparser_to_numpy(g["force"]), muparser_to_numpy(g["exact"])
    n = 8
    p = StructuredProblem(2, n, k=1, viscosity=1.0)
    p.set_force(lambda X: F(X)[:, :2])
    p.set_dirichlet([("noslip", 0, None)])
    x_ref, _, _ = newton_solve(p, tol=1e-10)
    ctx = context_for(p)
    x = cuda(p.apply_nonzero_constraints(np.zeros(p.n_dofs)))
    st = ctx.newton(x, tolerance=1e-10, max_iterations=10, lin_max_iterations=4000, restart=200,
                    relative_residual=1e-11, minimum_residual=1e-14)
    assert st["final_residual"] < 1e-10
    eta = ctx.kelly_estimate(x, 0).cpu().numpy()
    eta_ref = kelly_estimate(p, x_ref, 0)
    assert np.abs(eta - eta_ref).max() < 1e-7 * eta_ref.max()
    flags = sx.refine_fixed_number(eta.astype(np.float32), 0.3)
    assert np.array_equal(flags, sx.refine_fixed_number(eta_ref.astype(np.float32), 0.3))
    assert flags.sum() >= int(0.3 * n * n)
    # refined problem (hanging nodes), transferred initial guess
    mesh = sx.refined_cube(2, n, 1, 1, flags)
    q = StructuredProblem.from_refined(mesh, viscosity=1.0)
    lines = sx.hanging_dof_lines(mesh)
    q.set_hanging(*lines)
    q.hang_lines = lines
    q.set_dirichlet([("noslip", 0, None)])
    q.set_force(lambda X: F(X)[:, :2])
    x0 = q.apply_nonzero_constraints(sx.refined_interpolate(2, n, 1, 1, flags, x.cpu().numpy()))
    y_ref, _, _ = newton_solve(q, x0=x0.copy(), tol=1e-10)
    ctx2 = context_for(q)
    y = cuda(x0)
    st2 = ctx2.newton(y, tolerance=1e-10, max_iterations=10, lin_max_iterations=4000, restart=200,
                      relative_residual=1e-11, minimum_residual=1e-14)
    assert st2["final_residual"] < 1e-10
    ys = y.cpu().numpy()
    nv = 2 * q.n_vnodes
    assert np.abs(ys[:nv] - y_ref[:nv]).max() < 1e-8
    e0, _ = Oracle(p).l2_error(x.cpu().numpy(), E)
    e1, _ = Oracle(q).l2_error(ys, E)
    assert e1 < e0, (e0, e1)


@pytest.mark.parametrize("dim,k,kp", [(2, 2, 1), (3, 1, 1)])
def test_box_kelly_restatement_matches_uniform_oracle(dim, k, kp):
    """The face-search restatement for hanging meshes (oracle.kelly_estimate_boxes) equals the
    round-1 lattice restatement on a conforming mesh (an octree refined uniformly)."""
    from oracle.oracle import kelly_estimate_boxes
    p = _uniform(dim, 4, k, kp)
    m = dict(dim=dim, k=k, kp=kp, cell_vnodes=p.cell_vnodes, cell_pnodes=p.cell_pnodes if kp != k else p.cell_vnodes,
             cell_x0=p.cell_x0, cell_h=p.cell_h, n_vnodes=p.n_vnodes)
    sol = np.random.default_rng(SEED).uniform(-1, 1, p.n_dofs)
    for var in (0, 1):
        a = kelly_estimate_boxes(m, sol, var)
        b = kelly_estimate(p, sol, var)
        assert np.abs(a - b).max() <= 1e-12 * np.abs(b).max()


def _octree_kelly_mesh(dim, k, kp):
    t = sx.Octree(dim, 2)
    t.adapt(refine=np.ones(t.n_cells, np.int32))
    for _ in range(2):
        lev, x0, h = t.cells()
        f = (np.linalg.norm(x0 + 0.5 * h - 0.4, axis=1) < 0.5).astype(np.int32)
        t.adapt(refine=f, max_level=4)
    return t


@pytest.mark.gpu
@pytest.mark.parametrize("dim,k,kp", [(2, 1, 1), (2, 2, 1), (3, 1, 1), (3, 2, 2)])
def test_kelly_hanging_faces_gpu_vs_oracle(dim, k, kp):
    """Kelly on a multi-level mesh with hanging faces (gls_kelly_estimate_faces with the
    gls_octree_faces pieces) == the oracle's face-search restatement at 1e-12; on the uniform mesh
    the face form equals the conforming kernel."""
    from oracle.oracle import kelly_estimate_boxes
    from tests.gpu_util import context_for, cuda, relerr
    t = _octree_kelly_mesh(dim, k, kp)
    m = t.mesh(k, kp)
    assert m["cell_level"].max() >= 3
    p = StructuredProblem.from_refined(m, viscosity=1.0)
    lines = sx.hanging_dof_lines(m)
    p.set_hanging(*lines)
    p.hang_lines = lines
    rng = np.random.default_rng(SEED)
    sol = p.apply_nonzero_constraints(rng.uniform(-1, 1, p.n_dofs))
    ctx = context_for(p)
    faces = t.faces(k, kp)
    for var in (0, 1):
        eta = ctx.kelly_estimate_faces(cuda(sol), var, faces).cpu().numpy()
        ref = kelly_estimate_boxes(m, sol, var)
        assert relerr(eta, ref) < 1e-12, (var, relerr(eta, ref))
    u = sx.Octree(dim, 4)
    mu = u.mesh(k, kp)
    pu = StructuredProblem.from_refined(mu, viscosity=1.0)
    solu = rng.uniform(-1, 1, pu.n_dofs)
    cu = context_for(pu)
    for var in (0, 1):
        a = cu.kelly_estimate_faces(cuda(solu), var, u.faces(k, kp)).cpu().numpy()
        b = cu.kelly_estimate(cuda(solu), var).cpu().numpy()
        assert relerr(a, b) < 1e-12
