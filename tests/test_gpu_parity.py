"""GPU parity: HIP residual / Jacobian action / diagonal vs the CPU oracle on the same
seeded inputs (seed 20200200, U(-1,1)), through the C-ABI. FP64 tolerance: 1e-12 relative
(max-norm), the bar stated in BASELINE.json's north star ("stated floating-point tolerance")
and SURVEY §7 step 3. DoF indexing is bit-exact: both sides use the same cell->node arrays."""
import numpy as np
import pytest

from oracle.oracle import Oracle, StructuredProblem, muparser_to_numpy
from tests.gpu_util import context_for, cuda, relerr

TOL = 1e-12
SEED = 20200200

CASES = [
    # dim, n, k, kp, scheme, nu
    (3, 3, 1, 1, "steady", 1.0),
    (3, 2, 2, 2, "steady", 1.0),
    (3, 2, 2, 2, "bdf2", 0.01),
    (3, 2, 2, 1, "bdf1", 0.1),
    (3, 3, 1, 1, "bdf3", 0.01),
    (2, 4, 1, 1, "steady", 1.0),
    (2, 3, 2, 1, "sdirk2_1", 1.0),
    (2, 3, 2, 1, "sdirk2_2", 1.0),
    (2, 3, 2, 2, "sdirk3_3", 0.05),
    (2, 3, 3, 3, "bdf2", 0.02),
]


def _problem(dim, n, k, kp, scheme, nu, force=True, srf=False):
    p = StructuredProblem(dim, n, k=k, kp=kp, viscosity=nu, scheme=scheme, time_steps=(0.01, 0.013, 0.011, 0.009),
                          srf=srf, omega=(0.3, -0.2, 0.7))
    p.set_dirichlet([("noslip", 0, None)])
    if force:
        p.set_force(lambda X: np.stack([np.sin(X[:, 0] + 2 * X[:, 1]) for _ in range(dim)], 1) *
                    np.arange(1, dim + 1)[None, :])
    return p


def _states(p):
    rng = np.random.default_rng(SEED)
    return [rng.uniform(-1, 1, p.n_dofs) for _ in range(5)]


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES, ids=lambda c: "d%d_n%d_Q%dQ%d_%s" % c[:5])
def test_residual_jv_diag(case):
    p = _problem(*case)
    u, u1, u2, u3, v = _states(p)
    orc = Oracle(p)
    ctx = context_for(p)
    U, U1, U2, U3, V = map(cuda, (u, u1, u2, u3, v))
    ctx.set_state(U, U1, U2, U3)
    r = ctx.residual().cpu().numpy()
    assert relerr(r, orc.residual(u, u1, u2, u3)) < TOL
    d = ctx.jacobian_diagonal().cpu().numpy()
    assert relerr(d, orc.jacobian_diagonal(u, u1, u2, u3)) < TOL
    jv = ctx.jacobian_apply(V).cpu().numpy()
    assert relerr(jv, orc.jacobian_apply(u, v, u1, u2, u3)) < TOL
    # constrained rows: residual exactly 0, J.v = D_c v
    con = p.constrained.astype(bool)
    assert np.all(r[con] == 0.0)


@pytest.mark.gpu
@pytest.mark.parametrize("dim", [2, 3])
def test_srf_source(dim):
    p = _problem(dim, 3, 1, 1, "bdf1", 0.5, srf=True)
    u, u1, u2, u3, v = _states(p)
    orc = Oracle(p)
    ctx = context_for(p)
    ctx.set_state(cuda(u), cuda(u1))
    assert relerr(ctx.residual().cpu().numpy(), orc.residual(u, u1)) < TOL
    assert relerr(ctx.jacobian_apply(cuda(v)).cpu().numpy(), orc.jacobian_apply(u, v, u1)) < TOL


@pytest.mark.gpu
def test_jv_matches_assembled_matrix_and_linearity():
    """J.v equals the reference-style assembled CSR (constraint elimination + |diag| rule) times v,
    and is linear in v (size-independent property)."""
    p = _problem(3, 2, 2, 2, "bdf2", 0.02)
    u, u1, u2, u3, v = _states(p)
    w = np.random.default_rng(SEED + 1).uniform(-1, 1, p.n_dofs)
    A, _ = Oracle(p).matrix_and_rhs(u, u1, u2)
    ctx = context_for(p)
    ctx.set_state(cuda(u), cuda(u1), cuda(u2))
    jv = ctx.jacobian_apply(cuda(v)).cpu().numpy()
    assert relerr(jv, A @ v) < TOL
    jw = ctx.jacobian_apply(cuda(w)).cpu().numpy()
    jvw = ctx.jacobian_apply(cuda(2.0 * v - 3.0 * w)).cpu().numpy()
    assert relerr(jvw, 2.0 * jv - 3.0 * jw) < 1e-12
    d = ctx.jacobian_diagonal().cpu().numpy()
    assert relerr(d, A.diagonal()) < TOL


@pytest.mark.gpu
def test_product_mesh_builder_parity():
    """The C++ Morton-ordered mesh gives the same global vectors as the oracle's lexicographic mesh."""
    import softx_2020_200_amd as sx
    from softx_2020_200_amd.problem import build_context
    p = _problem(3, 4, 2, 2, "steady", 1.0, force=False)
    m = sx.hyper_cube(3, 4, 2, 2)
    from tests.gpu_util import vnode_mask_of
    ctx = build_context(m, viscosity=1.0, vnode_mask=vnode_mask_of(p))
    ctx.set_time("steady")
    u, _, _, _, v = _states(p)
    ctx.set_state(cuda(u))
    orc = Oracle(p)
    assert relerr(ctx.residual().cpu().numpy(), orc.residual(u)) < TOL
    assert relerr(ctx.jacobian_apply(cuda(v)).cpu().numpy(), orc.jacobian_apply(u, v)) < TOL


@pytest.mark.gpu
def test_empty_and_single_cell():
    p = StructuredProblem(3, 1, k=2)
    u, _, _, _, v = _states(p)
    ctx = context_for(p)
    ctx.set_state(cuda(u))
    assert relerr(ctx.residual().cpu().numpy(), Oracle(p).residual(u)) < TOL
    from softx_2020_200_amd import GLSContext
    e = GLSContext(3, 1, 1, np.zeros((0, 8), np.int32), None, np.zeros((0, 3)), 8, 8)
    e.set_time("steady")
    z = cuda(np.zeros(32))
    e.set_state(z)
    assert float(e.residual().abs().max()) == 0.0


def _morton_problem(n, k, scheme, nu, force=True, srf=False, periodic=()):
    """Oracle problem carrying the product's Morton-ordered hyper_cube arrays (brick-kernel layout)."""
    import softx_2020_200_amd as sx
    p = StructuredProblem(3, n, k=k, kp=k, viscosity=nu, scheme=scheme, time_steps=(0.01, 0.013, 0.011, 0.009),
                          srf=srf, omega=(0.3, -0.2, 0.7), periodic=periodic)
    m = sx.hyper_cube(3, n, k, k, -1.0, 1.0, periodic=periodic)
    p.cell_vnodes = np.ascontiguousarray(m["cell_vnodes"])
    p.cell_pnodes = np.ascontiguousarray(m["cell_pnodes"])
    p.cell_x0 = np.ascontiguousarray(m["cell_x0"])
    p.cell_h = np.ascontiguousarray(m["cell_h"])
    if not periodic:
        p.set_dirichlet([("noslip", 0, None)])
    if force:
        p.set_force(lambda X: np.stack([np.sin(X[:, 0] + 2 * X[:, 1]), np.cos(X[:, 2]), X[:, 0] * X[:, 1]], 1))
    return p


BRICK_CASES = [
    (4, 2, "steady", 1.0, False),
    (4, 2, "bdf2", 0.01, False),
    (2, 2, "bdf3", 0.02, True),
    (4, 1, "bdf1", 0.1, False),
    (4, 1, "sdirk3_2", 0.05, True),
    (2, 2, "sdirk2_2", 0.5, False),
]


@pytest.mark.gpu
@pytest.mark.parametrize("case", BRICK_CASES, ids=lambda c: "n%d_Q%d_%s_srf%d" % (c[0], c[1], c[2], c[4]))
def test_brick_kernels_vs_oracle(case):
    n, k, scheme, nu, srf = case
    p = _morton_problem(n, k, scheme, nu, srf=srf)
    u, u1, u2, u3, v = _states(p)
    ctx = context_for(p)
    assert ctx.uses_brick_kernels
    ctx.set_state(cuda(u), cuda(u1), cuda(u2), cuda(u3))
    orc = Oracle(p)
    assert relerr(ctx.residual().cpu().numpy(), orc.residual(u, u1, u2, u3)) < TOL
    # the brick path derives the diagonal in the linearization pass (incl. |K_ii| on constrained rows)
    assert relerr(ctx.jacobian_diagonal().cpu().numpy(), orc.jacobian_diagonal(u, u1, u2, u3)) < TOL
    assert relerr(ctx.jacobian_apply(cuda(v)).cpu().numpy(), orc.jacobian_apply(u, v, u1, u2, u3)) < TOL


@pytest.mark.gpu
def test_brick_periodic_wrap():
    """Periodic x: the brick at the high face shares nodes with the low-face brick (atomics path)."""
    p = _morton_problem(4, 2, "bdf1", 0.1, periodic=(0,))
    u, u1, u2, u3, v = _states(p)
    ctx = context_for(p)
    assert ctx.uses_brick_kernels
    ctx.set_state(cuda(u), cuda(u1))
    orc = Oracle(p)
    assert relerr(ctx.residual().cpu().numpy(), orc.residual(u, u1)) < TOL
    assert relerr(ctx.jacobian_diagonal().cpu().numpy(), orc.jacobian_diagonal(u, u1)) < TOL
    assert relerr(ctx.jacobian_apply(cuda(v)).cpu().numpy(), orc.jacobian_apply(u, v, u1)) < TOL


@pytest.mark.gpu
def test_brick_deterministic():
    """Brick kernels sum cells in LDS in a fixed order; repeated J.v launches agree bitwise on
    brick-interior DoFs and to rounding on shared ones."""
    p = _morton_problem(4, 2, "bdf2", 0.01)
    u, u1, u2, u3, v = _states(p)
    ctx = context_for(p)
    ctx.set_state(cuda(u), cuda(u1), cuda(u2))
    a = ctx.jacobian_apply(cuda(v)).cpu().numpy()
    b = ctx.jacobian_apply(cuda(v)).cpu().numpy()
    assert relerr(a, b) < 1e-14


@pytest.mark.gpu
def test_jv_linearization_cache(monkeypatch):
    """J.v reads the per-quadrature-point linearization (MODE_LIN once per state, MODE_JVQ per call).
    It equals the recompute-every-call kernel (GLS_JV_RECOMPUTE=1) and the oracle, and is refreshed
    by every state / time-step / viscosity change (a stale cache would fail the oracle checks)."""
    p = _morton_problem(4, 2, "bdf2", 0.02)
    u, u1, u2, u3, v = _states(p)
    ctx = context_for(p)
    monkeypatch.setenv("GLS_JV_RECOMPUTE", "1")
    ref_ctx = context_for(p)
    monkeypatch.delenv("GLS_JV_RECOMPUTE")
    orc = Oracle(p)
    for c in (ctx, ref_ctx):
        c.set_state(cuda(u), cuda(u1), cuda(u2))
    a = ctx.jacobian_apply(cuda(v)).cpu().numpy()
    assert relerr(a, ref_ctx.jacobian_apply(cuda(v)).cpu().numpy()) < 1e-14
    assert relerr(a, orc.jacobian_apply(u, v, u1, u2)) < TOL
    # new state through set_state
    ctx.set_state(cuda(u3), cuda(u1), cuda(u2))
    assert relerr(ctx.jacobian_apply(cuda(v)).cpu().numpy(), orc.jacobian_apply(u3, v, u1, u2)) < TOL
    # new time steps (alpha, tau's transient term) and viscosity
    p2 = _morton_problem(4, 2, "bdf2", 0.05)
    p2.time_steps = (0.02, 0.013, 0.011, 0.009)
    ctx.set_time("bdf2", p2.time_steps)
    ctx.set_viscosity(0.05)
    assert relerr(ctx.jacobian_apply(cuda(v)).cpu().numpy(), Oracle(p2).jacobian_apply(u3, v, u1, u2)) < TOL


TOL_F32 = 1e-5  # FP32 arithmetic (unit roundoff 6e-8) over ~100-term quadrature sums, max-norm relative


@pytest.mark.gpu
@pytest.mark.parametrize("case", BRICK_CASES, ids=lambda c: "n%d_Q%d_%s_srf%d" % (c[0], c[1], c[2], c[4]))
def test_brick_jv_f32_vs_oracle(case):
    """The mixed-precision V-cycle's operator (gls_jacobian_apply_f32: FP32 linearization copy,
    FP32 sweeps and pointwise algebra, FP64 vectors) is the oracle's J.v to FP32 accuracy, and
    follows state changes (the FP32 copy is refreshed with the FP64 linearization)."""
    n, k, scheme, nu, srf = case
    p = _morton_problem(n, k, scheme, nu, srf=srf)
    u, u1, u2, u3, v = _states(p)
    ctx = context_for(p)
    assert ctx.uses_brick_kernels
    orc = Oracle(p)
    ctx.set_state(cuda(u), cuda(u1), cuda(u2), cuda(u3))
    e1 = relerr(ctx.jacobian_apply_f32(cuda(v)).cpu().numpy(), orc.jacobian_apply(u, v, u1, u2, u3))
    ctx.set_state(cuda(u3), cuda(u1), cuda(u2), cuda(u))
    e2 = relerr(ctx.jacobian_apply_f32(cuda(v)).cpu().numpy(), orc.jacobian_apply(u3, v, u1, u2, u))
    print("FP32 J.v rel err %.2e %.2e" % (e1, e2))
    assert e1 < TOL_F32 and e2 < TOL_F32, (e1, e2)


@pytest.mark.gpu
@pytest.mark.parametrize("n,scheme,srf", [(2, "bdf2", False), (4, "bdf2", False), (6, "bdf1", False),
                                          (4, "steady", True)])
def test_pencil_kernels_and_structured_slab_sum(monkeypatch, n, scheme, srf):
    """The Q2 brick operators in the two dataflows agree: the pencil kernels (gls_brick_pencil.hip,
    default: residual, linearization + Jacobian diagonal, J.v, FP32 smoother J.v) and the lane-per-point
    kernels (GLS_PENCIL=0) to FP64 rounding (1e-13; the FP32 operator to FP32 rounding), both equal to the
    oracle; and the structured hyper_cube slab sum (k_slab_sum_cube, default on the cube) is BITWISE the
    node/offset/slot-map form (GLS_SLAB_CSR=1, read at context creation): same slots, same ascending
    order. n = 2, 4 leave the last brick triple short (1 and 2 of 3 bricks); the forcing and (case 4)
    the SRF source run the general instantiation."""
    p = _morton_problem(n, 2, scheme, 0.01, srf=srf)
    u, u1, u2, u3, v = _states(p)
    ctx = context_for(p)
    monkeypatch.setenv("GLS_SLAB_CSR", "1")
    csr = context_for(p)
    monkeypatch.delenv("GLS_SLAB_CSR")
    V = cuda(v)
    out = {}
    for tag, c, pencil in (("pencil", ctx, "1"), ("csr", csr, "1"), ("lpp", ctx, "0")):
        monkeypatch.setenv("GLS_PENCIL", pencil)
        c.set_state(cuda(u), cuda(u1), cuda(u2), cuda(u3))  # drops the cached linearization / diagonal
        out[tag] = [c.residual().cpu().numpy(), c.jacobian_diagonal().cpu().numpy(),
                    c.jacobian_apply(V).cpu().numpy(), c.jacobian_apply_f32(V).cpu().numpy()]
    monkeypatch.delenv("GLS_PENCIL")
    for a, b in zip(out["pencil"], out["csr"]):
        assert np.array_equal(a, b)
    names = ("residual", "diagonal", "J.v", "J.v f32")
    for i, (a, b) in enumerate(zip(out["pencil"], out["lpp"])):
        assert relerr(a, b) < (2e-6 if i == 3 else 1e-13), (names[i], relerr(a, b))
    orc = Oracle(p)
    assert relerr(out["pencil"][0], orc.residual(u, u1, u2, u3)) < TOL
    assert relerr(out["pencil"][1], orc.jacobian_diagonal(u, u1, u2, u3)) < TOL
    assert relerr(out["pencil"][2], orc.jacobian_apply(u, v, u1, u2, u3)) < TOL


@pytest.mark.gpu
@pytest.mark.parametrize("n,scheme,srf", [(2, "bdf2", False), (4, "bdf2", False), (4, "steady", True)])
def test_fused_residual_linearization_diagonal(monkeypatch, n, scheme, srf):
    """assemble_matrix_and_rhs as one pencil launch (MODE_RESLIN: residual, J.v linearization and Jacobian
    diagonal, gls_residual_and_diagonal) is BITWISE the separate residual / diagonal launches: the
    residual, the diagonal, and the J.v / FP32 J.v from the linearization it cached. Case 3 runs the
    forcing + SRF instantiation; GLS_NO_RESLIN=1 (the separate calls behind the same entry) agrees too."""
    p = _morton_problem(n, 2, scheme, 0.01, srf=srf)
    u, u1, u2, u3, v = _states(p)
    ctx = context_for(p)
    V = cuda(v)
    ctx.set_state(cuda(u), cuda(u1), cuda(u2), cuda(u3))
    sep = [ctx.residual().cpu().numpy(), ctx.jacobian_diagonal().cpu().numpy(),
           ctx.jacobian_apply(V).cpu().numpy(), ctx.jacobian_apply_f32(V).cpu().numpy()]
    for env in (None, "1"):
        if env:
            monkeypatch.setenv("GLS_NO_RESLIN", env)
        ctx.set_state(cuda(u), cuda(u1), cuda(u2), cuda(u3))  # drops the linearization / diagonal
        r, d = ctx.residual_and_diagonal()
        fused = [r.cpu().numpy(), d.cpu().numpy(), ctx.jacobian_apply(V).cpu().numpy(),
                 ctx.jacobian_apply_f32(V).cpu().numpy()]
        for name, a, b in zip(("residual", "diagonal", "J.v", "J.v f32"), fused, sep):
            assert np.array_equal(a, b), (env, name, relerr(a, b))
    orc = Oracle(p)
    assert relerr(sep[0], orc.residual(u, u1, u2, u3)) < TOL
