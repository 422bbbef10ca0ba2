"""Slip boundary conditions (reference: VectorTools::compute_no_normal_flux_constraints
in setup_dofs, gls_navier_stokes.cc:100-110 (nonzero_constraints) and 149-160 (zero_constraints)).

On the hyper_cube's axis-aligned faces n.u = 0 constrains the normal velocity component of every
face of that boundary id the node lies on (edges / corners: all of them), homogeneously; an
earlier boundary condition that already constrains a component wins (AffineConstraints keeps the
first line). The reference's slip tests run on gmsh cylinder meshes (out of scope), so parity is
pinned by the oracle's restatement of those semantics only (no reference golden).

CPU: the oracle's constrained components equal an independent lattice-index construction; the
product's Dirichlet builder (softx_2020_200_amd.problem) equals the oracle's.
GPU: residual / diagonal / J.v of the brick kernels (Q1, Q2) and of the general cell kernel (2D)
equal the oracle's with slip walls (1e-12), and the device Newton reaches the oracle's solution."""
import numpy as np
import pytest

from oracle.oracle import Oracle, StructuredProblem, newton_solve
import softx_2020_200_amd as sx
from softx_2020_200_amd.problem import dirichlet_from_bcs

SEED = 20200200
TOL = 1e-12


def lid(X):
    v = np.zeros((X.shape[0], X.shape[1]))
    v[:, 0] = 1.0 - X[:, 0] ** 2
    return v


BC_LISTS = {
    "all_slip_colorized": (True, [("slip", b, None) for b in range(6)]),
    "all_slip_id0": (False, [("slip", 0, None)]),
    "lid_first": (True, [("function", 3, lid)] + [("slip", b, None) for b in (0, 1, 2, 4, 5)]),
    "lid_last": (True, [("slip", b, None) for b in (0, 1, 2, 4, 5)] + [("function", 3, lid)]),
    "mixed": (True, [("noslip", 2, None), ("slip", 0, None), ("slip", 1, None), ("function", 3, lid),
                     ("slip", 4, None), ("noslip", 5, None)]),
}


def expected_components(p, colorize, bcs):
    """Independent construction on lattice indices: {dof: value} with the first-wins rule."""
    dim, nx = p.dim, p.k * p.n + 1
    idx = np.indices((nx,) * dim).reshape(dim, -1)[::-1].T
    X = p.lo + idx * (p.hi - p.lo) / (nx - 1)
    out = {}
    for typ, bid, f in bcs:
        for node in range(idx.shape[0]):
            faces = []
            for d in range(dim):
                if idx[node, d] == 0 and (2 * d if colorize else 0) == bid:
                    faces.append(d)
                if idx[node, d] == nx - 1 and (2 * d + 1 if colorize else 0) == bid:
                    faces.append(d)
            if not faces:
                continue
            comps = sorted(set(faces)) if typ == "slip" else range(dim)
            val = f(X[node:node + 1])[0] if typ == "function" else np.zeros(dim)
            for c in comps:
                out.setdefault(node * dim + c, float(val[c]))
    return out


@pytest.mark.parametrize("name", list(BC_LISTS))
@pytest.mark.parametrize("k", [1, 2])
def test_oracle_slip_components(name, k):
    colorize, bcs = BC_LISTS[name]
    p = StructuredProblem(3, 3, k=k, colorize=colorize)
    p.set_dirichlet(bcs)
    exp = expected_components(p, colorize, bcs)
    assert set(p.dirichlet) == set(exp)
    assert all(abs(p.dirichlet[d] - exp[d]) < 1e-15 for d in exp)
    assert set(np.nonzero(p.constrained)[0].tolist()) == set(exp)
    if name.startswith("all_slip"):  # face interiors: one component; edges: two; corners: three
        per_node = np.bincount(np.array(sorted(exp)) // 3, minlength=p.n_vnodes)
        assert per_node.max() == 3 and (per_node == 1).sum() == 6 * (k * 3 - 1) ** 2


@pytest.mark.parametrize("name", list(BC_LISTS))
def test_product_slip_matches_oracle(name):
    colorize, bcs = BC_LISTS[name]
    n, k = 4, 2
    m = sx.hyper_cube(3, n, k, k, -1.0, 1.0)
    mask, dofs, vals = dirichlet_from_bcs(m, n, -1.0, 1.0, colorize, bcs)
    p = StructuredProblem(3, n, k=k, colorize=colorize)
    p.set_dirichlet(bcs)
    assert sorted(dofs.tolist()) == sorted(p.dirichlet)
    got = dict(zip(dofs.tolist(), vals.tolist()))
    assert all(abs(got[d] - p.dirichlet[d]) < 1e-15 for d in got)
    comp = np.zeros((m["n_vnodes"], 3), dtype=bool)
    comp.reshape(-1)[dofs] = True
    assert np.array_equal(mask, (comp * np.array([1, 2, 4])).sum(1).astype(np.uint8))


def _morton_slip_problem(n, k, scheme, nu, name):
    colorize, bcs = BC_LISTS[name]
    p = StructuredProblem(3, n, k=k, kp=k, viscosity=nu, scheme=scheme, time_steps=(0.01, 0.013, 0.011, 0.009),
                          colorize=colorize)
    m = sx.hyper_cube(3, n, k, k, -1.0, 1.0)
    p.cell_vnodes = np.ascontiguousarray(m["cell_vnodes"])
    p.cell_pnodes = np.ascontiguousarray(m["cell_pnodes"])
    p.cell_x0 = np.ascontiguousarray(m["cell_x0"])
    p.cell_h = np.ascontiguousarray(m["cell_h"])
    p.set_dirichlet(bcs)
    p.set_force(lambda X: np.stack([np.sin(X[:, 0] + 2 * X[:, 1]), np.cos(X[:, 2]), X[:, 0] * X[:, 1]], 1))
    return p


@pytest.mark.gpu
@pytest.mark.parametrize("case", [(4, 2, "bdf2", 0.01, "mixed"), (4, 1, "steady", 1.0, "all_slip_colorized"),
                                  (2, 2, "bdf1", 0.1, "all_slip_id0"), (4, 2, "sdirk2_2", 0.05, "lid_last")],
                         ids=lambda c: "n%d_Q%d_%s_%s" % (c[0], c[1], c[2], c[4]))
def test_slip_brick_kernels_vs_oracle(case):
    from tests.gpu_util import context_for, cuda, relerr
    p = _morton_slip_problem(*case)
    rng = np.random.default_rng(SEED)
    u, u1, u2, u3, v = (rng.uniform(-1, 1, p.n_dofs) for _ in range(5))
    ctx = context_for(p)
    assert ctx.uses_brick_kernels
    ctx.set_state(cuda(u), cuda(u1), cuda(u2), cuda(u3))
    orc = Oracle(p)
    assert relerr(ctx.residual().cpu().numpy(), orc.residual(u, u1, u2, u3)) < TOL
    assert relerr(ctx.jacobian_diagonal().cpu().numpy(), orc.jacobian_diagonal(u, u1, u2, u3)) < TOL
    assert relerr(ctx.jacobian_apply(cuda(v)).cpu().numpy(), orc.jacobian_apply(u, v, u1, u2, u3)) < TOL


@pytest.mark.gpu
def test_slip_newton_2d_cell_kernel():
    """2D Q2-Q1 cavity: slip side walls and bottom, parabolic lid (first-wins at the lid corners);
    device Newton + GMRES(Jacobi) == the oracle's exact-solve Newton."""
    from tests.gpu_util import context_for, cuda

    def lid2(X):
        v = np.zeros((X.shape[0], 2))
        v[:, 0] = 1.0 - X[:, 0] ** 2
        return v
    p = StructuredProblem(2, 8, k=2, kp=1, viscosity=0.05, colorize=True)
    p.set_dirichlet([("function", 3, lid2), ("slip", 0, None), ("slip", 1, None), ("slip", 2, None)])
    x_ref, its, res = newton_solve(p, tol=1e-10)
    ctx = context_for(p)
    assert not ctx.uses_brick_kernels
    x = cuda(p.apply_nonzero_constraints(np.zeros(p.n_dofs)))
    st = ctx.newton(x, tolerance=1e-10, max_iterations=12, lin_max_iterations=4000, restart=200,
                    relative_residual=1e-11, minimum_residual=1e-14)
    assert st["final_residual"] < 1e-10, st
    xs = x.cpu().numpy()
    nv = 2 * p.n_vnodes
    assert np.abs(xs[:nv] - x_ref[:nv]).max() < 1e-8
    # the slip walls carry tangential flow: zero normal component only
    X = p.vnode_coords()
    left = np.nonzero(np.abs(X[:, 0] + 1) < 1e-12)[0]
    inner = left[(np.abs(X[left, 1]) < 0.9)]
    assert np.abs(xs[2 * inner]).max() == 0.0 and np.abs(xs[2 * inner + 1]).max() > 1e-4


def test_slip_normal_sets_edges_and_corners():
    """compute_no_normal_flux_constraints at edges / corners (gls_navier_stokes.cc:100-110): the
    face normals meeting at a node are grouped by direction and constrain as many components as
    independent directions meet -- box corners all components (2D: 2, 3D: 3), 3D box edges two, face
    nodes one (the axis normal); a smooth curved wall (hyper_shell, MappingQ2) one normal per node,
    equal to the averaged node normal of gls_fe_space_boundary_normals."""
    from softx_2020_200_amd.native import UMesh
    for dim, k in ((2, 2), (3, 1)):
        m = UMesh(dim, "hyper_cube", "-1 : 1 : false")
        m.refine_global(2)
        h = m.fe_space_handle(k, k)
        X = h.data["vnode_x"].reshape(-1, dim)
        cnt, nrm = h.boundary_normal_sets(0)
        on = (np.abs(np.abs(X) - 1) < 1e-12).sum(1)  # number of box faces the node lies on
        assert np.array_equal(cnt, on), (dim, np.unique(cnt), np.unique(on))
        one = on == 1
        n0 = nrm[one, 0]
        assert np.allclose(np.abs(n0).max(1), 1) and np.allclose(np.abs(n0).sum(1), 1)  # axis normals
        ax = np.argmax(np.abs(n0), 1)
        assert np.allclose(n0[np.arange(len(ax)), ax], np.sign(X[one][np.arange(len(ax)), ax]))
    m = UMesh(2, "hyper_shell", "0, 0 : 0.25 : 1 : 4 : true")
    m.refine_global(2)
    h = m.fe_space_handle(2, 2, qmapping_all=True)
    for bid in (0, 1):
        cnt, nrm = h.boundary_normal_sets(bid)
        avg = h.boundary_normals(bid)
        on = np.abs(avg).sum(1) > 0
        assert on.any() and np.array_equal(cnt[on], np.ones(on.sum(), np.int32)) and not cnt[~on].any()
        assert np.allclose(nrm[on, 0], avg[on], atol=1e-12)
