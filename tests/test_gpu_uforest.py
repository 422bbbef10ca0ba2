"""GPU tests of local adaptation on unstructured / curved meshes (gls_umesh_prepare / adapt, hanging
lines of gls_umesh_fe_space, gls_kelly_estimate_mapped):
  * the device Kelly kernel == the host evaluation of the same face pieces (tests/test_uforest.py pins
    the pieces against the oracle's box Kelly), on adapted gmsh / curved meshes, 2D and 3D;
  * the per-cell HIP operators with MappingQ geometry and hanging-node condensation == the oracle's
    condensed operators (residual, J.v, nonzero-constraint distribution) at 1e-12."""
import numpy as np
import pytest

from oracle.oracle import MappedProblem, Oracle
from tests.gpu_util import context_for, cuda, relerr
from tests.test_uforest import CASES, _numpy_kelly, apply_lines, make_mesh, random_adapt


def dof_lines(sp):
    """node-level lines {node: [(master, w)]} -> DoF-level CSR (as gls_set_hanging takes them)"""
    dim, nv = sp["dim"], sp["n_vnodes"]
    dofs, offs, mas, ws = [], [0], [], []
    for nd, ln in sorted(sp["vhang"].items()):
        for c in range(dim):
            dofs.append(nd * dim + c)
            mas.extend(m * dim + c for m, _ in ln)
            ws.extend(w for _, w in ln)
            offs.append(len(mas))
    for nd, ln in sorted(sp["phang"].items()):
        dofs.append(dim * nv + nd)
        mas.extend(dim * nv + m for m, _ in ln)
        ws.extend(w for _, w in ln)
        offs.append(len(mas))
    return (np.array(dofs, np.int64), np.array(offs, np.int64), np.array(mas, np.int64), np.array(ws))


def adapted_space(name, dim, spec, k, kp, qall=True):
    m = make_mesh(dim, spec)
    m.refine_global(1)
    random_adapt(m, 2 if dim == 2 else 1, seed=5, k=k)
    return m, m.fe_space_handle(k, kp, qmapping_all=qall)


def continuous_field(sp, rng):
    dim, nv = sp["dim"], sp["n_vnodes"]
    x = rng.uniform(-1, 1, dim * nv + sp["n_pnodes"])
    v = x[:dim * nv].reshape(-1, dim)
    for c in range(dim):
        v[:, c] = apply_lines(v[:, c], sp["vhang"])
    x[:dim * nv] = v.reshape(-1)
    x[dim * nv:] = apply_lines(x[dim * nv:], sp["phang"])
    return x


@pytest.mark.gpu
@pytest.mark.parametrize("name,dim,spec,flat", CASES, ids=[c[0] for c in CASES])
@pytest.mark.parametrize("k,kp", [(1, 1), (2, 1)])
def test_mapped_kelly_kernel_matches_host(name, dim, spec, flat, k, kp):
    m, h = adapted_space(name, dim, spec, k, kp)
    sp = h.data
    faces = h.kelly_faces(k + 2)
    p = MappedProblem(sp, viscosity=0.1)
    p.set_dirichlet([("noslip", 0, None)])
    ctx = context_for(p)
    x = continuous_field(sp, np.random.default_rng(6))
    for variable in (0, 1):
        eta = ctx.kelly_estimate_mapped(cuda(x), variable, faces).cpu().numpy()
        ref = _numpy_kelly(sp, faces, x, variable, dim)
        assert relerr(eta, ref) < 1e-12, (variable, relerr(eta, ref))


@pytest.mark.gpu
@pytest.mark.parametrize("name,dim,spec,flat", CASES, ids=[c[0] for c in CASES])
@pytest.mark.parametrize("k,kp,scheme", [(1, 1, "bdf2"), (2, 1, "steady"), (2, 2, "bdf1")])
def test_adapted_mapped_operators_match_oracle(name, dim, spec, flat, k, kp, scheme):
    m, h = adapted_space(name, dim, spec, k, kp)
    sp = h.data
    p = MappedProblem(sp, viscosity=0.05, scheme=scheme, time_steps=(0.01, 0.012, 0.011, 0.01))
    lines = dof_lines(sp)
    p.set_hanging(*lines)
    p.hang_lines = lines
    p.set_dirichlet([("noslip", 0, None)])
    p.set_force(lambda X: np.stack([np.sin(X[:, 0] + 2 * X[:, 1])] + [np.cos(X[:, d]) for d in range(1, dim)], 1))
    rng = np.random.default_rng(20200200)
    u, u1, u2, v = (rng.uniform(-1, 1, p.n_dofs) for _ in range(4))
    p.apply_nonzero_constraints(u)
    orc = Oracle(p)
    ctx = context_for(p)
    ctx.set_state(cuda(u), cuda(u1), cuda(u2))
    assert relerr(ctx.residual().cpu().numpy(), orc.residual(u, u1, u2)) < 1e-12
    assert relerr(ctx.jacobian_apply(cuda(v)).cpu().numpy(), orc.jacobian_apply(u, v, u1, u2)) < 1e-12
    x = rng.uniform(-1, 1, p.n_dofs)
    X = cuda(x)
    ctx.apply_dirichlet(X)
    assert np.abs(X.cpu().numpy() - p.apply_nonzero_constraints(x.copy())).max() < 1e-14


@pytest.mark.gpu
def test_per_cell_operators_bitwise_reproducible():
    """The per-cell kernels scatter through per-cell element vectors summed in a fixed order
    (gather_element_vectors), so repeated evaluations are bitwise identical (no atomics)."""
    m, h = adapted_space("square", 2, CASES[0][2], 2, 1)
    sp = h.data
    p = MappedProblem(sp, viscosity=0.05, scheme="bdf1", time_steps=(0.01, 0.01, 0.01, 0.01))
    lines = dof_lines(sp)
    p.set_hanging(*lines)
    p.hang_lines = lines
    p.set_dirichlet([("noslip", 0, None)])
    rng = np.random.default_rng(8)
    u, u1, v = (rng.uniform(-1, 1, p.n_dofs) for _ in range(3))
    ctx = context_for(p)
    ctx.set_state(cuda(u), cuda(u1))
    r0, j0 = ctx.residual().cpu().numpy(), ctx.jacobian_apply(cuda(v)).cpu().numpy()
    for _ in range(3):
        assert np.array_equal(ctx.residual().cpu().numpy(), r0)
        assert np.array_equal(ctx.jacobian_apply(cuda(v)).cpu().numpy(), j0)


@pytest.mark.gpu
@pytest.mark.parametrize("name,k,kp", [("square", 1, 1), ("square", 2, 1), ("rect3d", 2, 1), ("cylshell", 1, 1)])
def test_ilu_probed_matrix_with_hanging_nodes(name, k, kp):
    """gls_ilu_attach on an adapted mapped mesh: the probed CSR (the condensed operator's pattern:
    hanging nodes replaced by their masters, hanging rows diagonal) == the oracle's assembled,
    hanging-condensed system matrix; ILU(0)-GMRES then solves the Newton step."""
    case = [c for c in CASES if c[0] == name][0]
    m, h = adapted_space(*case[:3], k, kp)
    sp = h.data
    p = MappedProblem(sp, viscosity=0.05, scheme="bdf1", time_steps=(0.05,) * 4)
    lines = dof_lines(sp)
    p.set_hanging(*lines)
    p.hang_lines = lines
    p.set_dirichlet([("noslip", 0, None)])
    rng = np.random.default_rng(3)
    u = p.apply_nonzero_constraints(rng.uniform(-1, 1, p.n_dofs))
    u1 = p.apply_nonzero_constraints(rng.uniform(-1, 1, p.n_dofs))
    A, _ = Oracle(p).matrix_and_rhs(u, u1)
    ctx = context_for(p)
    ctx.set_state(cuda(u), cuda(u1))
    nnz, nprobe = ctx.attach_ilu()
    M = ctx.ilu_matrix()
    A = A.tocsr()
    d = (M - A).tocsr()
    assert np.abs(d.data).max() <= 1e-12 * np.abs(A.data).max() if d.nnz else True
    rhs = ctx.residual()
    x, its, res, ok = ctx.solve_linear(rhs, None, max_iterations=400, restart=60, relative_residual=1e-10,
                                       minimum_residual=1e-14)
    assert ok and its < 400, (its, res)
