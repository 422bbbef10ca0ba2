"""GPU: the geometric multigrid V-cycle on the octree refinement hierarchy (gls_mg_attach_transfers with
gls_octree_coarsen_to / gls_octree_mg_transfer levels) as the GMRES preconditioner of the
device Newton on multi-level adapted meshes with hanging-node constraints. The Newton solution equals the
oracle's direct Newton solution of the same condensed system (oracle/gls_oracle.c, 1e-8 on the velocity)
and the Jacobi-preconditioned device Newton's, in a fraction of the GMRES iterations. Parity is pinned by
the oracle only (no reference golden exists for these meshes)."""
import numpy as np
import pytest

import softx_2020_200_amd as sx
from oracle.oracle import StructuredProblem, newton_solve
from gpu_util import context_for, cuda
from test_octree_mg import adapted_tree


def level_problem(tree, k, kp, nu, scheme="steady"):
    mesh = tree.mesh(k, kp)
    dim = mesh["dim"]
    p = StructuredProblem.from_refined(mesh, viscosity=nu, scheme=scheme, time_steps=(0.05, 0.05, 0.05, 0.05))
    lines = sx.hanging_dof_lines(mesh)
    if len(lines[0]):
        p.set_hanging(*lines)
        p.hang_lines = lines
    p.set_dirichlet([("noslip", 0, None)])
    p.set_force(lambda X: np.stack([np.sin(X[:, 0] + 2 * X[:, 1]) * (1.0 + X[:, dim - 1]) for _ in range(dim)], 1))
    return p


def octree_hierarchy(tree, k, kp, nu, scheme="steady"):
    """level l = the forest coarsened to max_level - l, down to the uniform level-0 mesh"""
    L = tree.max_level
    trees = [tree.coarsen_to(L - l) for l in range(L + 1)]
    probs = [level_problem(t, k, kp, nu, scheme) for t in trees]
    xfer = []
    for l in range(L):
        hf, hc = trees[l].mesh_handle(k, kp), trees[l + 1].mesh_handle(k, kp)
        try:
            xfer.append(sx.octree_mg_transfer(hf, hc))
        finally:
            trees[l].free_mesh_handle(hf)
            trees[l + 1].free_mesh_handle(hc)
    return trees, probs, xfer


@pytest.mark.gpu
@pytest.mark.parametrize("dim,k,kp,steps,smoother", [(3, 1, 1, 3, "jacobi"), (3, 2, 2, 2, "jacobi"), (3, 2, 1, 2, "jacobi"),
                                                     (2, 2, 2, 4, "jacobi"), (2, 2, 1, 4, "jacobi"), (3, 2, 1, 2, "ilu"),
                                                     (2, 2, 1, 4, "ilu"), (3, 2, 2, 2, "ilu")])
def test_octree_multigrid_newton(dim, k, kp, steps, smoother):
    tree = adapted_tree(dim, 2, steps)
    assert tree.max_level >= 2
    trees, probs, xfer = octree_hierarchy(tree, k, kp, nu=0.1)
    p = probs[0]
    x_ref, _, _ = newton_solve(p, tol=1e-10)
    out = {}
    for mg in (False, True):
        ctxs = [context_for(q) for q in (probs if mg else probs[:1])]
        if mg:
            ctxs[0].attach_multigrid_transfers(ctxs[1:], xfer, pre_smooth=2 if smoother == "jacobi" else 1,
                                               post_smooth=2 if smoother == "jacobi" else 1, omega=0.6,
                                               coarse_direct=1, smoother=smoother)
        x = cuda(p.apply_nonzero_constraints(np.zeros(p.n_dofs)))
        st = ctxs[0].newton(x, tolerance=1e-10, max_iterations=10, lin_max_iterations=5000, restart=200,
                            relative_residual=1e-10, minimum_residual=1e-13)
        out[mg] = (x.cpu().numpy(), st)
        assert st["final_residual"] < 1e-10, (mg, st)
    nvd = dim * p.n_vnodes
    for mg in (False, True):
        assert np.abs(out[mg][0][:nvd] - x_ref[:nvd]).max() < 1e-8, mg
    its_mg, its_j = out[True][1]["linear_iterations"], out[False][1]["linear_iterations"]
    print("octree GMG %dD Q%dQ%d %s: %d levels, %d DoFs, GMRES its %d (Jacobi %d)" % (dim, k, kp, smoother, len(probs),
                                                                                    p.n_dofs, its_mg, its_j))
    # the V-cycle cuts the iterations > 4x, except Q2-Q1 under point-Jacobi smoothing (it sees only the PSPG
    # pressure diagonal): > 2x
    assert its_mg * (2 if (k != kp and smoother == "jacobi") else 4) < its_j, (out[True][1], out[False][1])


@pytest.mark.gpu
def test_octree_multigrid_transfers_match_host():
    """gls_mg_transfer on the attached octree hierarchy applies the host CSR (prolongation) and its
    transpose (restriction) exactly"""
    import scipy.sparse as sps
    tree = adapted_tree(3, 2, 2)
    trees, probs, xfer = octree_hierarchy(tree, 2, 2, nu=0.1)
    ctxs = [context_for(q) for q in probs]
    ctxs[0].attach_multigrid_transfers(ctxs[1:], xfer, coarse_direct=1)
    rng = np.random.default_rng(7)
    for l, (off, col, w, inj) in enumerate(xfer):
        nf, nc = probs[l].n_dofs, probs[l + 1].n_dofs
        P = sps.csr_matrix((w, col, off), shape=(nf, nc))
        xc, xf = rng.normal(size=nc), rng.normal(size=nf)
        yf = ctxs[0].mg_transfer(l, 1, cuda(xc), cuda(np.zeros(nf)))
        yc = ctxs[0].mg_transfer(l, 0, cuda(xf), cuda(np.zeros(nc)))
        assert np.abs(yf.cpu().numpy() - P @ xc).max() < 1e-13 * np.abs(P @ xc).max()
        assert np.abs(yc.cpu().numpy() - P.T @ xf).max() < 1e-13 * np.abs(P.T @ xf).max()


@pytest.mark.gpu
def test_octree_multigrid_mixed_precision():
    """the levels' forest bricks smooth with the FP32 pencil J.v (gls_mg_params.mixed_precision): the outer FP64
    Newton / GMRES reach the oracle's solution (1e-8), iterations within a few of the FP64 V-cycle's"""
    tree = adapted_tree(3, 2, 2)
    trees, probs, xfer = octree_hierarchy(tree, 2, 2, nu=0.1)
    p = probs[0]
    x_ref, _, _ = newton_solve(p, tol=1e-10)
    its = {}
    for mp in (0, 1):
        ctxs = [context_for(q) for q in probs]
        assert ctxs[0].forest_bricks() > 0
        ctxs[0].attach_multigrid_transfers(ctxs[1:], xfer, coarse_direct=1, mixed_precision=mp)
        x = cuda(p.apply_nonzero_constraints(np.zeros(p.n_dofs)))
        st = ctxs[0].newton(x, tolerance=1e-10, max_iterations=10, lin_max_iterations=5000, restart=200,
                            relative_residual=1e-10, minimum_residual=1e-13)
        assert st["final_residual"] < 1e-10, (mp, st)
        assert np.abs(x.cpu().numpy()[:3 * p.n_vnodes] - x_ref[:3 * p.n_vnodes]).max() < 1e-8, mp
        its[mp] = st["linear_iterations"]
    print("octree GMG FP64 / mixed: %d / %d GMRES its" % (its[0], its[1]))
    assert its[1] <= its[0] + 10
