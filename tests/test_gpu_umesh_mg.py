"""GPU: the geometric multigrid V-cycle on the refinement hierarchy of adapted unstructured / curved meshes
(gls_umesh_coarsen_to + gls_fe_space_mg_transfer levels, gls_mg_attach_transfers; MappingQ per-cell
kernels on every level, hanging-node lines) as the GMRES preconditioner of the device Newton. A linearized
solve (the Newton step at a smooth state) reaches the Jacobi-preconditioned GMRES's solution (1e-6 relative, both at residual 1e-11) in
fewer GMRES iterations; the level operators are the per-cell ones the oracle pins at 1e-12
(tests/test_gpu_uforest.py). Parity pinned by the oracle
only (the reference holds no multigrid)."""
import numpy as np
import pytest

from oracle.oracle import MappedProblem
from gpu_util import context_for, cuda
from tests.test_gpu_uforest import dof_lines
from tests.test_uforest import CASES, make_mesh, random_adapt


def mapped_level(sp, nu):
    dim = sp["dim"]
    p = MappedProblem(sp, viscosity=nu, scheme="bdf1", time_steps=(0.05, 0.05, 0.05, 0.05))
    if sp["vhang"] or sp["phang"]:
        lines = dof_lines(sp)
        p.set_hanging(*lines)
        p.hang_lines = lines
    bids = int(np.bitwise_or.reduce(sp["vnode_bid"].astype(np.int64)))
    p.set_dirichlet([("noslip", b, None) for b in range(32) if (bids >> b) & 1])  # enclosed flow
    p.set_force(lambda X: np.stack([np.sin(X[:, 0] + 2 * X[:, 1])] + [np.cos(X[:, d]) for d in range(1, dim)], 1))
    return p


@pytest.mark.gpu
@pytest.mark.parametrize("name,dim,spec,flat", [c for c in CASES if c[0] in ("shell", "cylshell", "rect3d")],
                         ids=["shell", "rect3d", "cylshell"])
@pytest.mark.parametrize("k,kp,smoother", [(1, 1, "jacobi"), (2, 2, "jacobi"), (2, 1, "ilu")])
def test_umesh_multigrid_linear_solve(name, dim, spec, flat, k, kp, smoother):
    m = make_mesh(dim, spec)
    m.refine_global(1)
    random_adapt(m, 2 if dim == 2 else 1, seed=5, k=k)
    hf = m.fe_space_handle(k, kp, qmapping_all=True)
    L = int(hf.data["cell_level"].max())
    handles = [hf] + [m.coarsen_to(L - l).fe_space_handle(k, kp, qmapping_all=True) for l in range(1, L + 1)]
    probs = [mapped_level(h.data, 0.1) for h in handles]
    xfer = [handles[l].mg_transfer_from(handles[l + 1]) for l in range(L)]
    p = probs[0]
    # one linearized solve at a smooth state (J x = R(u), the Newton step): the V-cycle-preconditioned and
    # the Jacobi-preconditioned GMRES reach the same x; the operators themselves equal the oracle's
    # (tests/test_gpu_uforest.py::test_adapted_mapped_operators_match_oracle, 1e-12)
    Xv = handles[0].data["vnode_x"]
    u = np.concatenate([np.stack([np.sin(Xv[:, 0] + Xv[:, d]) for d in range(dim)], 1).reshape(-1),
                        np.cos(handles[0].data["pnode_x"][:, 0])])
    p.apply_nonzero_constraints(u)
    out = {}
    for mg in (False, True):
        ctxs = [context_for(q) for q in (probs if mg else probs[:1])]
        if mg:
            sw = 2 if smoother == "jacobi" else 1
            ctxs[0].attach_multigrid_transfers(ctxs[1:], xfer, pre_smooth=sw, post_smooth=sw, omega=0.6, coarse_direct=1,
                                               smoother=smoother)
        U, U1 = cuda(u), cuda(np.zeros(p.n_dofs))
        ctxs[0].apply_dirichlet(U)
        ctxs[0].set_state(U, U1)
        rhs = ctxs[0].residual()
        x, its, res, ok = ctxs[0].solve_linear(rhs, ctxs[0].zeros(), max_iterations=5000, restart=200,
                                               relative_residual=1e-11, minimum_residual=1e-300, true_residual=True)
        out[mg] = (x.cpu().numpy(), its)
        assert ok and res <= 1e-11 * float(rhs.norm()) * 1.01, (mg, its, res)
    nvd = dim * p.n_vnodes
    # both at rel. residual 1e-11; the difference is that times the conditioning (~1e4 on the shells)
    assert np.abs(out[True][0][:nvd] - out[False][0][:nvd]).max() < 1e-6 * max(1.0, np.abs(out[False][0][:nvd]).max())
    its_mg, its_j = out[True][1], out[False][1]
    print("umesh GMG %s Q%dQ%d %s: %d levels %s DoFs, GMRES its %d (Jacobi %d)" % (name, k, kp, smoother, len(probs),
                                                                           [q.n_dofs for q in probs], its_mg, its_j))
    assert its_mg * 2 < its_j, (its_mg, its_j)


@pytest.mark.gpu
def test_large_coarsest_level_fp32_lu(monkeypatch, capfd):
    """a coarsest level above 8192 DoFs (the Q2-Q1 cylinder shell at refinement 2, 30816 DoFs, under its
    refinement-3 level): the FP32 unpivoted LU factored by the worker thread on the side stream, its check
    |A x - 1| / |1| taken (no pivoted fallback; the matrix kept banded in the probe CSR's Cuthill-McKee order), and
    the V-cycle-preconditioned GMRES converging"""
    from softx_2020_200_amd.native import UMesh
    m = UMesh(3, "cylinder_shell", "1 : 0.25 : 1 : 8 : 2")
    m.refine_global(3)
    hf = m.fe_space_handle(2, 1, qmapping_all=True)
    hc = m.coarsen_to(2).fe_space_handle(2, 1, qmapping_all=True)
    probs = [mapped_level(h.data, 1.0) for h in (hf, hc)]
    assert 8192 < probs[1].n_dofs <= 40000, probs[1].n_dofs
    p = probs[0]
    Xv = hf.data["vnode_x"]
    u = np.concatenate([np.stack([-Xv[:, 1], Xv[:, 0], 0.3 * np.sin(3 * Xv[:, 2])], 1).reshape(-1),
                        np.cos(hf.data["pnode_x"][:, 0])])
    p.apply_nonzero_constraints(u)
    ctxs = [context_for(q) for q in probs]
    monkeypatch.setenv("GLS_MG_VERBOSE", "1")
    ctxs[0].attach_multigrid_transfers(ctxs[1:], [hf.mg_transfer_from(hc)], pre_smooth=1, post_smooth=1, omega=0.6,
                                       coarse_direct=1, smoother="ilu")
    U = cuda(u)
    ctxs[0].apply_dirichlet(U)
    ctxs[0].set_state(U, cuda(np.zeros(p.n_dofs)))
    rhs = ctxs[0].residual()
    x, its, res, ok = ctxs[0].solve_linear(rhs, ctxs[0].zeros(), max_iterations=200, restart=50,
                                           relative_residual=1e-8, minimum_residual=1e-300, true_residual=True)
    monkeypatch.delenv("GLS_MG_VERBOSE")
    import ctypes
    ctypes.CDLL(None).fflush(None)  # the library's printf lines (stdout is a pipe under pytest: block-buffered)
    log = capfd.readouterr().out
    import re
    lines = [l for l in log.splitlines() if "unpivoted LU" in l and "check" in l]
    checks = [float(re.search(r"= ([0-9.eE+-]+)", l).group(1)) for l in lines]
    refined = ["refinement step" in l for l in lines]
    print("large coarsest level: %d DoFs, GMRES its %d, LU checks %s, refined %s" % (probs[1].n_dofs, its, checks, refined))
    assert ok and res <= 1e-8 * float(rhs.norm()) * 1.01, (its, res)
    # the check decides: below 1e-2 as it is, up to 0.5 with one refinement step, else pivoted
    assert checks and max(checks) < 0.5, log[-2000:]
    assert all(r == (c >= 1e-2) for r, c in zip(refined, checks)), lines
    assert "pivoted LU + inverse" not in log, log[-2000:]
    assert its <= 40, its
