"""In-library RCCL transport (gls_rccl_create / gls_dist_attach_rccl) on the box's one GPU: a
single-rank communicator (RCCL refuses two ranks on one device, so the multi-rank exchange runs on
the driver's 8-GPU node). The rank's context goes through the distributed code path -- owned-DoF
dot products reduced with ncclAllReduce on the context stream -- and must reproduce the plain
context's residual, J.v and Newton/GMRES solve."""
import numpy as np
import pytest


@pytest.mark.gpu
def test_single_rank_rccl_matches_plain_context():
    import torch

    import softx_2020_200_amd as sx
    from softx_2020_200_amd.dist import DistributedProblem, local_vector
    from softx_2020_200_amd.problem import build_context, dirichlet_from_bcs
    n = 4
    m = sx.hyper_cube(3, n, 2, 2)
    bcs = [("noslip", b, None) for b in (0, 1, 2, 4, 5)] + [("function", 3, (1.0, 0.0, 0.0))]
    mask, ddofs, dvals = dirichlet_from_bcs(m, n, -1.0, 1.0, True, bcs)
    ts = (0.01, 0.012, 0.01, 0.01)
    g = build_context(m, viscosity=0.05, vnode_mask=mask)
    g.set_time("bdf2", ts)
    g.set_dirichlet(ddofs, dvals)
    N = g.n_dofs
    rng = np.random.default_rng(20200200)
    u, u1, u2, v = (rng.uniform(-1, 1, N) for _ in range(4))
    u[ddofs] = dvals
    cu = lambda a: torch.tensor(a, dtype=torch.float64, device="cuda")
    g.set_state(cu(u), cu(u1), cu(u2))
    r_g = g.residual().cpu().numpy()
    jv_g = g.jacobian_apply(cu(v)).cpu().numpy()
    dp = DistributedProblem(m, 0, 1, "cuda", viscosity=0.05, vnode_mask=mask, dirichlet=(ddofs, dvals), impl="native")
    assert dp.exchanger is None
    c = dp.ctx
    c.set_time("bdf2", ts)
    lv = lambda a: cu(local_vector(dp.plan, a, m["n_vnodes"]))
    c.set_state(lv(u), lv(u1), lv(u2))
    back = lambda x: x  # one rank: the local numbering is the global one restricted to owned nodes
    l2g = dp.plan["local_to_global"]
    nl = l2g.shape[0]
    def to_global(loc):
        out = np.zeros(N)
        nv = m["n_vnodes"]
        out[(3 * l2g[:, None] + np.arange(3)[None, :]).ravel()] = loc[:3 * nl]
        out[3 * nv + l2g] = loc[3 * nl:]
        return out
    rel = lambda a, b: float(np.abs(a - b).max() / np.abs(b).max())
    assert rel(to_global(c.residual().cpu().numpy()), r_g) < 1e-12
    assert rel(to_global(c.jacobian_apply(lv(v)).cpu().numpy()), jv_g) < 1e-12
    # Newton/GMRES: every Gram-Schmidt dot goes through ncclAllReduce
    x_g = cu(u1.copy())
    x_g[ddofs] = cu(dvals)
    stg = g.newton(x_g, cu(u1), cu(u2), tolerance=1e-9, max_iterations=6, lin_max_iterations=400, restart=60,
                   relative_residual=1e-6, minimum_residual=1e-13)
    x0 = u1.copy()
    x0[ddofs] = dvals
    x_d = lv(x0)
    std = c.newton(x_d, lv(u1), lv(u2), tolerance=1e-9, max_iterations=6, lin_max_iterations=400, restart=60,
                   relative_residual=1e-6, minimum_residual=1e-13)
    assert std["newton_iterations"] == stg["newton_iterations"]
    assert abs(std["linear_iterations"] - stg["linear_iterations"]) <= 1
    nvd = 3 * m["n_vnodes"]
    assert np.abs(to_global(x_d.cpu().numpy())[:nvd] - x_g.cpu().numpy()[:nvd]).max() < 1e-8
