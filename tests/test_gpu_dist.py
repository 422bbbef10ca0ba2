"""Multi-rank GPU path through the C-ABI (gls_dist_attach): 2 ranks on the box's one GPU,
exchange via torch.distributed gloo (host-staged; the bench uses nccl = RCCL). The distributed
residual, J.v, diagonal and a full Newton/GMRES solve must match the single-rank results."""
import os

import numpy as np
import pytest


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist

    import softx_2020_200_amd as sx
    from softx_2020_200_amd.dist import DistributedProblem, dist_import, local_vector, owned_global_dofs
    from softx_2020_200_amd.problem import build_context, dirichlet_from_bcs
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        n = 4
        m = sx.hyper_cube(3, n, 2, 2)
        bcs = [("noslip", b, None) for b in (0, 1, 2, 4, 5)] + [("function", 3, (1.0, 0.0, 0.0))]
        mask, ddofs, dvals = dirichlet_from_bcs(m, n, -1.0, 1.0, True, bcs)
        ts = (0.01, 0.012, 0.01, 0.01)
        # single-rank reference (same process, same GPU)
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
        d_g = g.jacobian_diagonal().cpu().numpy()
        # distributed
        dp = DistributedProblem(m, rank, world, "cuda", viscosity=0.05, vnode_mask=mask, dirichlet=(ddofs, dvals),
                                backend="gloo")
        c = dp.ctx
        c.set_time("bdf2", ts)
        lv = lambda a: cu(local_vector(dp.plan, a, m["n_vnodes"]))
        U, U1, U2, V = lv(u), lv(u1), lv(u2), lv(v)
        dist_import(c, U1)
        dist_import(c, U2)
        c.set_state(U, U1, U2)
        loc, glo = owned_global_dofs(dp.plan, m["n_vnodes"])
        rel = lambda a, b: float(np.abs(a - b).max() / np.abs(b).max())
        errs = {}
        errs["res"] = rel(c.residual().cpu().numpy()[loc], r_g[glo])
        errs["diag"] = rel(c.jacobian_diagonal().cpu().numpy()[loc], d_g[glo])
        errs["jv"] = rel(c.jacobian_apply(V).cpu().numpy()[loc], jv_g[glo])
        # Newton: one BDF2 step from u1
        x_g = cu(u1.copy())
        x_g[ddofs] = cu(dvals)
        stg = g.newton(x_g, cu(u1), cu(u2), tolerance=1e-9, max_iterations=6, lin_max_iterations=400, restart=60,
                       relative_residual=1e-6, minimum_residual=1e-13)
        x0 = u1.copy()
        x0[ddofs] = dvals
        X = lv(x0)
        std = c.newton(X, U1, U2, tolerance=1e-9, max_iterations=6, lin_max_iterations=400, restart=60,
                       relative_residual=1e-6, minimum_residual=1e-13)
        xg = x_g.cpu().numpy()
        xd = X.cpu().numpy()[loc]
        nvel = 3 * m["n_vnodes"]
        velmask = glo < nvel
        errs["newton_u"] = float(np.abs(xd[velmask] - xg[glo][velmask]).max())
        errs["newton_res"] = (stg["final_residual"], std["final_residual"])
        errs["lin_its"] = (stg["linear_iterations"], std["linear_iterations"])
        q.put((rank, errs))
    except Exception as e:  # report instead of hanging the parent
        import traceback
        traceback.print_exc()
        q.put((rank, {"error": repr(e)}))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_two_ranks_one_gpu_matches_single_rank():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29700 + os.getpid() % 500
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(2)]
    for p in procs:
        p.join(timeout=60)
    for rank, e in res:
        assert "error" not in e, e
        assert e["res"] < 1e-12 and e["jv"] < 1e-12 and e["diag"] < 1e-12, (rank, e)
        assert e["newton_res"][1] < 1e-9, (rank, e)
        assert e["newton_u"] < 1e-7, (rank, e)
