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


def _mg_worker(rank, world, port, q, replica=False):
    """Distributed multigrid (every level partitioned, nested rank boxes) vs the single-rank V-cycle:
    the preconditioned GMRES and one Newton step must agree (same iterations, same solution).
    replica: the bench's cycle -- 2 + 2 sweeps on 4^3 and an exact LU on 2^3 -- on one rank, and on N
    ranks the distributed levels down to 4^3 with that remainder run on a replica of the 4^3 level
    (gls_mg_set_coarse_replica)."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist

    import softx_2020_200_amd as sx
    from softx_2020_200_amd.dist import (DistributedProblem, attach_distributed_multigrid, dist_import,
                                         local_vector, multigrid_levels, owned_global_dofs)
    from softx_2020_200_amd.problem import CavityProblem, dirichlet_from_bcs
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        n, nu, ts = 8, 0.02, (0.01, 0.01, 0.01, 0.01)
        opts = dict(pre_smooth=1, post_smooth=1, omega=0.9, mixed_precision=True) if replica else {}
        if replica:
            single = CavityProblem(dim=3, n=n, k=2, viscosity=nu, multigrid=True, mg_coarsest=2,
                                   level_sweeps={-2: (2, 2)}, **opts)
        else:
            single = CavityProblem(dim=3, n=n, k=2, viscosity=nu, multigrid=True, mg_coarsest=4)
        g = single.ctx
        g.set_time("bdf2", ts)
        m = single.mesh
        N = g.n_dofs
        rng = np.random.default_rng(20200200 + 1)
        u1, u2, xt = (0.3 * rng.uniform(-1, 1, N) for _ in range(3))
        u1[single.dir_dofs] = single.dir_vals
        u2[single.dir_dofs] = single.dir_vals
        xt[single.dir_dofs] = 0.0
        cu = lambda a: torch.tensor(a, dtype=torch.float64, device="cuda")
        g.set_state(cu(u1), cu(u1), cu(u2))
        # consistent right-hand side (J has the constant-pressure null vector of the enclosed cavity)
        b = g.jacobian_apply(cu(xt)).cpu().numpy()
        xg, its_g, res_g, ok_g = g.solve_linear(cu(b), max_iterations=200, restart=30, relative_residual=1e-6)
        # distributed levels with the same boundary data
        bcs = [("noslip", bb, None) for bb in (0, 1, 2, 4, 5)] + [("function", 3, (1.0, 0.0, 0.0))]
        levels = []
        for mm_n in [n] + multigrid_levels(n, world, 4):
            mm = sx.hyper_cube(3, mm_n, 2, 2, -1.0, 1.0)
            mk, dd, dv = dirichlet_from_bcs(mm, mm_n, -1.0, 1.0, True, bcs)
            levels.append(DistributedProblem(mm, rank, world, "cuda", viscosity=nu, vnode_mask=mk, dirichlet=(dd, dv),
                                             backend="gloo"))
        if replica:
            assert len(levels) == len(single.levels)  # the 2^3 level lives in the replica
            rep = CavityProblem(dim=3, n=4, k=2, viscosity=nu, multigrid=True, mg_coarsest=2, pre_smooth=2,
                                post_smooth=2, omega=0.9, mixed_precision=True)
            attach_distributed_multigrid(levels, replica=rep, coarse_direct=-1, **opts)
        else:
            assert len(levels) == 1 + len(single.levels)
            attach_distributed_multigrid(levels)
        dp = levels[0]
        c = dp.ctx
        c.set_time("bdf2", ts)
        lv = lambda a: cu(local_vector(dp.plan, a, m["n_vnodes"]))
        U1, U2, B = lv(u1), lv(u2), lv(b)
        dist_import(c, U1)
        dist_import(c, U2)
        c.set_state(U1, U1, U2)
        xd, its_d, res_d, ok_d = c.solve_linear(B, max_iterations=200, restart=30, relative_residual=1e-6)
        loc, glo = owned_global_dofs(dp.plan, m["n_vnodes"])
        xgn = xg.cpu().numpy()
        vel = glo < 3 * m["n_vnodes"]  # pressure is determined up to a constant
        errs = {"lin_its": (its_g, its_d), "ok": (ok_g, ok_d),
                "x_rel": float(np.abs(xd.cpu().numpy()[loc][vel] - xgn[glo][vel]).max() / np.abs(xgn).max())}
        # one Newton step with the multigrid-preconditioned GMRES
        x_g = cu(u1.copy())
        stg = g.newton(x_g, cu(u1), cu(u2), tolerance=1e-30, max_iterations=1, lin_max_iterations=100,
                       relative_residual=1e-6)
        X = lv(u1.copy())
        std = c.newton(X, U1, U2, tolerance=1e-30, max_iterations=1, lin_max_iterations=100, relative_residual=1e-6)
        xs = x_g.cpu().numpy()
        errs["newton_lin_its"] = (stg["linear_iterations"], std["linear_iterations"])
        errs["newton_x"] = float(np.abs(X.cpu().numpy()[loc] - xs[glo]).max() / np.abs(xs).max())
        q.put((rank, errs))
    except Exception as e:
        import traceback
        traceback.print_exc()
        q.put((rank, {"error": repr(e)}))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("world,replica", [(2, False), (4, False), (2, True), (4, True)])
def test_distributed_multigrid_matches_single_rank(world, replica):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 30300 + 10 * world + 5 * int(replica) + os.getpid() % 400
    procs = [ctx.Process(target=_mg_worker, args=(r, world, port, q, replica)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    for rank, e in res:
        assert "error" not in e, e
        assert e["ok"] == (True, True), (rank, e)
        tol_its = 0 if replica else 1  # the replica's cycle is the one-rank cycle: identical counts
        assert abs(e["lin_its"][0] - e["lin_its"][1]) <= tol_its, (rank, e)
        assert e["x_rel"] < 1e-7, (rank, e)
        assert abs(e["newton_lin_its"][0] - e["newton_lin_its"][1]) <= tol_its, (rank, e)
        assert e["newton_x"] < 1e-7, (rank, e)


def _split_worker(rank, world, port, q):
    """The overlapped J.v's brick split (boundary bricks: a cell holds a ghost or exported node;
    interior bricks read no ghost value) on a real partition: with the callback transport and
    GLS_SPLIT_DIST=1 the J.v runs as interior + boundary subset launches after the import; it must be
    bitwise the single launch, and both must match the single-rank J.v."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist

    import softx_2020_200_amd as sx
    from softx_2020_200_amd.dist import DistributedProblem, dist_import, local_vector, owned_global_dofs
    from softx_2020_200_amd.problem import build_context, dirichlet_from_bcs
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        n = 8
        m = sx.hyper_cube(3, n, 2, 2)
        bcs = [("noslip", b, None) for b in (0, 1, 2, 4, 5)] + [("function", 3, (1.0, 0.0, 0.0))]
        mask, ddofs, dvals = dirichlet_from_bcs(m, n, -1.0, 1.0, True, bcs)
        ts = (0.01, 0.012, 0.01, 0.01)
        g = build_context(m, viscosity=0.05, vnode_mask=mask)
        g.set_time("bdf2", ts)
        N = g.n_dofs
        rng = np.random.default_rng(20200200 + 7)
        u, u1, u2, v = (rng.uniform(-1, 1, N) for _ in range(4))
        u[ddofs] = dvals
        cu = lambda a: torch.tensor(a, dtype=torch.float64, device="cuda")
        g.set_state(cu(u), cu(u1), cu(u2))
        jv_g = g.jacobian_apply(cu(v)).cpu().numpy()
        dp = DistributedProblem(m, rank, world, "cuda", viscosity=0.05, vnode_mask=mask, dirichlet=(ddofs, dvals),
                                backend="gloo")
        c = dp.ctx
        c.set_time("bdf2", ts)
        lv = lambda a: cu(local_vector(dp.plan, a, m["n_vnodes"]))
        U, U1, U2 = lv(u), lv(u1), lv(u2)
        dist_import(c, U1)
        dist_import(c, U2)
        c.set_state(U, U1, U2)
        plain = c.jacobian_apply(lv(v)).cpu().numpy()
        os.environ["GLS_SPLIT_DIST"] = "1"
        split = c.jacobian_apply(lv(v)).cpu().numpy()
        del os.environ["GLS_SPLIT_DIST"]
        loc, glo = owned_global_dofs(dp.plan, m["n_vnodes"])
        q.put((rank, {"bitwise": bool(np.array_equal(plain, split)),
                      "rel": float(np.abs(split[loc] - jv_g[glo]).max() / np.abs(jv_g).max())}))
    except Exception as e:
        import traceback
        traceback.print_exc()
        q.put((rank, {"error": repr(e)}))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 4])
def test_split_jv_on_partition_bitwise(world):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 31300 + 10 * world + os.getpid() % 400
    procs = [ctx.Process(target=_split_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    for rank, e in res:
        assert "error" not in e, e
        assert e["bitwise"] and e["rel"] < 1e-12, (rank, e)
