"""Row e2 + f1: the refinement-hierarchy multigrid across ranks (gls_mg_attach_replica). The fine level of an
adapted, curved unstructured mesh with hanging-node lines is partitioned over 2 / 3 / 4 ranks on the box's one GPU
(gls_gpart_* + gls_dist_attach_dofs, gloo ghost exchange); the coarser levels run on every rank as one
single-rank context with its own hierarchy (the replica), fed by the all-reduced restriction of the owned rows.
With Jacobi smoothing the distributed V-cycle is the single-rank one (the distributed diagonal and J.v equal the
single-rank ones on owned DoFs, tests/test_gpu_dist_general.py), so the linearized solve takes the same GMRES
iterations and reaches the same solution; with ILU smoothing the fine level becomes block-Jacobi ILU per rank
(the reference's Ifpack additive Schwarz, gls_navier_stokes.cc:1131-1176) and the iterations stay close.
Parity pinned by the single-rank hierarchy multigrid (tests/test_gpu_umesh_mg.py), whose level operators the
oracle pins at 1e-12 (the reference holds no geometric multigrid)."""
import os

import numpy as np
import pytest

SOLVE = dict(max_iterations=3000, restart=200, relative_residual=1e-10, minimum_residual=1e-300, true_residual=True)


def _levels(case):
    """(fine space dict for the partition, level problems fine -> coarsest, transfers, fine hanging lines, state)"""
    import softx_2020_200_amd as sx
    from tests.test_gpu_umesh_mg import mapped_level
    from tests.test_gpu_uforest import dof_lines
    from tests.test_uforest import CASES, make_mesh, random_adapt
    name, k, kp, smoother, two_level = case
    if name == "octree3d":  # adapted hyper_cube forest: affine per-cell levels; the ranks see its mapped form
        from tests.test_gpu_octree_mg import octree_hierarchy
        from tests.test_octree_mg import adapted_tree
        tree = adapted_tree(3, 2, 2)
        trees, probs, xfer = octree_hierarchy(tree, k, kp, nu=0.1)
        if two_level:
            raise ValueError("octree: full hierarchy only")
        mesh = trees[0].mesh(k, kp)
        space = dict(mesh, cell_support=np.ascontiguousarray(mesh["vnode_x"][mesh["cell_vnodes"]]))
        lines = sx.hanging_dof_lines(mesh)
        Xv, Xp, dim = mesh["vnode_x"], mesh["pnode_x"], 3
    else:
        _, dim, spec, _ = [c for c in CASES if c[0] == name][0]
        m = make_mesh(dim, spec)
        m.refine_global(1)
        random_adapt(m, 2 if dim == 2 else 1, seed=5, k=k)
        hf = m.fe_space_handle(k, kp, qmapping_all=True)
        L = L0 = int(hf.data["cell_level"].max())
        if two_level:  # fine + one coarser level: the replica is the coarsest, solved exactly on every rank
            L = 1
        handles = [hf] + [m.coarsen_to(L0 - l).fe_space_handle(k, kp, qmapping_all=True) for l in range(1, L + 1)]
        probs = [mapped_level(h.data, 0.1) for h in handles]
        xfer = [handles[l].mg_transfer_from(handles[l + 1]) for l in range(L)]
        space = handles[0].data
        lines = dof_lines(space) if (space["vhang"] or space["phang"]) else None
        Xv, Xp = space["vnode_x"], space["pnode_x"]
    u = np.concatenate([np.stack([np.sin(Xv[:, 0] + Xv[:, d]) for d in range(dim)], 1).reshape(-1), np.cos(Xp[:, 0])])
    probs[0].apply_nonzero_constraints(u)
    return space, probs, xfer, lines, u, dim


def _worker(rank, world, port, q, case):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist

    from softx_2020_200_amd.dist import DistributedGeneralProblem, attach_replica_multigrid, owned_dofs
    from tests.gpu_util import context_for, cuda, vnode_mask_of
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        smoother, two_level = case[3], case[4]
        space, probs, xfer, lines, u, dim = _levels(case)
        L = len(probs) - 1
        p = probs[0]
        sw = 2 if smoother == "jacobi" else 1
        mg = dict(pre_smooth=sw, post_smooth=sw, omega=0.6, smoother=smoother)

        def coarse_hierarchy(levels):
            ctxs = [context_for(q_) for q_ in levels]
            if len(ctxs) > 1:
                ctxs[0].attach_multigrid_transfers(ctxs[1:], xfer[L + 1 - len(levels):], coarse_direct=1, **mg)
            return ctxs

        out = {"levels": [q_.n_dofs for q_ in probs]}
        # single rank: the whole hierarchy on one context
        ctxs = coarse_hierarchy(probs)
        U = cuda(u)
        ctxs[0].apply_dirichlet(U)
        ctxs[0].set_state(U, cuda(np.zeros(p.n_dofs)))
        rhs = ctxs[0].residual()
        xs, its_s, res_s, ok_s = ctxs[0].solve_linear(rhs, ctxs[0].zeros(), **SOLVE)
        out["single"] = (its_s, ok_s, res_s / float(rhs.norm()))
        # ranks: fine level partitioned, levels 1..L replicated on every rank
        dirs = np.array(sorted(p.dirichlet), np.int64)
        dp = DistributedGeneralProblem(space, rank, world, "cuda", viscosity=0.1, vnode_mask=vnode_mask_of(p),
                                       dirichlet=(dirs, np.array([p.dirichlet[d] for d in dirs])), lines=lines,
                                       force_q=p.force_q)
        c = dp.ctx
        c.set_time(p.scheme, p.time_steps)
        replica = coarse_hierarchy(probs[1:])
        attach_replica_multigrid(dp, replica[0], xfer[0], coarse_direct=int(two_level), **mg)
        Ud = cuda(dp.local(u))
        c.apply_dirichlet(Ud)
        c.set_state(Ud, cuda(np.zeros(len(dp.plan["l2g_dofs"]))))
        rd = c.residual()
        loc, glo = owned_dofs(dp.plan)
        r_s = rhs.cpu().numpy()
        out["rhs_err"] = float(np.abs(rd.cpu().numpy()[loc] - r_s[glo]).max() / np.abs(r_s).max())
        # one V-cycle application: equal on the owned rows for the Jacobi smoother
        zs = ctxs[0].apply_preconditioner(rhs).cpu().numpy()
        zd = c.apply_preconditioner(rd).cpu().numpy()
        out["vcycle_err"] = float(np.abs(zd[loc] - zs[glo]).max() / np.abs(zs).max())
        xd, its_d, res_d, ok_d = c.solve_linear(rd, c.zeros(), **SOLVE)
        out["dist"] = (its_d, ok_d, res_d)
        nvd = dim * p.n_vnodes
        vel = glo < nvd
        xsn = xs.cpu().numpy()
        out["x_err"] = float(np.abs(xd.cpu().numpy()[loc][vel] - xsn[glo][vel]).max() / np.abs(xsn[:nvd]).max())
        out["n_ghost_recv"] = int(dp.plan["recv_off"][-1])
        q.put((rank, out))
    except Exception as e:
        import traceback
        traceback.print_exc()
        q.put((rank, {"error": repr(e)}))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3, 4])
@pytest.mark.parametrize("case", [("shell", 2, 2, "jacobi", False), ("cylshell", 2, 1, "jacobi", False),
                                  ("cylshell", 2, 1, "ilu", False), ("cylshell", 2, 1, "jacobi", True),
                                  ("octree3d", 2, 2, "jacobi", False)],
                         ids=["shell-q2q2-jacobi", "cylshell-q2q1-jacobi", "cylshell-q2q1-ilu", "cylshell-q2q1-two-level",
                              "octree3d-q2q2-jacobi"])
def test_hierarchy_multigrid_across_ranks_matches_single_rank(world, case):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 33100 + 17 * world + 5 * (hash(case) % 7) + os.getpid() % 300
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, case)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=400) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    for rank, e in res.items():
        assert "error" not in e, (rank, e)
    print(case, world, res[0])
    assert sum(e["n_ghost_recv"] for e in res.values()) > 0  # lowest-rank ownership: rank 0 may receive none
    for rank, e in res.items():
        assert e["rhs_err"] < 1e-12, (rank, e)
        its_s, ok_s, _ = e["single"]
        its_d, ok_d, _ = e["dist"]
        assert ok_s and ok_d, (rank, e)
        assert e["x_err"] < 1e-6, (rank, e)
        if case[3] == "jacobi":
            assert e["vcycle_err"] < 1e-10, (rank, e)
            assert abs(its_d - its_s) <= 1, (rank, e)
        else:
            assert its_d <= 2 * its_s + 5, (rank, e)
