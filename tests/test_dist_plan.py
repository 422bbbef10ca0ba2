"""Multi-GPU path, host side (CPU, gloo): the C++ partition plan (softx_2020_200_amd/csrc/gls_dist.cpp)
and the ghost-exchange protocol, checked end to end with the oracle as the per-rank compute:
sum over ranks of (local residual, export-added to owners) == the global residual."""
import os

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

import softx_2020_200_amd as sx
from softx_2020_200_amd.dist import local_vector, owned_global_dofs, partition



def _box(l2g, n1d):
    x, y, z = l2g % n1d, (l2g // n1d) % n1d, l2g // (n1d * n1d)
    lo = np.array([x.min(), y.min(), z.min()])
    dims = np.array([x.max(), y.max(), z.max()]) - lo + 1
    return lo, dims, int(np.prod(dims)) == l2g.size


@pytest.mark.parametrize("world", [2, 4, 8])
def test_partitions_are_nested_boxes(world):
    """Distributed multigrid precondition (gls_set_lattice / gls_mg_attach): on 2^j ranks every
    rank's nodes fill a box of the node lattice, and the rank's box on the n/2 mesh is every
    second node of its box on the n mesh (coarse cells = parents of the fine cells)."""
    from softx_2020_200_amd.dist import multigrid_levels
    n, k = 8, 2
    levels = [n] + multigrid_levels(n, world, 2)
    assert levels[1] == 4
    for r in range(world):
        boxes = []
        for m in levels:
            mesh = sx.hyper_cube(3, m, k, k)
            p = partition(mesh["cell_vnodes"], mesh["n_vnodes"], r, world)
            lo, dims, full = _box(p["local_to_global"], k * m + 1)
            assert full, (world, r, m)
            boxes.append((lo, dims))
        for (flo, fd), (clo, cd) in zip(boxes[:-1], boxes[1:]):
            assert np.array_equal(flo, 2 * clo) and np.array_equal(fd, 2 * cd - 1)


@pytest.mark.parametrize("world", [2, 3, 4, 8])
def test_partition_invariants(world):
    m = sx.hyper_cube(3, 4, 2, 2)
    cv, nv = m["cell_vnodes"], m["n_vnodes"]
    plans = [partition(cv, nv, r, world) for r in range(world)]
    owned = np.concatenate([p["local_to_global"][:p["n_owned"]] for p in plans])
    assert np.array_equal(np.sort(owned), np.arange(nv))          # every node owned exactly once
    assert sum(p["cell_end"] - p["cell_begin"] for p in plans) == m["n_cells"]
    for r, p in enumerate(plans):
        assert (p["cell_end"] - p["cell_begin"]) % 8 == 0            # whole bricks
        l2g = p["local_to_global"]
        assert np.array_equal(l2g[p["local_cells"]], cv[p["cell_begin"]:p["cell_end"]])
        for i, s in enumerate(p["nbrs"]):
            # my recv list from s == s's send list to me (same global ids, same order)
            q = plans[s]
            j = list(q["nbrs"]).index(r)
            mine = l2g[p["recv_nodes"][p["recv_off"][i]:p["recv_off"][i + 1]]]
            theirs = q["local_to_global"][q["send_nodes"][q["send_off"][j]:q["send_off"][j + 1]]]
            assert np.array_equal(mine, theirs)
            mine_s = l2g[p["send_nodes"][p["send_off"][i]:p["send_off"][i + 1]]]
            theirs_r = q["local_to_global"][q["recv_nodes"][q["recv_off"][j]:q["recv_off"][j + 1]]]
            assert np.array_equal(mine_s, theirs_r)
        # ghosts are owned by lower ranks only (lowest-rank ownership)
        gh = l2g[p["n_owned"]:]
        for other in range(r, world):
            po = plans[other]
            assert not np.intersect1d(gh, po["local_to_global"][:po["n_owned"]]).size or other < r


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    from oracle.oracle import Oracle, StructuredProblem
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        m = sx.hyper_cube(3, 4, 2, 2)
        p = StructuredProblem(3, 4, k=2, viscosity=0.05, scheme="bdf1", time_steps=(0.01,) * 4)
        p.cell_vnodes, p.cell_x0, p.cell_h = m["cell_vnodes"], m["cell_x0"], m["cell_h"]
        p.cell_pnodes = m["cell_pnodes"]
        p.set_dirichlet([("noslip", 0, None)])
        rng = np.random.default_rng(20200200)
        u, u1 = rng.uniform(-1, 1, p.n_dofs), rng.uniform(-1, 1, p.n_dofs)
        r_glob = Oracle(p).residual(u, u1)
        plan = partition(m["cell_vnodes"], m["n_vnodes"], rank, world)
        # rank-local problem for the oracle (local mesh, local vectors with ghost values)
        l2g = plan["local_to_global"]
        nl = len(l2g)
        cb, ce = plan["cell_begin"], plan["cell_end"]
        pl = StructuredProblem(3, 4, k=2, viscosity=0.05, scheme="bdf1", time_steps=(0.01,) * 4)
        pl.cell_vnodes = plan["local_cells"]
        pl.cell_pnodes = plan["local_cells"]
        pl.cell_x0, pl.cell_h = m["cell_x0"][cb:ce], m["cell_h"][cb:ce]
        pl.n_vnodes = pl.n_pnodes = nl
        pl.n_dofs = 4 * nl
        pl.constrained = local_vector(plan, p.constrained.astype(float), m["n_vnodes"]).astype(np.uint8)
        r_loc = Oracle(pl).residual(local_vector(plan, u, m["n_vnodes"]), local_vector(plan, u1, m["n_vnodes"]))
        # export-add: ghost contributions -> owners (the protocol of gls_dist_attach, phase 1)
        y = torch.tensor(r_loc)
        pieces = []
        for i, nbr in enumerate(plan["nbrs"]):
            rn = plan["recv_nodes"][plan["recv_off"][i]:plan["recv_off"][i + 1]]
            sn = plan["send_nodes"][plan["send_off"][i]:plan["send_off"][i + 1]]
            pieces.append((int(nbr), rn, sn))
        reqs, bufs = [], []
        for nbr, rn, sn in pieces:
            if len(rn):
                out = torch.tensor(np.stack([r_loc[3 * rn], r_loc[3 * rn + 1], r_loc[3 * rn + 2], r_loc[3 * nl + rn]], 1)
                                   .reshape(-1).copy())
                reqs.append(dist.isend(out, nbr))
                bufs.append(out)
            if len(sn):
                inc = torch.zeros(4 * len(sn), dtype=torch.float64)
                reqs.append(dist.irecv(inc, nbr))
                bufs.append((sn, inc))
        for w in reqs:
            w.wait()
        for b in bufs:
            if isinstance(b, tuple):
                sn, inc = b
                inc = inc.numpy().reshape(-1, 4)
                for c in range(3):
                    np.add.at(r_loc, 3 * sn + c, inc[:, c])
                np.add.at(r_loc, 3 * nl + sn, inc[:, 3])
        loc, glo = owned_global_dofs(plan, m["n_vnodes"])
        con = p.constrained.astype(bool)
        err = np.abs(np.where(con[glo], 0.0, r_loc[loc]) - r_glob[glo]).max() / np.abs(r_glob).max()
        q.put((rank, float(err)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_distributed_residual_equals_global_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + world * 7 + os.getpid() % 500
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for pr in procs:
        pr.join(timeout=60)
    for rank, err in res:
        assert err < 1e-13, (rank, err)


# ---- general meshes (row e2): gls_gpart_* on adapted mapped meshes with hanging-node lines
def _adapted_space(dim, k, kp):
    from tests.test_uforest import make_mesh, random_adapt
    spec = dict(grid=("hyper_shell", "0, 0 : 0.25 : 1 : 6 : true")) if dim == 2 else \
        dict(grid=("cylinder_shell", "1 : 0.25 : 1 : 8 : 2"))
    m = make_mesh(dim, spec)
    m.refine_global(1)
    random_adapt(m, 2 if dim == 2 else 1, seed=5, k=k)
    return m.fe_space(k, kp, qmapping_all=True)


@pytest.mark.parametrize("dim,k,kp", [(2, 2, 1), (2, 1, 1), (3, 2, 1)])
@pytest.mark.parametrize("world", [2, 3, 4])
def test_general_partition_covers_and_closes(dim, k, kp, world):
    """Every global DoF is owned by exactly one rank; each rank's local DoFs hold its cells' DoFs and
    the masters of every hanging line on them; a rank's send list to a neighbour equals (as global
    DoFs, in order) the neighbour's receive list from it, and receives only ghost DoFs."""
    from softx_2020_200_amd.dist import gpartition, owned_dofs
    from tests.test_gpu_uforest import dof_lines
    sp = _adapted_space(dim, k, kp)
    lines = dof_lines(sp)
    assert len(lines[0]) > 0
    plans = [gpartition(sp, r, world, lines) for r in range(world)]
    ndof = plans[0]["n_global_dofs"]
    owned = np.concatenate([owned_dofs(p)[1] for p in plans])
    assert np.array_equal(np.sort(owned), np.arange(ndof))
    ld, lo, lm = (np.asarray(a) for a in lines[:3])
    line_of = {int(d): i for i, d in enumerate(ld)}
    for r, p in enumerate(plans):
        loc = set(p["l2g_dofs"].tolist())
        cells = range(p["cell_begin"], p["cell_end"])
        nvg = sp["n_vnodes"]
        for c in cells:
            for nd in sp["cell_vnodes"][c]:
                for cc in range(dim):
                    g = int(nd) * dim + cc
                    assert g in loc
                    if g in line_of:
                        i = line_of[g]
                        assert set(lm[lo[i]:lo[i + 1]].tolist()) <= loc, (r, g)
            for pn in (sp["cell_pnodes"][c] if kp != k else sp["cell_vnodes"][c]):
                assert dim * nvg + int(pn) in loc
        # local cell maps agree with the global ones
        lv = p["vl2g"][p["local_cv"]]
        assert np.array_equal(lv, sp["cell_vnodes"][p["cell_begin"]:p["cell_end"]])
        # owned-first numbering
        n_own = p["n_owned_v"]
        assert np.all(np.diff(p["vl2g"][:n_own]) > 0)
    for a, pa in enumerate(plans):
        for i, b in enumerate(pa["nbrs"]):
            pb = plans[int(b)]
            j = list(pb["nbrs"]).index(a)
            sent = pa["l2g_dofs"][pa["send_dofs"][pa["send_off"][i]:pa["send_off"][i + 1]]]
            got = pb["l2g_dofs"][pb["recv_dofs"][pb["recv_off"][j]:pb["recv_off"][j + 1]]]
            assert np.array_equal(sent, got), (a, int(b))
            own_b = set(owned_dofs(pb)[1].tolist())
            assert not (set(got.tolist()) & own_b)


@pytest.mark.parametrize("world", [2, 3])
def test_replica_transfer_rows_and_injection(world):
    """gls_mg_attach_replica's per-rank arrays (dist.replica_transfer): every rank's local fine rows carry the
    global prolongation's rows (replica columns unchanged), and each level-1 DoF's state is injected by exactly
    one rank, the owner of the fine DoF it is taken from."""
    from softx_2020_200_amd.dist import gpartition, owned_dofs, replica_transfer
    from tests.test_gpu_uforest import dof_lines
    from tests.test_uforest import make_mesh, random_adapt
    m = make_mesh(3, dict(grid=("cylinder_shell", "1 : 0.25 : 1 : 8 : 2")))
    m.refine_global(1)
    random_adapt(m, 1, seed=5, k=2)
    hf = m.fe_space_handle(2, 1, qmapping_all=True)
    L = int(hf.data["cell_level"].max())
    hc = m.coarsen_to(L - 1).fe_space_handle(2, 1, qmapping_all=True)
    off, col, w, inj = hf.mg_transfer_from(hc)
    lines = dof_lines(hf.data)
    nc = len(inj)
    hits = np.zeros(nc, np.int64)
    for r in range(world):
        plan = gpartition(hf.data, r, world, lines)
        lo, lc, lw, li = replica_transfer(plan, off, col, w, inj)
        l2g = np.asarray(plan["l2g_dofs"])
        assert len(lo) == len(l2g) + 1
        for i in range(0, len(l2g), max(1, len(l2g) // 200)):
            g = l2g[i]
            assert np.array_equal(lc[lo[i]:lo[i + 1]], col[off[g]:off[g + 1]])
            assert np.array_equal(lw[lo[i]:lo[i + 1]], w[off[g]:off[g + 1]])
        loc, glo = owned_dofs(plan)
        sel = li >= 0
        assert np.isin(li[sel], loc).all()
        assert np.array_equal(l2g[li[sel]], inj[sel])
        hits += sel
    assert (hits == 1).all()


# ---- distributed forest: gls_dpart_create from each rank's local part only
@pytest.mark.parametrize("dim,k,kp", [(2, 2, 1), (2, 1, 1), (3, 2, 1)])
@pytest.mark.parametrize("world", [2, 3, 4, 8])
def test_local_part_plan_equals_replicated_plan(dim, k, kp, world):
    """A rank's plan from its local part alone (owned cells + ghost layer, node keys = global ids) is the plan
    the replicated global mesh gives: same local cells, node order, owned counts, neighbours and exchange lists."""
    from softx_2020_200_amd.dist import dplan, gpartition, local_part
    from tests.test_gpu_uforest import dof_lines
    sp = _adapted_space(dim, k, kp)
    lines = dof_lines(sp)
    for r in range(world):
        g = gpartition(sp, r, world, lines)
        part = local_part(sp, r, world, lines)
        assert len(part["cell_owner"]) < sp["n_cells"] or world == 1
        d = dplan(part, r, world)
        assert np.array_equal(d["vl2k"], g["vl2g"]) and np.array_equal(d["pl2k"], g["pl2g"]), r
        for key in ("local_cv", "local_cp", "nbrs", "send_off", "send_dofs", "recv_off", "recv_dofs"):
            assert np.array_equal(d[key], g[key]), (r, key)
        assert (d["n_owned_v"], d["n_owned_p"]) == (g["n_owned_v"], g["n_owned_p"])


@pytest.mark.parametrize("world", [2, 3])
def test_local_part_plan_with_sparse_keys(world):
    """Node keys need not be a numbering: with scattered 64-bit keys the plans still pair up (a rank's send list to
    a neighbour is, as DoF keys and in order, that neighbour's receive list), owned cells map back to their keys,
    and every DoF is owned by exactly one rank."""
    from softx_2020_200_amd.dist import dplan, local_part
    from tests.test_gpu_uforest import dof_lines
    sp = _adapted_space(3, 2, 1)
    lines = dof_lines(sp)
    rng = np.random.default_rng(3)
    vkey = rng.choice(2 ** 40, sp["n_vnodes"], replace=False) * 7 + 5
    pkey = rng.choice(2 ** 40, sp["n_pnodes"], replace=False) * 3 + 1

    def rekey(part):
        d1 = part["dim"] + 1
        def kv(dk):
            pres = dk % d1 == part["dim"]
            out = np.empty_like(dk)
            out[pres] = pkey[dk[pres] // d1]
            out[~pres] = vkey[dk[~pres] // d1]
            return out * d1 + dk % d1
        q = dict(part, cell_vkeys=vkey[part["cell_vkeys"]], cell_pkeys=pkey[part["cell_pkeys"]])
        ld, lo, lm, lw = part["lines"]
        q["lines"] = (kv(ld), lo, kv(lm), lw)
        return q
    plans, parts = [], []
    for r in range(world):
        part = rekey(local_part(sp, r, world, lines))
        parts.append(part)
        plans.append(dplan(part, r, world))
    owned = []
    for r, (pl, pa) in enumerate(zip(plans, parts)):
        own = pa["cell_owner"] == r
        assert np.array_equal(pl["vl2k"][pl["local_cv"]], pa["cell_vkeys"][own])
        assert np.array_equal(pl["pl2k"][pl["local_cp"]], pa["cell_pkeys"][own])
        n = pl["n_vnodes"]
        owned.append(np.concatenate([pl["l2k_dofs"][:3 * pl["n_owned_v"]], pl["l2k_dofs"][3 * n:3 * n + pl["n_owned_p"]]]))
    allown = np.concatenate(owned)
    assert len(np.unique(allown)) == len(allown) == 3 * sp["n_vnodes"] + sp["n_pnodes"]
    for a, pa in enumerate(plans):
        for i, b in enumerate(pa["nbrs"]):
            pb = plans[int(b)]
            j = list(pb["nbrs"]).index(a)
            sent = pa["l2k_dofs"][pa["send_dofs"][pa["send_off"][i]:pa["send_off"][i + 1]]]
            got = pb["l2k_dofs"][pb["recv_dofs"][pb["recv_off"][j]:pb["recv_off"][j + 1]]]
            assert np.array_equal(sent, got), (a, int(b))


def _numbering_worker(rank, world, port, q, part):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    from softx_2020_200_amd.dist import dpartition
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        pl = dpartition(part, rank, world)
        q2 = dict(l2k=pl["l2k_dofs"], l2g=pl["l2g_dofs"], n=pl["n_global_dofs"], no=(pl["n_owned_v"], pl["n_owned_p"]),
                  nv=pl["n_vnodes"])
        q.put((rank, q2))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_distributed_numbering_gloo(world):
    """dpartition's global numbering (owned counts all-reduced, ghost ids from their owners): every rank's owned
    DoFs are one contiguous range, the ranges tile [0, n), and a DoF key has the same global id on every rank that
    holds it. Each worker process receives only its local part."""
    from softx_2020_200_amd.dist import local_part
    from tests.test_gpu_uforest import dof_lines
    sp = _adapted_space(3, 2, 1)
    lines = dof_lines(sp)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29800 + world * 11 + os.getpid() % 400
    procs = [ctx.Process(target=_numbering_worker, args=(r, world, port, q, local_part(sp, r, world, lines)))
             for r in range(world)]
    for pr in procs:
        pr.start()
    res = dict(q.get(timeout=300) for r in range(world))
    for pr in procs:
        pr.join(timeout=60)
    n = 3 * sp["n_vnodes"] + sp["n_pnodes"]
    key2g = {}
    ranges = []
    for r in range(world):
        e = res[r]
        assert e["n"] == n
        nov, nop = e["no"]
        own = np.concatenate([e["l2g"][:3 * nov], e["l2g"][3 * e["nv"]:3 * e["nv"] + nop]])
        ranges.append(np.sort(own))
        for kk, gg in zip(e["l2k"].tolist(), e["l2g"].tolist()):
            assert key2g.setdefault(kk, gg) == gg
    allown = np.concatenate(ranges)
    assert np.array_equal(np.sort(allown), np.arange(n))
    assert len(set(key2g.values())) == len(key2g)


@pytest.mark.parametrize("world", [2, 5])
def test_local_part_plan_on_an_adapted_octree(world):
    """The same equality on an adapted hyper_cube forest (octree leaves with hanging faces, Q2-Q2): the local part's
    ghost layer closes over the hanging lines, and the plan equals the replicated one."""
    import softx_2020_200_amd as sx
    from softx_2020_200_amd.dist import dplan, gpartition, local_part
    from tests.test_octree_mg import adapted_tree
    mesh = adapted_tree(3, 2, 2).mesh(2, 2)
    space = dict(mesh, cell_support=np.ascontiguousarray(mesh["vnode_x"][mesh["cell_vnodes"]]))
    lines = sx.hanging_dof_lines(mesh)
    assert len(lines[0]) > 0
    for r in range(world):
        g = gpartition(space, r, world, lines)
        d = dplan(local_part(space, r, world, lines), r, world)
        assert np.array_equal(d["vl2k"], g["vl2g"]), r
        for key in ("local_cv", "nbrs", "send_off", "send_dofs", "recv_off", "recv_dofs"):
            assert np.array_equal(d[key], g[key]), (r, key)
