"""Multi-GPU driver glue: one process per GPU, torch.distributed ("nccl" = RCCL over xGMI).

The partition plan and every kernel (pack/unpack, operators, GMRES, Newton) live in
libgls_native.so (csrc/gls_dist.cpp, gls_api.cpp). This module only
  * calls gls_part_* to get the rank-local mesh and exchange lists,
  * owns the device exchange buffers (4 doubles per exchanged node: u, v, w, p),
  * implements the two callbacks the C++ side calls: ghost exchange (grouped point-to-point
    isend/irecv to the neighbour ranks) and the sum all-reduce of dot products.
Backend "nccl" exchanges device buffers directly (RCCL P2P over xGMI); backend "gloo" stages
through host memory (used by the CPU/one-GPU tests).
"""
from __future__ import annotations

import ctypes as C
import traceback

import numpy as np

from .native import GLSContext, GLSError, check, load

EXCHANGE_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_int)
ALLREDUCE_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_int)


def _bind(L):
    if getattr(L, "_dist_bound", False):
        return L
    i64, vp = C.c_int64, C.c_void_p
    L.gls_part_create.argtypes = [C.c_int, C.c_int, C.POINTER(C.c_int32), C.c_int, C.c_int, C.c_int, C.POINTER(vp)]
    L.gls_part_sizes.argtypes = [vp] + [C.POINTER(i64)] * 4 + [C.POINTER(C.c_int)] + [C.POINTER(i64)] * 2
    L.gls_part_get.argtypes = [vp, C.POINTER(C.c_int32), C.POINTER(i64), C.POINTER(C.c_int), C.POINTER(i64),
                               C.POINTER(C.c_int32), C.POINTER(i64), C.POINTER(C.c_int32)]
    L.gls_part_destroy.argtypes = [vp]
    L.gls_dist_attach.argtypes = [vp, i64, C.c_int, C.POINTER(i64), C.POINTER(C.c_int32), C.POINTER(i64),
                                  C.POINTER(C.c_int32), vp, vp, vp, EXCHANGE_FN, ALLREDUCE_FN, vp]
    L.gls_dist_import.argtypes = [vp, vp]
    L.gls_rccl_unique_id.argtypes = [C.POINTER(C.c_ubyte)]
    L.gls_rccl_create.argtypes = [C.POINTER(C.c_ubyte), C.c_int, C.c_int, C.POINTER(vp)]
    L.gls_rccl_destroy.argtypes = [vp]
    L.gls_rccl_info.argtypes = [vp, C.POINTER(C.c_int), C.POINTER(C.c_int)]
    L.gls_dist_attach_rccl.argtypes = [vp, vp, i64, C.c_int, C.POINTER(C.c_int), C.POINTER(i64), C.POINTER(C.c_int32),
                                       C.POINTER(i64), C.POINTER(C.c_int32)]
    i32p, i64p = C.POINTER(C.c_int32), C.POINTER(i64)
    L.gls_gpart_create.argtypes = [C.c_int, C.c_int, C.c_int, i64, i32p, i32p, i64, i64, i64, i64p, i64p, i64p, C.c_int,
                                   C.c_int, C.POINTER(vp)]
    L.gls_gpart_sizes.argtypes = [vp] + [i64p] * 6 + [C.POINTER(C.c_int)] + [i64p] * 2
    L.gls_gpart_get.argtypes = [vp, i32p, i32p, i64p, i64p, C.POINTER(C.c_int), i64p, i32p, i64p, i32p]
    L.gls_gpart_map_dofs.argtypes = [vp, i64, i64p, i64p]
    L.gls_gpart_destroy.argtypes = [vp]
    L.gls_dpart_create.argtypes = [C.c_int, C.c_int, C.c_int, i64, i32p, i64p, i64p, i64, i64p, i64p, i64p, C.c_int,
                                   C.c_int, C.POINTER(vp)]
    L.gls_dist_attach_dofs.argtypes = [vp, i64, i64, C.c_int, i64p, i32p, i64p, i32p, vp, vp, vp, EXCHANGE_FN,
                                       ALLREDUCE_FN, vp]
    L.gls_dist_attach_dofs_rccl.argtypes = [vp, vp, i64, i64, C.c_int, C.POINTER(C.c_int), i64p, i32p, i64p, i32p]
    L._dist_bound = True
    return L


def partition(cell_vnodes, n_vnodes, rank, world):
    """Partition plan (C++): returns dict with the rank-local mesh and exchange lists."""
    L = _bind(load())
    cv = np.ascontiguousarray(cell_vnodes, dtype=np.int32)
    h = C.c_void_p()
    check(L.gls_part_create(cv.shape[0], cv.shape[1], cv.ctypes.data_as(C.POINTER(C.c_int32)), int(n_vnodes), rank,
                            world, C.byref(h)), "gls_part_create")
    try:
        cb, ce, no, nl, ns, nr = (C.c_int64() for _ in range(6))
        nn = C.c_int()
        check(L.gls_part_sizes(h, C.byref(cb), C.byref(ce), C.byref(no), C.byref(nl), C.byref(nn), C.byref(ns),
                               C.byref(nr)), "gls_part_sizes")
        nc = ce.value - cb.value
        out = dict(cell_begin=cb.value, cell_end=ce.value, n_owned=no.value, n_local=nl.value,
                   local_cells=np.zeros((nc, cv.shape[1]), dtype=np.int32),
                   local_to_global=np.zeros(nl.value, dtype=np.int64),
                   nbrs=np.zeros(nn.value, dtype=np.int32), send_off=np.zeros(nn.value + 1, dtype=np.int64),
                   send_nodes=np.zeros(ns.value, dtype=np.int32), recv_off=np.zeros(nn.value + 1, dtype=np.int64),
                   recv_nodes=np.zeros(nr.value, dtype=np.int32))
        check(L.gls_part_get(h, out["local_cells"].ctypes.data_as(C.POINTER(C.c_int32)),
                             out["local_to_global"].ctypes.data_as(C.POINTER(C.c_int64)),
                             out["nbrs"].ctypes.data_as(C.POINTER(C.c_int)),
                             out["send_off"].ctypes.data_as(C.POINTER(C.c_int64)),
                             out["send_nodes"].ctypes.data_as(C.POINTER(C.c_int32)),
                             out["recv_off"].ctypes.data_as(C.POINTER(C.c_int64)),
                             out["recv_nodes"].ctypes.data_as(C.POINTER(C.c_int32))), "gls_part_get")
        if nn.value == 0:
            out["send_off"] = np.zeros(1, dtype=np.int64)
            out["recv_off"] = np.zeros(1, dtype=np.int64)
        return out
    finally:
        L.gls_part_destroy(h)


class Exchanger:
    """Device exchange buffers + the C callbacks (torch.distributed point-to-point / all-reduce)."""

    def __init__(self, plan, device, backend="nccl", group=None, width=4):
        import torch
        self.torch = torch
        self.dist = torch.distributed
        self.plan = plan
        self.backend = backend
        self.group = group
        self.width = width  # doubles per exchange entry: 4 per node (brick meshes), 1 per DoF (general meshes)
        ns, nr = int(plan["send_off"][-1]), int(plan["recv_off"][-1])
        self.send_buf = torch.zeros(max(ns, 1) * width, dtype=torch.float64, device=device)
        self.recv_buf = torch.zeros(max(nr, 1) * width, dtype=torch.float64, device=device)
        self.red_buf = torch.zeros(256, dtype=torch.float64, device=device)
        self._xchg = EXCHANGE_FN(self._exchange)
        self._allred = ALLREDUCE_FN(self._allreduce)

    def _segments(self, phase):
        p = self.plan
        sb, rb = (self.send_buf, self.recv_buf) if phase == 0 else (self.recv_buf, self.send_buf)
        so, ro = (p["send_off"], p["recv_off"]) if phase == 0 else (p["recv_off"], p["send_off"])
        w = self.width
        for i, nbr in enumerate(p["nbrs"]):
            yield int(nbr), sb[w * so[i]:w * so[i + 1]], rb[w * ro[i]:w * ro[i + 1]]

    def _exchange(self, user, phase):
        try:
            d = self.dist
            if self.backend == "nccl":
                ops = []
                for nbr, s, r in self._segments(phase):
                    if s.numel():
                        ops.append(d.P2POp(d.isend, s, nbr, group=self.group))
                    if r.numel():
                        ops.append(d.P2POp(d.irecv, r, nbr, group=self.group))
                if ops:
                    for w in d.batch_isend_irecv(ops):
                        w.wait()
            else:  # gloo: stage through host memory
                segs = list(self._segments(phase))
                host_s = [s.cpu() for _, s, _ in segs]
                host_r = [self.torch.empty(r.numel(), dtype=self.torch.float64) for _, _, r in segs]
                reqs = []
                for (nbr, s, r), hs, hr in zip(segs, host_s, host_r):
                    if hs.numel():
                        reqs.append(d.isend(hs, nbr, group=self.group))
                    if hr.numel():
                        reqs.append(d.irecv(hr, nbr, group=self.group))
                for q in reqs:
                    q.wait()
                for (_, _, r), hr in zip(segs, host_r):
                    if r.numel():
                        r.copy_(hr.to(r.device))
            return 0
        except Exception:
            traceback.print_exc()
            return -1

    def _allreduce(self, user, dev_ptr, n):
        try:
            assert dev_ptr == self.red_buf.data_ptr() and n <= self.red_buf.numel()
            view = self.red_buf[:n]
            if self.backend == "nccl":
                self.dist.all_reduce(view, group=self.group)
            else:
                h = view.cpu()
                self.dist.all_reduce(h, group=self.group)
                view.copy_(h.to(view.device))
            return 0
        except Exception:
            traceback.print_exc()
            return -1


def attach(ctx: GLSContext, plan, exchanger: Exchanger):
    L = _bind(load())
    p = plan
    check(L.gls_dist_attach(ctx.h, int(p["n_owned"]), len(p["nbrs"]),
                            p["send_off"].ctypes.data_as(C.POINTER(C.c_int64)),
                            p["send_nodes"].ctypes.data_as(C.POINTER(C.c_int32)),
                            p["recv_off"].ctypes.data_as(C.POINTER(C.c_int64)),
                            p["recv_nodes"].ctypes.data_as(C.POINTER(C.c_int32)),
                            C.c_void_p(exchanger.send_buf.data_ptr()), C.c_void_p(exchanger.recv_buf.data_ptr()),
                            C.c_void_p(exchanger.red_buf.data_ptr()), exchanger._xchg, exchanger._allred, None),
          "gls_dist_attach")
    ctx._exchanger = exchanger  # keep callbacks alive
    ctx._plan = plan


_RCCL = {}


def rccl_comm(rank, world, group=None):
    """The process's in-library RCCL communicator (gls_rccl_create), created once and shared by every
    context (all multigrid levels); rank 0's unique id travels through torch.distributed."""
    key = (rank, world, id(group))
    if key not in _RCCL:
        import torch.distributed as dist
        L = _bind(load())
        buf = (C.c_ubyte * 128)()
        if rank == 0:
            check(L.gls_rccl_unique_id(buf), "gls_rccl_unique_id")
        obj = [bytes(buf) if rank == 0 else None]
        if world > 1:
            dist.broadcast_object_list(obj, src=0, group=group)
        idb = (C.c_ubyte * 128).from_buffer_copy(obj[0])
        h = C.c_void_p()
        check(L.gls_rccl_create(idb, rank, world, C.byref(h)), "gls_rccl_create")
        _RCCL[key] = h
    return _RCCL[key]


def drop_rccl():
    """Forget the cached in-library communicators without calling into them (a pre-flight that failed on some
    rank may have left one mid-collective; the fallback transport does not use it)."""
    _RCCL.clear()


def rccl_info(comm):
    """(rank, size) of an in-library RCCL communicator as RCCL itself reports them."""
    L = _bind(load())
    r, w = C.c_int(), C.c_int()
    check(L.gls_rccl_info(comm, C.byref(r), C.byref(w)), "gls_rccl_info")
    return r.value, w.value


def attach_rccl(ctx: GLSContext, plan, comm):
    """Attach the rank-local context to the in-library RCCL transport (no Python on the data path)."""
    L = _bind(load())
    p = plan
    nbrs = np.ascontiguousarray(p["nbrs"], dtype=np.int32)
    check(L.gls_dist_attach_rccl(ctx.h, comm, int(p["n_owned"]), len(nbrs), nbrs.ctypes.data_as(C.POINTER(C.c_int)),
                                 p["send_off"].ctypes.data_as(C.POINTER(C.c_int64)),
                                 p["send_nodes"].ctypes.data_as(C.POINTER(C.c_int32)),
                                 p["recv_off"].ctypes.data_as(C.POINTER(C.c_int64)),
                                 p["recv_nodes"].ctypes.data_as(C.POINTER(C.c_int32))), "gls_dist_attach_rccl")
    ctx._plan = plan


def dist_import(ctx, x):
    L = _bind(load())
    check(L.gls_dist_import(ctx.h, C.c_void_p(x.data_ptr())), "gls_dist_import")


def local_vector(plan, global_vec, n_vnodes_global, dim=3):
    """Restrict a global [vel interleaved | pressure] vector to the rank-local layout (Qk-Qk)."""
    l2g = plan["local_to_global"]
    nl = l2g.shape[0]
    out = np.zeros(dim * nl + nl)
    gv = np.asarray(global_vec)
    for c in range(dim):
        out[c:dim * nl:dim] = gv[dim * l2g + c]
    out[dim * nl:] = gv[dim * n_vnodes_global + l2g]
    return out


def owned_global_dofs(plan, n_vnodes_global, dim=3):
    """(local dof indices of owned DoFs, their global dof indices)."""
    l2g = plan["local_to_global"]
    nl, no = l2g.shape[0], plan["n_owned"]
    loc, glo = [], []
    for c in range(dim):
        loc.append(dim * np.arange(no) + c)
        glo.append(dim * l2g[:no] + c)
    loc.append(dim * nl + np.arange(no))
    glo.append(dim * n_vnodes_global + l2g[:no])
    return np.concatenate(loc), np.concatenate(glo)


class DistributedProblem:
    """Rank-local GLS context on a Morton brick mesh (3D Qk-Qk), attached to the exchanger."""

    def __init__(self, mesh, rank, world, device, viscosity=1.0, vnode_mask=None, dirichlet=None, force_q=None,
                 backend="nccl", group=None, impl="torch"):
        if mesh["k"] != mesh["kp"] or mesh["dim"] != 3:
            raise GLSError("distributed path: 3D Qk-Qk only")
        plan = partition(mesh["cell_vnodes"], mesh["n_vnodes"], rank, world)
        self.plan = plan
        cb, ce = plan["cell_begin"], plan["cell_end"]
        l2g = plan["local_to_global"]
        nl = l2g.shape[0]
        self.n_vnodes_global = mesh["n_vnodes"]
        lmask = vnode_mask[l2g] if vnode_mask is not None else None
        fq = force_q[cb:ce] if force_q is not None else None
        self.ctx = GLSContext(3, mesh["k"], mesh["kp"], plan["local_cells"], None, mesh["cell_h"][cb:ce], nl, nl,
                              viscosity=viscosity, cell_x0=mesh["cell_x0"][cb:ce], vnode_mask=lmask, force_q=fq)
        if dirichlet is not None:
            gdofs, gvals = dirichlet
            g2l = np.full(mesh["n_vnodes"], -1, dtype=np.int64)
            g2l[l2g] = np.arange(nl)
            node = g2l[gdofs // 3]
            sel = node >= 0
            self.ctx.set_dirichlet(3 * node[sel] + gdofs[sel] % 3, np.asarray(gvals)[sel])
        if impl == "native":  # in-library RCCL: ncclSend / ncclRecv / ncclAllReduce on the context stream
            self.exchanger = None
            attach_rccl(self.ctx, plan, rccl_comm(rank, world, group))
        else:  # torch.distributed callbacks ("nccl" = RCCL through torch, "gloo" through the host)
            self.exchanger = Exchanger(plan, device, backend=backend, group=group)
            attach(self.ctx, plan, self.exchanger)
        self.n_dofs_local = self.ctx.n_dofs

    def set_lattice(self):
        """Declare this rank's nodes as a box of the global hyper_cube node lattice (multigrid)."""
        n1d = int(round(self.n_vnodes_global ** (1.0 / 3.0)))
        self.ctx.set_lattice(n1d, self.plan["local_to_global"])


def multigrid_levels(n, world, coarsest=4):
    """Cells per direction of the nested levels below n usable by a distributed V-cycle: every level
    keeps whole 2x2x2 bricks and a brick count divisible by the rank count (nested partitions)."""
    out = []
    m = n
    while m % 2 == 0 and m // 2 >= coarsest and ((m // 2) ** 3 // 8) % world == 0 and (m // 2) % 2 == 0:
        m //= 2
        out.append(m)
    return out


def attach_distributed_multigrid(levels, replica=None, **mg_opts):
    """levels: [DistributedProblem] on nested hyper_cubes (fine first), same ranks / boundary data.
    replica: optional single-rank problem object (``.ctx``, ``.mesh``; e.g. a CavityProblem with its own
    multigrid) on the WHOLE mesh of the coarsest distributed level: below that level every rank runs the
    replica's cycle on the gathered right-hand side (gls_mg_set_coarse_replica), so that the N-rank
    V-cycle is the one-rank one."""
    for lv in levels:
        lv.set_lattice()
    levels[0].ctx.attach_multigrid([lv.ctx for lv in levels[1:]], **mg_opts)
    levels[0]._mg_levels = levels
    if replica is not None:
        cl = levels[-1]
        l2g = cl.plan["local_to_global"].astype(np.int64)
        nvg = cl.n_vnodes_global
        loc = np.concatenate([(l2g[:, None] * 3 + np.arange(3)[None, :]).reshape(-1), 3 * nvg + l2g])
        levels[0].ctx.set_coarse_replica(replica.ctx, loc)
        levels[0]._replica = replica



# ---------------------------------------------------------------------------------------------------
# General meshes (adaptive / unstructured / curved forests, row e2): DoF-level partition and exchange
# ---------------------------------------------------------------------------------------------------
def gpartition(space, rank, world, lines=None):
    """gls_gpart_create on a (replicated) global mesh description: space = gls_fe_space-style dict
    (dim, k, kp, n_cells, cell_vnodes, cell_pnodes, n_vnodes, n_pnodes); lines = global DoF-level
    lines (dofs, offsets, masters[, weights]) or None. Returns the plan dict (local cells, node maps,
    owned counts, DoF exchange lists) and the C handle's global -> local DoF map as a function."""
    L = _bind(load())
    dim, k, kp = int(space["dim"]), int(space["k"]), int(space["kp"])
    cv = np.ascontiguousarray(space["cell_vnodes"], dtype=np.int32)
    sep = kp != k
    cp = np.ascontiguousarray(space["cell_pnodes"], dtype=np.int32) if sep else None
    nv, npn = int(space["n_vnodes"]), int(space["n_pnodes"])
    if lines is None or len(lines[0]) == 0:
        ld, lo, lm = np.zeros(0, np.int64), np.zeros(1, np.int64), np.zeros(0, np.int64)
    else:
        ld, lo, lm = (np.ascontiguousarray(a, dtype=np.int64) for a in lines[:3])
    p64 = lambda a: a.ctypes.data_as(C.POINTER(C.c_int64))  # noqa: E731
    p32 = lambda a: a.ctypes.data_as(C.POINTER(C.c_int32)) if a is not None else C.POINTER(C.c_int32)()  # noqa: E731
    h = C.c_void_p()
    check(L.gls_gpart_create(dim, k, kp, cv.shape[0], p32(cv), p32(cp), nv, npn, len(ld), p64(ld), p64(lo), p64(lm),
                             rank, world, C.byref(h)), "gls_gpart_create")
    out = _plan_from_handle(L, h, dim, cv.shape[1], cp.shape[1] if sep else None)
    # global DoF ids of the local DoFs (velocity node*dim + c, pressure dim*NV + p)
    g = np.concatenate([(out["vl2g"][:, None] * dim + np.arange(dim)[None, :]).reshape(-1), dim * nv + out["pl2g"]])
    out["l2g_dofs"] = g
    out["n_global_dofs"] = dim * nv + npn
    return out


def _plan_from_handle(L, h, dim, nvpc, npc):
    """gls_gpart_sizes / _get into a plan dict (and destroy the handle); npc None = equal order"""
    p64 = lambda a: a.ctypes.data_as(C.POINTER(C.c_int64))  # noqa: E731
    p32 = lambda a: a.ctypes.data_as(C.POINTER(C.c_int32)) if a is not None else C.POINTER(C.c_int32)()  # noqa: E731
    try:
        cb, ce, nvl, npl, nov, nop, ns, nr = (C.c_int64() for _ in range(8))
        nn = C.c_int()
        check(L.gls_gpart_sizes(h, C.byref(cb), C.byref(ce), C.byref(nvl), C.byref(npl), C.byref(nov), C.byref(nop),
                                C.byref(nn), C.byref(ns), C.byref(nr)), "gls_gpart_sizes")
        nc = ce.value - cb.value
        sep = npc is not None
        out = dict(cell_begin=cb.value, cell_end=ce.value, n_vnodes=nvl.value, n_pnodes=npl.value,
                   n_owned_v=nov.value, n_owned_p=nop.value, dim=dim,
                   local_cv=np.zeros((nc, nvpc), np.int32),
                   local_cp=np.zeros((nc, npc), np.int32) if sep else None,
                   vl2g=np.zeros(nvl.value, np.int64), pl2g=np.zeros(npl.value, np.int64),
                   nbrs=np.zeros(nn.value, np.int32), send_off=np.zeros(nn.value + 1, np.int64),
                   send_dofs=np.zeros(ns.value, np.int32), recv_off=np.zeros(nn.value + 1, np.int64),
                   recv_dofs=np.zeros(nr.value, np.int32))
        check(L.gls_gpart_get(h, p32(out["local_cv"]), p32(out["local_cp"]), p64(out["vl2g"]), p64(out["pl2g"]),
                              out["nbrs"].ctypes.data_as(C.POINTER(C.c_int)), p64(out["send_off"]),
                              p32(out["send_dofs"]), p64(out["recv_off"]), p32(out["recv_dofs"])), "gls_gpart_get")
        if nn.value == 0:
            out["send_off"] = np.zeros(1, np.int64)
            out["recv_off"] = np.zeros(1, np.int64)
        if not sep:
            out["local_cp"] = out["local_cv"]
        return out
    finally:
        L.gls_gpart_destroy(h)


# ---------------------------------------------------------------------------------------------------
# Distributed forest: a rank's plan from its local part only (gls_dpart_create)
# ---------------------------------------------------------------------------------------------------
def _dof_node(g, dim, nv, sep):
    """unified node id of global DoF ids (velocity nodes [0, nv), pressure nodes nv + p when separate)"""
    g = np.asarray(g, np.int64)
    nvd = dim * nv
    return np.where(g < nvd, g // dim, (nv if sep else 0) + g - nvd)


def _dof_key(g, dim, nv):
    """DoF key (node key * (dim + 1) + c, c = dim for pressure) of global DoF ids, keys = global node ids"""
    g = np.asarray(g, np.int64)
    nvd = dim * nv
    return np.where(g < nvd, (g // dim) * (dim + 1) + g % dim, (g - nvd) * (dim + 1) + dim)


def local_part(space, rank, world, lines=None, dirichlet=None, vnode_mask=None, force_q=None):
    """What a p::d triangulation hands rank `rank` of the forest `space` (the partitioner's hand-off; the rank
    itself never sees the global arrays): its owned cells (the equal-count range of the space-filling cell
    order) plus the ghost layer (every cell touching a node of an owned cell, a master node of a hanging line on
    one, or the DoF node of a line one of whose masters it touches -- gls_dpart_create's contract), with owners, node keys (= global node ids), the lines on those cells in DoF keys, and the per-cell /
    per-node data the rank's context needs (cell_support and force_q of the owned cells, vnode_mask and Dirichlet
    rows on the provided nodes). Feeds dpartition / DistributedGeneralProblem(part=...)."""
    dim, k, kp = int(space["dim"]), int(space["k"]), int(space["kp"])
    sep = kp != k
    cv = np.asarray(space["cell_vnodes"], np.int64)
    cp = np.asarray(space["cell_pnodes"], np.int64) if sep else None
    nv = int(space["n_vnodes"])
    npn = int(space["n_pnodes"]) if sep else nv
    nc = cv.shape[0]
    cb = [nc * r // world for r in range(world + 1)]
    owner = np.searchsorted(np.asarray(cb[1:]), np.arange(nc), side="right").astype(np.int32)
    U = np.concatenate([cv, cp + nv], 1) if sep else cv
    nun = nv + (npn if sep else 0)
    S = np.zeros(nun, bool)
    S[U[cb[rank]:cb[rank + 1]].ravel()] = True
    if lines is not None and len(lines[0]):
        ld, lo, lm = (np.asarray(a, np.int64) for a in lines[:3])
        dn = _dof_node(ld, dim, nv, sep)
        mn = _dof_node(lm, dim, nv, sep)
        mline = np.repeat(np.arange(len(ld)), np.diff(lo))
        add = np.zeros(nun, bool)
        add[mn[S[dn[mline]]]] = True   # masters of the lines on the owned cells' nodes
        add[dn[mline[S[mn]]]] = True   # DoF nodes of the lines whose master an owned cell touches
        S |= add
    prov = np.nonzero(S[U].any(1))[0]
    nodes = np.zeros(nun, bool)
    nodes[U[prov].ravel()] = True
    part = dict(dim=dim, k=k, kp=kp, cell_owner=owner[prov], cell_vkeys=np.ascontiguousarray(cv[prov]),
                cell_pkeys=np.ascontiguousarray(cp[prov]) if sep else None)
    own = slice(cb[rank], cb[rank + 1])
    if "cell_support" in space:
        part["cell_support"] = np.ascontiguousarray(space["cell_support"][own])
    if force_q is not None:
        part["force_q"] = np.ascontiguousarray(np.asarray(force_q)[own])
    if lines is not None and len(lines[0]):
        ld, lo, lm = (np.asarray(a, np.int64) for a in lines[:3])
        lw = np.asarray(lines[3]) if len(lines) > 3 else np.ones(len(lm))
        keep = np.nonzero(nodes[_dof_node(ld, dim, nv, sep)])[0]
        lens = np.diff(lo)[keep]
        idx = np.repeat(lo[keep], lens) + (np.arange(lens.sum()) - np.repeat(np.cumsum(lens) - lens, lens))
        part["lines"] = (_dof_key(ld[keep], dim, nv), np.concatenate([[0], np.cumsum(lens)]).astype(np.int64),
                         _dof_key(lm[idx], dim, nv), lw[idx])
    vk = np.nonzero(nodes[:nv])[0]
    part["vnode_keys"] = vk
    if vnode_mask is not None:
        part["vnode_mask"] = np.ascontiguousarray(np.asarray(vnode_mask)[vk])
    if dirichlet is not None:
        gd, gv = (np.asarray(a) for a in dirichlet)
        sel = nodes[_dof_node(gd, dim, nv, sep)]
        part["dirichlet"] = (_dof_key(gd[sel], dim, nv), gv[sel])
    return part


def part_dof_keys(part):
    """sorted DoF keys of every DoF on the part's provided cells"""
    d1 = part["dim"] + 1
    vk = np.unique(part["cell_vkeys"])
    pk = np.unique(part["cell_pkeys"]) if part["cell_pkeys"] is not None else vk
    return np.unique(np.concatenate([(vk[:, None] * d1 + np.arange(part["dim"])[None, :]).ravel(), pk * d1 + part["dim"]]))


def dplan(part, rank, world):
    """gls_dpart_create on the rank's local part: plan dict as gpartition's with the local nodes' keys (vl2k,
    pl2k, l2k_dofs) in place of global ids."""
    L = _bind(load())
    dim, k, kp = int(part["dim"]), int(part["k"]), int(part["kp"])
    owner = np.ascontiguousarray(part["cell_owner"], np.int32)
    cv = np.ascontiguousarray(part["cell_vkeys"], np.int64)
    cp = part["cell_pkeys"]
    cp = np.ascontiguousarray(cp, np.int64) if cp is not None else None
    lines = part.get("lines")
    if lines is None or len(lines[0]) == 0:
        ld, lo, lm = np.zeros(0, np.int64), np.zeros(1, np.int64), np.zeros(0, np.int64)
    else:
        ld, lo, lm = (np.ascontiguousarray(a, dtype=np.int64) for a in lines[:3])
    p64 = lambda a: a.ctypes.data_as(C.POINTER(C.c_int64)) if a is not None else C.POINTER(C.c_int64)()  # noqa: E731
    h = C.c_void_p()
    check(L.gls_dpart_create(dim, k, kp, cv.shape[0], owner.ctypes.data_as(C.POINTER(C.c_int32)), p64(cv), p64(cp),
                             len(ld), p64(ld), p64(lo), p64(lm), rank, world, C.byref(h)), "gls_dpart_create")
    out = _plan_from_handle(L, h, dim, cv.shape[1], cp.shape[1] if cp is not None else None)
    out["vl2k"], out["pl2k"] = out.pop("vl2g"), out.pop("pl2g")
    d1 = dim + 1
    out["l2k_dofs"] = np.concatenate([(out["vl2k"][:, None] * d1 + np.arange(dim)[None, :]).reshape(-1),
                                      out["pl2k"] * d1 + dim])
    return out


def dpartition(part, rank, world, device="cpu", backend="gloo", group=None):
    """dplan, then the distributed global numbering (deal.II's: each rank's owned DoFs one contiguous range, by an
    all-reduce of the owned counts and one owner -> ghost exchange of the ghost DoFs' ids): adds l2g_dofs,
    n_global_dofs (velocity node * dim + c, pressure dim * NV + node, as gpartition's)."""
    import torch
    out = dplan(part, rank, world)
    dim = out["dim"]
    # distributed numbering: owned counts -> offsets; owners send their ids to the ghosting ranks
    dev = device if backend == "nccl" else "cpu"
    cnt = torch.zeros(2 * world, dtype=torch.int64, device=dev)
    cnt[2 * rank], cnt[2 * rank + 1] = out["n_owned_v"], out["n_owned_p"]
    torch.distributed.all_reduce(cnt, group=group)
    cnt = cnt.cpu().numpy().reshape(world, 2)
    nv_g, np_g = int(cnt[:, 0].sum()), int(cnt[:, 1].sum())
    voff, poff = int(cnt[:rank, 0].sum()), int(cnt[:rank, 1].sum())
    nvl = out["n_vnodes"]
    g = np.full(len(out["l2k_dofs"]), -1, np.int64)
    nov, nop = out["n_owned_v"], out["n_owned_p"]
    g[:dim * nov] = ((voff + np.arange(nov))[:, None] * dim + np.arange(dim)[None, :]).ravel()
    g[dim * nvl:dim * nvl + nop] = dim * nv_g + poff + np.arange(nop)
    ex = Exchanger(out, dev, backend=backend, group=group, width=1)
    ns, nr = int(out["send_off"][-1]), int(out["recv_off"][-1])
    if ns:
        ex.send_buf[:ns] = torch.as_tensor(g[out["send_dofs"]].astype(np.float64), device=dev)
    if ex._exchange(None, 0) != 0:
        raise GLSError("dpartition: the numbering exchange failed")
    if nr:
        g[out["recv_dofs"]] = ex.recv_buf[:nr].cpu().numpy().astype(np.int64)
    if (g < 0).any():
        raise GLSError("dpartition: rank %d holds DoFs no exchange numbered" % rank)
    out["l2g_dofs"] = g
    out["n_global_dofs"] = dim * nv_g + np_g
    out["n_global_vnodes"] = nv_g
    return out


def owned_dofs(plan):
    """(local ids, global ids) of the rank's owned DoFs (velocity of owned nodes, pressure of owned nodes)"""
    d = plan["dim"]
    nvl = plan["n_vnodes"]
    loc = np.concatenate([np.arange(d * plan["n_owned_v"]), d * nvl + np.arange(plan["n_owned_p"])])
    return loc, plan["l2g_dofs"][loc]


def attach_dofs(ctx: GLSContext, plan, exchanger: Exchanger):
    L = _bind(load())
    p = plan
    p64 = lambda a: a.ctypes.data_as(C.POINTER(C.c_int64))  # noqa: E731
    p32 = lambda a: a.ctypes.data_as(C.POINTER(C.c_int32))  # noqa: E731
    check(L.gls_dist_attach_dofs(ctx.h, int(p["n_owned_v"]), int(p["n_owned_p"]), len(p["nbrs"]), p64(p["send_off"]),
                                 p32(p["send_dofs"]), p64(p["recv_off"]), p32(p["recv_dofs"]),
                                 C.c_void_p(exchanger.send_buf.data_ptr()), C.c_void_p(exchanger.recv_buf.data_ptr()),
                                 C.c_void_p(exchanger.red_buf.data_ptr()), exchanger._xchg, exchanger._allred, None),
          "gls_dist_attach_dofs")
    ctx._exchanger = exchanger
    ctx._plan = plan


class DistributedGeneralProblem:
    """Rank-local GLS context on a general (mapped, adapted) mesh: the rank's cells of the global
    space, Dirichlet rows and hanging lines mapped to local DoFs, DoF-level ghost exchange through
    torch.distributed (gloo / nccl callbacks)."""

    def __init__(self, space, rank, world, device, viscosity=1.0, vnode_mask=None, dirichlet=None, lines=None,
                 backend="gloo", group=None, qmapping=True, force_q=None, part=None):
        """space = the replicated global mesh (gpartition), or part = this rank's local part only (local_part's
        dict; space, vnode_mask, dirichlet, lines and force_q then come from the part, in node / DoF keys)."""
        if part is not None:  # distributed forest: nothing global on this rank
            plan = dpartition(part, rank, world, device, backend, group)
            dim, k, kp = int(part["dim"]), int(part["k"]), int(part["kp"])
            vk = np.asarray(part["vnode_keys"])
            lmask = np.ascontiguousarray(part["vnode_mask"][np.searchsorted(vk, plan["vl2k"])]) \
                if "vnode_mask" in part else None
            support, fq = part["cell_support"], part.get("force_q")
            lines, dirichlet = part.get("lines"), part.get("dirichlet")
            keys = plan["l2k_dofs"]
            order = np.argsort(keys)

            def to_local(ids):
                ids = np.asarray(ids, np.int64)
                pos = np.minimum(np.searchsorted(keys, ids, sorter=order), len(keys) - 1)
                loc = order[pos]
                return np.where(keys[loc] == ids, loc, -1)
        else:
            plan = gpartition(space, rank, world, lines)
            cb, ce = plan["cell_begin"], plan["cell_end"]
            dim, k, kp = int(space["dim"]), int(space["k"]), int(space["kp"])
            lmask = np.ascontiguousarray(vnode_mask[plan["vl2g"]]) if vnode_mask is not None else None
            support = space["cell_support"][cb:ce]
            fq = None if force_q is None else force_q[cb:ce]
            g2l = np.full(plan["n_global_dofs"], -1, np.int64)
            g2l[plan["l2g_dofs"]] = np.arange(len(plan["l2g_dofs"]))
            self.g2l = g2l

            def to_local(ids):
                return g2l[np.asarray(ids, np.int64)]
        self.plan = plan
        self.ctx = GLSContext(dim, k, kp, plan["local_cv"], plan["local_cp"] if kp != k else None, None,
                              plan["n_vnodes"], plan["n_pnodes"], viscosity=viscosity, vnode_mask=lmask,
                              map_degree=k, cell_support=np.ascontiguousarray(support),
                              force_q=None if fq is None else np.ascontiguousarray(fq))
        if lines is not None and len(lines[0]):
            ld, lo, lm = (np.asarray(a) for a in lines[:3])
            lw = np.asarray(lines[3])
            lloc = to_local(ld)
            keep = np.nonzero(lloc >= 0)[0]
            mloc = to_local(lm)
            dofs, offs, mas, ws = [], [0], [], []
            for i in keep:
                m = mloc[lo[i]:lo[i + 1]]
                if (m < 0).any():
                    raise GLSError("line master not local on rank %d" % rank)
                dofs.append(lloc[i])
                mas.extend(m.tolist())
                ws.extend(lw[lo[i]:lo[i + 1]].tolist())
                offs.append(len(mas))
            if dofs:
                self.ctx.set_hanging(np.array(dofs, np.int64), np.array(offs, np.int64), np.array(mas, np.int64),
                                     np.array(ws))
        if dirichlet is not None:
            gd, gv = (np.asarray(a) for a in dirichlet)
            ld_ = to_local(gd)
            sel = ld_ >= 0
            self.ctx.set_dirichlet(ld_[sel], gv[sel])
        self.exchanger = Exchanger(plan, device, backend=backend, group=group, width=1)
        attach_dofs(self.ctx, plan, self.exchanger)

    def local(self, global_vec):
        return np.ascontiguousarray(np.asarray(global_vec)[self.plan["l2g_dofs"]])


def replica_transfer(plan, p_off, p_col, p_w, inject):
    """gls_mg_attach_replica's arrays for this rank from the GLOBAL prolongation (fine DoFs x level-1 DoFs, CSR)
    and injection (level-1 DoF -> fine DoF): P restricted to the rank's local fine rows (owned and ghost, local
    order), and for every level-1 DoF the local fine DoF it takes its state from where this rank owns that DoF
    (-1 elsewhere)."""
    l2g = np.asarray(plan["l2g_dofs"], np.int64)
    p_off, p_col, p_w = (np.asarray(a) for a in (p_off, p_col, p_w))
    lens = p_off[l2g + 1] - p_off[l2g]
    off = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    idx = np.repeat(p_off[l2g], lens) + (np.arange(off[-1]) - np.repeat(off[:-1], lens))
    loc, glo = owned_dofs(plan)
    g2l_own = np.full(int(plan["n_global_dofs"]), -1, np.int64)
    g2l_own[glo] = loc
    return off, p_col[idx].astype(np.int32), p_w[idx].astype(np.float64), g2l_own[np.asarray(inject, np.int64)]


def attach_replica_multigrid(dp, replica_ctx, p_global, **opts):
    """The refinement-hierarchy V-cycle across ranks: dp (DistributedGeneralProblem of the fine level) smooths
    its rows, replica_ctx (single-rank context of the whole level-1 mesh with its own hierarchy attached) runs
    the coarser levels on every rank (gls_mg_attach_replica); p_global = (off, col, w, inject) from level 1 to
    the fine level, global numbering (FESpaceHandle.mg_transfer_from / octree transfers)."""
    off, col, w, inj = replica_transfer(dp.plan, *p_global)
    dp.ctx.attach_multigrid_replica(replica_ctx, off, col, w, inj, **opts)
