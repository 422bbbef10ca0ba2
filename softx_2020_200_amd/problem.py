"""Problem setup on the product side: hyper_cube mesh (C++ builder), boundary
classification and Dirichlet constraints (setup_dofs, gls_navier_stokes.cc:80-184),
and the 3D lid-driven cavity of the benchmark.
"""
from __future__ import annotations

import numpy as np

from .native import GLSContext, hyper_cube


def vnode_boundary_ids(mesh, n, lo, hi, colorize):
    """per velocity node: bitmask of hyper_cube boundary ids it lies on (colorize: x-=0,x+=1,y-=2,...)."""
    dim, k = mesh["dim"], mesh["k"]
    nx = k * n + 1
    idx = np.indices((nx,) * dim).reshape(dim, -1)[::-1].T  # lexicographic, x fastest
    bits = np.zeros(idx.shape[0], dtype=np.int64)
    for d in range(dim):
        lo_b = 1 << (2 * d if colorize else 0)
        hi_b = 1 << (2 * d + 1 if colorize else 0)
        bits |= np.where(idx[:, d] == 0, lo_b, 0)
        bits |= np.where(idx[:, d] == nx - 1, hi_b, 0)
    coords = lo + idx * ((hi - lo) / (k * n))
    return bits, coords


def dirichlet_from_bcs(mesh, n, lo, hi, colorize, bcs):
    """bcs: list of (type, boundary_id, values) in bc order, type in {noslip, function, slip};
    values: callable(coords[m,dim]) -> [m,dim] or a constant tuple. deal.II first-wins rule.
    slip: compute_no_normal_flux_constraints (gls_navier_stokes.cc:100-110, 149-160) on the box's
    axis-aligned faces, i.e. the normal component(s) of the faces with that id are set to 0.
    Returns (vnode_mask uint8, dofs int64, values float64)."""
    dim, k = mesh["dim"], mesh["k"]
    bits, X = vnode_boundary_ids(mesh, n, lo, hi, colorize)
    nx = k * n + 1
    idx = np.indices((nx,) * dim).reshape(dim, -1)[::-1].T
    nv = bits.shape[0]
    taken = np.zeros((nv, dim), dtype=bool)
    vals = np.zeros((nv, dim))
    for typ, bid, f in bcs:
        sel = np.nonzero(bits & (1 << bid))[0]
        if sel.size == 0:
            continue
        comps = np.ones((sel.size, dim), dtype=bool)
        if typ == "noslip":
            v = np.zeros((sel.size, dim))
        elif typ == "function":
            v = np.asarray(f(X[sel]) if callable(f) else np.broadcast_to(np.asarray(f, dtype=float)[:dim],
                                                                          (sel.size, dim)), dtype=float)
        elif typ == "slip":
            v = np.zeros((sel.size, dim))
            for d in range(dim):
                on_lo = (idx[sel, d] == 0) & ((2 * d if colorize else 0) == bid)
                on_hi = (idx[sel, d] == nx - 1) & ((2 * d + 1 if colorize else 0) == bid)
                comps[:, d] = on_lo | on_hi
        else:
            raise ValueError("unsupported bc type %s" % typ)
        free = ~taken[sel] & comps
        vals[sel] = np.where(free, v, vals[sel])
        taken[sel] |= comps
    mask = np.zeros(nv, dtype=np.uint8)
    for c in range(dim):
        mask |= (taken[:, c].astype(np.uint8) << c)
    nodes, comps = np.nonzero(taken)
    dofs = nodes.astype(np.int64) * dim + comps
    return mask, dofs, vals[nodes, comps]


def build_context(mesh, viscosity=1.0, vnode_mask=None, force_q=None, srf=False, omega=(0, 0, 0), stream=None):
    return GLSContext(mesh["dim"], mesh["k"], mesh["kp"], mesh["cell_vnodes"], mesh["cell_pnodes"], mesh["cell_h"],
                      mesh["n_vnodes"], mesh["n_pnodes"], viscosity=viscosity, cell_x0=mesh["cell_x0"],
                      vnode_mask=vnode_mask, force_q=force_q, srf=srf, omega=omega, stream=stream)


class CavityProblem:
    """3D (or 2D) lid-driven cavity on hyper_cube(-1, 1, colorize=true): walls noslip, lid y=+1
    (boundary id 3) u=(1,0,0) — examples/01-cavity/cavity.prm:46-55 extended to 3D.
    The lid bc is listed last so the wall edges keep u=0 (first bc wins)."""

    def __init__(self, dim=3, n=8, k=2, kp=None, viscosity=0.01, stream=None, multigrid=False, mg_coarsest=4,
                 **mg_opts):
        kp = k if kp is None else kp
        self.dim, self.n, self.k, self.kp = dim, n, k, kp
        self.mesh = hyper_cube(dim, n, k, kp, -1.0, 1.0)
        walls = [i for i in range(2 * dim) if i != 3]
        bcs = [("noslip", b, None) for b in walls] + [("function", 3, (1.0, 0.0, 0.0))]
        self.vnode_mask, self.dir_dofs, self.dir_vals = dirichlet_from_bcs(self.mesh, n, -1.0, 1.0, True, bcs)
        self.ctx = build_context(self.mesh, viscosity=viscosity, vnode_mask=self.vnode_mask, stream=stream)
        self.ctx.set_dirichlet(self.dir_dofs, self.dir_vals)
        self.n_dofs = self.ctx.n_dofs
        self.levels = []
        if multigrid:  # nested hyper_cube levels n/2, n/4, ... down to mg_coarsest cells per direction
            m = n
            while m % 2 == 0 and m // 2 >= mg_coarsest:
                m //= 2
                self.levels.append(CavityProblem(dim, m, k, kp, viscosity, stream))
            self.ctx.attach_multigrid([lv.ctx for lv in self.levels], **mg_opts)


def octree_lid_tree(n=4, steps=3, dim=3, base=2):
    """An adapted forest for the cavity: n^dim cells (a base^dim forest refined globally to n per
    direction, so the multigrid hierarchy reaches down to base^dim cells), then `steps` refinements of
    the cells next to the lid (y = +1) and its two upper edges, each step one level deeper and one half
    thinner (a Kelly-like boundary-layer grading: gls_octree_adapt with the vertex 2:1 balance)."""
    from .native import Octree
    base = base if n % base == 0 and (n // base) & (n // base - 1) == 0 else n
    t = Octree(dim, base)
    g = 0
    while base << g < n:
        t.adapt(refine=np.ones(t.n_cells, np.int32))
        g += 1
    for s in range(steps):
        lev, x0, h = t.cells()
        c = x0 + 0.5 * h
        band = 1.0 - 2.0 ** -s
        near = (c[:, 1] > band) | ((c[:, 1] > 0.0) & (np.abs(c[:, 0]) > band))
        t.adapt(refine=near.astype(np.int32), max_level=g + s + 1)
    return t


def octree_dirichlet(mesh, lo=-1.0, hi=1.0):
    """CavityProblem's boundary conditions on an octree mesh (walls noslip, lid y = hi u = (1, 0, 0),
    wall edges keep u = 0): (vnode_mask, dofs, values); hanging nodes carry no mask bit (their lines
    give their values)."""
    dim, X = mesh["dim"], mesh["vnode_x"]
    tol = 1e-12 * (hi - lo)
    on = [(np.abs(X[:, d] - lo) < tol, np.abs(X[:, d] - hi) < tol) for d in range(dim)]
    wall = np.zeros(len(X), bool)
    for d in range(dim):
        wall |= on[d][0] | (on[d][1] if d != 1 else False)
    lid = on[1][1] & ~wall
    bnd = wall | lid
    hang = np.zeros(len(X), bool)
    hang[mesh["vhang"][0]] = True
    bnd &= ~hang
    mask = np.where(bnd, (1 << dim) - 1, 0).astype(np.uint8)
    nodes = np.nonzero(bnd)[0]
    dofs = (nodes[:, None] * dim + np.arange(dim)[None]).reshape(-1).astype(np.int64)
    vals = np.zeros((len(nodes), dim))
    vals[lid[nodes], 0] = 1.0
    return mask, dofs, vals.reshape(-1)


class AdaptiveCavityProblem:
    """CavityProblem's lid-driven cavity on an adapted octree forest (hanging-node constraints,
    gls_set_hanging; per-cell kernels). multigrid=True: the GMRES preconditioner is the V-cycle on the
    refinement hierarchy (gls_mg_attach_transfers) -- levels = the forest coarsened one level at a time
    (gls_octree_coarsen_to), transfers = gls_octree_mg_transfer, and the uniform level-0 mesh as the
    brick context of a CavityProblem (the same lexicographic node numbering) with an exact LU solve."""

    def __init__(self, tree, k=2, kp=None, viscosity=0.01, stream=None, multigrid=False, **mg_opts):
        from .native import hanging_dof_lines, octree_mg_transfer
        kp = k if kp is None else kp
        self.dim, self.k, self.kp, self.tree = tree.dim, k, kp, tree
        L = tree.max_level
        self.trees = [tree.coarsen_to(L - l) for l in range(L + 1)] if multigrid else [tree]
        self.levels, self.meshes = [], []
        for l, t in enumerate(self.trees):
            mesh = t.mesh(k, kp)
            self.meshes.append(mesh)
            lines = hanging_dof_lines(mesh)
            if multigrid and l == len(self.trees) - 1 and len(lines[0]) == 0:
                base = CavityProblem(tree.dim, tree.n, k, kp, viscosity, stream)
                nx = k * tree.n + 1
                idx = np.indices((nx,) * tree.dim).reshape(tree.dim, -1)[::-1].T
                if not np.allclose(mesh["vnode_x"], -1.0 + idx * (2.0 / (k * tree.n)), atol=1e-13):
                    raise RuntimeError("level-0 numbering differs from the hyper_cube's")
                self.levels.append(base.ctx)
                continue
            mask, dofs, vals = octree_dirichlet(mesh)
            ctx = build_context(mesh, viscosity=viscosity, vnode_mask=mask, stream=stream)
            if len(lines[0]):
                ctx.set_hanging(*lines)
            ctx.set_dirichlet(dofs, vals)
            self.levels.append(ctx)
        self.ctx = self.levels[0]
        self.mesh = self.meshes[0]
        self.n_dofs = self.ctx.n_dofs
        if multigrid:
            xfer = []
            for l in range(len(self.trees) - 1):
                hf, hc = self.trees[l].mesh_handle(k, kp), self.trees[l + 1].mesh_handle(k, kp)
                try:
                    xfer.append(octree_mg_transfer(hf, hc))
                finally:
                    self.trees[l].free_mesh_handle(hf)
                    self.trees[l + 1].free_mesh_handle(hc)
            self.ctx.attach_multigrid_transfers(self.levels[1:], xfer, **mg_opts)
