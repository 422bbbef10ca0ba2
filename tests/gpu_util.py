"""Helpers shared by the GPU parity tests: build a product context from an oracle problem."""
import numpy as np


def vnode_mask_of(p):
    """zero_constraints mask of the Dirichlet DoFs (hanging DoFs are passed as lines, not masked)."""
    c = p.constrained[:p.dim * p.n_vnodes].copy()
    if getattr(p, "hang", None) is not None:
        c[np.nonzero(p.hang[0][1:p.dim * p.n_vnodes + 1] > p.hang[0][:p.dim * p.n_vnodes])[0]] = 0
    c = c.reshape(p.n_vnodes, p.dim).astype(np.uint8)
    m = np.zeros(p.n_vnodes, dtype=np.uint8)
    for d in range(p.dim):
        m |= c[:, d] << d
    return m


def context_for(p, **kw):
    from softx_2020_200_amd import GLSContext
    mapped = getattr(p, "cell_support", None) is not None
    if mapped:
        kw = dict(kw, map_degree=p.map_degree, cell_support=p.cell_support)
    ctx = GLSContext(p.dim, p.k, p.kp, p.cell_vnodes, p.cell_pnodes if p.kp != p.k else None,
                     None if mapped else p.cell_h, p.n_vnodes, p.n_pnodes, viscosity=p.viscosity,
                     cell_x0=None if mapped else p.cell_x0, vnode_mask=vnode_mask_of(p),
                     force_q=p.force_q, srf=p.srf, omega=p.omega, **kw)
    ctx.set_time(p.scheme, p.time_steps)
    if getattr(p, "hang_lines", None) is not None:
        ctx.set_hanging(*p.hang_lines)
    if p.dirichlet:
        dofs = np.array(sorted(p.dirichlet), dtype=np.int64)
        ctx.set_dirichlet(dofs, np.array([p.dirichlet[d] for d in dofs]))
    return ctx


def cuda(a):
    import torch
    return torch.tensor(np.asarray(a), dtype=torch.float64, device="cuda")


def relerr(a, b):
    a = np.asarray(a)
    b = np.asarray(b)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-300))
