"""Feasibility probe (not product code): monolithic geometric multigrid V-cycle preconditioner for
the GLS Jacobian on nested hyper_cube levels, using the HIP operators of each level through the
C-ABI, exact Qk prolongation on the node lattice, damped-Jacobi smoothing. Measures GMRES
iterations vs plain Jacobi. Usage: python tools/gmg_probe.py N_FINE [k]"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from softx_2020_200_amd.problem import CavityProblem  # noqa: E402

nf = int(sys.argv[1]) if len(sys.argv) > 1 else 32
k = int(sys.argv[2]) if len(sys.argv) > 2 else 2
omega = float(os.environ.get("OMEGA", "0.6"))
nsm = int(os.environ.get("NSMOOTH", "2"))
ncoarse = int(os.environ.get("NCOARSE", "4"))
dev = "cuda"


def prolong_1d(nc_cells, k):
    """(k*2n+1) x (k*n+1) interpolation of Qk nodal values from the coarse to the fine lattice."""
    nfine, ncoarse_n = k * 2 * nc_cells + 1, k * nc_cells + 1
    P = np.zeros((nfine, ncoarse_n))
    xn = np.linspace(0, 1, k + 1)
    for i in range(nfine):
        x = i / (2.0 * k)  # position in coarse-cell units
        c = min(int(x), nc_cells - 1)
        xi = x - c
        for a in range(k + 1):
            L = 1.0
            for b in range(k + 1):
                if b != a:
                    L *= (xi - xn[b]) / (xn[a] - xn[b])
            P[i, c * k + a] += L
    return torch.tensor(P, dtype=torch.float64, device=dev)


class Level:
    def __init__(self, n):
        self.n = n
        self.p = CavityProblem(dim=3, n=n, k=k, viscosity=0.01)
        self.ctx = self.p.ctx
        self.ctx.set_time("bdf2", (0.01,) * 4)
        self.nx = k * n + 1
        self.N = self.ctx.n_dofs
        self.nv = self.p.mesh["n_vnodes"]
        con = np.zeros(self.N, dtype=bool)
        con[self.p.dir_dofs] = True
        self.free = torch.tensor(~con, device=dev).double()

    def split(self, x):
        v = x[:3 * self.nv].view(self.nx, self.nx, self.nx, 3)
        p = x[3 * self.nv:].view(self.nx, self.nx, self.nx)
        return v, p


def restrict_state(fine: Level, coarse: Level, x):
    v, p = fine.split(x)
    vc = v[::2, ::2, ::2, :].reshape(-1)
    pc = p[::2, ::2, ::2].reshape(-1)
    out = torch.cat([vc, pc]).contiguous()
    out[torch.tensor(coarse.p.dir_dofs, device=dev)] = torch.tensor(coarse.p.dir_vals, device=dev)
    return out


def apply_sep(P, a, axes):
    # a: [z][y][x](,c) ; apply P along the three spatial axes
    a = torch.einsum("iz,zyx...->iyx...", P, a)
    a = torch.einsum("jy,iyx...->ijx...", P, a)
    a = torch.einsum("kx,ijx...->ijk...", P, a)
    return a


def prolong(coarse: Level, fine: Level, P, xc):
    v, p = coarse.split(xc)
    vf = apply_sep(P, v, None).reshape(-1)
    pf = apply_sep(P, p, None).reshape(-1)
    return torch.cat([vf, pf]) * fine.free


def restrict(fine: Level, coarse: Level, P, rf):
    v, p = fine.split(rf * fine.free)
    PT = P.t().contiguous()
    vc = apply_sep(PT, v, None).reshape(-1)
    pc = apply_sep(PT, p, None).reshape(-1)
    return torch.cat([vc, pc]) * coarse.free


def main():
    ns = [nf]
    while ns[-1] // 2 >= ncoarse:
        ns.append(ns[-1] // 2)
    levels = [Level(n) for n in ns]
    Ps = [prolong_1d(levels[i + 1].n, k) for i in range(len(levels) - 1)]
    L0 = levels[0]
    m1 = torch.from_numpy(bench.smooth_state(L0.p.mesh, nf, 3, L0.p.dir_dofs, L0.p.dir_vals, 0.0)).to(dev)
    m2 = torch.from_numpy(bench.smooth_state(L0.p.mesh, nf, 3, L0.p.dir_dofs, L0.p.dir_vals, 0.3)).to(dev)
    states = [(m1, m1.clone(), m2)]
    for i in range(1, len(levels)):
        u, a, b = states[-1]
        states.append(tuple(restrict_state(levels[i - 1], levels[i], t) for t in (u, a, b)))
    for L, (u, a, b) in zip(levels, states):
        L.state = (u, a, b)
        L.ctx.set_state(u, a, b)
        L.diag = L.ctx.jacobian_diagonal().clone()

    def A(L, x):
        return L.ctx.jacobian_apply(x.contiguous())

    def smooth(L, x, b, steps):
        for _ in range(steps):
            x = x + omega * (b - A(L, x)) / L.diag
        return x

    def vcycle(li, b):
        L = levels[li]
        if li == len(levels) - 1:
            return smooth(L, torch.zeros_like(b), b, 30)
        x = smooth(L, torch.zeros_like(b), b, nsm)
        r = b - A(L, x)
        xc = vcycle(li + 1, restrict(L, levels[li + 1], Ps[li], r))
        x = x + prolong(levels[li + 1], L, Ps[li], xc)
        return smooth(L, x, b, nsm)

    rhs = L0.ctx.residual().clone()

    def gmres(M, b, tol, maxit=300, m=60):
        x = torch.zeros_like(b)
        beta = b.norm().item()
        hist = [beta]
        V = [b / beta]
        H = np.zeros((m + 1, m))
        its = 0
        g = np.zeros(m + 1)
        g[0] = beta
        Z = []
        cs, sn = np.zeros(m), np.zeros(m)
        for j in range(m):
            z = M(V[j])
            Z.append(z)
            w = A(L0, z)
            for i in range(j + 1):
                H[i, j] = torch.dot(V[i], w).item()
                w = w - H[i, j] * V[i]
            H[j + 1, j] = w.norm().item()
            V.append(w / H[j + 1, j])
            for i in range(j):
                t = cs[i] * H[i, j] + sn[i] * H[i + 1, j]
                H[i + 1, j] = -sn[i] * H[i, j] + cs[i] * H[i + 1, j]
                H[i, j] = t
            r = np.hypot(H[j, j], H[j + 1, j])
            cs[j], sn[j] = H[j, j] / r, H[j + 1, j] / r
            H[j, j] = r
            g[j + 1] = -sn[j] * g[j]
            g[j] = cs[j] * g[j]
            its += 1
            hist.append(abs(g[j + 1]))
            if abs(g[j + 1]) < tol:
                break
        return its, hist

    tol = 1e-4 * rhs.norm().item()
    for name, M in [("jacobi", lambda v: v / L0.diag), ("gmg", lambda v: vcycle(0, v))]:
        torch.cuda.synchronize()
        t = time.time()
        its, hist = gmres(M, rhs, tol, m=100 if name == "gmg" else 300)
        torch.cuda.synchronize()
        print("%-7s n=%d levels=%s omega=%.2f nsmooth=%d: %d its, rel res %.2e, %.2f s; hist %s" % (
            name, nf, ns, omega, nsm, its, hist[-1] / hist[0], time.time() - t,
            " ".join("%.1e" % (h / hist[0]) for h in hist[::max(1, len(hist) // 12)])), flush=True)


if __name__ == "__main__":
    main()
