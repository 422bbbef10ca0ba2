"""Preconditioner study for the configs[4] problem (tooling, CPU, not product code): can a p-multigrid
(Q2-Q1 -> Q1-Q1 on the same mapped mesh) replace the multicolor ILU(0) of the adaptive path (60 GMRES
iterations per Newton step on the GPU)? Assembles with the oracle (oracle/gls_oracle.c) the Q2-Q1 Jacobian
of apps/cases/cylinder3d_extruded.msh at the bench's synthetic BDF2 state and the Q1-Q1 one at the
injected state, builds the geometry-independent Q1 -> Q2 interpolation per cell (pressure: the same Q1
space), and runs scipy GMRES(30) to rel 1e-4 with a V(1,1) cycle: damped-Jacobi smoothing on Q2,
restriction = P^T, a coarse solve, prolongation. Results: profiles/r04_pmg_prototype.txt.
Usage: python tools/pmg_prototype.py   (several minutes; ~3 GB)"""
import os
import sys
import time

import numpy as np
import scipy.sparse as sps
import scipy.sparse.linalg as spla

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle.oracle import MappedProblem, Oracle  # noqa: E402
from softx_2020_200_amd.native import UMesh  # noqa: E402


def problem(m, k, kp):
    sp = m.fe_space(k, kp)
    p = MappedProblem(sp, viscosity=0.005, scheme="bdf2", time_steps=(0.05,) * 4)
    inlet = lambda X: np.stack([np.ones(len(X)), 0 * X[:, 0], 0 * X[:, 0]], 1)  # noqa: E731
    p.set_dirichlet([("noslip", 0, None), ("function", 1, inlet), ("slip", 2, None), ("slip", 4, None),
                     ("slip", 5, None)])
    return sp, p


def state(X, npn):  # bench.cylinder3d_context's synthetic state
    r2 = X[:, 0] ** 2 + X[:, 1] ** 2
    vel = np.zeros((len(X), 3))
    vel[:, 0] = 1.0 - np.exp(-r2 / 4.0) * (1.0 + 0.2 * np.sin(X[:, 2]))
    vel[:, 1] = 0.1 * np.exp(-r2 / 4.0) * X[:, 1]
    return np.concatenate([vel.reshape(-1), np.zeros(npn)])


def prolongation(spF, spC, nF, nC):
    cvF = np.asarray(spF["cell_vnodes"]).reshape(-1, 27)
    cvC = np.asarray(spC["cell_vnodes"]).reshape(-1, 8)
    cpF = np.asarray(spF["cell_pnodes"]).reshape(-1, 8)
    cpC = np.asarray(spC["cell_pnodes"]).reshape(-1, 8)
    nvF, nvC = spF["n_vnodes"], spC["n_vnodes"]
    rows, cols, vals = [], [], []
    seen = np.zeros(nvF, bool)
    xi = (0.0, 0.5, 1.0)
    for c in range(cvF.shape[0]):
        for a in range(27):
            i = cvF[c, a]
            if seen[i]:
                continue
            seen[i] = True
            ax, ay, az = a % 3, (a // 3) % 3, a // 9
            for v in range(8):
                w = ((xi[ax] if v & 1 else 1 - xi[ax]) * (xi[ay] if (v >> 1) & 1 else 1 - xi[ay]) *
                     (xi[az] if v >> 2 else 1 - xi[az]))
                if w:
                    for comp in range(3):
                        rows.append(3 * i + comp)
                        cols.append(3 * cvC[c, v] + comp)
                        vals.append(w)
    pm = {int(cpF[c, v]): int(cpC[c, v]) for c in range(cpF.shape[0]) for v in range(8)}
    for i, j in pm.items():
        rows.append(3 * nvF + i)
        cols.append(3 * nvC + j)
        vals.append(1.0)
    return sps.csr_matrix((vals, (rows, cols)), shape=(nF, nC))


def main():
    m = UMesh(3, gmsh=os.path.join(ROOT, "apps", "cases", "cylinder3d_extruded.msh"))
    spF, pF = problem(m, 2, 1)
    spC, pC = problem(m, 1, 1)
    uF = state(spF["vnode_x"], spF["n_pnodes"])
    pF.apply_nonzero_constraints(uF)
    uC = state(spC["vnode_x"], spC["n_pnodes"])
    pC.apply_nonzero_constraints(uC)
    AF, b = Oracle(pF).matrix_and_rhs(uF, uF, uF)
    AC, _ = Oracle(pC).matrix_and_rhs(uC, uC, uC)
    AF, AC = sps.csr_matrix(AF), sps.csr_matrix(AC)
    conF, conC = pF.constrained.astype(bool), pC.constrained.astype(bool)
    P = prolongation(spF, spC, pF.n_dofs, pC.n_dofs)
    R = P.T.tocsr()
    d = AF.diagonal()
    print("Q2-Q1 %d DoFs (%d nnz), Q1-Q1 %d DoFs (%d nnz)" % (AF.shape[0], AF.nnz, AC.shape[0], AC.nnz), flush=True)
    luC = spla.splu(AC.tocsc())
    iluC = spla.spilu(AC.tocsc(), drop_tol=0.0, fill_factor=1.0, permc_spec="NATURAL")

    def run(M, tag):
        its = [0]
        x, info = spla.gmres(AF, b, M=M, restart=30, rtol=1e-4, atol=0, maxiter=10,
                             callback=lambda r: its.__setitem__(0, its[0] + 1), callback_type="pr_norm")
        rel = np.linalg.norm(b - AF @ x) / np.linalg.norm(b)
        print("%-52s GMRES(30) its %4d  converged %s  true rel. residual %.2e" % (tag, its[0], info == 0, rel), flush=True)

    def vcycle(r, om, coarse):
        z = om * r / d
        res = r - AF @ z
        rc = R @ res
        rc[conC] = 0.0
        e = P @ (luC.solve(rc) if coarse == "lu" else iluC.solve(rc))
        e[conF] = 0.0
        z = z + e
        return z + om * (r - AF @ z) / d

    run(spla.LinearOperator(AF.shape, lambda r: r / d), "Jacobi")
    for om, coarse in ((0.7, "lu"), (0.7, "ilu")):
        run(spla.LinearOperator(AF.shape, lambda r, om=om, coarse=coarse: vcycle(r, om, coarse)),
            "p-MG V(1,1) Jacobi w%.1f, coarse %s" % (om, "exact LU" if coarse == "lu" else "one ILU(0) apply"))


if __name__ == "__main__":
    main()
