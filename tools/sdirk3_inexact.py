"""SDIRK3 Taylor-Green golden (taylor-green-vortex_gls_sdirk3.mpirun=2.output: 1.38223e-4) under the
reference's INEXACT Newton: tolerance 1e-6, max 5 iterations, GMRES(30) to max(1e-4 ||rhs||, 1e-9)
from a zero guess (solve_system_GMRES, gls_navier_stokes.cc:1242-1289), with several stand-ins for
the reference's Trilinos ILU(1) (not reproducible here). Exact linear solves give 1.38239e-4.
Tooling (oracle-based experiment), not a test. Usage: python tools/sdirk3_inexact.py"""
import os
import sys

import numpy as np
import scipy.sparse as sp
import scipy.sparse.linalg as spla

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle.oracle import Oracle, StructuredProblem  # noqa: E402
from tests.test_oracle_goldens import G, muparser_to_numpy  # noqa: E402


def newton_inexact(p, orc, x0, u1, u2, u3, prec, tol=1e-6, max_it=5):
    x = np.array(x0)
    p.apply_nonzero_constraints(x)
    pin = p.dim * p.n_vnodes
    last_res = cur_res = 1.0
    it = 0
    while cur_res > tol and it < max_it:
        A, rhs = orc.matrix_and_rhs(x, u1, u2, u3)
        if it == 0:
            cur_res = last_res = np.linalg.norm(rhs)
        A = A.tolil()
        A[pin, :] = 0
        A[:, pin] = 0
        A[pin, pin] = 1.0
        A = sp.csc_matrix(A)
        b = rhs.copy()
        b[pin] = 0.0
        if prec == "exact":
            dx = spla.spsolve(A, b)
        else:
            if prec == "jacobi":
                d = A.diagonal()
                M = spla.LinearOperator(A.shape, lambda v: v / d)
            else:
                ilu = spla.spilu(A, drop_tol=float(prec), fill_factor=4)
                M = spla.LinearOperator(A.shape, ilu.solve)
            tol_abs = max(1e-4 * np.linalg.norm(b), 1e-9)
            dx, info = spla.gmres(A, b, M=M, restart=30, maxiter=200, atol=tol_abs, rtol=0.0)
        dx[p.constrained.astype(bool)] = 0.0
        alpha = 1.0
        while alpha > 1e-3:
            xt = x + alpha * dx
            p.apply_nonzero_constraints(xt)
            cur_res = np.linalg.norm(orc.residual(xt, u1, u2, u3))
            if cur_res < 0.9 * last_res or last_res < tol:
                break
            alpha *= 0.5
        x = xt
        last_res = cur_res
        it += 1
    return x, it, cur_res


def run(prec):
    c = G["tgv_common"]
    IC = muparser_to_numpy(c["initial_condition"])
    p = StructuredProblem(2, 64, k=2, kp=1, lo=c["domain"][0], hi=c["domain"][1], colorize=True, periodic=(0, 1),
                          time_steps=(0.1,) * 4, viscosity=c["viscosity"])
    orc = Oracle(p)
    x = orc.l2_projection(IC)
    hist = [x.copy(), None, None]
    its = []
    for si, st in enumerate(["sdirk3_1", "sdirk3_2", "sdirk3_3"]):
        p.scheme = st
        x, it, res = newton_inexact(p, orc, x, hist[0], hist[1], hist[2], prec)
        its.append((it, res))
        if si < 2:
            hist[si + 1] = x.copy()
    nu, t = c["viscosity"], 0.1
    E = lambda X: np.stack([np.exp(-2 * nu * t) * np.cos(X[:, 0]) * np.sin(X[:, 1]),
                            -np.sin(X[:, 0]) * np.cos(X[:, 1]) * np.exp(-2 * nu * t), 0 * X[:, 0]], 1)
    return orc.l2_error(x, E)[0], its


if __name__ == "__main__":
    print("reference golden 1.38223e-04")
    for prec in ["exact", "jacobi", "1e-2", "1e-3", "1e-4"]:
        e, its = run(prec)
        print("%-7s L2 error velocity %.6e  Newton (its, final residual) per stage %s" % (prec, e, its), flush=True)
