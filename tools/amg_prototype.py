"""AMG study for the configs[4] problem (tooling, CPU, not product code): the Q2-Q1 -> Q1-Q1 p-multigrid of
tools/pmg_prototype.py with a smoothed-aggregation AMG on the Q1-Q1 level instead of its exact LU (which gave 6
GMRES iterations; one ILU(0) apply there gave 173). The reference preconditions `method = amg` with Trilinos ML
(setup_AMG, gls_navier_stokes.cc:1180-1240: smoothed aggregation, ILU smoother); this restates the method on the
oracle's assembled matrices to choose the aggregation / smoother before the device build.
Node-block aggregation (4 DoFs per Q1 node: u, v, w, p), tentative prolongator with identity blocks, Jacobi
smoothed (omega = 4/3 / rho(D^-1 A)), Galerkin R A P, down to <= 2000 DoFs (dense LU).
Usage: python tools/amg_prototype.py   (the first run assembles with the oracle and caches /tmp/amg_proto.npz)"""
import os
import sys
import time

import numpy as np
import scipy.sparse as sps
import scipy.sparse.linalg as spla

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

CACHE = "/tmp/amg_proto.npz"


def assemble():
    from oracle.oracle import Oracle
    from pmg_prototype import problem, prolongation, state
    from softx_2020_200_amd.native import UMesh
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
    P = prolongation(spF, spC, pF.n_dofs, pC.n_dofs)
    np.savez(CACHE, AF_data=AF.data, AF_ind=AF.indices, AF_ptr=AF.indptr, AF_shape=AF.shape,
             AC_data=AC.data, AC_ind=AC.indices, AC_ptr=AC.indptr, AC_shape=AC.shape,
             P_data=P.data, P_ind=P.indices, P_ptr=P.indptr, P_shape=P.shape, b=b,
             conF=pF.constrained.astype(bool), conC=pC.constrained.astype(bool), nvC=spC["n_vnodes"])


def load():
    if not os.path.exists(CACHE):
        assemble()
    z = np.load(CACHE)
    mk = lambda t: sps.csr_matrix((z[t + "_data"], z[t + "_ind"], z[t + "_ptr"]), shape=tuple(z[t + "_shape"]))  # noqa: E731
    return mk("AF"), mk("AC"), mk("P"), z["b"], z["conF"], z["conC"], int(z["nvC"])


def node_of_dofs(nv):
    """Q1-Q1 DoF layout [3 nv velocity, interleaved | nv pressure] -> node id per DoF"""
    return np.concatenate([np.repeat(np.arange(nv), 3), np.arange(nv)])


def aggregate(S, n):
    """Vanek's greedy aggregation on the node graph S (CSR, strong connections, symmetric pattern)"""
    agg = -np.ones(n, np.int64)
    na = 0
    # phase 1: nodes whose whole strong neighbourhood is free start an aggregate
    for i in range(n):
        if agg[i] >= 0:
            continue
        nb = S.indices[S.indptr[i]:S.indptr[i + 1]]
        if (agg[nb] < 0).all():
            agg[i] = na
            agg[nb] = na
            na += 1
    # phase 2: free nodes join a neighbouring aggregate (the strongest connection)
    for i in range(n):
        if agg[i] >= 0:
            continue
        nb = S.indices[S.indptr[i]:S.indptr[i + 1]]
        w = S.data[S.indptr[i]:S.indptr[i + 1]]
        cand = [(wj, j) for wj, j in zip(w, nb) if agg[j] >= 0]
        if cand:
            agg[i] = -2 - agg[max(cand)[1]]  # mark, resolve after the sweep (phase-1 aggregates only)
    for i in range(n):
        if agg[i] <= -2:
            agg[i] = -2 - agg[i]
    # phase 3: the rest form aggregates with their free neighbours
    for i in range(n):
        if agg[i] >= 0:
            continue
        agg[i] = na
        for j in S.indices[S.indptr[i]:S.indptr[i + 1]]:
            if agg[j] < 0:
                agg[j] = na
        na += 1
    return agg, na


def build_hierarchy(A, nodes, nn, theta=0.08, smooth=True, max_coarse=2000, bs=4):
    levels = []
    while A.shape[0] > max_coarse and len(levels) < 10:
        # node-block strength: |A_ij|_F between nodes, scaled by the diagonal blocks
        Ab = sps.csr_matrix((np.abs(A.data) ** 2, A.indices, A.indptr), shape=A.shape)
        G = sps.csr_matrix((np.ones(len(nodes)), (nodes, np.arange(len(nodes)))), shape=(nn, A.shape[0]))
        B = (G @ Ab @ G.T).tocsr()
        B.data = np.sqrt(B.data)
        dg = np.sqrt(np.maximum(B.diagonal(), 1e-300))
        Bc = B.tocoo()
        keep = (Bc.row != Bc.col) & (Bc.data > theta * dg[Bc.row] * dg[Bc.col])
        S = sps.csr_matrix((Bc.data[keep], (Bc.row[keep], Bc.col[keep])), shape=B.shape)
        S = S.maximum(S.T).tocsr()
        agg, na = aggregate(S, nn)
        # tentative prolongator: DoF d of node i -> DoF (agg[i], slot) with the DoF's slot within its node
        slot = np.zeros(A.shape[0], np.int64)
        order = np.argsort(nodes, kind="stable")
        cnt = np.zeros(nn, np.int64)
        for d in order:
            slot[d] = cnt[nodes[d]]
            cnt[nodes[d]] += 1
        Pt = sps.csr_matrix((np.ones(A.shape[0]), (np.arange(A.shape[0]), agg[nodes] * bs + slot)),
                            shape=(A.shape[0], na * bs))
        Pt = Pt[:, np.unique(Pt.indices)].tocsr() if Pt.shape[1] != len(np.unique(Pt.indices)) else Pt
        d = A.diagonal()
        Dinv = sps.diags(1.0 / d)
        if smooth:
            x = np.random.default_rng(0).uniform(-1, 1, A.shape[0])
            for _ in range(15):
                x = Dinv @ (A @ x)
                x /= np.linalg.norm(x)
            rho = np.linalg.norm(Dinv @ (A @ x))
            P = (Pt - (4.0 / 3.0 / rho) * (Dinv @ (A @ Pt))).tocsr()
        else:
            P = Pt
        R = P.T.tocsr()
        Ac = (R @ A @ P).tocsr()
        levels.append(dict(A=A, P=P, R=R, d=d))
        # coarse nodes: aggregates, DoFs slot-major inside each
        nodes = np.repeat(np.arange(na), bs)[:Ac.shape[0]] if Pt.shape[1] == na * bs else np.repeat(np.arange(na), bs)
        nn = na
        A = Ac
    levels.append(dict(A=A, lu=spla.splu(A.tocsc())))
    return levels


def amg_vcycle(levels, b, l=0, nu=1, om=0.7, smoother="jacobi"):
    L = levels[l]
    if "lu" in L:
        return L["lu"].solve(b)
    A, d = L["A"], L["d"]
    if smoother == "ilu":
        if "ilu" not in L:
            L["ilu"] = spla.spilu(A.tocsc(), drop_tol=0.0, fill_factor=1.0, permc_spec="NATURAL")
        sm = lambda r: L["ilu"].solve(r)  # noqa: E731
    else:
        sm = lambda r: om * r / d  # noqa: E731
    x = sm(b)
    for _ in range(nu - 1):
        x = x + sm(b - A @ x)
    r = b - A @ x
    x = x + L["P"] @ amg_vcycle(levels, L["R"] @ r, l + 1, nu, om, smoother)
    for _ in range(nu):
        x = x + sm(b - A @ x)
    return x


def main():
    t0 = time.time()
    AF, AC, P, b, conF, conC, nvC = load()
    R = P.T.tocsr()
    d = AF.diagonal()
    print("Q2-Q1 %d DoFs, Q1-Q1 %d DoFs (%d nnz), loaded in %.1f s" % (AF.shape[0], AC.shape[0], AC.nnz, time.time() - t0),
          flush=True)
    nodes = node_of_dofs(nvC)

    def run(M, tag):
        its = [0]
        x, info = spla.gmres(AF, b, M=M, restart=30, rtol=1e-4, atol=0, maxiter=10,
                             callback=lambda r: its.__setitem__(0, its[0] + 1), callback_type="pr_norm")
        rel = np.linalg.norm(b - AF @ x) / np.linalg.norm(b)
        print("%-70s its %4d conv %s rel %.2e" % (tag, its[0], info == 0, rel), flush=True)

    for theta, smooth in ((0.08, True), (0.02, True), (0.08, False)):
        t1 = time.time()
        lev = build_hierarchy(AC, nodes, nvC, theta=theta, smooth=smooth)
        sizes = [L["A"].shape[0] for L in lev]
        print("AMG theta %.2f smooth %s: levels %s, setup %.1f s" % (theta, smooth, sizes, time.time() - t1), flush=True)
        for cyc, nu, smo in ((1, 1, "jacobi"), (1, 2, "jacobi"), (2, 1, "jacobi"), (1, 1, "ilu")):
            def coarse(rc, cyc=cyc, nu=nu, smo=smo):
                x = amg_vcycle(lev, rc, nu=nu, smoother=smo)
                for _ in range(cyc - 1):
                    x = x + amg_vcycle(lev, rc - AC @ x, nu=nu, smoother=smo)
                return x

            def vcycle(r, om=0.7):
                z = om * r / d
                res = r - AF @ z
                rc = R @ res
                rc[conC] = 0.0
                e = P @ coarse(rc)
                e[conF] = 0.0
                z = z + e
                return z + om * (r - AF @ z) / d
            run(spla.LinearOperator(AF.shape, vcycle), "p-MG Jacobi(1,1) + AMG(theta %.2f, %s) x%d V(%d,%d) %s" % (
                theta, "SA" if smooth else "UA", cyc, nu, nu, smo))


if __name__ == "__main__":
    main()
