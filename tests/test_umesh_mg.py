"""Multigrid levels of adapted unstructured / curved meshes (gls_umesh_coarsen_to, gls_fe_space_mg_transfer;
SURVEY §8 f1/f2: the reference preconditions these meshes with ILU / ML-AMG, gls_navier_stokes.cc:1161-1240).
CPU: the coarsened triangulations tile the same domain with fewer cells down to the coarse mesh; the
prolongation is FE_Q's embedding (child -> parent reference coordinates): a partition of unity on every fine
master row, empty fine hanging rows, coarse masters as columns, the exact interpolation of linear fields on
straight-sided meshes (in both isoparametric spaces); the injection maps each coarse node onto the fine node at the same point,
on curved meshes too (children's vertices are the parents' manifold points). No reference golden covers a
multigrid hierarchy: the checks are algebraic."""
import numpy as np
import pytest
import scipy.sparse as sps

from tests.test_uforest import CASES, make_mesh, random_adapt

SEED = 20200200


def adapted(name, dim, spec, k):
    m = make_mesh(dim, spec)
    m.refine_global(1)
    random_adapt(m, 2 if dim == 2 else 1, seed=5, k=k)
    return m


def hanging_dofs(sp):
    dim = sp["dim"]
    out = set()
    for nd in sp["vhang"]:
        out |= {nd * dim + c for c in range(dim)}
    return out | {dim * sp["n_vnodes"] + nd for nd in sp["phang"]}


@pytest.mark.parametrize("name,dim,spec,flat", CASES, ids=[c[0] for c in CASES])
@pytest.mark.parametrize("k,kp", [(1, 1), (2, 1), (2, 2)])
def test_umesh_mg_transfer(name, dim, spec, flat, k, kp):
    m = adapted(name, dim, spec, k)
    hf = m.fe_space_handle(k, kp, qmapping_all=True)
    sf = hf.data
    L = int(sf["cell_level"].max())
    assert L >= 2
    prev = sf["n_cells"]
    for lev in range(L - 1, -1, -1):  # the levels tile the domain with fewer cells down to the coarse mesh
        sl = m.coarsen_to(lev).fe_space(k, kp, qmapping_all=True)
        assert sl["cell_level"].max() <= lev and sl["n_cells"] < prev
        assert abs(sl["volume"] - sf["volume"]) < 1e-9 * sf["volume"] or not flat
        prev = sl["n_cells"]
    mc = m.coarsen_to(L - 1)
    hc = mc.fe_space_handle(k, kp, qmapping_all=True)
    sc = hc.data
    off, col, w, inj = hf.mg_transfer_from(hc)
    nf = dim * sf["n_vnodes"] + sf["n_pnodes"]
    nc = dim * sc["n_vnodes"] + sc["n_pnodes"]
    P = sps.csr_matrix((w, col, off), shape=(nf, nc))
    hang_f, hang_c = hanging_dofs(sf), hanging_dofs(sc)
    assert len(hang_f) > 0
    rows = np.array(sorted(set(range(nf)) - hang_f))
    assert all(off[i] == off[i + 1] for i in hang_f)
    assert not (set(np.unique(col).tolist()) & hang_c)
    assert np.abs(np.asarray(P.sum(1)).ravel()[rows] - 1.0).max() < 1e-12
    # injection: the coarse node's point is the fine node's point
    Xf = np.concatenate([np.repeat(sf["vnode_x"], dim, axis=0), sf["pnode_x"]])
    Xc = np.concatenate([np.repeat(sc["vnode_x"], dim, axis=0), sc["pnode_x"]])
    assert np.abs(Xf[inj] - Xc).max() < 1e-12 * max(1.0, np.abs(Xf).max())
    if flat:  # straight-sided (multilinear) cells: every linear field lies in both spaces, interpolated exactly
        rng = np.random.default_rng(SEED + 7 * dim + k)
        a = rng.normal(size=(dim + 1, dim + 1))

        def field(sp):
            lin = lambda X, r: r[0] + X @ r[1:]  # noqa: E731
            vel = np.stack([lin(sp["vnode_x"], a[c]) for c in range(dim)], 1).reshape(-1)
            return np.concatenate([vel, lin(sp["pnode_x"], a[dim])])
        uf, uc = field(sf), field(sc)
        assert np.abs((P @ uc)[rows] - uf[rows]).max() < 1e-10 * max(1.0, np.abs(uf).max())


@pytest.mark.parametrize("name,dim,spec,flat", CASES, ids=[c[0] for c in CASES])
@pytest.mark.parametrize("kf,kpf", [(2, 1), (2, 2)])
def test_p_level_transfer(name, dim, spec, flat, kf, kpf):
    """The p-level pair of gls_fe_space_mg_transfer (same cells, Qkf-Qkpf -> Q1-Q1, the coarse space below a
    hierarchy's base mesh): a partition of unity on every fine master row, empty fine hanging rows, the
    injection a right inverse of P (P maps each coarse nodal vector onto fine nodes that reproduce it at the
    coarse nodes), the exact Q2 interpolant of a Q1 field: the values at the vertices and the averages at the
    midpoints of every cell's reference lattice, on adapted meshes with hanging nodes in both spaces."""
    m = adapted(name, dim, spec, kf)
    hf = m.fe_space_handle(kf, kpf, qmapping_all=True)
    hc = m.fe_space_handle(1, 1, qmapping_all=True)
    sf, sc = hf.data, hc.data
    off, col, w, inj = hf.mg_transfer_from(hc)
    nf = dim * sf["n_vnodes"] + sf["n_pnodes"]
    nc = dim * sc["n_vnodes"] + sc["n_pnodes"]
    P = sps.csr_matrix((w, col, off), shape=(nf, nc))
    hf_d, hc_d = hanging_dofs(sf), hanging_dofs(sc)
    rows = np.diff(off)
    for i in range(nf):
        if i in hf_d:
            assert rows[i] == 0
        else:
            assert abs(P[i].sum() - 1.0) < 1e-12, i
    assert not set(col.tolist()) & hc_d
    assert (inj >= 0).all()
    rng = np.random.default_rng(SEED)
    xc = rng.uniform(-1, 1, nc)
    for nd, ln in sc["vhang"].items():  # a conforming coarse field
        for c in range(dim):
            xc[nd * dim + c] = sum(wt * xc[mm * dim + c] for mm, wt in ln)
    for nd, ln in sc["phang"].items():
        xc[dim * sc["n_vnodes"] + nd] = sum(wt * xc[dim * sc["n_vnodes"] + mm] for mm, wt in ln)
    xf = P @ xc
    free = np.array([j for j in range(nc) if j not in hc_d])
    assert np.abs(xf[inj[free]] - xc[free]).max() < 1e-12
    # cell by cell: the fine lattice values are the Q1 interpolant of the cell's vertex values
    kf1 = kf + 1
    cvf = np.asarray(sf["cell_vnodes"]).reshape(sf["n_cells"], -1)
    cvc = np.asarray(sc["cell_vnodes"]).reshape(sc["n_cells"], -1)
    fh = {nd for nd in sf["vhang"]}
    for cell in range(0, sf["n_cells"], max(1, sf["n_cells"] // 25)):
        for a in range(cvf.shape[1]):
            if cvf[cell, a] in fh:
                continue
            ia = [(a // kf1 ** d) % kf1 for d in range(dim)]
            want = 0.0
            for b in range(2 ** dim):
                wb = np.prod([(ia[d] / kf) if (b >> d) & 1 else 1 - ia[d] / kf for d in range(dim)])
                want += wb * xc[cvc[cell, b] * dim]
            assert abs(xf[cvf[cell, a] * dim] - want) < 1e-12
