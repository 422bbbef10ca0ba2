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
