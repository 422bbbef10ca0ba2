"""Multigrid on the octree refinement hierarchy (the reference's GLS solver preconditions
with ILU / ML-AMG, gls_navier_stokes.cc:1161-1240, on a p4est forest, navier_stokes_base.cc:55-60): the
global-coarsening level meshes (gls_octree_coarsen_to) and their grid transfers (gls_octree_mg_transfer).

CPU: the truncated forests tile the cube and nest (every fine leaf inside one coarse leaf); the
prolongation is the FE interpolation between nested conforming spaces, so it reproduces every global
Q_k / Q_kp field exactly at the fine masters, leaves the fine hanging rows empty and has coarse masters as
its only columns; the injection maps each coarse node onto the coincident fine node. No reference golden
covers a multigrid hierarchy (the reference has none): exactness is checked against polynomials."""
import numpy as np
import pytest
import scipy.sparse as sps

import softx_2020_200_amd as sx

SEED = 20200200


def adapted_tree(dim, n, steps, seed=3, max_level=4):
    """the adaptation of tests/test_hanging.py::octree_mesh, returning the forest"""
    t = sx.Octree(dim, n)
    rng = np.random.default_rng(seed)
    for _ in range(steps):
        lev, x0, h = t.cells()
        near = np.linalg.norm(x0 + 0.5 * h - 0.55, axis=1) < 0.6
        t.adapt(refine=near.astype(np.int32), coarsen=(~near & (rng.uniform(size=len(lev)) < 0.5)).astype(np.int32),
                max_level=max_level)
    return t


def poly(X, c):
    v = np.zeros(X.shape[0])
    for idx in np.ndindex(*c.shape):
        t = np.full(X.shape[0], c[idx])
        for d in range(X.shape[1]):
            t = t * X[:, d] ** idx[d]
        v += t
    return v


def field(mesh, dim, k, kp, cv, cp):
    """DoF vector [velocity node-major | pressure] of global polynomials (coefficients cv[c], cp)"""
    vel = np.stack([poly(mesh["vnode_x"], cv[c]) for c in range(dim)], 1).reshape(-1)
    return np.concatenate([vel, poly(mesh["pnode_x"], cp)])


@pytest.mark.parametrize("dim,n,steps", [(2, 2, 3), (3, 2, 2)])
def test_coarsen_to_levels_nest(dim, n, steps):
    t = adapted_tree(dim, n, steps)
    L = t.max_level
    assert L >= 2
    lev_f, x0_f, h_f = t.cells()
    for l in range(L + 1):
        tc = t.coarsen_to(l)
        lev, x0, h = tc.cells()
        assert lev.max() <= l and tc.max_level == min(l, L)
        assert abs(np.prod(h, axis=1).sum() - 2.0 ** dim) < 1e-12  # tiles [-1, 1]^dim
        # every fine leaf lies in exactly one coarse leaf, which is its ancestor-or-self on level <= l
        ctr = x0_f + 0.5 * h_f
        inside = np.all((ctr[:, None, :] > x0[None]) & (ctr[:, None, :] < x0[None] + h[None]), axis=2)
        assert (inside.sum(1) == 1).all()
        owner = inside.argmax(1)
        assert (np.minimum(lev_f, l) == lev[owner]).all()
        assert np.all(x0[owner] <= x0_f + 1e-14) and np.all(x0_f + h_f <= x0[owner] + h[owner] + 1e-14)
    same = t.coarsen_to(L)
    assert all(np.array_equal(a, b) for a, b in zip(same.cells(), t.cells()))


@pytest.mark.parametrize("dim,k,kp,gap", [(2, 2, 1, 1), (2, 1, 1, 1), (3, 2, 2, 1), (3, 1, 1, 1), (3, 2, 2, 2)])
def test_mg_transfer_reproduces_qk(dim, k, kp, gap):
    t = adapted_tree(dim, 2, 3 if dim == 2 else 2)
    tc = t.coarsen_to(t.max_level - gap)
    hf, hc = t.mesh_handle(k, kp), tc.mesh_handle(k, kp)
    try:
        off, col, w, inj = sx.octree_mg_transfer(hf, hc)
    finally:
        t.free_mesh_handle(hf)
        tc.free_mesh_handle(hc)
    mf, mc = t.mesh(k, kp), tc.mesh(k, kp)
    nf = dim * mf["n_vnodes"] + mf["n_pnodes"]
    nc = dim * mc["n_vnodes"] + mc["n_pnodes"]
    assert len(off) == nf + 1 and len(inj) == nc
    rng = np.random.default_rng(SEED + dim + k)
    cv = rng.normal(size=(dim,) + (k + 1,) * dim)
    cp = rng.normal(size=(kp + 1,) * dim)
    uf, uc = field(mf, dim, k, kp, cv, cp), field(mc, dim, k, kp, cv, cp)
    P = sps.csr_matrix((w, col, off), shape=(nf, nc))

    def hanging_dofs(m):
        hv = m["vhang"][0]
        return set((hv[:, None] * dim + np.arange(dim)[None]).reshape(-1).tolist()) | set(
            (dim * m["n_vnodes"] + m["phang"][0]).tolist())

    hang_f, hang_c = hanging_dofs(mf), hanging_dofs(mc)
    assert len(hang_f) > 0
    rows = np.array(sorted(set(range(nf)) - hang_f))
    # coarse masters only, empty fine hanging rows, exact interpolation of the Q_k field
    assert not (set(np.unique(col).tolist()) & hang_c)
    assert all(off[i] == off[i + 1] for i in hang_f)
    err = np.abs((P @ uc)[rows] - uf[rows]).max()
    assert err < 1e-11 * max(1.0, np.abs(uf).max()), err
    # rows of a partition of unity (constants are reproduced)
    assert np.abs(np.asarray(P.sum(1)).ravel()[rows] - 1.0).max() < 1e-12
    # injection: the coincident fine DoF
    assert np.abs(uf[inj] - uc).max() < 1e-12 * max(1.0, np.abs(uf).max())


@pytest.mark.parametrize("dim,k", [(2, 2), (3, 2), (3, 1)])
def test_mg_transfer_below_the_base(dim, k):
    """a uniform level below an adapted forest's level-0 grid (two forests, bases 4 and 2): the
    transfer between the base-4 level-0 mesh and the 2^dim mesh is the same exact interpolation"""
    fine, coarse = sx.Octree(dim, 4), sx.Octree(dim, 2)
    hf, hc = fine.mesh_handle(k, k), coarse.mesh_handle(k, k)
    try:
        off, col, w, inj = sx.octree_mg_transfer(hf, hc)
    finally:
        fine.free_mesh_handle(hf)
        coarse.free_mesh_handle(hc)
    mf, mc = fine.mesh(k, k), coarse.mesh(k, k)
    nf, nc = dim * mf["n_vnodes"] + mf["n_pnodes"], dim * mc["n_vnodes"] + mc["n_pnodes"]
    rng = np.random.default_rng(SEED + 11 * dim + k)
    cv, cp = rng.normal(size=(dim,) + (k + 1,) * dim), rng.normal(size=(k + 1,) * dim)
    uf, uc = field(mf, dim, k, k, cv, cp), field(mc, dim, k, k, cv, cp)
    P = sps.csr_matrix((w, col, off), shape=(nf, nc))
    assert np.abs(P @ uc - uf).max() < 1e-11 * max(1.0, np.abs(uf).max())
    assert np.abs(uf[inj] - uc).max() < 1e-12 * max(1.0, np.abs(uf).max())
