"""Multi-level adaptive hyper_cube (gls_octree_*; the reference's p4est forest adaptation,
navier_stokes_base.cc:592-780, and make_hanging_node_constraints + close(), gls_navier_stokes.cc:84,
143): vertex 2:1 balance, coarsening of complete sibling groups, hanging lines that reproduce the
Qk space exactly and make the field continuous across every non-conforming face, and an exact
SolutionTransfer for Qk fields. Host-only (CPU) tests."""
import itertools

import numpy as np
import pytest

from softx_2020_200_amd.native import Octree, octree_transfer, refined_cube


def lag(k, a, x):
    v = np.ones_like(x)
    for b in range(k + 1):
        if b != a:
            v = v * (x - b / k) / ((a - b) / k)
    return v


def apply_lines(vals, lines):
    node, off, master, w = lines
    out = vals.copy()
    for i, nd in enumerate(node):
        out[nd] = np.dot(w[off[i]:off[i + 1]], vals[master[off[i]:off[i + 1]]])
    return out


def eval_cell(m, key, c, xi, nodal):
    dim = m["dim"]
    k = m["k"] if key == "v" else m["kp"]
    cn = m["cell_vnodes"][c] if key == "v" else m["cell_pnodes"][c]
    s = 0.0
    for a, nd in enumerate(cn):
        w = 1.0
        r = a
        for d in range(dim):
            w *= lag(k, r % (k + 1), np.asarray(xi[d]))
            r //= k + 1
        s = s + w * nodal[nd]
    return s


def vertex_balanced(tree):
    lev, x0, h = tree.cells()
    dim = tree.dim
    hi = x0 + h
    for i in range(len(lev)):
        touch = np.all((x0 <= hi[i] + 1e-12) & (hi >= x0[i] - 1e-12), axis=1)
        if np.any(np.abs(lev[touch] - lev[i]) > 1):
            return False
    return True


def adapted(dim, n, steps, seed=3):
    t = Octree(dim, n)
    rng = np.random.default_rng(seed)
    for s in range(steps):
        lev, x0, h = t.cells()
        # refine cells near a corner point, coarsen a random half of the others
        ctr = x0 + 0.5 * h
        near = np.linalg.norm(ctr - 0.55, axis=1) < 0.6
        t.adapt(refine=near.astype(np.int32), coarsen=(~near & (rng.uniform(size=len(lev)) < 0.5)).astype(np.int32),
                max_level=4)
    return t


@pytest.mark.parametrize("dim", [2, 3])
def test_balance_and_counts(dim):
    t = Octree(dim, 2)
    assert t.n_cells == 2 ** dim and t.max_level == 0
    t.adapt(refine=np.ones(t.n_cells, np.int32))
    assert t.n_cells == 4 ** dim and t.max_level == 1
    for _ in range(3):  # refine the cell at the low corner repeatedly: the balance grades the mesh
        lev, x0, h = t.cells()
        f = np.zeros(len(lev), np.int32)
        f[np.argmin(np.linalg.norm(x0 + 1.0, axis=1))] = 1
        t.adapt(refine=f)
        assert vertex_balanced(t)
    assert t.max_level == 4
    lev, x0, h = t.cells()
    vol = np.prod(h, axis=1).sum()
    assert abs(vol - 2.0 ** dim) < 1e-12  # the leaves tile the cube


@pytest.mark.parametrize("dim", [2, 3])
def test_coarsening(dim):
    t = Octree(dim, 2)
    t.adapt(refine=np.ones(t.n_cells, np.int32))
    n1 = t.n_cells
    t.adapt(coarsen=np.ones(n1, np.int32))  # every sibling group complete and flagged
    assert t.n_cells == 2 ** dim
    t.adapt(refine=np.ones(t.n_cells, np.int32))
    lev, x0, h = t.cells()
    f = np.zeros(len(lev), np.int32)
    f[0] = 1
    t.adapt(refine=f)  # one level-2 patch
    n2 = t.n_cells
    lev, x0, h = t.cells()
    # coarsening the level-1 group next to the level-2 patch would break the 2:1 balance: refused
    t.adapt(coarsen=(lev == 1).astype(np.int32))
    assert vertex_balanced(t)
    assert t.n_cells < n2  # but the groups away from it were coarsened
    t.adapt(coarsen=np.zeros(t.n_cells, np.int32), min_level=1)
    assert vertex_balanced(t)


@pytest.mark.parametrize("dim,k,kp", [(2, 1, 1), (2, 2, 1), (2, 2, 2), (3, 1, 1), (3, 2, 1)])
def test_hanging_lines_reproduce_qk_and_continuity(dim, k, kp):
    t = adapted(dim, 2, 3 if dim == 2 else 2)
    assert t.max_level >= 2  # multi-level: chained constraints occur
    m = t.mesh(k, kp)
    rng = np.random.default_rng(1)
    for key, kk in (("v", k), ("p", kp)):
        X = m[key + "node_x"]
        lines = m[key + "hang"]
        # masters are never constrained (closed chains)
        assert not set(lines[2].tolist()) & set(lines[0].tolist())
        # a Qk polynomial is reproduced exactly
        coef = rng.uniform(-1, 1, (kk + 1,) * dim)
        def poly(P):
            v = 0.0
            for e in itertools.product(range(kk + 1), repeat=dim):
                term = coef[e]
                for d in range(dim):
                    term = term * P[:, d] ** e[d]
                v = v + term
            return v
        exact = poly(X)
        assert np.abs(apply_lines(exact, lines) - exact).max() < 1e-12
        # random master values: the constrained field is continuous across every face
        vals = apply_lines(rng.uniform(-1, 1, len(X)), lines)
        x0, h = m["cell_x0"], m["cell_h"]
        hi = x0 + h
        pts = rng.uniform(size=(6, dim))
        for i in range(m["n_cells"]):
            for d in range(dim):
                for side in (0, 1):
                    fx = x0[i, d] + side * h[i, d]
                    # neighbours sharing (part of) this face
                    other = np.where((np.abs((x0[:, d] if side else hi[:, d]) - fx) < 1e-12) &
                                     np.all(np.delete((x0 < hi[i] - 1e-12) & (hi > x0[i] + 1e-12), d, axis=1), axis=1))[0]
                    for j in other:
                        lo_ = np.maximum(x0[i], x0[j])
                        up_ = np.minimum(hi[i], hi[j])
                        P = lo_ + pts * (up_ - lo_)
                        P[:, d] = fx
                        a = eval_cell(m, key, i, ((P - x0[i]) / h[i]).T, vals)
                        b = eval_cell(m, key, j, ((P - x0[j]) / h[j]).T, vals)
                        assert np.abs(a - b).max() < 1e-11, (key, i, j)


@pytest.mark.parametrize("dim,k,kp", [(2, 2, 1), (3, 1, 1)])
def test_one_level_matches_refined_cube(dim, k, kp):
    """One refinement of flagged cells == the round-1 builder (same nodes, same hanging lines)."""
    n = 4
    flags = np.zeros(n ** dim, np.int32)
    flags[[0, 5, n ** dim - 1]] = 1
    a = refined_cube(dim, n, k, kp, flags)
    t = Octree(dim, n)
    lev, x0, h = t.cells()
    # the octree lists level-0 cells in Morton order: map the lexicographic flags onto it
    ijk = np.rint((x0 + 1.0) / h).astype(int)
    lexi = sum(ijk[:, d] * n ** d for d in range(dim))
    t.adapt(refine=flags[lexi])
    b = t.mesh(k, kp)
    for key in ("v", "p"):
        assert np.array_equal(a[key + "node_x"], b[key + "node_x"])
        la, lb = a[key + "hang"], b[key + "hang"]
        def lines(l):
            return {int(nd): dict(zip(l[2][l[1][i]:l[1][i + 1]].tolist(), l[3][l[1][i]:l[1][i + 1]].tolist()))
                    for i, nd in enumerate(l[0])}
        A, B = lines(la), lines(lb)
        assert A.keys() == B.keys()
        for nd in A:
            assert A[nd].keys() == B[nd].keys() and all(abs(A[nd][q] - B[nd][q]) < 1e-14 for q in A[nd])


@pytest.mark.parametrize("dim,k,kp", [(2, 2, 1), (3, 2, 2)])
def test_transfer_exact_for_qk(dim, k, kp):
    t = Octree(dim, 2)
    t.adapt(refine=np.ones(t.n_cells, np.int32))
    old = t.mesh_handle(k, kp)
    mo = t.mesh(k, kp)
    lev, x0, h = t.cells()
    f = np.zeros(len(lev), np.int32)
    f[: len(lev) // 3] = 1
    c = np.zeros(len(lev), np.int32)
    c[-(2 ** dim):] = 1
    t.adapt(refine=f, coarsen=c)
    new = t.mesh_handle(k, kp)
    mn = t.mesh(k, kp)
    rng = np.random.default_rng(7)
    cv, cp = rng.uniform(-1, 1, (dim, 3)), rng.uniform(-1, 1, 3)
    def field(m):
        Xv, Xp = m["vnode_x"], m["pnode_x"]
        vel = np.stack([cv[c, 0] + cv[c, 1] * Xv[:, 0] * Xv[:, 1] + cv[c, 2] * Xv[:, -1] ** min(k, 2) for c in range(dim)], 1)
        pre = cp[0] + cp[1] * Xp[:, 0] + cp[2] * Xp[:, 1] * (Xp[:, 0] if kp > 1 else 1)
        return np.concatenate([vel.ravel(), pre])
    out = octree_transfer(old, new, field(mo), dim * mn["n_vnodes"] + mn["n_pnodes"])
    assert np.abs(out - field(mn)).max() < 1e-12
    t.free_mesh_handle(old)
    t.free_mesh_handle(new)


@pytest.mark.parametrize("dim", [2, 3])
def test_octree_faces_tile_the_interior(dim):
    """The face pieces cover every interior face exactly once: their total area equals the sum of
    the interior face areas of the finest-level decomposition of the cube."""
    t = adapted(dim, 2, 2)
    fa, fb, fd, ra, rb = t.faces(1)
    lev, x0, h = t.cells()
    area = 0.0
    for e in range(len(fa)):
        a = 1.0
        for j, ax in enumerate([x for x in range(dim) if x != fd[e]]):
            a *= (ra[e, 2 * j + 1] - ra[e, 2 * j]) * h[fa[e], ax]
            # both descriptions of the piece have the same physical extent
            assert abs((ra[e, 2 * j + 1] - ra[e, 2 * j]) * h[fa[e], ax] - (rb[e, 2 * j + 1] - rb[e, 2 * j]) * h[fb[e], ax]) < 1e-14
        area += a
    # interior area of [-1, 1]^dim cut by the leaves: sum over cells of their high faces inside the cube
    ref = 0.0
    for i in range(len(lev)):
        for d in range(dim):
            if x0[i, d] + h[i, d] < 1.0 - 1e-12:
                ref += np.prod(np.delete(h[i], d))
    assert abs(area - ref) < 1e-12


def _leaves(t):
    lev, x0, h = t.cells()
    return [(int(l), tuple(int(round(v)) for v in (x - t.lo) / hh)) for l, x, hh in zip(lev, x0, h)]


def test_refine_coarsen_pd_matches_oracle():
    """gls_refine_coarsen_pd (p::d::GridRefinement with coarsening, navier_stokes_base.cc:654-667) equals
    the oracle restatement bit for bit: flags and both thresholds, with ties, zeros, the element cap and
    meshes already above it."""
    from oracle.oracle import pd_refine_coarsen
    from softx_2020_200_amd import refine_coarsen_pd
    rng = np.random.default_rng(1)
    for t in range(200):
        n = int(rng.integers(1, 300))
        dim = int(rng.integers(2, 4))
        c = (rng.random(n) ** 3).astype(np.float32)
        if t % 5 == 0:
            c[rng.integers(0, n, n // 3)] = 0
        if t % 7 == 0:
            c = np.round(c * 4) / 4
        top, bot = float(rng.random() * 0.5), (float(rng.random() * 0.4) if t % 3 else 0.0)
        ft = ("number", "fraction")[t % 2]
        mx = int(rng.integers(1, 3 * n + 2))
        a, b = refine_coarsen_pd(c, dim, top, bot, ft, mx), pd_refine_coarsen(c, dim, top, bot, ft, mx)
        assert (a[0] == b[0]).all() and (a[1] == b[1]).all() and a[2] == b[2], (t, a[2], b[2])
        assert not (a[0] & a[1]).any()
    # at the cap, fixed number coarsens (n - max) / (1 - 2^-dim) cells and refines none
    c = np.arange(1, 101, dtype=np.float32)
    r, k, _ = refine_coarsen_pd(c, 2, 0.3, 0.0, "number", 76)
    assert r.sum() == 0 and k.sum() == 32 and k[:32].all()


@pytest.mark.parametrize("dim", [2, 3])
def test_prepare_matches_oracle_and_is_consistent(dim):
    """gls_octree_prepare (Triangulation::prepare_coarsening_and_refinement with the reference's mesh
    smoothing, navier_stokes_base.cc:55-60, 682) equals the oracle restatement on random multi-level
    trees and flags; a second call changes nothing (deal.II's promise); the adaptation then executes
    exactly the prepared flags (no extra balance refinement) and keeps the vertex 2:1 rule."""
    from oracle.oracle import prepare_coarsening_and_refinement
    rng = np.random.default_rng(7 + dim)
    for case in range(12 if dim == 2 else 5):
        n = 1 + case % 2
        t = Octree(dim, n)
        for _ in range(3 if dim == 2 else 2):
            t.adapt(np.ones(t.n_cells, np.int32))
            if dim == 3:
                break
        for step in range(3 if dim == 2 else 2):
            nc = t.n_cells
            r = (rng.random(nc) < rng.random() * 0.4).astype(np.int32)
            c = ((rng.random(nc) < rng.random() * 0.7) & (r == 0)).astype(np.int32)
            pr, pc, loops = t.prepare(r, c)
            orr, occ = prepare_coarsening_and_refinement(dim, n, _leaves(t), r, c)
            assert (pr == orr).all() and (pc == occ).all(), (case, step)
            again = t.prepare(pr, pc)
            assert (again[0] == pr).all() and (again[1] == pc).all()
            assert not (pr & pc).any() and pc.sum() % 2 ** dim == 0
            t.adapt(pr, pc)
            assert t.n_cells == nc + (2 ** dim - 1) * int(pr.sum()) - (2 ** dim - 1) * int(pc.sum()) // 2 ** dim
            assert vertex_balanced(t)


def test_prepare_islands():
    """The smoothing rules on a uniform 8x8 mesh: an isolated flagged cell loses its flag
    (eliminate_refined_inner_islands), and so do four cells that touch only at corners; a cell with
    three flagged face neighbours is refined too (eliminate_unrefined_islands); a 2x2 block stays as
    flagged."""
    t = Octree(2, 1)
    for _ in range(3):
        t.adapt(np.ones(t.n_cells, np.int32))
    lev, x0, h = t.cells()
    ij = np.round((x0 + 1) / h).astype(int)
    at = {(int(a), int(b)): i for i, (a, b) in enumerate(ij)}
    z = np.zeros(t.n_cells, np.int32)
    r = z.copy()
    r[at[3, 3]] = 1
    assert t.prepare(r, z)[0].sum() == 0
    r = z.copy()
    for p in [(3, 4), (5, 4), (4, 3), (4, 5)]:
        r[at[p]] = 1
    assert t.prepare(r, z)[0].sum() == 0
    r = z.copy()
    for p in [(3, 4), (3, 3), (4, 3), (5, 4), (5, 3)]:
        r[at[p]] = 1
    pr = t.prepare(r, z)[0]
    assert pr[at[4, 4]] == 1 and pr.sum() == 6
    r = z.copy()
    for p in [(2, 2), (2, 3), (3, 2), (3, 3)]:
        r[at[p]] = 1
    assert (t.prepare(r, z)[0] == r).all()
