"""Local adaptation of unstructured / curved meshes (gls_umesh_prepare / gls_umesh_adapt, hanging lines
and levels in gls_umesh_fe_space, hierarchy-based gls_fe_space_transfer, Kelly face pieces with
MappingQ geometry): the reference's p::d::Triangulation adaptation on gmsh / generator meshes
(navier_stokes_base.cc:55-60, 592-780; make_hanging_node_constraints, gls_navier_stokes.cc:84, 143).
Host-only (CPU) tests:
  * on an axis-aligned hyper_cube the unstructured hierarchy reproduces the octree (gls_octree_*,
    itself checked against the oracle's restatement of prepare_coarsening_and_refinement): the same
    smoothed flags, the same active cells, the same Q1 hanging nodes;
  * hanging lines make every field continuous across every face piece (both sides evaluated at the
    pieces' paired reference points) and reproduce linear functions on flat meshes;
  * SolutionTransfer refine -> coarsen returns the original field;
  * the Kelly face pieces (host geometry) give the oracle's box Kelly indicator on the hyper_cube.
"""
import os

import numpy as np
import pytest

from oracle.oracle import kelly_estimate_boxes
from softx_2020_200_amd.native import Octree, UMesh

HERE = os.path.dirname(os.path.abspath(__file__))
MESHES = os.path.join(HERE, "golden", "meshes")


def lag(k, a, x):
    v = np.ones_like(np.asarray(x, dtype=np.float64))
    for b in range(k + 1):
        if b != a:
            v = v * (x - b / k) / ((a - b) / k)
    return v


def dlag(k, a, x):
    x = np.asarray(x, dtype=np.float64)
    tot = np.zeros_like(x)
    for c in range(k + 1):
        if c == a:
            continue
        t = np.full_like(x, 1.0 / ((a - c) / k))
        for b in range(k + 1):
            if b != a and b != c:
                t = t * (x - b / k) / ((a - b) / k)
        tot = tot + t
    return tot


def cell_centres(sp):
    """centre of each active cell = mean of its corner support points"""
    dim, k = sp["dim"], sp["k"]
    S = sp["cell_support"]
    corners = [sum(((v >> d) & 1) * k * (k + 1) ** d for d in range(dim)) for v in range(1 << dim)]
    return S[:, corners, :].mean(axis=1)


def apply_lines(vals, lines):
    out = vals.copy()
    for nd, ln in lines.items():
        out[nd] = sum(w * vals[m] for m, w in ln)
    return out


def eval_at(sp, key, c, xi, nodal):
    dim = sp["dim"]
    k = sp["k"] if key == "v" else sp["kp"]
    cn = sp["cell_vnodes"][c] if key == "v" else sp["cell_pnodes"][c]
    s = 0.0
    for a, nd in enumerate(cn):
        w = 1.0
        r = a
        for d in range(dim):
            w *= lag(k, r % (k + 1), xi[d])
            r //= k + 1
        s += w * nodal[nd]
    return s


def random_adapt(m, cycles, seed, k=1, frac=0.3):
    """prepare + adapt with flags from a seeded score (refine the top `frac`, coarsen the bottom 30%)"""
    rng = np.random.default_rng(seed)
    for _ in range(cycles):
        sp = m.fe_space(k)
        ctr = cell_centres(sp)
        score = rng.uniform(size=len(ctr)) + np.exp(-4 * np.linalg.norm(ctr - ctr.mean(0) * 0.8, axis=1))
        order = np.argsort(-score)
        r = np.zeros(len(ctr), np.int32)
        c = np.zeros(len(ctr), np.int32)
        r[order[:int(frac * len(ctr))]] = 1
        c[order[-int(0.3 * len(ctr)):]] = 1
        r, c = m.prepare(r, c)
        m.adapt(r, c)
    return m


def _key(level, ctr):
    return (int(level),) + tuple(np.round(ctr, 9))


@pytest.mark.parametrize("dim", [2, 3])
def test_adapt_matches_octree(dim):
    t = Octree(dim, 1)
    m = UMesh(dim, "hyper_cube", "-1 : 1 : false")
    for _ in range(2):
        t.adapt(refine=np.ones(t.n_cells, np.int32))
    m.refine_global(2)
    rng = np.random.default_rng(11)
    for cycle in range(3 if dim == 2 else 2):
        lev, x0, h = t.cells()
        tk = {_key(lev[i], x0[i] + 0.5 * h[i]): i for i in range(len(lev))}
        sp = m.fe_space(1)
        uk = [_key(sp["cell_level"][i], c) for i, c in enumerate(cell_centres(sp))]
        assert sorted(uk) == sorted(tk)  # the same active cells
        perm = np.array([tk[u] for u in uk])  # umesh cell i == octree leaf perm[i]
        score = rng.uniform(size=len(lev))
        r_t = (score > 0.7).astype(np.int32)
        c_t = (score < 0.35).astype(np.int32)
        r2, c2, _ = t.prepare(r_t, c_t)
        r_u, c_u = m.prepare(r_t[perm], c_t[perm])
        assert np.array_equal(r_u, r2[perm]) and np.array_equal(c_u, c2[perm]), cycle
        t.adapt(refine=r2, coarsen=c2)
        m.adapt(r_u, c_u)
    lev, x0, h = t.cells()
    sp = m.fe_space(1)
    assert sorted(_key(sp["cell_level"][i], c) for i, c in enumerate(cell_centres(sp))) == \
        sorted(_key(lev[i], x0[i] + 0.5 * h[i]) for i in range(len(lev)))
    assert max(sp["cell_level"]) >= 3
    # Q1: the same nodes and the same hanging nodes (positions)
    om = t.mesh(1, 1)
    assert sp["n_vnodes"] == om["n_vnodes"]
    hx = sorted(tuple(np.round(sp["vnode_x"][n], 9)) for n in sp["vhang"])
    ox = sorted(tuple(np.round(om["vnode_x"][n], 9)) for n in om["vhang"][0])
    assert hx == ox


CASES = [
    ("square", 2, dict(gmsh="square.msh"), True),
    ("shell", 2, dict(grid=("hyper_shell", "0, 0 : 0.25 : 1 : 6 : true")), False),
    ("rect3d", 3, dict(grid=("subdivided_hyper_rectangle", "2,1,1 : 0,0,0 : 2,1,1 : false")), True),
    ("cylshell", 3, dict(grid=("cylinder_shell", "1 : 0.5 : 1 : 6 : 1")), False),
]


def make_mesh(dim, spec):
    if "gmsh" in spec:
        return UMesh(dim, gmsh=os.path.join(MESHES, spec["gmsh"]))
    return UMesh(dim, *spec["grid"])


@pytest.mark.parametrize("name,dim,spec,flat", CASES, ids=[c[0] for c in CASES])
@pytest.mark.parametrize("k,kp", [(1, 1), (2, 1), (2, 2)])
def test_hanging_lines_continuity(name, dim, spec, flat, k, kp):
    if dim == 3 and (k, kp) == (2, 2):
        pytest.skip("covered by (2, 1) for the velocity space")
    m = make_mesh(dim, spec)
    m.refine_global(1)
    random_adapt(m, 2 if dim == 2 else 1, seed=5, k=k)
    h = m.fe_space_handle(k, kp, qmapping_all=True)
    sp = h.data
    assert max(sp["cell_level"]) - min(sp["cell_level"]) >= 1
    assert sp["vhang"], "no hanging nodes"
    faces = h.kelly_faces(k + 2)
    rng = np.random.default_rng(2)
    for key, kk in (("v", k), ("p", kp)):
        lines = sp[key + "hang"]
        assert not set(m_ for ln in lines.values() for m_, _ in ln) & set(lines)  # closed chains
        for ln in lines.values():
            assert abs(sum(w for _, w in ln) - 1.0) < 1e-12  # partition of unity
        X = sp[key + "node_x"]
        nodal = apply_lines(rng.uniform(-1, 1, len(X)), lines)
        # continuity at every paired face point (the pieces' own parametrisation)
        for e in range(0, len(faces["ca"]), max(1, len(faces["ca"]) // 200)):
            for q in range(faces["nqf"]):
                ua = eval_at(sp, key, faces["ca"][e], faces["xi"][e, q, 0], nodal)
                ub = eval_at(sp, key, faces["cb"][e], faces["xi"][e, q, 1], nodal)
                assert abs(ua - ub) < 1e-11, (key, e, q, ua, ub)
        if flat:  # linear functions are reproduced exactly at the hanging nodes
            f = 0.3 + X @ np.array([1.0, -2.0, 0.5][:dim])
            g = apply_lines(f, lines)
            assert np.abs(g - f).max() < 1e-12


@pytest.mark.parametrize("name,dim,spec,flat", CASES[:3], ids=[c[0] for c in CASES[:3]])
def test_transfer_refine_coarsen_roundtrip(name, dim, spec, flat):
    m = make_mesh(dim, spec)
    m.refine_global(1)
    h0 = m.fe_space_handle(2, 1)
    sp0 = h0.data
    rng = np.random.default_rng(4)
    x0 = rng.uniform(-1, 1, dim * sp0["n_vnodes"] + sp0["n_pnodes"])
    ctr = cell_centres(sp0)
    r = (np.linalg.norm(ctr - ctr[0], axis=1) < np.median(np.linalg.norm(ctr - ctr[0], axis=1))).astype(np.int32)
    r, c = m.prepare(r, np.zeros_like(r))
    m.adapt(r, c)
    h1 = m.fe_space_handle(2, 1)
    x1 = h1.transfer_from(h0, x0)
    sp1 = h1.data
    assert sp1["n_cells"] > sp0["n_cells"]
    # the transferred field satisfies the new hanging constraints (it is the old continuous field)
    for key, off in (("v", 0), ("p", dim * sp1["n_vnodes"])):
        for nd, ln in sp1[key + "hang"].items():
            for comp in (range(dim) if key == "v" else [0]):
                idx = (lambda n: n * dim + comp) if key == "v" else (lambda n: off + n)
                assert abs(x1[idx(nd)] - sum(w * x1[idx(mm)] for mm, w in ln)) < 1e-12
    # coarsen every new family back: the original mesh and field return
    lv = sp1["cell_level"]
    back = (lv > 1).astype(np.int32)
    rb, cb = m.prepare(np.zeros_like(back), back)
    m.adapt(rb, cb)
    h2 = m.fe_space_handle(2, 1)
    assert h2.data["n_cells"] == sp0["n_cells"]
    x2 = h2.transfer_from(h1, x1)
    assert np.abs(x2 - x0).max() < 1e-12


def _numpy_kelly(sp, faces, nodal, variable, dim):
    """eta from the face pieces with the host's own evaluation of g . grad_xi u on both sides"""
    k = sp["k"] if variable == 0 else sp["kp"]
    cn = sp["cell_vnodes"] if variable == 0 else sp["cell_pnodes"]
    nv = sp["n_vnodes"]
    ncomp = dim if variable == 0 else 1
    loc = np.indices((k + 1,) * dim).reshape(dim, -1)[::-1].T
    acc = np.zeros(sp["n_cells"])
    for e in range(len(faces["ca"])):
        tot = 0.0
        for q in range(faces["nqf"]):
            dn = np.zeros((2, ncomp))
            for side, c in enumerate((faces["ca"][e], faces["cb"][e])):
                xi, g = faces["xi"][e, q, side], faces["g"][e, q, side]
                for a, ia in enumerate(loc):
                    gphi = 0.0
                    for d in range(dim):
                        t = g[d] * dlag(k, ia[d], xi[d])
                        for o in range(dim):
                            if o != d:
                                t = t * lag(k, ia[o], xi[o])
                        gphi += t
                    node = cn[c][a]
                    vals = nodal[node * dim:(node + 1) * dim] if variable == 0 else nodal[dim * nv + node:dim * nv + node + 1]
                    dn[side] += gphi * vals
            tot += faces["jxw"][e, q] * ((dn[0] - dn[1]) ** 2).sum()
        acc[faces["ca"][e]] += tot
        acc[faces["cb"][e]] += tot
    return np.sqrt(faces["diam"] / 24.0 * acc)


@pytest.mark.parametrize("dim,k,kp", [(2, 1, 1), (2, 2, 1), (3, 1, 1)])
def test_kelly_faces_match_box_oracle(dim, k, kp):
    m = UMesh(dim, "hyper_cube", "-1 : 1 : false")
    m.refine_global(2 if dim == 2 else 1)
    random_adapt(m, 2 if dim == 2 else 1, seed=9)
    h = m.fe_space_handle(k, kp)
    sp = dict(h.data)
    S = sp["cell_support"]
    sp["cell_x0"] = S[:, 0, :]
    sp["cell_h"] = S[:, -1, :] - S[:, 0, :]
    faces = h.kelly_faces(k + 2)
    rng = np.random.default_rng(3)
    nodal = rng.uniform(-1, 1, dim * sp["n_vnodes"] + sp["n_pnodes"])
    # constrained (continuous) field
    v = nodal[:dim * sp["n_vnodes"]].reshape(-1, dim)
    for comp in range(dim):
        v[:, comp] = apply_lines(v[:, comp], sp["vhang"])
    nodal[:dim * sp["n_vnodes"]] = v.reshape(-1)
    nodal[dim * sp["n_vnodes"]:] = apply_lines(nodal[dim * sp["n_vnodes"]:], sp["phang"])
    for variable in (0, 1):
        ref = kelly_estimate_boxes(sp, nodal, variable)
        got = _numpy_kelly(sp, faces, nodal, variable, dim)
        assert np.abs(got - ref).max() <= 1e-12 * np.abs(ref).max(), variable


@pytest.mark.parametrize("name,dim,spec,flat", CASES, ids=[c[0] for c in CASES])
@pytest.mark.parametrize("k,kp", [(2, 1)])
def test_vectorised_kelly_equals_loop_restatement(name, dim, spec, flat, k, kp):
    """oracle.kelly_from_face_pieces (used by the app pipeline tests on larger meshes) equals the
    plain-loop evaluation of the same face pieces on adapted meshes, for velocity and pressure."""
    from oracle.oracle import kelly_from_face_pieces
    m = make_mesh(dim, spec)
    m.refine_global(1)
    random_adapt(m, 1, seed=3, k=k)
    h = m.fe_space_handle(k, kp, qmapping_all=True)
    sp = h.data
    faces = h.kelly_faces(k + 2)
    x = np.random.default_rng(9).uniform(-1, 1, dim * sp["n_vnodes"] + sp["n_pnodes"])
    for variable in (0, 1):
        a = kelly_from_face_pieces(sp, faces, x, variable)
        b = _numpy_kelly(sp, faces, x, variable, dim)
        assert np.abs(a - b).max() <= 1e-12 * np.abs(b).max(), variable
