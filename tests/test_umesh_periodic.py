"""Periodic boundaries under local refinement on general (GridGenerator / gmsh) meshes:
the reference adds the periodic face pairs to its p::d triangulation (add_periodicity, source/core/grids.cc:
41-58) and closes make_periodicity_constraints with the hanging-node constraints
(source/solvers/gls_navier_stokes.cc:80-184, periodic at :128-134, :162-168). No reference case combines
periodicity with adaptation, so these checks pin the constraint algebra and the mesh rules directly:
  * refinement levels differ by at most one across the periodic boundary (the vertex 2:1 balance and the
    mesh smoothing see across it, gls_umesh_set_periodic);
  * every constraint line (hanging nodes of either side, nodes of a finer periodic face constrained to the
    coarser face across the boundary) reproduces every field of the space that is periodic: g(y) (2D) and
    g(y, z) (3D) polynomials of the element degree, which the discrete space holds exactly;
  * the Kelly face pieces tile the interior faces plus the periodic boundary (their JxW sum equals the
    interior face measure + one periodic face), and on a uniform mesh a field repeating every cell gives
    every cell the same number of pieces."""
import numpy as np
import pytest

from softx_2020_200_amd.native import UMesh


def _rect(dim, nx, L=2.0):
    if dim == 2:
        return UMesh(2, grid_type="subdivided_hyper_rectangle", grid_arguments="%d,2 : 0,0 : %g,1 : true" % (nx, L))
    return UMesh(3, grid_type="subdivided_hyper_rectangle", grid_arguments="%d,2,2 : 0,0,0 : %g,1,1 : true" % (nx, L))


def _refine_near(m, dim, k, x_lo, x_hi, times):
    """refine (with the smoothing / balance) the cells whose centre lies in x_lo < x < x_hi, `times` times"""
    for _ in range(times):
        sp = m.fe_space(1)
        cx = sp["cell_support"][:, :, 0].mean(axis=1)
        r = ((cx > x_lo) & (cx < x_hi)).astype(np.int32)
        r, c = m.prepare(r, np.zeros_like(r))
        m.adapt(r, c)


def _lines_reproduce(sp, key, X, g):
    lines = sp[key]
    err = 0.0
    for n, line in lines.items():
        err = max(err, abs(g(X[n]) - sum(w * g(X[mm]) for mm, w in line)))
    return lines, err


@pytest.mark.parametrize("dim,k", [(2, 1), (2, 2), (3, 1), (3, 2)])
def test_periodic_refined_constraints_reproduce_periodic_fields(dim, k):
    m = _rect(dim, 4)
    per = [(0, 1, 0)]
    m.set_periodic(per)
    _refine_near(m, dim, k, 1.5, 2.1, 2)  # two levels at the x = L side only
    sp = m.fe_space(k, 1, periodic=per)
    lev = sp["cell_level"]
    cx = sp["cell_support"][:, :, 0].mean(axis=1)
    assert lev.max() == 2
    # 2:1 across the periodic boundary: the x = 0 column was refined by the balance
    assert lev[cx < 0.5 / 1].min() >= 1, np.bincount(lev[cx < 0.5])
    X = sp["vnode_x"]
    on_x0 = np.abs(X[:, 0]) < 1e-12
    on_xl = np.nonzero(np.abs(X[:, 0] - 2.0) < 1e-12)[0]  # x = L nodes without a partner at x = 0
    g = (lambda x: 1.0 + x[1] + 0.7 * x[1] ** 2 * (k > 1)) if dim == 2 else \
        (lambda x: 1.0 + x[1] - 2 * x[2] + 0.5 * x[1] * x[2] + 0.7 * (x[1] ** 2 - x[2] ** 2) * (k > 1))
    lines, err = _lines_reproduce(sp, "vhang", X, g)
    assert err < 1e-12, err
    # partnered x = L nodes are identified with x = 0 nodes; the others (the finer face's extra nodes) are
    # constrained to the coarser face at x = 0, so the check is not vacuous
    assert len(on_xl) > 0 and all(int(n) in lines for n in on_xl), (len(on_xl), len(lines))
    assert all(any(on_x0[mm] for mm, _ in lines[int(n)]) for n in on_xl)
    _, errp = _lines_reproduce(sp, "phang", sp["pnode_x"], lambda x: 1.0 + x[1] + (x[2] if dim == 3 else 0.0))
    assert errp < 1e-12


@pytest.mark.parametrize("dim", [2, 3])
def test_periodic_space_without_refinement_matches_unconstrained_count(dim):
    """uniform mesh: the periodic space identifies the x = L nodes with the x = 0 ones and has no lines"""
    m = _rect(dim, 4)
    per = [(0, 1, 0)]
    a = m.fe_space(2, 1)
    b = m.fe_space(2, 1, periodic=per)
    nface = 5 if dim == 2 else 25  # Q2 nodes on the x = L face: (2*2+1)^(dim-1)
    assert b["n_vnodes"] == a["n_vnodes"] - nface
    assert not b["vhang"]


@pytest.mark.parametrize("dim", [2, 3])
def test_periodic_kelly_faces_tile_faces(dim):
    """The periodic space's Kelly pieces are the plain space's (interior faces, hanging ones split into the
    fine side's pieces) plus pieces tiling the periodic boundary once (measure 1), before and after local
    refinement on either side of it."""
    m = _rect(dim, 4)
    per = [(0, 1, 0)]
    m.set_periodic(per)
    for stage in range(3):
        sp = m.fe_space_handle(2, 1, periodic=per)
        kf = sp.kelly_faces(3)
        plain = m.fe_space_handle(2, 1).kelly_faces(3)
        d = sp.data
        cx = d["cell_support"][:, :, 0].mean(axis=1)
        across = np.abs(cx[kf["ca"]] - cx[kf["cb"]]) > 1.0  # pieces joining the two periodic sides
        assert abs(kf["jxw"][across].sum() - 1.0) < 1e-12, (stage, kf["jxw"][across].sum())
        assert abs(kf["jxw"].sum() - plain["jxw"].sum() - 1.0) < 1e-12, stage
        assert len(kf["ca"]) - across.sum() == len(plain["ca"])
        if stage == 0:  # uniform: every cell has the same number of pieces (one y (and z) wall each)
            cnt = np.bincount(np.concatenate([kf["ca"], kf["cb"]]), minlength=d["n_cells"])
            assert (cnt == cnt[0]).all() and cnt[0] == 2 + (dim - 1)
        else:  # levels on the two sides differ: irregular periodic pieces from the finer side
            lev = d["cell_level"]
            assert (lev[kf["ca"][across]] != lev[kf["cb"][across]]).any() or stage == 2
        _refine_near(m, dim, 2, 1.5 if stage == 0 else -0.1, 2.1 if stage == 0 else 0.3, 1)
