"""CPU-side checks of the C-ABI library (no GPU calls): it loads, exports every symbol
include/gls_native.h declares, and its host-only building blocks match the reference KATs."""
import json
import os
import re

import numpy as np

import softx_2020_200_amd as sx
from softx_2020_200_amd.native import EXPORTS, load
from oracle.oracle import StructuredProblem

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
G = json.load(open(os.path.join(ROOT, "tests", "golden", "reference_goldens.json")))


def test_header_symbols_exported():
    hdr = open(os.path.join(ROOT, "include", "gls_native.h")).read()
    declared = set(re.findall(r"^(?:int|void|const char \*)\s*(gls_\w+)\s*\(", hdr, re.M))
    assert declared, "no declarations parsed"
    L = load()
    for name in sorted(declared):
        assert hasattr(L, name), name
    assert declared == set(EXPORTS)


def test_bdf_kat():
    g = G["bdf_01"]
    for order in (1, 2, 3):
        a = sx.bdf_coefficients(order, g["time_steps"])
        for v, w in zip(a, g["order%d" % order]):
            assert abs(v - w) <= 0.5e-5 * abs(w) + 1e-12


def test_sdirk_tables():
    c = sx.sdirk_coefficients(2, 0.1)
    a = (2 - np.sqrt(2)) / 2
    assert np.isclose(c[1, 1], -(2 * a - 1) / a / a / 0.1)
    c3 = sx.sdirk_coefficients(3, 0.2)
    assert np.isclose(c3[1, 2], -1.48472100564154 / 0.2)


def test_newton_kat():
    x = sx.newton_selftest()
    gold = G["newton_01"]["solution"]
    assert abs(x[0] - gold[0]) < 1e-5 and abs(x[1] - gold[1]) < 1e-12


def test_skip_newton_kat():
    """SkipNewton KAT: the Jacobian of the first iteration is reused by every later one (a chord
    iteration), which still reaches the printed 1.22474 -1.50000 within 10 iterations."""
    gold = G["skip_newton_01"]["solution"]
    x = sx.skip_newton_selftest(1)
    assert abs(x[0] - gold[0]) < 0.5e-5 and abs(x[1] - gold[1]) < 0.5e-5
    # the chord iteration is not quadratic: after 10 steps it is still visibly off the root
    # (Newton reaches it to machine precision), so the template really froze the Jacobian
    assert 1e-12 < abs(x[0] - np.sqrt(1.5)) < 1e-6
    xn = sx.newton_selftest()
    assert abs(xn[0] - np.sqrt(1.5)) < 1e-12


def test_hyper_cube_dof_numbering_matches_oracle():
    """bit-exact DoF indexing: the C++ mesh builder (Morton cells) and the oracle's lexicographic
    builder give the same node ids for every cell."""
    for dim, n, k, kp, per in [(3, 4, 2, 2, ()), (3, 3, 2, 1, ()), (2, 8, 1, 1, ()), (2, 4, 2, 1, (0, 1)),
                               (3, 4, 1, 1, (2,))]:
        m = sx.hyper_cube(dim, n, k, kp, -1.0, 1.0, periodic=per)
        p = StructuredProblem(dim, n, k=k, kp=kp, periodic=per)
        assert m["n_vnodes"] == p.n_vnodes and m["n_pnodes"] == p.n_pnodes
        # match cells by lower corner
        key_m = {tuple(np.round(x, 12)): i for i, x in enumerate(m["cell_x0"])}
        for c in range(p.n_cells):
            i = key_m[tuple(np.round(p.cell_x0[c], 12))]
            assert np.array_equal(m["cell_vnodes"][i], p.cell_vnodes[c])
            assert np.array_equal(m["cell_pnodes"][i], p.cell_pnodes[c])


def test_morton_order():
    m = sx.hyper_cube(3, 4, 1, 1)
    ijk = np.round((m["cell_x0"] + 1.0) / 0.5).astype(int)
    # first 8 cells = the first octant's 2x2x2 block (z-order, x fastest)
    assert [tuple(v) for v in ijk[:8]] == [(0, 0, 0), (1, 0, 0), (0, 1, 0), (1, 1, 0),
                                           (0, 0, 1), (1, 0, 1), (0, 1, 1), (1, 1, 1)]


def test_cavity_constraints_first_bc_wins():
    from softx_2020_200_amd.problem import dirichlet_from_bcs
    m = sx.hyper_cube(3, 2, 1, 1)
    bcs = [("noslip", b, None) for b in (0, 1, 2, 4, 5)] + [("function", 3, (1.0, 0.0, 0.0))]
    mask, dofs, vals = dirichlet_from_bcs(m, 2, -1.0, 1.0, True, bcs)
    # every boundary node constrained in all comps; lid interior node (x=0,y=1,z=0) has u=1
    assert mask.sum() > 0 and set(np.unique(mask)) <= {0, 7}
    nx = 3
    lid_center = 1 + nx * (2 + nx * 1)
    d = dict(zip(dofs.tolist(), vals.tolist()))
    assert d[lid_center * 3] == 1.0
    corner = 0 + nx * (2 + nx * 0)  # x=-1,y=1,z=-1: wall wins
    assert d[corner * 3] == 0.0


def test_missing_extension_fails_loudly(monkeypatch, tmp_path):
    import softx_2020_200_amd.native as nat
    monkeypatch.setattr(nat, "_lib", None)
    monkeypatch.setattr(nat, "LIB_PATH", str(tmp_path / "nope.so"))
    try:
        nat.load()
    except nat.GLSError as e:
        assert "no CPU fallback" in str(e)
    else:
        raise AssertionError("load() must raise without the HIP extension")
