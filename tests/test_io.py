"""Drop-in I/O surface (CPU): parameter-file parser, ParsedFunction expressions and the VTU/PVTU/PVD
writer (csrc/gls_io.cpp through the C-ABI). Parameter texts below are written for these tests in
the deal.II ParameterHandler format Lethe reads (source/core/parameters.cc)."""
import base64
import struct
import xml.etree.ElementTree as ET

import numpy as np
import pytest

import softx_2020_200_amd as sx
from softx_2020_200_amd.io import Expr, Prm, write_pvd, write_pvtu, write_vtu
from softx_2020_200_amd.native import GLSError

PRM = r"""
# cavity-like case
subsection simulation control
  set method                  = bdf2     # trailing comment
  set time step               = 0.01
  set output   name           = out-put
end
subsection physical properties
    set kinematic viscosity   = 0.01
end
subsection boundary conditions
  set number = 2
    subsection bc 0
        set id   = 3
        set type = function
        subsection u
            set Function expression = 1
        end
        subsection v
            set Function constants  = A=2, B=-0.5
            set Function expression = A*x + \
                                      B*y
        end
    end
    subsection bc 1
        set type = noslip
    end
end
"""


def test_prm_sections_comments_continuation():
    p = Prm(PRM)
    assert p.get("simulation control/method") == "bdf2"
    assert float(p.get("simulation control/time step")) == 0.01
    assert p.get("simulation control/output name") == "out-put"        # blanks collapsed like deal.II
    assert p.get("physical properties/kinematic  viscosity") == "0.01"
    assert p.get("boundary conditions/bc 0/v/Function expression") == "A*x + B*y"
    assert p.get("boundary conditions/bc 0/v/Function constants") == "A=2, B=-0.5"
    assert p.get("boundary conditions/bc 1/type") == "noslip"
    assert p.get("boundary conditions/bc 1/id") is None
    assert p.get("missing/key", "dflt") == "dflt"
    keys = dict(p.items())
    assert len(keys) == 11 and keys["boundary conditions/number"] == "2"


@pytest.mark.parametrize("bad", ["subsection a\nset x = 1\n", "end\n", "set x 1\n", "garbage line\n"])
def test_prm_errors(bad):
    with pytest.raises(GLSError):
        Prm(bad)


def test_expr_components_constants_functions():
    X = np.random.default_rng(1).uniform(-1, 1, (50, 4))
    x, y, z, t = X.T
    e = Expr("A*x + B*y ; sin(pi*x)*cos(Pi*y)^2 ; -x^2 ; exp(-2*nu*t)*atan2(y,x) ;", "x,y,z,t", "A=2, B=-0.5, nu=0.1")
    assert e.n_components == 4                      # one trailing empty component dropped
    out = e(X)
    np.testing.assert_allclose(out[:, 0], 2 * x - 0.5 * y, rtol=0, atol=1e-15)
    np.testing.assert_allclose(out[:, 1], np.sin(np.pi * x) * np.cos(np.pi * y) ** 2, rtol=1e-15, atol=1e-15)
    np.testing.assert_allclose(out[:, 2], -(x ** 2), rtol=0, atol=1e-15)   # sign binds looser than ^
    np.testing.assert_allclose(out[:, 3], np.exp(-0.2 * t) * np.arctan2(y, x), rtol=1e-14, atol=1e-15)
    e2 = Expr("if(x>0, ln(1+x), sqrt(abs(x))) ; x > 0 && y < 0 ? 1 : 0 ; max(x, y, z) ; log(2.0) ; 1./4*(2+3)", "x,y,z")
    o2 = e2(X[:, :3])
    np.testing.assert_allclose(o2[:, 0], np.where(x > 0, np.log1p(np.maximum(x, 0)), np.sqrt(np.abs(x))), rtol=1e-14)
    np.testing.assert_array_equal(o2[:, 1], ((x > 0) & (y < 0)).astype(float))
    np.testing.assert_array_equal(o2[:, 2], np.max(X[:, :3], axis=1))
    assert o2[0, 3] == pytest.approx(np.log(2.0), rel=1e-15)     # deal.II: log = natural log
    assert o2[0, 4] == 1.25


def test_expr_long_vector_expression_matches_numpy():
    """A long multi-component expression (nested powers, products of trig terms, literals like
    2. and 1e-3) against numpy."""
    expr = ("3*pi*(1.5-cos(2*pi*y))^2*sin(pi*x)*cos(pi*z) - (sin(pi*z)^3)*(cos(pi * x)^2)/(2.+y*y) + 1e-3*x*y*z ;"
            " 0 ; exp(-(x^2+y^2+z^2)/0.5) ; 0")
    X = np.random.default_rng(2).uniform(0, 1, (40, 3))
    x, y, z = X.T
    p = np.pi
    ref = (3 * p * (1.5 - np.cos(2 * p * y)) ** 2 * np.sin(p * x) * np.cos(p * z)
           - np.sin(p * z) ** 3 * np.cos(p * x) ** 2 / (2. + y * y) + 1e-3 * x * y * z)
    out = Expr(expr, "x,y,z")(X)
    assert out.shape == (40, 4)
    np.testing.assert_allclose(out[:, 0], ref, rtol=1e-13, atol=1e-13)
    np.testing.assert_allclose(out[:, 2], np.exp(-(x ** 2 + y ** 2 + z ** 2) / 0.5), rtol=1e-14)
    assert not out[:, 1].any() and not out[:, 3].any()


@pytest.mark.parametrize("bad", ["x +", "foo(x)", "w*2", "sin(x, y)", "(x", "x ; ; y"])
def test_expr_errors(bad):
    with pytest.raises(GLSError):
        Expr(bad, "x,y")


def _read_vtu(path):
    root = ET.parse(path).getroot()
    piece = root.find("UnstructuredGrid/Piece")
    arrays = {}
    for da in root.iter("DataArray"):
        raw = base64.b64decode(da.text.strip())
        n = struct.unpack("<Q", raw[:8])[0]
        dt = {"Float64": "<f8", "Int64": "<i8", "UInt8": "u1"}[da.get("type")]
        a = np.frombuffer(raw[8:8 + n], dtype=dt)
        nc = int(da.get("NumberOfComponents", "1"))
        arrays[da.get("Name", "points")] = a.reshape(-1, nc) if nc > 1 else a
    return int(piece.get("NumberOfPoints")), int(piece.get("NumberOfCells")), arrays


@pytest.mark.parametrize("k,sub", [(2, 2), (2, 1), (1, 1), (1, 3)])
def test_vtu_fields(tmp_path, k, sub):
    n = 2
    m = sx.hyper_cube(3, n, k, k, -1.0, 1.0)
    nx = k * n + 1
    g = np.linspace(-1, 1, nx)
    Z, Y, X = np.meshgrid(g, g, g, indexing="ij")
    # u = (-y + x, x, z) (linear: exactly represented), p = x*y
    vel = np.stack([-Y + X, X, Z], -1).reshape(-1, 3)
    sol = np.concatenate([vel.reshape(-1), (X * Y).reshape(-1)])
    f = str(tmp_path / "s.vtu")
    write_vtu(f, m, sol, subdivision=sub, subdomain=3)
    npts, ncells, A = _read_vtu(f)
    ppc = (sub + 1) ** 3
    assert npts == m["n_cells"] * ppc
    P = A["points"]
    np.testing.assert_allclose(A["velocity"][:, 0], -P[:, 1] + P[:, 0], atol=1e-13)
    np.testing.assert_allclose(A["velocity"][:, 1], P[:, 0], atol=1e-13)
    np.testing.assert_allclose(A["pressure"], P[:, 0] * P[:, 1], atol=1e-13)   # Q1 or Q2 interpolant of x*y
    np.testing.assert_allclose(A["vorticity"], np.tile([0.0, 0.0, 2.0], (npts, 1)), atol=1e-12)
    assert np.all(A["subdomain"] == 3)
    # q_criterion as the reference computes it: running sum over each patch's points of
    # |W|^2 - |S|^2 (post_processors.h keeps p1/r1 across the point loop), times 1/2
    G = np.array([[1.0, -1.0, 0.0], [1.0, 0.0, 0.0], [0.0, 0.0, 1.0]])
    W, S = 0.5 * (G - G.T), 0.5 * (G + G.T)
    per_point = (W * W).sum() - (S * S).sum()
    expect = np.tile(0.5 * per_point * np.arange(1, ppc + 1), m["n_cells"])
    np.testing.assert_allclose(A["q_criterion"], expect, rtol=1e-12, atol=1e-12)
    if k > 1:   # one Lagrange hexahedron per patch, VTK corner order first
        assert ncells == m["n_cells"] and np.all(A["types"] == 72)
        conn = A["connectivity"].reshape(ncells, ppc)
        c0 = P[conn[0, :8]]
        lo, hi = P[conn[0]].min(0), P[conn[0]].max(0)
        corners = np.array([[0, 0, 0], [1, 0, 0], [1, 1, 0], [0, 1, 0], [0, 0, 1], [1, 0, 1], [1, 1, 1], [0, 1, 1]])
        np.testing.assert_allclose(c0, lo + corners * (hi - lo))
        assert sorted(conn[0]) == list(range(ppc))
    else:
        assert ncells == m["n_cells"] * sub ** 3 and np.all(A["types"] == 12)


def test_pvtu_pvd(tmp_path):
    write_pvtu(str(tmp_path / "a.00001.pvtu"), 3, ["a.00001.00000.vtu", "a.00001.00001.vtu"])
    write_pvd(str(tmp_path / "a.pvd"), [(0.0, "a.00000.pvtu"), (0.05, "a.00001.pvtu")])
    r = ET.parse(str(tmp_path / "a.00001.pvtu")).getroot()
    assert [p.get("Source") for p in r.iter("Piece")] == ["a.00001.00000.vtu", "a.00001.00001.vtu"]
    names = [d.get("Name") for d in r.iter("PDataArray") if d.get("Name")]
    assert names == ["velocity", "pressure", "subdomain", "vorticity", "q_criterion"]
    ds = list(ET.parse(str(tmp_path / "a.pvd")).getroot().iter("DataSet"))
    assert [(float(d.get("timestep")), d.get("file")) for d in ds] == [(0.0, "a.00000.pvtu"), (0.05, "a.00001.pvtu")]


def _app(tmp_path, prm_text, *args):
    import os
    import subprocess
    app = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "apps", "gls_navier_stokes")
    f = tmp_path / "c.prm"
    f.write_text(prm_text)
    return subprocess.run([app, *args, str(f)], capture_output=True, text=True, timeout=60)


@pytest.mark.parametrize("text,msg", [
    ("subsection mesh\n  set grid type = hyper_ball\nend\n", "grid type 'hyper_ball' is not supported"),
    ("subsection simulation control\n  set method = rk4\nend\n", "unknown time stepping method"),
    ("subsection boundary conditions\n set number = 1\n subsection bc 0\n  set type = outlet\n end\nend\n", "outlet"),
    ("subsection source term\n set enable = true\n subsection xyz\n  set Function expression = q*2; 0; 0; 0\n"
     " end\nend\n", "unknown variable 'q'"),
    ("subsection mesh\n set initial refinement = 2\n", "not closed"),
    ("subsection simulation control\n set method = steady\n set number mesh adapt = 1\nend\n"
     "subsection mesh adaptation\n set type = kelly\n set fraction type = banana\nend\n", "fraction type 'banana' is unknown"),
    ("subsection simulation control\n set method = steady\n set number mesh adapt = 1\nend\n"
     "subsection mesh adaptation\n set type = kelly\n set fraction refinement = 0.97\nend\n",  # default coarsening 0.05
     "refinement + coarsening <= 1"),
    # linear solver/method (parameters.cc:519-532): only amg | gmres | bicgstab; the amg entries validated
    ("subsection linear solver\n set method = direct\nend\n", "method 'direct' is invalid"),
    ("subsection linear solver\n set method = amg\n set amg n cycles = 0\nend\n", "amg n cycles must be >= 1"),
    ("subsection linear solver\n set method = amg\n set amg preconditioner ilu fill = 1.5\nend\n",
     "amg preconditioner ilu fill = 1.5 is not supported"),
    ("subsection linear solver\n set verbosity = loud\nend\n", "Unknown verbosity mode"),
    # restart (parameters.cc:759-798): checkpoint / restart out of scope, never silently ignored
    ("subsection restart\n set restart = true\nend\n", "restart/restart = true"),
    ("subsection restart\n set checkpoint = true\n set frequency = 5\nend\n", "restart/checkpoint = true"),
])
def test_app_rejects_unsupported_input_before_touching_the_gpu(tmp_path, text, msg):
    out = _app(tmp_path, text, "--dim", "3")
    assert out.returncode == 1 and msg in out.stderr, out.stderr
