"""End-to-end drop-in check of the C++ application (apps/gls_navier_stokes): parameter files in the
reference's format are generated here from the golden fixture data (forcing / exact solution
expressions, mesh sizes, schemes of the reference's application tests), the app runs the full
prm -> mesh -> initial condition -> time loop -> Newton/GMRES on the GPU -> L2 error path, and its
errors are compared with the numbers the reference printed."""
import json
import os
import subprocess
import numpy as np

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
APP = os.path.join(ROOT, "apps", "gls_navier_stokes")
G = json.load(open(os.path.join(ROOT, "tests", "golden", "reference_goldens.json")))


def run_app(tmp_path, prm, dim, *extra):
    f = tmp_path / "case.prm"
    f.write_text(prm)
    if not os.path.exists(APP):
        pytest.fail("apps/gls_navier_stokes is not built (run __graft_entry__.build())")
    out = subprocess.run([APP, "--dim", str(dim), "--precision", "9", *extra, str(f)], cwd=str(tmp_path),
                         capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-2000:]
    return out.stdout


def table(stdout):
    """rows of the reference-format error table (ConvergenceTable: "-" = no rate -> nan)"""
    rows, on = [], False
    for line in stdout.splitlines():
        if line.startswith("cells ") or line.startswith(" time "):
            on = True
            continue
        if on and line.strip() and not line.startswith("newton_iterations"):
            rows.append([float("nan") if v == "-" else float(v) for v in line.split()])
    return rows


def values(stdout, key):
    """numbers of the reference's 'key : value' post-processing lines"""
    return [float(l.split(":")[1]) for l in stdout.splitlines() if l.startswith(key)]


def mms_prm(g, dim, refinement, adapt):
    zeros = "; ".join(["0"] * (dim + 1))
    return f"""
subsection simulation control
  set method            = steady
  set number mesh adapt = {adapt}
  set output frequency  = 0
end
subsection physical properties
  set kinematic viscosity = 1.0
end
subsection mesh
  set type               = dealii
  set grid type          = hyper_cube
  set grid arguments     = -1 : 1 : false
  set initial refinement = {refinement}
end
subsection mesh adaptation
  set type = uniform
end
subsection FEM
  set velocity order = 1
  set pressure order = 1
end
subsection boundary conditions
  set number = 1
  subsection bc 0
    set type = noslip
  end
end
subsection source term
  set enable = true
  subsection xyz
    set Function expression = {g["force"]}
  end
end
subsection initial conditions
  set type = nodal
  subsection uvwp
    set Function expression = {zeros}
  end
end
subsection analytical solution
  set enable = true
  subsection uvw
    set Function expression = {g["exact"]}
  end
end
subsection non-linear solver
  set tolerance      = 1e-10
  set max iterations = 10
  set verbosity      = verbose
end
subsection linear solver
  set max iters         = 2000
  set relative residual = 1e-12
  set minimum residual  = 1e-14
end
"""


def close(a, b, digits):
    """within half a unit of the last printed digit (relative, as tests/test_oracle_goldens.py)"""
    return abs(a - b) <= 0.5 * 10.0 ** (1 - digits) * abs(b) * 1.0000001


@pytest.mark.gpu
@pytest.mark.parametrize("precond", ["jacobi", "mg"])
def test_app_mms3d_with_uniform_refinement(tmp_path, precond):
    g = G["mms3d_gls"]
    out = run_app(tmp_path, mms_prm(g, 3, 2, 1), 3, "--precond", precond)
    rows = table(out)
    assert [int(r[0]) for r in rows] == [64, 512], out
    for i, r in enumerate(rows):
        assert close(r[1], g["error_velocity"][i], 5), (r, out)
        assert close(r[3], g["error_pressure"][i], 5), (r, out)
    assert (tmp_path / "L2Error.dat").exists()


@pytest.mark.gpu
def test_app_mms2d(tmp_path):
    g = G["mms2d_gls"]
    out = run_app(tmp_path, mms_prm(g, 2, 3, 2), 2)
    rows = table(out)
    assert [int(r[0]) for r in rows] == [64, 256, 1024]
    for i, r in enumerate(rows):
        assert close(r[1], g["error_velocity"][i], 5), (r, g)
        assert close(r[3], g["error_pressure"][i], 5), (r, g)


def tgv_prm(method, k, kp, refinement, dt, t_end, output_frequency=0):
    c = G["tgv_common"]
    nu = c["viscosity"]
    bcs = "\n".join(f"""  subsection bc {i}
    set type               = periodic
    set id                 = {a}
    set periodic_id        = {b}
    set periodic_direction = {d}
  end""" for i, (a, b, d) in enumerate(c["periodic"]))
    return f"""
subsection simulation control
  set method           = {method}
  set time step        = {dt}
  set time end         = {t_end}
  set output frequency = {output_frequency}
  set output name      = tgv
end
subsection physical properties
  set kinematic viscosity = {nu}
end
subsection mesh
  set type               = dealii
  set grid type          = hyper_cube
  set grid arguments     = {c["domain"][0]} : {c["domain"][1]} : true
  set initial refinement = {refinement}
end
subsection FEM
  set velocity order = {k}
  set pressure order = {kp}
end
subsection boundary conditions
  set number = {len(c["periodic"])}
{bcs}
end
subsection initial conditions
  set type = L2projection
  subsection uvwp
    set Function expression = {c["initial_condition"]}
  end
end
subsection analytical solution
  set enable    = true
  set verbosity = verbose
  subsection uvw
    set Function constants  = viscosity={nu}
    set Function expression = exp(-2*viscosity*t)*cos(x)*sin(y); -sin(x)*cos(y)*exp(-2*viscosity*t); 0
  end
end
subsection post-processing
  set verbosity                = verbose
  set calculate enstrophy      = true
  set calculate kinetic energy = true
end
subsection non-linear solver
  set tolerance      = {c["newton_tol"]}
  set max iterations = {c["newton_max_it"]}
  set verbosity      = quiet
end
subsection linear solver
  set max iters         = 5000
  set relative residual = 1e-13
  set minimum residual  = 1e-14
end
"""


@pytest.mark.gpu
def test_app_tgv_sdirk2_l2projection_periodic(tmp_path):
    g = G["tgv_sdirk2"]
    out = run_app(tmp_path, tgv_prm("sdirk2", g["k"], g["kp"], 6, g["dt"], g["t_end"]), 2)
    assert len(values(out, "L2 error velocity :")) == 1
    e = [r[1] for r in table(out)]  # the transient error table, printed with --precision 9
    assert len(e) == 1 and close(e[0], g["error_velocity_log"], 6), out
    # the initial state's kinetic energy and enstrophy of the TGV field are 1/4 and 1/2
    ke = values(out, "Kinetic energy :")
    en = values(out, "Enstrophy  :")
    assert abs(ke[0] - 0.25) < 1e-3 and abs(en[0] - 0.5) < 2e-3


@pytest.mark.gpu
def test_app_tgv_bdf1_first_step_and_output(tmp_path):
    g = G["tgv_bdf1"]
    out = run_app(tmp_path, tgv_prm("bdf1", g["k"], g["kp"], 5, g["dt"], g["dt"], output_frequency=1), 2)
    e = [r[1] for r in table(out)]
    assert close(e[0], g["checkpoints"]["0.01"], 5), out
    for f in ("tgv.pvd", "tgv.00000.pvtu", "tgv.00001.pvtu", "tgv.00001.00000.vtu"):
        assert (tmp_path / f).exists(), f


@pytest.mark.gpu
def test_app_mms2d_slip_walls_matches_oracle(tmp_path):
    """bc type = slip (compute_no_normal_flux_constraints, gls_navier_stokes.cc:100-110) on every wall of
    the mms2d case: the app's velocity L2 error equals the oracle's direct-Newton solution of the same
    constrained problem (no reference golden exists for slip on this mesh: parity pinned by the oracle)."""
    import numpy as np
    from oracle.oracle import Oracle, StructuredProblem, muparser_to_numpy, newton_solve
    g = G["mms2d_gls"]
    prm = mms_prm(g, 2, 3, 1).replace("    set type = noslip", "    set type = slip")
    out = run_app(tmp_path, prm, 2)
    rows = table(out)
    assert [int(r[0]) for r in rows] == [64, 256]  # initial refinement 3, one uniform adaptation
    F, E = muparser_to_numpy(g["force"]), muparser_to_numpy(g["exact"])
    for row, n in zip(rows, (8, 16)):
        p = StructuredProblem(2, n, k=1, viscosity=1.0)
        p.set_force(lambda X: F(X)[:, :2])
        p.set_dirichlet([("slip", 0, None)])
        x, its, res = newton_solve(p, tol=1e-10)
        eu, ep = Oracle(p).l2_error(x, E)
        assert abs(row[1] - eu) <= 1e-6 * eu, (row, eu)
        assert np.isfinite(ep)
    # slip is not noslip: the error differs from the reference's noslip golden
    assert abs(rows[0][1] - g["error_velocity"][0]) > 1e-3 * g["error_velocity"][0]


def _leaf_lex(tree, n_uniform):
    """lexicographic hyper_cube(n_uniform) cell index of each leaf of a uniform forest"""
    lev, x0, h = tree.cells()
    hc = (tree.hi - tree.lo) / n_uniform
    ij = np.round((x0 - tree.lo) / hc).astype(np.int64)
    return sum(ij[:, d] * n_uniform ** d for d in range(tree.dim))


@pytest.mark.gpu
@pytest.mark.parametrize("dim,variable,ftype,coarsen,adapts", [
    (2, "velocity", "number", 0.0, 1), (2, "pressure", "number", 0.0, 1), (3, "velocity", "number", 0.0, 1),
    (2, "velocity", "fraction", 0.0, 1), (2, "velocity", "number", 0.1, 3), (2, "pressure", "fraction", 0.05, 3),
    (3, "velocity", "number", 0.1, 2)])
def test_app_mms_kelly_adaptation_matches_oracle(tmp_path, dim, variable, ftype, coarsen, adapts):
    """mesh adaptation type = kelly (refine_mesh_kelly, navier_stokes_base.cc:610-780) in the app over
    `adapts` steady cycles of mms2d (8^2) / mms3d (8^3), Q1: Kelly on the device (conforming kernel on
    the uniform mesh, face-piece kernel on the adapted ones), p::d::GridRefinement marking with
    refinement 0.3 and coarsening, max / min level rules, prepare_coarsening_and_refinement smoothing,
    forest adaptation with hanging nodes, SolutionTransfer, Newton on each mesh. The first row equals
    the reference golden; every later row equals the oracle's own pipeline (oracle Kelly -> oracle
    marking -> oracle smoothing -> the forest -> condensed oracle Newton): cell counts exactly, errors
    at 1e-6. Parity unpinned beyond the oracle: the reference holds no Kelly golden on this mesh."""
    from oracle.oracle import (Oracle, StructuredProblem, kelly_estimate, kelly_estimate_boxes, muparser_to_numpy,
                               newton_solve, pd_refine_coarsen, prepare_coarsening_and_refinement)
    import softx_2020_200_amd as sx
    g = G["mms2d_gls" if dim == 2 else "mms3d_gls"]
    n, gi = (8, 0) if dim == 2 else (8, 1)  # 4^3: the discrete velocity is ~0, Kelly is roundoff
    prm = mms_prm(g, dim, 3, adapts).replace("  set type = uniform\n", f"""  set type = kelly
  set variable = {variable}
  set fraction type = {ftype}
  set fraction refinement = 0.3
  set fraction coarsening = {coarsen}
""")
    out = run_app(tmp_path, prm, dim, "--precond", "jacobi")
    rows = table(out)
    assert len(rows) == adapts + 1, out
    assert int(rows[0][0]) == n ** dim and close(rows[0][1], g["error_velocity"][gi], 5), (rows, out)
    # the oracle's pipeline on the same meshes
    F, E = muparser_to_numpy(g["force"]), muparser_to_numpy(g["exact"])
    p = StructuredProblem(dim, n, k=1, viscosity=1.0)
    p.set_force(lambda X: F(X)[:, :dim])
    p.set_dirichlet([("noslip", 0, None)])
    x, _, _ = newton_solve(p, tol=1e-10)
    tree = sx.Octree(dim, 1)
    for _ in range(3):
        tree.adapt(np.ones(tree.n_cells, np.int32))
    eta = kelly_estimate(p, x, 0 if variable == "velocity" else 1)[_leaf_lex(tree, n)]
    var = 0 if variable == "velocity" else 1
    leaves = lambda t: [(int(l), tuple(int(round(v)) for v in (x0 - t.lo) / hh)) for l, x0, hh in zip(*t.cells())]
    coarsened = 0
    for a in range(adapts):
        nc = tree.n_cells
        r, c, _ = pd_refine_coarsen(eta.astype(np.float32), dim, 0.3, coarsen, ftype)
        lev = tree.cells()[0]
        c[lev == 0] = 0  # min refinement level 0; max level 10 is not reached
        r0 = int(r.sum())
        c0 = int(c.sum())
        r, c = prepare_coarsening_and_refinement(dim, 1, leaves(tree), r, c)
        assert (f"kelly: {r0} of {nc} cells flagged for refinement, {c0} for coarsening (after smoothing: "
                f"{int(r.sum())}, {int(c.sum())})") in out
        coarsened += int(c.sum())
        tree.adapt(r, c)
        assert int(rows[a + 1][0]) == tree.n_cells == nc + (2 ** dim - 1) * (int(r.sum()) - int(c.sum()) // 2 ** dim), \
            (a, rows, int(r.sum()), int(c.sum()))
        mesh = tree.mesh(1, 1)
        q = StructuredProblem.from_refined(mesh, viscosity=1.0)
        lines = sx.hanging_dof_lines(mesh)
        q.set_hanging(*lines)
        q.hang_lines = lines
        q.set_dirichlet([("noslip", 0, None)])
        q.set_force(lambda X: F(X)[:, :dim])
        y, _, _ = newton_solve(q, tol=1e-10)
        eu, ep = Oracle(q).l2_error(y, E)
        assert abs(rows[a + 1][1] - eu) <= 1e-6 * eu, (a, rows[a + 1], eu)
        assert abs(rows[a + 1][3] - ep) <= 1e-6 * ep, (a, rows[a + 1], ep)
        eta = kelly_estimate_boxes(mesh, y, var)
    assert rows[-1][1] < rows[0][1]
    if coarsen == 0:  # (with coarsening, whether complete families survive the smoothing depends on the case)
        assert coarsened == 0, coarsened


SHELL_ROTATION_PRM = """
subsection simulation control
  set method            = steady
  set number mesh adapt = 1
  set output frequency  = 0
end
subsection FEM
  set velocity order = 2
  set pressure order = 1
  set qmapping all   = true
end
subsection physical properties
  set kinematic viscosity = 1.0
end
subsection mesh
  set type           = dealii
  set grid type      = hyper_shell
  set grid arguments = 0, 0 : 0.25 : 1 : 8 : true
  set initial refinement = 1
end
subsection boundary conditions
  set number = 2
  subsection bc 0
    set id = 0
    set type = function
    subsection u
      set Function expression = -y
    end
    subsection v
      set Function expression = x
    end
  end
  subsection bc 1
    set id = 1
    set type = {outer}
  end
end
subsection mesh adaptation
  set type = uniform
end
subsection analytical solution
  set enable = true
  subsection uvw
    set Function expression = -y*(1+1/(x*x+y*y))/17; x*(1+1/(x*x+y*y))/17; 0
  end
end
subsection non-linear solver
  set tolerance      = 1e-10
  set max iterations = 10
end
subsection linear solver
  set max iters         = 5000
  set relative residual = 1e-12
  set minimum residual  = 1e-14
end
"""


@pytest.mark.gpu
def test_app_slip_on_curved_wall_rigid_rotation(tmp_path):
    """slip on a curved wall (compute_no_normal_flux_constraints with node normals that are not axes,
    gls_navier_stokes.cc:100-110): the velocity component of largest |n_c| is constrained by the line
    u_c = -sum (n_d / n_c) u_d. Inner circle (r = 1/4) rotating with u = (-y, x), outer circle (r = 1)
    slip: with the reference's Laplacian viscous form the natural condition on the slip wall is
    d u_theta / dr = 0, so the exact flow is u_theta = (r + 1/r) / 17 (u_theta(1/4) = 1/4,
    u_theta'(1) = 0) with dp/dr = u_theta^2 / r; the velocity error against it falls with refinement,
    while a no-slip outer wall gives the Taylor-Couette profile, far from it. Parity unpinned (no
    reference case uses slip on a curved wall); checked against the analytic solution."""
    rows = table(run_app(tmp_path, SHELL_ROTATION_PRM.replace("{outer}", "slip"), 2))
    assert len(rows) == 2, rows
    assert rows[0][1] < 1e-2 and rows[1][1] < rows[0][1] / 4, rows  # Q2 velocity: ~h^3 on curved cells
    rows_ns = table(run_app(tmp_path, SHELL_ROTATION_PRM.replace("{outer}", "noslip"), 2))
    assert rows_ns[-1][1] > 10 * rows[-1][1], (rows, rows_ns)


@pytest.mark.gpu
def test_app_slip_on_curved_wall_kelly_hanging_chains(tmp_path):
    """Kelly adaptation next to a curved slip wall: a hanging node on the outer circle has master
    vertices whose u_cmax carries the slip line, so the hanging line's masters are themselves
    constrained; the app closes the chain (AffineConstraints::close(): the slip line's masters
    substituted with the weights multiplied) instead of aborting. Two Kelly cycles of the rigid
    rotation case above (fixed fraction 0.4 of the cells refined, so the refined region ends on the
    wall): it runs and the error against the analytic profile stays at the uniform runs' level and
    falls. Parity unpinned (no reference case uses slip on a curved wall); checked against the
    analytic solution."""
    prm = (SHELL_ROTATION_PRM.replace("{outer}", "slip").replace("number mesh adapt = 1", "number mesh adapt = 2")
           .replace("set type = uniform", "set type = kelly\n  set fraction type = number\n"
                    "  set fraction refinement = 0.4\n  set fraction coarsening = 0.0\n  set variable = velocity"))
    rows = table(run_app(tmp_path, prm, 2))
    assert len(rows) == 3, rows
    assert rows[0][1] < 1e-2 and rows[-1][1] < rows[0][1], rows
    # not uniform: the adapted meshes have fewer cells than 4^cycles x the initial mesh
    assert int(rows[-1][0]) < 16 * int(rows[0][0]), rows


PI_ = "3.14159265358979"
PERIODIC_MMS_FORCE = ("-12*{pi}*y^2*(y^2 - 1)^2*(3*cos({pi}*x) + 10)*sin({pi}*x)/25 + 6*{pi}^2*y*(y^2 - 1)*cos({pi}*x)/5 "
                      "- 12*y*(3*cos({pi}*x) + 10)/5 + {pi}*y*cos({pi}*x)/5 + 3*{pi}*(y^2 - 1)^2*(3*y^2 - 1)*"
                      "(3*cos({pi}*x) + 10)*sin({pi}*x)/25; 3*{pi}^2*y*(y^2 - 1)^3*(3*cos({pi}*x) + 10)*cos({pi}*x)/25 "
                      "+ 9*{pi}^2*y*(y^2 - 1)^3*sin({pi}*x)^2/25 + 3*{pi}^3*(y^2 - 1)^2*sin({pi}*x)/10 "
                      "- 6*{pi}*(3*y^2 - 1)*sin({pi}*x)/5 + sin({pi}*x)/5; 0").format(pi=PI_)
PERIODIC_MMS_EXACT = ("2*y*(y^2 - 1)*(3*cos({pi}*x) + 10)/5; 3*{pi}*(y^2 - 1)^2*sin({pi}*x)/10; "
                      "y*sin({pi}*x)/5").format(pi=PI_)


@pytest.mark.gpu
@pytest.mark.parametrize("k", [1, 2])
def test_app_periodic_kelly_adaptation(tmp_path, k):
    """Periodic boundaries under Kelly adaptation (gls_navier_stokes.cc:130-134, 164-168 with
    refine_mesh_kelly): a steady manufactured flow on [-1, 1]^2, periodic in x, no-slip walls at y = +-1,
    u = curl psi, psi = (1 - y^2)^2 (1 + 0.3 cos(pi x)), p = 0.2 y sin(pi x) (force from sympy). The
    forest wraps its neighbourhoods and identifies the periodic faces, hanging lines included; three
    Kelly cycles refine (hanging DoFs appear) and the velocity error vs the exact solution falls every
    cycle. Parity unpinned: no reference case combines periodicity with adaptation (the operator on such
    meshes is checked against the oracle in tests/test_hanging.py::test_periodic_octree_gpu_vs_oracle)."""
    prm = mms_prm({"force": PERIODIC_MMS_FORCE, "exact": PERIODIC_MMS_EXACT}, 2, 3, 2)
    prm = prm.replace("  set grid arguments     = -1 : 1 : false", "  set grid arguments     = -1 : 1 : true")
    prm = prm.replace("  set velocity order = 1\n  set pressure order = 1", f"  set velocity order = {k}\n  set pressure order = 1")
    prm = prm.replace("  set type = uniform\n", """  set type = kelly
  set variable = velocity
  set fraction type = number
  set fraction refinement = 0.3
  set fraction coarsening = 0.0
""")
    prm = prm.replace("""subsection boundary conditions
  set number = 1
  subsection bc 0
    set type = noslip
  end
end""", """subsection boundary conditions
  set number = 3
  subsection bc 0
    set type = periodic
    set id = 0
    set periodic_id = 1
    set periodic_direction = 0
  end
  subsection bc 1
    set type = noslip
    set id = 2
  end
  subsection bc 2
    set type = noslip
    set id = 3
  end
end""")
    out = run_app(tmp_path, prm, 2, "--precond", "jacobi")
    rows = table(out)
    assert len(rows) == 3, out
    cells = [int(r[0]) for r in rows]
    assert cells[0] == 64 and cells[1] > cells[0] and cells[2] > cells[1], cells
    errs = [r[1] for r in rows]
    assert errs[1] < errs[0] and errs[2] < errs[1], errs
    hang = [int(l.split(":")[1]) for l in out.splitlines() if "Hanging node DoFs" in l]
    assert hang and max(hang) > 0, out[-3000:]
    assert "kelly:" in out


@pytest.mark.gpu
@pytest.mark.parametrize("k", [1, 2])
def test_app_periodic_kelly_adaptation_general_mesh(tmp_path, k):
    """The same periodic manufactured flow on the GENERAL mesh path (GridGenerator
    subdivided_hyper_rectangle -> gls_umesh: MappingQ geometry, per-cell kernels): the triangulation
    carries the periodic pair (gls_umesh_set_periodic: the smoothing and the 2:1 balance see across it),
    the space identifies the partnered nodes and constrains the nodes of a finer periodic face to the
    coarser face across it, the Kelly faces include the periodic pieces. Three Kelly cycles refine and the
    velocity error falls every cycle. Parity unpinned (no reference case combines periodicity with
    adaptation; the constraint algebra is checked on the CPU in tests/test_umesh_periodic.py)."""
    prm = mms_prm({"force": PERIODIC_MMS_FORCE, "exact": PERIODIC_MMS_EXACT}, 2, 3, 2)
    prm = prm.replace("  set grid type          = hyper_cube\n  set grid arguments     = -1 : 1 : false",
                      "  set grid type          = subdivided_hyper_rectangle\n"
                      "  set grid arguments     = 1,1 : -1,-1 : 1,1 : true")
    assert "subdivided_hyper_rectangle" in prm
    prm = prm.replace("  set velocity order = 1\n  set pressure order = 1", f"  set velocity order = {k}\n  set pressure order = 1")
    prm = prm.replace("  set type = uniform\n", """  set type = kelly
  set variable = velocity
  set fraction type = number
  set fraction refinement = 0.3
  set fraction coarsening = 0.0
""")
    prm = prm.replace("""subsection boundary conditions
  set number = 1
  subsection bc 0
    set type = noslip
  end
end""", """subsection boundary conditions
  set number = 3
  subsection bc 0
    set type = periodic
    set id = 0
    set periodic_id = 1
    set periodic_direction = 0
  end
  subsection bc 1
    set type = noslip
    set id = 2
  end
  subsection bc 2
    set type = noslip
    set id = 3
  end
end""")
    out = run_app(tmp_path, prm, 2, "--precond", "jacobi")
    rows = table(out)
    assert len(rows) == 3, out
    cells = [int(r[0]) for r in rows]
    assert cells[0] == 64 and cells[1] > cells[0] and cells[2] > cells[1], cells
    errs = [r[1] for r in rows]
    assert errs[1] < errs[0] and errs[2] < errs[1], errs
    # the uniform first mesh equals the hyper_cube path's (same cells, same periodic identification)
    ref = run_app(tmp_path, prm.replace("  set grid type          = subdivided_hyper_rectangle\n"
                                        "  set grid arguments     = 1,1 : -1,-1 : 1,1 : true",
                                        "  set grid type          = hyper_cube\n  set grid arguments     = -1 : 1 : true"),
                  2, "--precond", "jacobi")
    r0 = table(ref)[0]
    assert abs(rows[0][1] - r0[1]) <= 1e-6 * r0[1], (rows[0], r0)


@pytest.mark.gpu
def test_app_transient_kelly_periodic_tgv(tmp_path):
    """Transient Kelly adaptation on a periodic hyper_cube (refine_mesh_kelly every step with the time
    history transferred, navier_stokes_base.cc:684-733): the reference's 2D Taylor-Green vortex prm
    (Q2-Q1, SDIRK2, periodic in x and y) on 16^2 cells, 3 steps of 0.05 with Kelly every step, against
    the same run on the uniform mesh: the adapted meshes carry hanging DoFs across the periodic faces and
    the velocity error vs the analytic decay stays at or below the uniform run's every step. Parity
    unpinned (no reference golden for an adapted TGV)."""
    base = open(os.path.join(os.path.dirname(__file__), "golden", "app_cases", "taylor-green-vortex_gls_sdirk2.prm")).read()
    prm = (base.replace("set time step               = 0.100", "set time step = 0.05")
               .replace("set time end                = 0.10", "set time end = 0.15")
               .replace("set output frequency        = 1 ", "set output frequency = 0 ")
               .replace("set initial refinement   = 6", "set initial refinement = 4")
               .replace("set tolerance               = 1e-6", "set tolerance = 1e-9")
               .replace("set relative residual                     = 1e-4", "set relative residual = 1e-10")
               .replace("set minimum residual                      = 1e-9", "set minimum residual = 1e-13"))
    assert "time step = 0.05" in prm and "initial refinement = 4" in prm and "tolerance = 1e-9" in prm, prm
    errs = {}
    for tag, adapt in (("uniform", "  set type                    = none"),
                       ("kelly", "  set type = kelly\n  set frequency = 1\n  set variable = velocity\n"
                                 "  set fraction type = number\n  set fraction refinement = 0.2\n"
                                 "  set fraction coarsening = 0.0\n  set max refinement level = 6")):
        d = tmp_path / tag
        d.mkdir()
        out = run_app(d, prm.replace("  set type                    = none", adapt), 2)
        errs[tag] = [float(l.split(":")[1]) for l in out.splitlines() if l.startswith("L2 error velocity")]
        if tag == "kelly":
            hang = [int(l.split(":")[1]) for l in out.splitlines() if "Hanging node DoFs" in l]
            assert hang and max(hang) > 0, out[-3000:]
    assert len(errs["uniform"]) == len(errs["kelly"]) == 3, errs
    for a, b in zip(errs["kelly"], errs["uniform"]):
        assert 0 < a <= 1.0001 * b, errs


@pytest.mark.gpu
def test_app_kelly_forest_multigrid(tmp_path):
    """3D Kelly adaptation of mms3d (Q1-Q1, two cycles with coarsening) with the hierarchy multigrid on the
    adapted hyper_cubes (--precond hmg; method = amg picks it too): the V-cycle on the forest's refinement
    hierarchy (gls_mg_attach_transfers, announced on stderr) gives the error table of the ILU-preconditioned run
    (method = gmres, the app's default there as the reference's setup_ILU, gls_navier_stokes.cc:1161-1176):
    same cell counts, errors at 1e-6 (converged solves)."""
    import subprocess
    g = G["mms3d_gls"]
    prm = mms_prm(g, 3, 3, 2).replace("  set type = uniform\n", """  set type = kelly
  set variable = velocity
  set fraction type = number
  set fraction refinement = 0.3
  set fraction coarsening = 0.1
""")
    res = {}
    for pc in ("hmg", "mg"):
        f = tmp_path / ("%s.prm" % pc)
        f.write_text(prm)
        out = subprocess.run([APP, "--dim", "3", "--precision", "9", "--stats", "--precond", pc, str(f)],
                             cwd=str(tmp_path), capture_output=True, text=True, timeout=600)
        assert out.returncode == 0, out.stderr[-2000:]
        its = [int(l.split("linear_iterations =")[1]) for l in out.stdout.splitlines() if "linear_iterations =" in l]
        res[pc] = (table(out.stdout), out.stderr, its)
    assert "refinement hierarchy" in res["hmg"][1], res["hmg"][1][-800:]
    assert "refinement hierarchy" not in res["mg"][1] and "ILU(" in res["mg"][1], res["mg"][1][-800:]
    rm, ri = res["hmg"][0], res["mg"][0]
    assert len(rm) == len(ri) == 3 and [r[0] for r in rm] == [r[0] for r in ri], (rm, ri)
    for a, b in zip(rm, ri):
        assert abs(a[1] - b[1]) <= 1e-6 * b[1] and abs(a[3] - b[3]) <= 1e-6 * b[3], (a, b)
    print("forest GMG linear iterations %s, ILU %s" % (res["hmg"][2], res["mg"][2]))
