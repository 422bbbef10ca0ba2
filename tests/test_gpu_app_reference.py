"""The reference's own application tests through the drop-in entry points: each case is the
reference's .prm (tests/golden/app_cases/, copied from applications_tests/ with its mesh fixtures in
tests/golden/meshes/) run by apps/gls_navier_stokes_{2d,3d} on the GPU; its stdout is diffed
against the reference's .output the way the reference's harness does, on the lines this build
prints: 'Number of active cells / degrees of freedom / Volume of triangulation' and the final
error table (cells, error_velocity, error_pressure and their log2 rates, printed digits).
Documented exceptions: the torque summary (forces are out of scope) is not produced; DoF counts
of periodic cases count identified nodes once (deal.II counts them twice and constrains one);
taylorcouette_gls's pressure column depends on the reference solver's free pressure constant
(tests/golden/reference_goldens.json, curved/taylorcouette_gls/pressure_note)."""
import os
import re
import shutil
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CASES = os.path.join(ROOT, "tests", "golden", "app_cases")
MESHES = os.path.join(ROOT, "tests", "golden", "meshes")


def run_case(tmp_path, name, dim, *extra, prm_edit=None):
    prm = open(os.path.join(CASES, name + ".prm")).read()
    prm = re.sub(r"(set file name\s*=\s*)\.\./", r"\1", prm)  # the fixtures sit next to the prm here
    if prm_edit is not None:
        prm = prm_edit(prm)
    for f in os.listdir(MESHES):
        shutil.copy(os.path.join(MESHES, f), tmp_path / f)
    (tmp_path / "case.prm").write_text(prm)
    app = os.path.join(ROOT, "apps", "gls_navier_stokes_%dd" % dim)
    if not os.path.exists(app):
        pytest.fail("%s is not built (run __graft_entry__.build())" % app)
    out = subprocess.run([app, *extra, "case.prm"], cwd=str(tmp_path), capture_output=True, text=True, timeout=900)
    assert out.returncode == 0, out.stderr[-3000:]
    return out.stdout


def setup_lines(text):
    return [l.strip() for l in text.splitlines() if l.strip().startswith(("Number of active cells", "Number of degrees",
                                                                         "Volume of triangulation"))]


def error_rows(text):
    rows, on = [], False
    for l in text.splitlines():
        if l.startswith("cells "):
            on = True
            continue
        if on and l.strip():
            rows.append(l.split())
    return rows


@pytest.mark.gpu
@pytest.mark.parametrize("name,dim,periodic,pressure", [
    ("mms2d_gls", 2, False, True), ("mms3d_gls", 3, False, True), ("mms2d-unstructured_gls", 2, False, True),
    ("taylorcouette-unstructured_gls", 2, False, True), ("taylorcouette_gls", 2, False, False),
    ("rigid-body-rotation_gls", 2, False, False), ("poiseuille_gls", 2, True, False),
    ("poiseuille3d_gls", 3, True, False), ("cylinder-rigid-body_gls", 3, False, False)])
def test_reference_application_case(tmp_path, name, dim, periodic, pressure):
    ref = open(os.path.join(CASES, name + ".output")).read()
    out = run_case(tmp_path, name, dim)
    ours, theirs = setup_lines(out), setup_lines(ref)
    assert len(ours) == len(theirs), out
    for a, b in zip(ours, theirs):  # periodic cases too: deal.II's DoF count (periodicity as a constraint)
        assert a == b, (a, b)
    ro, rr = error_rows(out), error_rows(ref)
    print(name, "ours", ro, "reference", rr)
    assert len(ro) == len(rr), out
    roundoff = name in ("rigid-body-rotation_gls", "cylinder-rigid-body_gls")  # exact solution: errors ~1e-11
    for a, b in zip(ro, rr):
        assert a[0] == b[0]  # cells
        if roundoff:  # the exact discrete solution, to the prm's Newton tolerance (1e-8 / 1e-9)
            assert float(a[1]) < 1e-7 and float(a[3]) < 1e-7, a
            continue
        if name == "poiseuille_gls":  # Newton tol 1e-6 / 3 its with GMRES rel 1e-4: the printed error's
            # last digit depends on the inexact solve (the exactly converged oracle gives 2.22743e-04,
            # the reference's 2.2274e-04); one unit of the last printed digit is allowed
            assert abs(float(a[1]) - float(b[1])) <= 1.01e-4 * float(b[1]), (name, a, b)
            continue
        assert a[1] == b[1], (name, a, b)  # error_velocity at the printed digits
        if len(b) > 2 and b[2] != "-":
            assert a[2] == b[2], (name, a, b)
        if pressure:
            assert a[3:] == b[3:], (name, a, b)
        elif name.startswith("poiseuille"):
            # the exact pressure (linear) lies in the Q1 space: both columns are the inexact solve's noise
            # (reference 2.5e-09..1.6e-08); bounded at the same scale instead of diffed
            assert float(a[3]) < 1e-7 and float(b[3]) < 1e-7, (name, a, b)
        elif name == "taylorcouette_gls":
            # the reference's column carries its solver's free pressure constant (pressure_note): ours,
            # without it, stays below the reference's on every level
            assert float(a[3]) < float(b[3]), (name, a, b)


@pytest.mark.gpu
@pytest.mark.parametrize("method", ["sdirk2", "sdirk3"])
def test_reference_tgv_sdirk_cases(tmp_path, method):
    """The reference's taylor-green-vortex_gls_{sdirk2,sdirk3} application tests as shipped (Q2-Q1,
    periodic, L2-projection IC, one step of 0.1, Newton tol 1e-6, GMRES rel 1e-4 -- an inexact
    Newton): enstrophy and kinetic energy before and after the step match the .output to all printed
    digits. The L2 error depends on where the inexact linear solves stop. For SDIRK3, exact solves
    give 1.38239e-4 (oracle); this build's ILU(1)-GMRES at the reference's tolerances gives
    1.38249e-4 (ILU(0): 1.38207e-4); the reference printed 1.38223e-4. The values differ by 1.9e-4
    relative: the DoF order of the ILU factors and AztecOO's GMRES internals decide where the inexact
    Newton stops. So the error is checked at that scale (3e-4 relative). SDIRK2 is checked at 1e-5
    relative (1.20259e-3 vs the printed 1.20258e-3)."""
    name = "taylor-green-vortex_gls_" + method
    prm = open(os.path.join(CASES, name + ".prm")).read()
    prm = re.sub(r"set output frequency\s*=\s*1 ", "set output frequency = 1000000 ", prm)
    (tmp_path / "case.prm").write_text(prm)
    app = os.path.join(ROOT, "apps", "gls_navier_stokes_2d")
    out = subprocess.run([app, "case.prm"], cwd=str(tmp_path), capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-3000:]
    ref = open(os.path.join(CASES, name + ".output")).read()
    pick = lambda t, key: [l.split(":")[1].strip() for l in t.splitlines() if l.startswith(key)]
    for key in ("Enstrophy", "Kinetic energy"):
        assert pick(out.stdout, key) == pick(ref, key), (key, pick(out.stdout, key), pick(ref, key))
    e, r = float(pick(out.stdout, "L2 error velocity")[0]), float(pick(ref, "L2 error velocity")[0])
    assert abs(e - r) <= (3e-4 if method == "sdirk3" else 1e-5) * r, (e, r)


@pytest.mark.gpu
def test_reference_cylinder_kelly_adaptation(tmp_path):
    """applications_tests/gls_navier_stokes_2d/cylinder_gls run as shipped (no prm edit): gmsh
    cylinder_structured.msh, Q1-Q1, slip walls, 3 steady Kelly adaptations (fraction type number,
    refine 0.3 / coarsen 0.1, max 70000 cells, max level 5), Newton 1e-4 and ILU(1)-GMRES rel 1e-4.
    The first two meshes reproduce the reference's counts exactly (1167/3750, 2247/7134). The third
    mesh has 4293 active cells and 13629 DoFs, against the reference's 4302 and 13653. The fourth has
    8256 and 26040, against 8268 and 26076.

    Remaining cause: the inexact solves. Kelly marks by a float threshold, and the solve stops at
    GMRES rel 1e-4. Where it stops depends on the ILU(1) factors, which depend on the DoF order:
    deal.II's Cuthill-McKee runs on deal.II's own initial DoF numbering, which this build cannot
    reproduce. It also depends on AztecOO's GMRES internals. With ILU(0) the third mesh had 4284
    cells. With converged solves (Newton 1e-10, GMRES rel 1e-12) all four meshes match the
    reference exactly (the second test below)."""
    ref = open(os.path.join(CASES, "cylinder_gls.output")).read()
    out = run_case(tmp_path, "cylinder_gls", 2)
    ours, theirs = setup_lines(out), setup_lines(ref)
    assert len(ours) == len(theirs) == 12, (ours, theirs)
    assert ours[:6] == theirs[:6], (ours, theirs)
    count = lambda l: int(l.split(":")[1])
    for a, b in zip(ours[6:], theirs[6:]):
        if a.startswith("Volume"):
            assert a == b
        else:  # inexact-solve spread of the Kelly marking (the measured values are in the docstring)
            assert abs(count(a) - count(b)) <= 0.005 * count(b), (a, b)


@pytest.mark.gpu
def test_reference_cylinder_kelly_adaptation_converged(tmp_path):
    """The same case with the solves converged (Newton 1e-10, GMRES rel 1e-12): the discrete solution
    no longer depends on the preconditioner, and every cycle's active-cell and DoF counts equal the
    reference's (1167/3750, 2247/7134, 4302/13653, 8268/26076)."""
    ref = open(os.path.join(CASES, "cylinder_gls.output")).read()
    out = run_case(tmp_path, "cylinder_gls", 2, prm_edit=lambda t: t.replace(
        "set tolerance               = 1e-4", "set tolerance = 1e-10").replace(
        "set relative residual       = 1e-4", "set relative residual = 1e-12").replace(
        "set minimum residual        = 1e-9", "set minimum residual = 1e-14"))
    ours, theirs = setup_lines(out), setup_lines(ref)
    assert ours == theirs, (ours, theirs)


@pytest.mark.gpu
@pytest.mark.parametrize("method", ["gmres", "bicgstab", "amg"])
def test_reference_mms2d_every_linear_solver_method(tmp_path, method):
    """'linear solver/method' (parameters.cc:519-532) is honoured, not ignored: the reference's mms2d_gls
    with each of gmres, bicgstab (solve_system_BiCGStab, gls_navier_stokes.cc:1293-1340) and amg
    (solve_system_AMG, :1344-1391; the ML hierarchy is substituted explicitly, announced on stderr)
    reproduces the golden error table; the app states the solver / preconditioner it used."""
    app = os.path.join(ROOT, "apps", "gls_navier_stokes_2d")
    prm = open(os.path.join(CASES, "mms2d_gls.prm")).read()
    prm, n = re.subn(r"(subsection linear solver.*?set method\s*=\s*)\w+", r"\g<1>" + method, prm, flags=re.S)
    assert n == 1
    (tmp_path / "case.prm").write_text(prm)
    out = subprocess.run([app, "case.prm"], cwd=str(tmp_path), capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-3000:]
    want = {"gmres": "-> GMRES + ILU(", "bicgstab": "-> BiCGStab + ILU(", "amg": "-> GMRES + ILU("}[method]
    line = [l for l in out.stderr.splitlines() if l.startswith("linear solver: method = " + method)]
    assert len(line) == 1 and want in line[0], out.stderr[-2000:]
    if method == "amg":
        assert "ML AMG substituted" in line[0]
    ref = open(os.path.join(CASES, "mms2d_gls.output")).read()
    assert error_rows(out.stdout) == error_rows(ref), (error_rows(out.stdout), error_rows(ref))


@pytest.mark.gpu
def test_reference_cylinder_kelly_flag_flips_are_within_the_inexact_solve_perturbation(tmp_path):
    """Why the shipped cylinder_gls run (Newton 1e-4, GMRES rel 1e-4) does not reproduce the reference's
    third and fourth meshes exactly while the converged run does: run both with --dump, recompute on the
    oracle side, for each cycle on the common mesh, the Kelly indicator of each run's solution
    (kelly_from_face_pieces: MappingQ1 face pieces, QGauss(3)) and the p::d fixed-number marking
    (pd_refine_coarsen: refine 0.3 / coarsen 0.1, max 70000 cells). At the first cycle whose flags
    differ, EVERY differing cell K must satisfy |eta_conv(K) - theta_conv| <= |eta_ship(K) - eta_conv(K)|
    + |theta_ship - theta_conv| (theta: that flag's threshold): the flip is explained by how far the
    inexact solve moved that cell's indicator and the threshold, not by a difference in the
    estimator, the marking or the mesh. The measured perturbation and the flipped cells are printed."""
    from oracle.oracle import kelly_from_face_pieces, pd_refine_coarsen
    from softx_2020_200_amd.native import UMesh
    from tests.test_gpu_app_configs import read_dumps
    converged = lambda t: t.replace("set tolerance               = 1e-4", "set tolerance = 1e-10").replace(  # noqa: E731
        "set relative residual       = 1e-4", "set relative residual = 1e-12").replace(
        "set minimum residual        = 1e-9", "set minimum residual = 1e-14")
    runs = {}
    for tag, edit in (("shipped", None), ("converged", converged)):
        d = tmp_path / tag
        d.mkdir()
        (d / "dump").mkdir()
        run_case(d, "cylinder_gls", 2, "--dump", str(d / "dump"), prm_edit=edit)
        runs[tag] = read_dumps(str(d / "dump"))
    assert len(runs["shipped"]) == len(runs["converged"]) == 4
    m = UMesh(2, gmsh=os.path.join(MESHES, "cylinder_structured.msh"))
    first_diff = None
    for cyc in range(3):
        h = m.fe_space_handle(1, 1)
        sp = h.data
        ds, dc = runs["shipped"][cyc], runs["converged"][cyc]
        assert int(ds["n_cells"]) == int(dc["n_cells"]) == sp["n_cells"], cyc
        faces = h.kelly_faces(3)
        es = np.asarray(kelly_from_face_pieces(sp, faces, ds["x"], 0), dtype=np.float32).astype(np.float64)
        ec = np.asarray(kelly_from_face_pieces(sp, faces, dc["x"], 0), dtype=np.float32).astype(np.float64)
        rs, cs, (ts, bs) = pd_refine_coarsen(es, 2, 0.3, 0.1, "number", 70000)
        rc, cc, (tc, bc) = pd_refine_coarsen(ec, 2, 0.3, 0.1, "number", 70000)
        lev = np.asarray(sp["cell_level"])
        for r_ in (rs, rc):
            r_[lev >= 5] = 0  # max refinement level
        flip_r, flip_c = np.nonzero(rs != rc)[0], np.nonzero(cs != cc)[0]
        if len(flip_r) or len(flip_c):
            d_eta = np.abs(es - ec)
            slack = 1e-6 * max(abs(tc), abs(bc), 1e-30)  # float32 indicators
            print("cycle %d: %d cells, %d refine / %d coarsen flags differ; max |eta_s - eta_c| %.3e (eta max %.3e), "
                  "refine threshold %.6e vs %.6e, coarsen threshold %.6e vs %.6e"
                  % (cyc, sp["n_cells"], len(flip_r), len(flip_c), d_eta.max(), ec.max(), ts, tc, bs, bc))
            for K in flip_r:
                assert abs(ec[K] - tc) <= d_eta[K] + abs(ts - tc) + slack, (cyc, K, ec[K], es[K], tc, ts)
            for K in flip_c:
                assert abs(ec[K] - bc) <= d_eta[K] + abs(bs - bc) + slack, (cyc, K, ec[K], es[K], bc, bs)
            first_diff = cyc
            break
        r, c = m.prepare(rc, cc)
        m.adapt(r, c)
    # the shipped run's third mesh differs from the reference's (4293 vs 4302 cells): the flags differ
    # at cycle 1 at the latest
    assert first_diff is not None and first_diff <= 1, first_diff
