"""The adaptive BASELINE configurations through the drop-in application, checked step by step
against the oracle (the app runs with --dump: every iteration's final state -- scheme, time steps,
mesh size, present solution and time history -- is written for the test to read):

  * configs[3] (examples/02-taylor-couette in 3D: cylinder_shell, Q2-Q1, MappingQ2 on all cells,
    slip end caps, steady, Kelly adaptation with hanging-node constraints): the shipped
    apps/cases/taylor-couette3d_q2q1_kelly.prm, two Kelly cycles;
  * configs[4] (examples/03-cylinder in 3D: Re 200 flow past the extruded gmsh cylinder, Q2-Q1,
    BDF2, slip walls, Kelly every 2nd step with the solution history transferred to the adapted
    general mesh): apps/cases/cylinder3d_q2q1_re200_kelly.prm on a 1-layer extrusion of the
    reference's cylinder_structured.msh (tests/golden/meshes/cylinder3d_1layer.msh, made by
    tools/extrude_gmsh.py), three time steps.

Each runs on one rank and across ranks (--np: the reference's mpirun, every rank's context on its
cells of the partitioned forest, row e2; on one GPU the ranks exchange through host shared memory);
the dumps are the gathered global state. For every iteration of the app:
  1. the oracle's GLS residual (gls_oracle.c restating assembleGLS, hanging lines condensed,
     nonzero constraints from the prm's boundary conditions) at the app's solution, with the app's
     scheme, time steps and history, is below the Newton tolerance: the app solved the reference's
     discrete equations on that mesh;
  2. the next mesh follows from the oracle-side Kelly indicator of that solution
     (kelly_from_face_pieces), the oracle's p::d fixed-number marking (pd_refine_coarsen), the
     level rules and the triangulation's smoothing / adaptation: cell counts exactly;
  3. (configs[3]) the printed L2 errors equal the oracle's L2 errors of the app's solution;
     (configs[4]) the history the app solved with after the adaptation equals the SolutionTransfer
     of the previous step's state.
The oracle's own Newton (sparse direct solves) is not run here: at 20-70 k DoFs of 3D Q2-Q1 it takes
minutes per solve on one core; the residual check pins the same solution."""
import os
import re
import shutil
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CASES = os.path.join(ROOT, "apps", "cases")
MESHES = os.path.join(ROOT, "tests", "golden", "meshes")


def read_dumps(d):
    out = []
    for f in sorted(x for x in os.listdir(d) if x.endswith(".meta")):
        meta = {}
        for line in open(os.path.join(d, f)):
            k, *v = line.split()
            meta[k] = [float(x) for x in v] if k == "time_steps" else float(v[0])
        n = int(meta["n_dofs"])
        raw = np.fromfile(os.path.join(d, f[:-5] + ".bin"), dtype=np.float64)
        assert raw.size == 4 * n, (f, raw.size, n)
        meta["x"], meta["m1"], meta["m2"], meta["m3"] = raw.reshape(4, n)
        out.append(meta)
    return out


def run_app(tmp_path, prm_text, files=(), extra=()):
    for f in files:
        shutil.copy(f, tmp_path / os.path.basename(f))
    (tmp_path / "case.prm").write_text(prm_text)
    dump = tmp_path / "dump"
    dump.mkdir()
    app = os.path.join(ROOT, "apps", "gls_navier_stokes_3d")
    if not os.path.exists(app):
        pytest.fail("apps/gls_navier_stokes_3d is not built (run __graft_entry__.build())")
    fo, fe = tmp_path / "stdout.txt", tmp_path / "stderr.txt"
    with open(fo, "w") as o, open(fe, "w") as e:
        try:  # the app line-buffers stdout: a run cut off at the limit still shows how far it got
            r = subprocess.run([app, "--stats", *extra, "--dump", str(dump), "case.prm"], cwd=str(tmp_path), stdout=o,
                               stderr=e, timeout=float(os.environ.get("GLS_APP_TIMEOUT", "170")))
        except subprocess.TimeoutExpired:
            pytest.fail("app timed out; stdout tail:\n%s\nstderr tail:\n%s" % (fo.read_text()[-3000:], fe.read_text()[-2000:]))
    assert r.returncode == 0, fe.read_text()[-3000:] + "\nstdout tail:\n" + fo.read_text()[-2000:]
    return fo.read_text(), read_dumps(str(dump))


def setprm(text, key, value):
    new, n = re.subn(r"(set %s\s*=\s*)[^\n#]*" % re.escape(key), r"\g<1>%s" % value, text)
    assert n >= 1, key
    return new


def mark(sp, eta, frac_r, frac_c, max_level, min_level=0):
    """refine_mesh_kelly's marking (navier_stokes_base.cc:654-680): p::d fixed number on the float
    indicator, then the max / min level rules"""
    from oracle.oracle import pd_refine_coarsen
    r, c, _ = pd_refine_coarsen(eta.astype(np.float32), 3, frac_r, frac_c, "number")
    counts = (int(r.sum()), int(c.sum()))  # the app's "kelly: ..." line counts before the level rules
    lev = np.asarray(sp["cell_level"])
    if lev.max() + 1 > max_level:
        r[lev >= max_level] = 0
    c[lev == min_level] = 0
    return r.astype(np.int32), c.astype(np.int32), counts


def problem(sp, nu, bcs, scheme="steady", ts=(1.0,) * 4):
    from oracle.oracle import MappedProblem
    from tests.test_gpu_uforest import dof_lines
    p = MappedProblem(sp, viscosity=nu, scheme=scheme, time_steps=tuple(ts))
    lines = dof_lines(sp)
    if len(lines[0]):
        p.set_hanging(*lines)
    p.set_dirichlet(bcs)
    return p


SCHEME_NAMES = {0: "steady", 1: "bdf1", 2: "bdf2", 3: "bdf3"}


@pytest.mark.gpu
@pytest.mark.parametrize("np_ranks", [1, 4])
def test_configs3_taylor_couette3d_kelly_pipeline(tmp_path, np_ranks):
    prm = open(os.path.join(CASES, "taylor-couette3d_q2q1_kelly.prm")).read()
    tol = 1e-8
    out, dumps = run_app(tmp_path, prm, extra=("--precision", "9", "--np", str(np_ranks)))
    assert "Running on %d MPI rank(s)" % np_ranks in out
    check_configs3_pipeline(out, dumps, tol)


def check_configs3_pipeline(out, dumps, tol):
    """every cycle's dump: the oracle's residual at it <= tol on the oracle's own copy of the mesh, the
    printed error = the oracle's, the Kelly marking = the oracle's (then the oracle adapts its copy)"""
    from oracle.oracle import Oracle, kelly_from_face_pieces
    from softx_2020_200_amd.native import UMesh
    assert len(dumps) == 3, out
    rows = [l.split() for l in out.splitlines() if re.match(r"^\s*\d+\s+\d\.\d+e[-+]\d+", l)]
    m = UMesh(3, "cylinder_shell", "1 : 0.25 : 1 : 8 : 2")
    m.refine_global(1)
    eta_, ri = 0.25, 0.25

    def exact(X):
        r = np.sqrt(X[:, 0] ** 2 + X[:, 1] ** 2)
        ut = -(eta_ ** 2) / (1 - eta_ ** 2) * r + ri ** 2 / (1 - eta_ ** 2) / r
        th = np.arctan2(X[:, 1], X[:, 0])
        return np.stack([-np.sin(th) * ut, np.cos(th) * ut, 0 * r, 0 * r], 1)

    bcs = [("function", 0, lambda X: np.stack([-X[:, 1], X[:, 0], 0 * X[:, 0]], 1)), ("noslip", 1, None),
           ("slip", 2, None), ("slip", 3, None)]
    for cyc, d in enumerate(dumps):
        h = m.fe_space_handle(2, 1, qmapping_all=True)
        sp = h.data
        assert int(d["n_cells"]) == sp["n_cells"] and int(d["n_dofs"]) == 3 * sp["n_vnodes"] + sp["n_pnodes"], cyc
        p = problem(sp, 1.0, bcs)
        orc = Oracle(p)
        res = np.linalg.norm(orc.residual(d["x"]))
        assert res <= 1.01 * tol, (cyc, res)
        eu, ep = orc.l2_error(d["x"], exact)
        assert int(rows[cyc][0]) == sp["n_cells"], (rows, cyc)
        assert abs(float(rows[cyc][1]) - eu) <= 1e-7 * eu, (cyc, rows[cyc], eu)
        if cyc + 1 < len(dumps):
            eta = kelly_from_face_pieces(sp, h.kelly_faces(4), d["x"], 0)
            r0, c0, (nr, ncs) = mark(sp, eta, 0.3, 0.0, 4)
            r, c = m.prepare(r0, c0)
            assert "kelly: %d of %d cells flagged for refinement, %d for coarsening (after smoothing: %d, %d)" % (
                nr, sp["n_cells"], ncs, r.sum(), c.sum()) in out, (cyc, out)
            m.adapt(r, c)


@pytest.mark.gpu
@pytest.mark.parametrize("np_ranks,precond", [(1, None), (2, None), (1, "hmg")])
def test_configs4_cylinder3d_re200_bdf2_kelly_pipeline(tmp_path, np_ranks, precond):
    """precond hmg: the hierarchy multigrid with the Q1-Q1 p-level on the base mesh (dense LU) below it -- on the
    first (unadapted) mesh the whole hierarchy is that p-level pair"""
    from oracle.oracle import Oracle, kelly_from_face_pieces
    from softx_2020_200_amd.native import UMesh
    prm = open(os.path.join(CASES, "cylinder3d_q2q1_re200_kelly.prm")).read()
    prm = setprm(prm, "file name", "cylinder3d_1layer.msh")
    prm = setprm(prm, "time end", "0.15")
    tol = 1e-8
    prm = setprm(prm, "tolerance", "%g" % tol)
    prm = setprm(prm, "relative residual", "1e-10")
    prm = setprm(prm, "minimum residual", "1e-13")
    out, dumps = run_app(tmp_path, prm, [os.path.join(MESHES, "cylinder3d_1layer.msh")],
                         extra=("--np", str(np_ranks)) + (("--precond", precond) if precond else ()))
    assert len(dumps) == 3, out
    if precond == "hmg":
        err = (tmp_path / "stderr.txt").read_text()
        assert "Q1-Q1 p-level on the base mesh, dense LU" in err, err[-1500:]
    assert "Running on %d MPI rank(s)" % np_ranks in out
    nu = 0.005
    m = UMesh(3, gmsh=os.path.join(MESHES, "cylinder3d_1layer.msh"))
    inlet = lambda X: np.stack([np.ones(len(X)), 0 * X[:, 0], 0 * X[:, 0]], 1)
    bcs = [("noslip", 0, None), ("function", 1, inlet), ("slip", 2, None), ("slip", 4, None), ("slip", 5, None)]
    h_prev, prev = None, None
    adapted = 0
    for it, d in enumerate(dumps, start=1):
        if it > 1 and it % 2 == 0:  # Kelly on the previous step's solution, then the history transfer
            sp_old = h_prev.data
            eta = kelly_from_face_pieces(sp_old, h_prev.kelly_faces(4), prev["x"], 0)
            r, c, (nr, ncs) = mark(sp_old, eta, 0.1, 0.05, 2)
            r, c = m.prepare(r, c)
            assert "kelly: %d of %d cells flagged for refinement, %d for coarsening (after smoothing: %d, %d)" % (
                nr, sp_old["n_cells"], ncs, r.sum(), c.sum()) in out, (it, out)
            m.adapt(r, c)
            h = m.fe_space_handle(2, 1)
            adapted += 1
            # the app solved step `it` with m1 = previous present, m2 = previous m1 (transferred)
            for key, src in (("m1", "x"), ("m2", "m1")):
                ref = h.transfer_from(h_prev, prev[src])
                assert np.abs(d[key] - ref).max() <= 1e-12 * max(np.abs(ref).max(), 1.0), (it, key)
        else:
            h = h_prev if h_prev is not None else m.fe_space_handle(2, 1)
        sp = h.data
        assert int(d["n_cells"]) == sp["n_cells"] and int(d["n_dofs"]) == 3 * sp["n_vnodes"] + sp["n_pnodes"], it
        scheme = SCHEME_NAMES[int(d["scheme"])]
        p = problem(sp, nu, bcs, scheme, d["time_steps"])
        res = np.linalg.norm(Oracle(p).residual(d["x"], d["m1"], d["m2"], d["m3"]))
        assert res <= 1.01 * tol, (it, scheme, res)
        h_prev, prev = h, d
    assert adapted == 1 and dumps[1]["n_cells"] > dumps[0]["n_cells"], [x["n_cells"] for x in dumps]


@pytest.mark.gpu
def test_configs3_taylor_couette3d_kelly_hierarchy_multigrid(tmp_path):
    """configs[3]'s adaptive pipeline with the geometric multigrid on the triangulation's refinement
    hierarchy as the GMRES preconditioner (--precond hmg: gls_umesh_coarsen_to levels, gls_fe_space_mg_transfer,
    gls_mg_attach_transfers; MappingQ2 per-cell kernels on every level, hanging and slip lines) instead of the
    reference's ILU: the same oracle checks as the ILU pipeline above (converged residual at every cycle's
    state, error table, Kelly marking), the preconditioner announced on stderr, the GMRES iteration totals
    of both runs printed (the two runs' meshes may differ from the third cycle on: the marking of cells at
    the refinement threshold depends on the inexact solves, as with the shipped cylinder_gls settings)."""
    prm = open(os.path.join(CASES, "taylor-couette3d_q2q1_kelly.prm")).read()
    its = {}
    # the prm's method = amg runs the hierarchy multigrid by default (the ML hierarchy substituted);
    # --precond ilu forces the ILU that ML would smooth with, for the comparison
    for pc in ("ilu", "mg", "hmg"):
        d = tmp_path / pc
        d.mkdir()
        out, dumps = run_app(d, prm, extra=("--precision", "9", "--precond", pc))
        err = (d / "stderr.txt").read_text()
        if pc == "ilu":
            assert "refinement hierarchy" not in err
        else:
            assert "triangulation's refinement hierarchy" in err and "ML AMG substituted" in err, err[-1500:]
            check_configs3_pipeline(out, dumps, 1e-8)
        its[pc] = [l for l in out.splitlines() if "linear_iterations =" in l]
    print("configs[3] GMRES totals: ILU %s, amg -> hierarchy GMG %s, --precond hmg %s" % (its["ilu"], its["mg"], its["hmg"]))


@pytest.mark.gpu
def test_configs3_hierarchy_multigrid_across_ranks(tmp_path):
    """configs[3] at --np 4 with --precond hmg: the fine level partitioned over the ranks, the coarser levels of
    the triangulation's hierarchy replicated on every rank (gls_mg_attach_replica; the exact LU on the coarsest
    when the replica is the only coarser level), the same oracle checks as the one-rank pipeline. The GMRES
    totals of the 4-rank run stay within 2x of the one-rank run's (the fine level's ILU(0) smoother becomes one
    block per rank, as the reference's Ifpack additive Schwarz)."""
    prm = open(os.path.join(CASES, "taylor-couette3d_q2q1_kelly.prm")).read()
    its = {}
    for npr in (1, 4):
        d = tmp_path / ("np%d" % npr)
        d.mkdir()
        out, dumps = run_app(d, prm, extra=("--precision", "9", "--precond", "hmg", "--np", str(npr), "--stats"))
        err = (d / "stderr.txt").read_text()
        assert "Running on %d MPI rank(s)" % npr in out
        assert "triangulation's refinement hierarchy" in err, err[-1500:]
        check_configs3_pipeline(out, dumps, 1e-8)
        its[npr] = [int(x) for x in re.findall(r"linear_iterations = (\d+)", out)]
    print("configs[3] hmg GMRES totals: 1 rank %s, 4 ranks %s" % (its[1], its[4]))
    assert its[1] and its[4] and sum(its[4]) <= 2 * sum(its[1]) + 10, its
