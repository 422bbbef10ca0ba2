"""BASELINE configs[0]: the reference's examples/01-cavity (2D lid-driven cavity, Q1-Q1, hyper_cube
refined 6 times = 64 x 64 cells, nu = 1, steady, two uniform mesh adaptations, Newton tol 1e-8, ILU(1)
GMRES rel 1e-9), committed as tests/golden/app_cases/example-01-cavity.prm.

CPU (the reference's CPU path, restated by the oracle): the exact-solve Newton (oracle newton_solve)
and the CPU baseline's Newton iteration (gls_oracle_newton_csr: CSR assembly, ILU(0), GMRES(30), line
search -- solve_system_GMRES) converge on the 64 x 64 cavity to the same discrete solution.

GPU: the drop-in application runs the shipped prm unchanged (--dump writes every solve's state); on each
of its three meshes (64^2, 128^2, 256^2) the oracle's GLS residual at the app's solution is below the
prm's Newton tolerance, and on 64^2 the app's velocity equals the oracle's exact-Newton solution."""
import os
import subprocess

import numpy as np
import pytest

from oracle.oracle import Oracle, StructuredProblem, newton_csr, newton_solve

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PRM = os.path.join(ROOT, "tests", "golden", "app_cases", "example-01-cavity.prm")


def cavity(n):
    """examples/01-cavity/cavity.prm: hyper_cube -1 : 1 : colorize, bc 0..2 noslip, bc 3 (y = 1) u = (1, 0)"""
    p = StructuredProblem(2, n, k=1, kp=1, viscosity=1.0, scheme="steady", colorize=True)
    p.set_dirichlet([("noslip", 0, None), ("noslip", 1, None), ("noslip", 2, None),
                     ("function", 3, lambda X: np.stack([np.ones(len(X)), 0 * X[:, 0]], 1))])
    return p


_EXACT = {}


def exact_solution(n):
    if n not in _EXACT:
        p = cavity(n)
        x, its, res = newton_solve(p, tol=1e-12, max_it=20)
        assert res < 1e-12, res
        _EXACT[n] = (p, x)
    return _EXACT[n]


def test_configs0_cpu_newton_paths_agree():
    p, x_ref = exact_solution(64)
    x = p.apply_nonzero_constraints(np.zeros(p.n_dofs))
    hist = []
    for _ in range(10):  # complete Newton iterations of the CPU baseline's path until converged
        st = newton_csr(p, x, threads=min(8, os.cpu_count() or 1), rel=1e-12, minres=1e-16)
        hist.append(st["res1"])
        if st["res1"] < 1e-10:
            break
    assert hist[-1] < 1e-10, hist
    nv = 2 * p.n_vnodes  # enclosed flow: the pressure is determined up to a constant
    assert np.abs(x[:nv] - x_ref[:nv]).max() < 1e-8
    r = Oracle(p).residual(x)
    assert np.linalg.norm(r) < 1e-8


@pytest.mark.gpu
def test_configs0_example_cavity_through_the_app(tmp_path):
    from tests.test_gpu_app_configs import read_dumps
    dump = tmp_path / "dump"
    dump.mkdir()
    app = os.path.join(ROOT, "apps", "gls_navier_stokes_2d")
    if not os.path.exists(app):
        pytest.fail("apps/gls_navier_stokes_2d is not built (run __graft_entry__.build())")
    (tmp_path / "cavity.prm").write_text(open(PRM).read())
    out = subprocess.run([app, "--dump", str(dump), "cavity.prm"], cwd=str(tmp_path), capture_output=True,
                         text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-3000:]
    assert "linear solver: method = gmres" in out.stderr, out.stderr[-2000:]
    dumps = read_dumps(str(dump))
    assert [int(d["n_dofs"]) for d in dumps] == [3 * (n + 1) ** 2 for n in (64, 128, 256)], out.stdout[-2000:]
    for d, n in zip(dumps, (64, 128, 256)):
        p = cavity(n)
        r = Oracle(p).residual(d["x"])
        assert np.linalg.norm(r) < 1e-8, (n, np.linalg.norm(r))
        bc = p.apply_nonzero_constraints(d["x"].copy())
        assert np.array_equal(bc, d["x"])  # the prm's boundary values are applied exactly
    p, x_ref = exact_solution(64)
    nv = 2 * p.n_vnodes
    assert np.abs(dumps[0]["x"][:nv] - x_ref[:nv]).max() < 1e-7
