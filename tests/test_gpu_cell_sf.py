"""The sum-factorized per-cell J.v (softx_2020_200_amd/csrc/gls_cell_sf.hip: 3D Q2-Q1 and Q2-Q2 cells, the
default for every per-cell J.v from the linearization cache) against the dense per-cell kernel (GLS_CELL_SF=0,
read per launch), the MFMA variant of the dense contractions (GLS_CELL_SF=2, v_mfma_f64_16x16x4f64) and the oracle's assembled, constraint-eliminated operator (gls_navier_stokes.cc:548-622):
MappingQ2 curved cells (cylinder shell, cylinder, unstructured gmsh), adapted meshes with hanging lines,
axis-aligned boxes on the per-cell path, transient and steady schemes, SRF. FP64 throughout: 1e-12 against
the oracle, 1e-13 between the two kernels (same per-point arithmetic, different summation order)."""
import os

import numpy as np
import pytest

from oracle.oracle import MappedProblem, Oracle, StructuredProblem
from softx_2020_200_amd.native import UMesh
from tests.gpu_util import context_for, cuda, relerr
from tests.test_gpu_uforest import adapted_space, dof_lines
from tests.test_uforest import CASES

MESHES = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "meshes")


def _mapped(kind):
    if kind == "cshell":
        return UMesh(3, "cylinder_shell", "0.5 : 0.25 : 1 : 8 : 2")
    if kind == "cylinder":
        m = UMesh(3, "cylinder", "1 : 1")
        m.refine_global(1)
        return m
    return UMesh(3, gmsh=os.path.join(MESHES, "cylinder_unstructured.msh"))


def _check(monkeypatch, p, ctx, seed=20200200):
    rng = np.random.default_rng(seed)
    u, u1, u2, v = (rng.uniform(-1, 1, p.n_dofs) for _ in range(4))
    if getattr(p, "hang_lines", None) is not None:
        p.apply_nonzero_constraints(u)
    ctx.set_state(cuda(u), cuda(u1), cuda(u2))
    V = cuda(v)
    sf = ctx.jacobian_apply(V).cpu().numpy()
    assert np.array_equal(ctx.jacobian_apply(V).cpu().numpy(), sf)  # fixed-order sums: bitwise repeatable
    monkeypatch.setenv("GLS_CELL_SF", "0")
    dense = ctx.jacobian_apply(V).cpu().numpy()
    monkeypatch.setenv("GLS_CELL_SF", "2")  # the MFMA contractions (A/B variant)
    mfma = ctx.jacobian_apply(V).cpu().numpy()
    monkeypatch.delenv("GLS_CELL_SF")
    ref = Oracle(p).jacobian_apply(u, v, u1, u2)
    e_d, e_o, e_m = relerr(sf, dense), relerr(sf, ref), relerr(mfma, ref)
    print("sum-factorized J.v vs dense %.2e, vs oracle %.2e; MFMA J.v vs oracle %.2e" % (e_d, e_o, e_m))
    assert e_d < 1e-13 and e_o < 1e-12 and e_m < 1e-12, (e_d, e_o, e_m)


MAPPED = [("cshell", 1, "bdf2", False), ("cshell", 2, "steady", True), ("cylinder", 1, "bdf1", True),
          ("cylinder", 2, "bdf2", False), ("cylu", 1, "steady", False)]


@pytest.mark.gpu
@pytest.mark.parametrize("kind,kp,scheme,srf", MAPPED, ids=["%s_Q2Q%d_%s%s" % (c[0], c[1], c[2], "_srf" if c[3] else "")
                                                           for c in MAPPED])
def test_sum_factorized_jv_mapped(monkeypatch, kind, kp, scheme, srf):
    sp = _mapped(kind).fe_space(2, kp, qmapping_all=True)
    p = MappedProblem(sp, viscosity=0.02, scheme=scheme, time_steps=(0.01, 0.012, 0.011, 0.01), srf=srf,
                      omega=(0.3, -0.2, 1.1))
    p.set_dirichlet([("noslip", 0, None)])
    _check(monkeypatch, p, context_for(p))


@pytest.mark.gpu
@pytest.mark.parametrize("name,spec", [(c[0], c[2]) for c in CASES if c[1] == 3], ids=[c[0] for c in CASES if c[1] == 3])
@pytest.mark.parametrize("kp,scheme", [(1, "steady"), (2, "bdf2")])
def test_sum_factorized_jv_adapted_hanging(monkeypatch, name, spec, kp, scheme):
    _, h = adapted_space(name, 3, spec, 2, kp)
    sp = h.data
    p = MappedProblem(sp, viscosity=0.05, scheme=scheme, time_steps=(0.01, 0.012, 0.011, 0.01))
    lines = dof_lines(sp)
    p.set_hanging(*lines)
    p.hang_lines = lines
    p.set_dirichlet([("noslip", 0, None)])
    _check(monkeypatch, p, context_for(p))


@pytest.mark.gpu
@pytest.mark.parametrize("kp,scheme", [(1, "bdf2"), (2, "steady")])
def test_sum_factorized_jv_boxes(monkeypatch, kp, scheme):
    """axis-aligned cells on the per-cell path (the brick kernels off): the box instantiation"""
    p = StructuredProblem(3, 3, k=2, kp=kp, viscosity=0.01, scheme=scheme, time_steps=(0.01, 0.012, 0.01, 0.01))
    p.set_dirichlet([("noslip", 0, None)])
    monkeypatch.setenv("GLS_DISABLE_BRICK", "1")
    ctx = context_for(p)
    monkeypatch.delenv("GLS_DISABLE_BRICK")
    assert not ctx.uses_brick_kernels
    _check(monkeypatch, p, ctx)
