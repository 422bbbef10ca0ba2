"""GPU: sum-factorised kernels on adapted leaves. On an adapted octree
(3D Q2-Q2, hanging nodes) the complete sibling groups of leaves run the pencil kernel (cached
linearization, element-vector output) and the other cells the per-cell kernel; the condensed J.v equals
the oracle's (1e-12) and the all-per-cell path's (GLS_OCT_BRICKS=0), the diagonal the per-cell one's, at
steady and BDF2 states. Parity pinned by the oracle (oracle/gls_oracle.c)."""
import numpy as np
import pytest

from oracle.oracle import Oracle
from gpu_util import context_for, cuda, relerr
from test_hanging import octree_problem


@pytest.mark.gpu
@pytest.mark.parametrize("scheme", ["steady", "bdf2"])
def test_forest_bricks_match_oracle_and_per_cell(monkeypatch, scheme):
    p, mesh = octree_problem(3, 2, 2, 2, 3, scheme=scheme)
    rng = np.random.default_rng(20200200)
    u, u1, u2, v = (rng.uniform(-1, 1, p.n_dofs) for _ in range(4))
    p.apply_nonzero_constraints(u)
    ref = Oracle(p).jacobian_apply(u, v, u1, u2)
    out = {}
    for flag in ("0", "1"):
        monkeypatch.setenv("GLS_OCT_BRICKS", flag)
        ctx = context_for(p)
        U, U1, U2, V = cuda(u), cuda(u1), cuda(u2), cuda(v)
        ctx.set_state(U, U1, U2)
        jv1 = ctx.jacobian_apply(V).cpu().numpy()  # linearization computed on demand
        d = ctx.jacobian_diagonal().cpu().numpy()  # per-cell + pencil diagonal (and the cache again)
        jv2 = ctx.jacobian_apply(V).cpu().numpy()
        out[flag] = (ctx.forest_bricks(), jv1, d, jv2)
    assert out["0"][0] == 0 and out["1"][0] > 0, (out["0"][0], out["1"][0])
    nb = out["1"][0]
    print("forest bricks: %d of %d cells" % (8 * nb, mesh["n_cells"]))
    for jv in (out["1"][1], out["1"][3]):
        assert relerr(jv, ref) < 1e-12, relerr(jv, ref)
        assert relerr(jv, out["0"][1]) < 1e-13
    assert relerr(out["1"][2], out["0"][2]) < 1e-13, relerr(out["1"][2], out["0"][2])
