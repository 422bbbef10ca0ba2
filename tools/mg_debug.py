"""Debug helper: linearity / magnitude of the multigrid preconditioner on a small steady problem
with the MMS-style forcing (not product code). Usage: python tools/mg_debug.py [n] [k] [direct]"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import softx_2020_200_amd as sx  # noqa: E402
from softx_2020_200_amd.io import Expr  # noqa: E402
from softx_2020_200_amd.problem import build_context, dirichlet_from_bcs  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4
k = int(sys.argv[2]) if len(sys.argv) > 2 else 1
direct = int(sys.argv[3]) if len(sys.argv) > 3 else 0
G = json.load(open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden",
                                "reference_goldens.json")))
F = Expr(G["mms3d_gls"]["force"], "x,y,z")


def level(m_):
    mesh = sx.hyper_cube(3, m_, k, k, -1.0, 1.0)
    mask, dd, dv = dirichlet_from_bcs(mesh, m_, -1.0, 1.0, False, [("noslip", 0, None)])
    xg = np.polynomial.legendre.leggauss(k + 1)[0] * 0.5 + 0.5
    Q = np.stack(np.meshgrid(xg, xg, xg, indexing="ij")[::-1], -1).reshape(-1, 3)
    X = (mesh["cell_x0"][:, None, :] + mesh["cell_h"][:, None, :] * Q[None]).reshape(-1, 3)
    fq = F(X)[:, :3].reshape(mesh["n_cells"], -1, 3)
    ctx = build_context(mesh, viscosity=1.0, vnode_mask=mask, force_q=fq)
    ctx.set_dirichlet(dd, dv)
    ctx.set_time("steady")
    return mesh, ctx


levels = []
m_ = n
while m_ >= 2:
    levels.append(level(m_))
    m_ //= 2
mesh, ctx = levels[0]
ctx.attach_multigrid([c for _, c in levels[1:]], pre_smooth=1, post_smooth=1, omega=0.9, coarse_sweeps=100,
                     coarse_omega=0.7, coarse_direct=direct)
N = ctx.n_dofs
u = torch.zeros(N, dtype=torch.float64, device="cuda")
ctx.set_state(u)
r = ctx.residual().clone()
rng = torch.Generator(device="cpu").manual_seed(1)
a = torch.rand(N, generator=rng, dtype=torch.float64).cuda()
b = torch.rand(N, generator=rng, dtype=torch.float64).cuda()
os.environ["GLS_MG_VERBOSE"] = "1"
za = ctx.apply_preconditioner(a).clone()
za2 = ctx.apply_preconditioner(a).clone()
zb = ctx.apply_preconditioner(b).clone()
zab = ctx.apply_preconditioner(a + b).clone()
zr = ctx.apply_preconditioner(r).clone()
nv = 3 * mesh["n_vnodes"]
print("n=%d k=%d direct=%d levels=%s" % (n, k, direct, [lv[0]["n_cells"] for lv in levels]))
print("repeat diff %.3e  linearity %.3e" % ((za - za2).abs().max().item(),
                                             (zab - za - zb).abs().max().item() / zab.abs().max().item()))
for name, z in (("a", za), ("r", zr)):
    print("%s: |z_u|max %.3e |z_p|max %.3e mean(z_p) %.3e" % (name, z[:nv].abs().max().item(), z[nv:].abs().max().item(),
                                                             z[nv:].mean().item()))
y = ctx.jacobian_apply(zr)
print("|J M r - r| / |r| = %.3e" % ((y - r).norm() / r.norm()).item())
x, its, res, ok = ctx.solve_linear(r, max_iterations=300, restart=30, relative_residual=1e-10, minimum_residual=1e-14)
print("gmres: its %d res %.3e ok %s" % (its, res, ok))
print("r: |r_u| %.3e |r_p| %.3e" % (r[:nv].abs().max().item(), r[nv:].abs().max().item()))
os.environ["GLS_GMRES_VERBOSE"] = "1"
x = torch.zeros(N, dtype=torch.float64, device="cuda")
st = ctx.newton(x, tolerance=1e-10, max_iterations=3, verbosity=1, lin_max_iterations=200, restart=30,
                relative_residual=1e-12, minimum_residual=1e-14)
print(st)
