"""Time the matrix-free J.v / residual / diagonal launches on the Q2 cavity (HIP events on the ctx stream)."""
import os, sys, time
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench
from softx_2020_200_amd.problem import CavityProblem

n = int(sys.argv[1]) if len(sys.argv) > 1 else 128
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
k = int(os.environ.get("GLS_K", "2"))
prob = CavityProblem(dim=3, n=n, k=k, viscosity=0.01)
ctx = prob.ctx
ctx.set_time("bdf2", (0.01,) * 4)
m1 = torch.from_numpy(bench.smooth_state(prob.mesh, n, 3, prob.dir_dofs, prob.dir_vals, 0.0)).cuda()
m2 = torch.from_numpy(bench.smooth_state(prob.mesh, n, 3, prob.dir_dofs, prob.dir_vals, 0.3)).cuda()
ctx.set_state(m1, m1, m2)
v = torch.rand(ctx.n_dofs, dtype=torch.float64, device="cuda")
y = torch.empty_like(v)
ctx.timing(True)
ctx.jacobian_apply(v, y); ctx.residual(y); torch.cuda.synchronize()
ms_l, n_l = ctx.timing_get(3)
ctx.timing(True)
for _ in range(reps):
    ctx.jacobian_apply(v, y)
for _ in range(reps // 4 + 1):
    ctx.residual(y)
d_out = torch.empty_like(v)
ctx.jacobian_diagonal(out=d_out)  # k_copy of n_dofs doubles: PMC byte calibration (tools/pmc_traffic.sh)
if ctx.uses_brick_kernels and not os.environ.get("GLS_JV_RECOMPUTE"):  # FP32 smoother J.v (slot 4; cached path only)
    for _ in range(reps):
        ctx.jacobian_apply_f32(v, y)
ms_jv, n_jv = ctx.timing_get(1)
ms_f, n_f = ctx.timing_get(4)
ms_s, n_s = ctx.timing_get(5)
ms_r, n_r = ctx.timing_get(0)
ms_d, n_d = ctx.timing_get(2)
print("n=%d k=%d brick=%s  J.v %.3f ms  J.v(f32) %.3f ms  slab sum %.3f ms  residual %.3f ms  diag %.3f ms  "
      "linearize %.3f ms (cells %d, dofs %d)" % (n, k, ctx.uses_brick_kernels, ms_jv / n_jv, ms_f / max(n_f, 1),
                                                 ms_s / max(n_s, 1), ms_r / n_r, ms_d / max(n_d, 1),
                                                 ms_l / max(n_l, 1), prob.mesh["n_cells"], ctx.n_dofs))
