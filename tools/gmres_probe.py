import sys, os, time, torch, numpy as np
sys.path.insert(0, os.getcwd())
os.environ["GLS_GMRES_VERBOSE"] = "1"
import bench
from softx_2020_200_amd.problem import CavityProblem
n = int(sys.argv[1]); restart = int(sys.argv[2])
prob = CavityProblem(dim=3, n=n, k=2, viscosity=0.01)
ctx = prob.ctx
ctx.set_time("bdf2", (0.01,)*4)
m1 = torch.from_numpy(bench.smooth_state(prob.mesh, n, 3, prob.dir_dofs, prob.dir_vals, 0.0)).cuda()
m2 = torch.from_numpy(bench.smooth_state(prob.mesh, n, 3, prob.dir_dofs, prob.dir_vals, 0.3)).cuda()
x = m1.clone()
t = time.time()
st = ctx.newton(x, m1, m2, tolerance=1e-30, max_iterations=2, lin_max_iterations=600, restart=restart, relative_residual=1e-4, minimum_residual=1e-14, verbosity=1)
print(st, time.time() - t, flush=True)
