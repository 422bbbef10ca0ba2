"""ILU attach diagnostics on a periodic 2D Q2-Q1 problem (the TGV setting): nnz, probes, CSR checksum,
and the GMRES iterations of one ILU-preconditioned solve. Run with PYTHONPATH selecting the library tree."""
import sys

import numpy as np

from oracle.oracle import StructuredProblem
from tests.gpu_util import context_for, cuda
import softx_2020_200_amd.native as nat

print("lib", nat.LIB_PATH)
for n, per in ((8, 3), (16, 3), (16, 0)):
    p = StructuredProblem(2, n, k=2, kp=1, viscosity=0.01, scheme="sdirk2_1", time_steps=(0.1,) * 4,
                          periodic=(0, 1)) if per else StructuredProblem(2, n, k=2, kp=1, viscosity=0.01, scheme="sdirk2_1", time_steps=(0.1,) * 4)
    if not per:
        p.set_dirichlet([("noslip", 0, None)])
    rng = np.random.default_rng(1)
    u = rng.uniform(-1, 1, p.n_dofs)
    ctx = context_for(p)
    ctx.set_state(cuda(u), cuda(u))
    nnz, npr = ctx.attach_ilu(1e-5, 1.0)
    M = ctx.ilu_matrix().tocsr()
    rhs = ctx.residual()
    x, its, res, ok = ctx.solve_linear(rhs, None, max_iterations=2000, restart=100, relative_residual=1e-8)
    print(n, per, "nnz", nnz, "probes", npr, "sum|M|", float(np.abs(M.data).sum()), "its", its, ok)
