"""Generate tests/golden/gls_vectors.npz: per-DoF GLS residual and J.v golden vectors.

Made by the CPU oracle (oracle/gls_oracle.c, restating gls_navier_stokes.cc:230-777), itself pinned
end to end against the reference's goldens (tests/test_oracle_goldens.py); the reference holds no
per-DoF vectors, so these freeze the oracle's pinned output as data. Cavity meshes on
hyper_cube(-1, 1, colorize=true): walls noslip, lid (id 3) u = (1, 0[, 0]); Q1-Q1 2D 4x4, Q1-Q1 3D 2^3,
Q2-Q2 3D 2^3; inputs u, u_m1, u_m2, v ~ U(-1, 1) from numpy default_rng(20200200) (stored);
schemes steady / bdf1 / bdf2 / sdirk2_1, nu in {1, 0.01}, dt = 0.01. Every DoF is keyed by its support
point and component (dof_x, dof_c), so a product with another DoF numbering can be compared.

    python tests/golden/make_vectors.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle.oracle import Oracle, StructuredProblem  # noqa: E402

MESHES = {"2d_q1_4": (2, 4, 1), "3d_q1_2": (3, 2, 1), "3d_q2_2": (3, 2, 2)}
SCHEMES = ["steady", "bdf1", "bdf2", "sdirk2_1"]
NUS = [1.0, 0.01]
DT = (0.01, 0.01, 0.01, 0.01)
SEED = 20200200


def cavity(dim, n, k, nu, scheme):
    p = StructuredProblem(dim, n, k=k, kp=k, colorize=True, viscosity=nu, scheme=scheme, time_steps=DT)
    lid = lambda X: np.tile([1.0] + [0.0] * (dim - 1), (X.shape[0], 1))
    p.set_dirichlet([("noslip", b, None) for b in range(2 * dim) if b != 3] + [("function", 3, lid)])
    return p


def main():
    out = {}
    for name, (dim, n, k) in MESHES.items():
        p0 = cavity(dim, n, k, 1.0, "steady")
        X = p0.vnode_coords()
        nv = p0.n_vnodes
        out[name + "/dof_x"] = np.concatenate([np.repeat(X, dim, axis=0), X])
        out[name + "/dof_c"] = np.concatenate([np.tile(np.arange(dim), nv), np.full(nv, dim)]).astype(np.int32)
        rng = np.random.default_rng(SEED)
        u, u1, u2, v = (rng.uniform(-1, 1, p0.n_dofs) for _ in range(4))
        for key, a in (("u", u), ("u_m1", u1), ("u_m2", u2), ("v", v)):
            out[f"{name}/{key}"] = a
        for scheme in SCHEMES:
            for nu in NUS:
                orc = Oracle(cavity(dim, n, k, nu, scheme))
                tag = f"{name}/{scheme}/nu{nu:g}"
                out[tag + "/residual"] = orc.residual(u, u1, u2)
                out[tag + "/jv"] = orc.jacobian_apply(u, v, u1, u2)
    np.savez_compressed(os.path.join(os.path.dirname(os.path.abspath(__file__)), "gls_vectors.npz"), **out)
    print("wrote %d arrays" % len(out))


if __name__ == "__main__":
    main()
