"""Back-to-back per-cell J.v launches on configs[3]'s mapped Q2-Q1 problem (tooling: the PMC / timing driver of the
per-cell kernels; GLS_CELL_SF selects the kernel: 1 sweeps, 0 dense VALU, 2 MFMA).
Usage: python tools/cell_jv_bench.py [refine=3] [reps=20]   (refine 3: 1.72 M DoFs, 65,536 cells)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    import bench
    r = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    m = bench.taylorcouette3d_mesh(r + 1)
    ctx, sp, x = bench.taylorcouette3d_context(m.fe_space(2, 1, qmapping_all=True))
    ctx.set_time("steady", (0.0,) * 4)
    dev = torch.device("cuda", 0)
    u = torch.from_numpy(x).to(dev)
    ctx.set_state(u)
    v = torch.rand(ctx.n_dofs, dtype=torch.float64, device=dev)
    y = torch.empty_like(v)
    ctx.jacobian_apply(v, y)  # the diagonal pass fills the linearization cache
    torch.cuda.synchronize()
    ctx.timing(True)
    for _ in range(reps):
        ctx.jacobian_apply(v, y)
    ms, n = ctx.timing_get(1)
    ctx.timing(False)
    print("GLS_CELL_SF=%s n_dofs %d cells %d: J.v %.4f ms per launch (%d launches)" % (
        os.environ.get("GLS_CELL_SF", "1"), ctx.n_dofs, sp["n_cells"], ms / max(n, 1), n))


if __name__ == "__main__":
    main()
