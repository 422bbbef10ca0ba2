"""bench.py — nonlinear (Newton) iterations/s of the GLS Navier–Stokes hot path on MI355X.

Workload (BASELINE.json configs[2], the metric's config): 3D lid-driven cavity, Q2-Q2,
128^3 cells (67,898,372 DoFs), transient BDF2, nu = 0.01, dt = 0.01.
One "step" = one Newton iteration of NewtonNonLinearSolver::solve
(include/core/newton_non_linear_solver.h:90-137): evaluation_point = present; residual + Jacobian
diagonal (matrix-free "assemble_matrix_and_rhs"); GMRES(30) on the matrix-free Jacobian, right
preconditioned by a geometric-multigrid V-cycle (levels 64^3..2^3, FP32 damped-Jacobi smoothing,
2+2 sweeps on the 4^3 level, exact LU solve of the 2^3 level's 500 DoFs; Jacobi with --precond
jacobi; on N GPUs the levels down to 4^3 are partitioned like the fine mesh and every rank runs the
rest of the same cycle -- 4^3 sweeps, LU on 2^3 -- on a replica of the 4^3 level from the all-reduced
right-hand side), relative residual 1e-4, max `--lin-max` iterations; alpha line search with
residual re-assembly. Every step restarts from the same synthetic state so the work per step is
fixed; linear iterations and residual evaluations are reported.

Launch: python bench.py [--gpus N --steps K --warmup W]. For N > 1 either under torch.distributed.run
(WORLD_SIZE must equal --gpus, else exit 1) or directly: without WORLD_SIZE the process starts N fresh
rank processes itself (before anything touches the GPU; RANK / LOCAL_RANK / WORLD_SIZE / MASTER_*
127.0.0.1), waits for them, exits non-zero if one fails and re-prints rank 0's JSON line.
Multi-GPU (N>1): the 128^3 mesh is partitioned into contiguous Morton brick ranges (one per GPU,
p4est-like); ghost import / export-add and the GMRES dot products go over the library's own RCCL
communicator (gls_dist_attach_rccl; the ghost import of the J.v overlaps the interior bricks on a
second stream; --dist-impl torch: torch.distributed callbacks instead). Before the warm-up a pre-flight
checks the N-rank residual and J.v of a 16^3 cavity (same transport) against a single-rank context on
rank 0 (abort above 1e-12; `preflight_relerr`). Fixed total problem -> "scaling": "strong"; value =
nonlinear iterations/s of the whole job; `rccl_ranks` = the in-library communicator's size as RCCL
reports it, `devices` = distinct GPUs behind the ranks.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0       # MI355X_MICROARCH.md chip table (spec)


def cell_jv_kernel_name(kp):
    """the per-cell J.v kernel a 3D Q2 cell runs (gls_cell_sf.hip: GLS_CELL_SF, read per launch, 1 by default)"""
    mode = os.environ.get("GLS_CELL_SF", "1")
    return {"0": "gls_cell_kernel<3,2,%d,3,MODE_JV,GEN> (dense per-cell)" % kp,
            "2": "k_cell_mfma_jv<%d,GEN> (MFMA per-cell)" % kp}.get(mode, "k_cell_sf_jv<%d,GEN> (sum-factorized per-cell)" % kp)
PMC_TRAFFIC_FILE = "r04_pmc_traffic_pencil_128.txt"  # tools/pmc_traffic.sh summary of the pencil J.v (fallback)
LDS_MODEL_FILE = "r05_lds_model.json"                # tools/lds_model.py (static model, source-hash tagged)
FP64_PEAK_TFS = 78.6        # MI355X FP64 (vector = matrix) spec; measured 61-64 TF (profiles/r01_microbench_fp64.txt)


def smooth_state(mesh, n, dim, dir_dofs, dir_vals, phase=0.0):
    """A smooth synthetic cavity-like velocity field (rotating vortex + lid shear), Dirichlet values applied."""
    k = mesh["k"]
    nx = k * n + 1
    g = np.linspace(-1.0, 1.0, nx)
    nv, npn = mesh["n_vnodes"], mesh["n_pnodes"]
    x = np.zeros(dim * nv + npn)
    Z, Y, X = np.meshgrid(g, g, g, indexing="ij") if dim == 3 else (None,) + tuple(np.meshgrid(g, g, indexing="ij"))
    wall = (1 - X ** 2) * (1 - Y ** 2) * ((1 - Z ** 2) if dim == 3 else 1.0)
    ux = (0.5 * (1 + Y)) ** 2 * wall * (1.0 + 0.1 * np.sin(phase))
    uy = -0.5 * X * wall
    vel = np.zeros((nv, dim))
    vel[:, 0] = ux.reshape(-1)
    vel[:, 1] = uy.reshape(-1)
    if dim == 3:
        vel[:, 2] = (0.2 * X * Y * wall).reshape(-1)
    x[:dim * nv] = vel.reshape(-1)
    x[dim * nv:] = 0.05 * (X * Y).reshape(-1) if mesh["kp"] == k else 0.0
    x[dir_dofs] = dir_vals
    return x


def pmc_traffic(path, kernel_mode, n_dofs):
    """HBM bytes per launch of gls_brick_kernel<k, mode> (+ its k_slab_sum) from a tools/pmc_traffic.sh summary
    (separate rocprofv3 --pmc passes for FETCH_SIZE and WRITE_SIZE, KiB per dispatch), corrected
    with the k_copy calibration in the same file (it moves 8 * n_dofs bytes each way; on gfx950
    FETCH_SIZE reports half of a streaming read, MI355X_MICROARCH.md 'HBM')."""
    if not os.path.exists(path):
        return None
    cur, vals = None, {}
    for line in open(path):
        if not line.startswith(" "):
            cur = line.strip()
            continue
        f = line.split()
        if cur and f and f[0] in ("FETCH_SIZE", "WRITE_SIZE"):
            vals.setdefault(cur, {})[f[0]] = float(f[1]) * 1024.0
    copy = next((v for k_, v in vals.items() if "k_copy" in k_), None)
    kern = next((v for k_, v in vals.items() if ("gls_pencil_kernel<double, %d" % kernel_mode in k_
                                                 or "gls_brick_kernel<2, %d, double>" % kernel_mode in k_)), None)
    slab = next((v for k_, v in vals.items() if "k_slab_sum<double" in k_ or "k_slab_sum_cube<double, false" in k_), {})
    if not copy or not kern or len(copy) < 2 or len(kern) < 2:
        return None
    fetch_corr = 8.0 * n_dofs / copy["FETCH_SIZE"]
    write_corr = 8.0 * n_dofs / copy["WRITE_SIZE"]
    # the J.v's slab node sum (one k_slab_sum per brick launch, same size for every mode)
    t = sum(d.get("FETCH_SIZE", 0.0) * fetch_corr + d.get("WRITE_SIZE", 0.0) * write_corr for d in (kern, slab))
    return t, fetch_corr, write_corr


def live_pmc_traffic(n, k, n_dofs, timeout=180):
    """HBM bytes per launch of the J.v (pencil kernel + its slab sum) MEASURED NOW: two separate
    `rocprofv3 --pmc FETCH_SIZE` / `--pmc WRITE_SIZE` passes (MI355X_MICROARCH.md "HBM": one TCC counter
    group per pass) over tools/jv_bench.py in a child process (this process keeps its GPU state; nothing is
    exec'ed), calibrated on the k_copy of n_dofs doubles in the same run (gfx950 counts half of a
    streaming read in FETCH_SIZE). Returns (bytes, fetch_corr, write_corr) or raises."""
    import csv
    import glob
    import shutil
    import subprocess
    import tempfile
    prof = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    out = tempfile.mkdtemp(prefix="gls_pmc_", dir=os.environ.get("TMPDIR", "/tmp"))
    vals = {}
    for i, ctr in enumerate(("FETCH_SIZE", "WRITE_SIZE")):
        cmd = [prof, "--pmc", ctr, "--kernel-include-regex", "gls_pencil_kernel|gls_brick_kernel|k_copy|k_slab_sum",
               "-d", os.path.join(out, "p%d" % i), "-o", "run", "--output-format", "csv", "--",
               sys.executable, os.path.join(ROOT, "tools", "jv_bench.py"), str(n), "4"]
        subprocess.run(cmd, timeout=timeout, capture_output=True, check=True, cwd=out, env=dict(os.environ, GLS_K=str(k)))
        for f in glob.glob(os.path.join(out, "p%d" % i, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                vals.setdefault(r["Kernel_Name"], {}).setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]) * 1024.0)
    shutil.rmtree(out, ignore_errors=True)
    mean = {kn: {c: sum(v) / len(v) for c, v in d.items()} for kn, d in vals.items()}
    copy = next(v for kn, v in mean.items() if "k_copy" in kn)
    kern = next(v for kn, v in mean.items() if "gls_pencil_kernel<double, 4" in kn or "gls_brick_kernel<%d, 4, double>" % k in kn)
    slab = next((v for kn, v in mean.items() if "k_slab_sum_cube<double, false" in kn or "k_slab_sum<double" in kn), {})
    fc, wc = 8.0 * n_dofs / copy["FETCH_SIZE"], 8.0 * n_dofs / copy["WRITE_SIZE"]
    t = sum(d.get("FETCH_SIZE", 0.0) * fc + d.get("WRITE_SIZE", 0.0) * wc for d in (kern, slab))
    return t, fc, wc


def step_bytes_model(n, k, m, L, f32_fine, k_hist=2):
    """Algorithmic HBM bytes of one Newton iteration of the cube (SURVEY §8d formulas, every array touched
    once per operator call): assemble_matrix_and_rhs (B_res + the diagonal's 8N), L line-search residuals
    (B_res), m FP64 J.v (B_Jv), the V-cycles' smoother J.v (B_Jv at the level's size: `f32_fine` measured
    launches on the fine level, 2 per V-cycle on each coarser level), their transfers (restriction reads the
    fine and writes the coarse vector, prolongation reads the coarse one and updates the fine x: 8 (3 N_l + 2
    N_l+1)) and first Jacobi sweeps (b, D, x: 24 N_l), and the Gram-Schmidt passes (multi-dot over j + 1
    vectors and the projection over j + 2 at step j, the final update over m + 2)."""
    def sz(c):  # (velocity nodes, DoFs) of the Qk-Qk c^3 cube
        nv = (k * c + 1) ** 3
        return nv, 4 * nv
    def b_jv(c):
        nv, N = sz(c)
        return 8 * N * 3 + 8 * k_hist * 3 * nv + 4 * c ** 3 * (k + 1) ** 3 + 32 * c ** 3 + nv
    def b_res(c):
        nv, N = sz(c)
        return 8 * N * 2 + 8 * k_hist * 3 * nv + 4 * c ** 3 * (k + 1) ** 3 + 32 * c ** 3
    N = sz(n)[1]
    levels = []
    c = n
    while c > 2:
        levels.append(c)
        c //= 2
    levels.append(2)
    vcyc = max(f32_fine // 2, 1)
    parts = {"assemble_matrix_and_rhs": b_res(n) + 8 * N, "line_search_residuals": L * b_res(n),
             "jacobian_apply_fp64": m * b_jv(n), "smoother_jv_fine": f32_fine * b_jv(n),
             "smoother_jv_coarse": vcyc * sum(2 * b_jv(c) for c in levels[1:-1]),
             "transfers": vcyc * sum(8 * (3 * sz(a)[1] + 2 * sz(b)[1]) for a, b in zip(levels[:-1], levels[1:])),
             "jacobi_first_sweeps": vcyc * sum(24 * sz(c)[1] for c in levels[:-1]),
             "orthogonalisation": 8 * N * (sum(2 * j + 3 for j in range(1, int(m) + 1)) + int(m) + 2)}
    return sum(parts.values()), parts


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_threads():
    """Host threads of the CPU legs and why: OMP_NUM_THREADS when set -- on the GPU box the pool sets it to
    this job's CPU share (16 host threads per GPU; the affinity mask shows the whole machine, whose other
    cores belong to other jobs) -- else every CPU in the process's affinity."""
    env = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    aff = len(os.sched_getaffinity(0))
    if env:
        return env, ("OMP_NUM_THREADS=%d: the job's CPU share (the affinity mask lists %d CPUs of the whole "
                     "machine, shared with other jobs)" % (env, aff))
    return aff, "every CPU in the process's affinity mask (%d)" % aff


def cpu_baseline(k, kp, nu, seconds, threads):
    """Oracle (CPU restatement of assembleGLS, 'port') timed on bounded samples, with the
    reference-cell tables precomputed as deal.II's FEValues does (gls_oracle_set_fast_tables):
      * element matrix + rhs and rhs-only throughput on `threads` OpenMP threads and on 1 thread;
      * CSR SpMV throughput (scipy, 1 thread) on the assembled Q2 matrix of a 10^3-cell cavity;
      * host copy bandwidth (numpy) for the GMRES orthogonalisation passes.
    Returns raw timings; main() extrapolates them to one Newton step of the GPU run's (m, L)."""
    import ctypes as C

    import scipy.sparse as sp

    from oracle.oracle import Oracle, StructuredProblem, _dp, lib
    L = lib()
    L.gls_oracle_set_fast_tables.argtypes = [C.c_int]
    L.gls_oracle_set_fast_tables(1)
    p = StructuredProblem(3, 6, k=k, kp=kp, viscosity=nu, scheme="bdf2", time_steps=(0.01,) * 4)
    u = np.random.default_rng(20200200).uniform(-1, 1, p.n_dofs)
    P = p.struct()
    res = {}
    for key, wm, thr, share in (("matrix", 1, threads, 0.35), ("rhs", 0, threads, 0.35),
                                ("matrix_1core", 1, 1, 0.1), ("rhs_1core", 0, 1, 0.1)):
        cnt = 8
        while True:
            t0 = time.perf_counter()
            L.gls_oracle_time_local_systems(C.byref(P), _dp(u), _dp(u), _dp(u), _dp(u), 0, cnt, wm, thr)
            dt = time.perf_counter() - t0
            if dt > seconds * share or cnt > 1 << 22:
                break
            cnt = int(cnt * max(2.0, min(8.0, (seconds * share) / max(dt, 1e-3))))
        res[key] = (cnt, dt)
    L.gls_oracle_set_fast_tables(0)
    # CSR SpMV (what the reference's Trilinos GMRES applies per iteration) on an assembled Q2 matrix
    q = StructuredProblem(3, 10, k=k, kp=kp, viscosity=nu, scheme="bdf2", time_steps=(0.01,) * 4)
    uq = np.random.default_rng(20200200).uniform(-1, 1, q.n_dofs)
    A, _ = Oracle(q).matrix_and_rhs(uq, uq, uq, None)
    A = sp.csr_matrix(A)
    x = np.random.default_rng(1).uniform(-1, 1, A.shape[0])
    reps, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds * 0.1:
        A @ x
        reps += 1
    res["spmv"] = (A.nnz, A.shape[0], (time.perf_counter() - t0) / reps)
    big = np.ones(1 << 25)
    dst = np.empty_like(big)
    t0 = time.perf_counter()
    for _ in range(4):
        np.copyto(dst, big)
    res["copy_gbs"] = 4 * 2 * big.nbytes / (time.perf_counter() - t0) / 1e9
    return res


def cpu_newton(k, kp, n, nu, scheme, dt, threads):
    """One complete Newton iteration of the reference's CPU path on the assembled system (oracle
    gls_oracle_newton_csr: CSR assembly on `threads`, ILU(0) setup, GMRES(30)+ILU(0) to rel 1e-4,
    line search; the sparsity pattern is setup_dofs work, timed separately) on the n^3 cavity with
    this bench's synthetic state. Returns the oracle's timing dict plus n_dofs."""
    import ctypes as C
    from oracle.oracle import StructuredProblem, lib, newton_csr
    L = lib()
    L.gls_oracle_set_fast_tables.argtypes = [C.c_int]
    L.gls_oracle_set_fast_tables(1)  # reference-cell tables precomputed, as FEValues does
    p = StructuredProblem(3, n, k=k, kp=kp, viscosity=nu, scheme=scheme, time_steps=(dt,) * 4, colorize=True)
    one = lambda X: np.stack([np.ones(len(X)), 0 * X[:, 0], 0 * X[:, 0]], 1)  # noqa: E731
    p.set_dirichlet([("noslip", b, None) for b in (0, 1, 2, 4, 5)] + [("function", 3, one)])
    mesh = dict(k=k, kp=kp, n_vnodes=p.n_vnodes, n_pnodes=p.n_pnodes)
    dd = np.array(sorted(p.dirichlet), dtype=np.int64)
    dv = np.array([p.dirichlet[d] for d in dd])
    x = smooth_state(mesh, n, 3, dd, dv, 0.0)
    u2 = smooth_state(mesh, n, 3, dd, dv, 0.3)
    st = newton_csr(p, x, x.copy(), u2, threads=threads, rel=1e-4, minres=1e-14)
    L.gls_oracle_set_fast_tables(0)
    st["n_dofs"] = p.n_dofs
    st["seconds"] = st["t_assemble"] + st["t_ilu"] + st["t_gmres"] + st["t_linesearch"]
    return st


def general_context(sp, bcs, nu, state, k=2, kp=1):
    """A GLS context on a general (mapped) FE space: bcs = [(type, boundary id, values)] in prm order, type
    noslip / function (values: X -> (n, 3)) / slip on an axis-aligned wall (the normal component, as
    compute_no_normal_flux_constraints there); state: X -> (n, 3) synthetic velocity, Dirichlet values applied."""
    from softx_2020_200_amd.native import GLSContext
    nv, X, bid = sp["n_vnodes"], sp["vnode_x"], sp["vnode_bid"].astype(np.int64)
    con = np.zeros((nv, 3), dtype=bool)
    val = np.zeros((nv, 3))
    scale = float(np.abs(X).max())
    for typ, b, fn in bcs:
        on = ((bid >> b) & 1).astype(bool)
        comps = np.ones(3, dtype=bool)
        if typ == "slip":
            flat = [d for d in range(3) if len(np.unique(np.round(X[on, d] / (1e-9 * scale)))) <= 2]
            comps = np.array([d == flat[0] for d in range(3)])
        vals = fn(X) if typ == "function" else np.zeros((nv, 3))
        for c in range(3):
            if not comps[c]:
                continue
            sel = on & ~con[:, c]
            con[sel, c] = True
            val[sel, c] = vals[sel, c]
    mask = (con[:, 0] * 1 + con[:, 1] * 2 + con[:, 2] * 4).astype(np.uint8)
    ctx = GLSContext(3, k, kp, sp["cell_vnodes"], sp["cell_pnodes"], None, nv, sp["n_pnodes"], viscosity=nu,
                     vnode_mask=mask, map_degree=k, cell_support=sp["cell_support"])
    dofs = np.nonzero(con.reshape(-1))[0].astype(np.int64)
    ctx.set_dirichlet(dofs, val.reshape(-1)[dofs])
    x = np.concatenate([state(X).reshape(-1), np.zeros(sp["n_pnodes"])])
    x[dofs] = val.reshape(-1)[dofs]
    return ctx, sp, x


def cylinder3d_mesh(refine=0):
    from softx_2020_200_amd.native import UMesh
    m = UMesh(3, gmsh=os.path.join(ROOT, "apps", "cases", "cylinder3d_extruded.msh"))
    if refine:
        m.refine_global(refine)
    return m


def cylinder3d_context(k=2, kp=1, nu=0.005, refine=0, space=None):
    """BASELINE configs[4]'s discrete problem on one GPU (apps/cases/cylinder3d_q2q1_re200_kelly.prm):
    the reference's cylinder_structured.msh extruded to 3D (4 layers, apps/cases/cylinder3d_extruded.msh),
    Q2-Q1 with MappingQ2 on the boundary cells, nu = 0.005 (Re 200); boundary conditions in the prm's
    order: id 0 noslip (cylinder), id 1 u = (1, 0, 0) (inlet), slip on the planar ids 2, 4, 5 (n.u = 0,
    the normal component; compute_no_normal_flux_constraints on axis-aligned walls). refine: global
    refinements of the mesh (flat: no manifold on the extruded gmsh mesh); space: that FE space given."""
    sp = space if space is not None else cylinder3d_mesh(refine).fe_space(k, kp)
    inlet = lambda X: np.stack([np.ones(len(X)), 0 * X[:, 0], 0 * X[:, 0]], 1)  # noqa: E731

    def state(X):  # the free stream with a smooth wake-like perturbation
        r2 = X[:, 0] ** 2 + X[:, 1] ** 2
        vel = np.zeros((len(X), 3))
        vel[:, 0] = 1.0 - np.exp(-r2 / 4.0) * (1.0 + 0.2 * np.sin(X[:, 2]))
        vel[:, 1] = 0.1 * np.exp(-r2 / 4.0) * X[:, 1]
        return vel
    return general_context(sp, [("noslip", 0, None), ("function", 1, inlet), ("slip", 2, None), ("slip", 4, None),
                                ("slip", 5, None)], nu, state, k, kp)


def taylorcouette3d_mesh(refine=1):
    from softx_2020_200_amd.native import UMesh
    m = UMesh(3, "cylinder_shell", "1 : 0.25 : 1 : 8 : 2")
    m.refine_global(refine)
    return m


def taylorcouette3d_context(space, k=2, kp=1, nu=1.0):
    """BASELINE configs[3]'s discrete problem (apps/cases/taylor-couette3d_q2q1_kelly.prm): cylinder_shell
    (inner radius 0.25, outer 1, length 1) with its cylindrical manifold, Q2-Q1 with MappingQ2 on every cell
    (qmapping all), nu = 1, steady; id 0 (inner) u = (-y, x, 0), id 1 noslip, slip end caps ids 2, 3."""
    rot = lambda X: np.stack([-X[:, 1], X[:, 0], 0 * X[:, 0]], 1)  # noqa: E731

    def state(X):  # the Couette profile u_theta(r) with an axial modulation
        r = np.sqrt(X[:, 0] ** 2 + X[:, 1] ** 2)
        eta, ri = 0.25, 0.25
        ut = (-(eta ** 2) / (1 - eta ** 2) * r + ri ** 2 / (1 - eta ** 2) / r) * (1.0 + 0.1 * np.sin(np.pi * X[:, 2]))
        th = np.arctan2(X[:, 1], X[:, 0])
        return np.stack([-np.sin(th) * ut, np.cos(th) * ut, 0.02 * np.sin(np.pi * X[:, 2]) * (1 - r)], 1)
    return general_context(space, [("function", 0, rot), ("noslip", 1, None), ("slip", 2, None), ("slip", 3, None)],
                           nu, state, k, kp)


def bench_cylinder3d(args):
    """--workload cylinder3d: one Newton iteration per step of BDF2 on configs[4]'s problem (single
    GPU, unadapted extruded mesh): residual, ILU(0) setup (probe + factor, multicolor order) and
    GMRES(30)+ILU to rel 1e-4, line search; the per-cell J.v kernel's roofline. --workload taylorcouette3d:
    the same on configs[3]'s problem (steady, cylinder_shell refined --cyl-refine + 1 times)."""
    import torch
    t_setup = time.perf_counter()
    tc = args.workload == "taylorcouette3d"
    scheme, ts = ("steady", (0.0,) * 4) if tc else ("bdf2", (0.05,) * 4)
    refine = args.cyl_refine + (1 if tc else 0)  # configs[3]'s prm starts from one global refinement
    mesh = (lambda r: taylorcouette3d_mesh(r)) if tc else (lambda r: cylinder3d_mesh(r))
    make = (lambda sp_: taylorcouette3d_context(sp_)) if tc else (lambda sp_: cylinder3d_context(space=sp_))
    qall = tc  # configs[3]: MappingQ2 on every cell
    levels, sw, pre, post = None, 0, 0, 0
    if args.cyl_precond == "hmg":  # the refinement hierarchy of the globally refined mesh
        if refine < 1 and not (args.cyl_plevel or args.cyl_hp):
            sys.exit("bench.py: --cyl-precond hmg needs --cyl-refine >= 1 or the p-level (a level below the fine mesh)")
        m = mesh(refine)
        base = m.coarsen_to(0)
        if args.cyl_hp:  # p first: Q2-Q1 fine -> Q1-Q1 on the same mesh -> the Q1-Q1 refinement hierarchy
            handles = [m.fe_space_handle(2, 1, qmapping_all=qall), m.fe_space_handle(1, 1, qmapping_all=qall)] + [
                m.coarsen_to(refine - l).fe_space_handle(1, 1, qmapping_all=qall) for l in range(1, refine)] + (
                [base.fe_space_handle(1, 1, qmapping_all=qall)] if refine >= 1 else [])
            kps = [(2, 1)] + [(1, 1)] * (len(handles) - 1)
        else:
            handles = [m.fe_space_handle(2, 1, qmapping_all=qall)] + [
                m.coarsen_to(refine - l).fe_space_handle(2, 1, qmapping_all=qall) for l in range(1, refine)] + (
                [base.fe_space_handle(2, 1, qmapping_all=qall)] if refine >= 1 else [])
            kps = [(2, 1)] * len(handles)
            if args.cyl_plevel:  # p-level below the base mesh: Q1-Q1 on the same cells, solved exactly
                handles.append(base.fe_space_handle(1, 1, qmapping_all=qall))
                kps.append((1, 1))
        xfer = [handles[l].mg_transfer_from(handles[l + 1]) for l in range(len(handles) - 1)]
        levels = [(taylorcouette3d_context(h.data, k=k_, kp=kp_) if tc else cylinder3d_context(k=k_, kp=kp_, space=h.data))
                  for h, (k_, kp_) in zip(handles, kps)]
        ctx, sp, x = levels[0]
        for c_, _, _ in levels:
            c_.set_time(scheme, ts)
        sw = 1 if args.cyl_smoother == "ilu" else 2
        # configs[3] (steady, nu 1): post-smoothing only, V(0,1), 7 GMRES its in 160 ms against V(1,1)'s 5 in 176;
        # configs[4]: V(1,1) (V(0,1) 184 ms, V(2,1) 175; profiles/r06_hmg_sweeps.txt)
        pre, post = args.cyl_sweeps if args.cyl_sweeps else ((0, 1) if tc and args.cyl_smoother == "ilu" else (sw, sw))
        nco = levels[-1][0].n_dofs
        ctx.attach_multigrid_transfers([c_ for c_, _, _ in levels[1:]], xfer, pre_smooth=pre if pre > 0 else -1,
                                       post_smooth=post,
                                       coarse_sweeps=args.mg_coarse_sweeps_cyl, omega=args.mg_omega_cyl,
                                       coarse_direct=1 if nco <= args.direct_max else -1, smoother=args.cyl_smoother)
    else:
        ctx, sp, x = make(mesh(refine).fe_space(2, 1, qmapping_all=qall))
        ctx.set_time(scheme, ts)
        ctx.attach_ilu(1e-5, 1.0, fill=args.ilu_fill, ordering="multicolor" if args.ilu_fill == 0 else "cm")
    dev = torch.device("cuda", 0)
    ctx.set_time(scheme, ts)
    t_setup = time.perf_counter() - t_setup
    m1 = torch.from_numpy(x).to(dev)
    m2 = m1.clone()
    present = m1.clone()

    def one_step():
        present.copy_(m1)
        return ctx.newton(present, m1, m2, tolerance=1e-30, max_iterations=1, lin_max_iterations=args.lin_max,
                          restart=args.restart, relative_residual=1e-4, minimum_residual=1e-9)
    for _ in range(args.warmup):
        one_step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    stats = [one_step() for _ in range(args.steps)]
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    ctx.set_state(present, m1, m2)
    v = torch.rand(ctx.n_dofs, dtype=torch.float64, device=dev)
    y = torch.empty_like(v)
    ctx.jacobian_apply(v, y)
    ctx.timing(True)
    for _ in range(args.jv_reps):
        ctx.jacobian_apply(v, y)
    jv_ms, jv_n = ctx.timing_get(1)
    ctx.timing(False)
    N, nc = ctx.n_dofs, sp["n_cells"]
    # algorithmic bytes of one per-cell J.v launch (gls_cell_kernel MODE_JV, element-vector output):
    # v and the linearization state u (8N each; the GLS Jacobian needs the full strong residual of u,
    # p), the cell node maps (4 B x (27 + 8) per cell), the MappingQ geometry per quadrature point
    # (22 doubles: x_q, JxW, J^-1, G = J^-1 J^-T, the Hessian correction -- FEValues' per-q data) and
    # the element vectors written (8 B x (3 x 27 + 8) per cell; summed into Jv by the gather kernel)
    B = 16 * N + 4 * nc * (27 + 8) + 22 * 8 * 27 * nc + 8 * nc * (3 * 27 + 8)
    ms = jv_ms / max(jv_n, 1)
    its_per_s = args.steps / el
    out = {
        "metric": ("nonlinear iters/sec (3D Taylor-Couette, Q2-Q1 mapped, steady)" if tc else
                   "nonlinear iters/sec (3D cylinder Re 200, Q2-Q1 mapped, BDF2)"), "value": its_per_s,
        "unit": "nonlinear_iters/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": 1e3 * el / args.steps, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "f64", "data": ("synthetic (Couette profile with an axial modulation, prm boundary values)" if tc else
                                 "synthetic (free stream with a smooth wake-like perturbation, prm boundary values)"),
        "config": {"workload": ("BASELINE configs[3] problem on one GPU: cylinder_shell 1:0.25:1:8:2 refined %d times "
                                "globally (cylindrical manifold), Q2-Q1 MappingQ2 on every cell, nu 1, steady" % refine)
                   if tc else ("BASELINE configs[4] problem on one GPU: apps/cases/cylinder3d_extruded.msh "
                               "(unadapted%s), Q2-Q1 MappingQ2, nu 0.005, BDF2 dt 0.05" % (
                                   ", %d global refinements (flat)" % args.cyl_refine if args.cyl_refine else "")),
                   "n_dofs": N, "n_cells": nc,
                   "linear_solver": ("GMRES(%d)+GMG V(%d,%d) on the %s (%d levels, %s smoothing, "
                                     "%s on the base mesh), rel 1e-4" % (
                                         args.restart, pre, post,
                                         "h-p hierarchy (Q2-Q1 fine, Q1-Q1 on the fine mesh and its refinement "
                                         "hierarchy)" if args.cyl_hp else "refinement hierarchy", len(levels),
                                         {"ilu": "multicolor ILU(0)", "jacobi": "damped-Jacobi",
                                          "ilu-coarse": "damped-Jacobi on the finest, multicolor ILU(0) below"}[
                                             args.cyl_smoother],
                                         ("exact LU of the Q1-Q1 level" if args.cyl_plevel or args.cyl_hp else "exact LU")
                                         if levels[-1][0].n_dofs <= args.direct_max else "%d sweeps" % args.mg_coarse_sweeps_cyl))
                   if levels else "GMRES(%d)+ILU(%d) %s, rel 1e-4" % (
                       args.restart, args.ilu_fill, "multicolor" if args.ilu_fill == 0 else "Cuthill-McKee")},
        "setup_s": t_setup,
        "mdof_per_s": N * its_per_s / 1e6,
        "linear_iterations_per_step": float(np.mean([s_["linear_iterations"] for s_ in stats])),
        "roofline": {"bound": "hbm", "kernel": cell_jv_kernel_name(1), "achieved": B / (ms * 1e-3) / 1e9,
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": B / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, "traffic": None,
                     "algorithmic_bytes_per_launch": B, "launch_ms": ms},
    }
    print(json.dumps(out))


def bench_octree(args):
    """--workload octree: the lid-driven cavity on an adapted octree forest (hanging-node constraints;
    base --cells^3, --octree-steps levels of lid / edge refinement, softx_2020_200_amd.problem.octree_lid_tree),
    Q2-Q2 BDF2, one Newton iteration per step: residual + diagonal, preconditioner setup, GMRES(--restart) to
    rel 1e-4, line search. --precond mg: the V-cycle on the refinement hierarchy (gls_mg_attach_transfers;
    per-cell FP64 smoothing on the hanging levels, exact LU on the uniform level 0); --precond ilu: the
    assembled multicolor ILU(0) (the adaptive path's default before)."""
    import torch
    from softx_2020_200_amd.problem import AdaptiveCavityProblem, octree_lid_tree
    dev = torch.device("cuda", 0)
    tree = octree_lid_tree(args.n, args.octree_steps)
    mg = args.precond == "mg"
    prob = AdaptiveCavityProblem(tree, k=args.k, kp=args.kp, viscosity=args.nu, multigrid=mg,
                                 pre_smooth=args.mg_smooth[0], post_smooth=args.mg_smooth[1], omega=args.mg_omega,
                                 coarse_direct=1, mixed_precision=int(args.mg_precision == "f32"),
                                 smoother=args.oct_smoother)
    ctx = prob.ctx
    if not mg:
        ctx.attach_ilu(1e-5, 1.0, fill=0, ordering="multicolor")
    ctx.set_time("bdf2", (args.dt,) * 4)
    X = prob.mesh["vnode_x"]
    vel = np.zeros((len(X), 3))
    vel[:, 0] = ((X[:, 1] + 1.0) / 2.0) ** 2 * (1.0 - X[:, 0] ** 2) * (1.0 - X[:, 2] ** 2)
    vel[:, 1] = 0.1 * np.sin(np.pi * X[:, 0]) * (1.0 - X[:, 1] ** 2)
    m1 = torch.from_numpy(np.concatenate([vel.reshape(-1), np.zeros(prob.mesh["n_pnodes"])])).to(dev)
    ctx.apply_dirichlet(m1)
    m2 = m1.clone()
    present = m1.clone()

    def one_step():
        present.copy_(m1)
        return ctx.newton(present, m1, m2, tolerance=1e-30, max_iterations=1, lin_max_iterations=args.lin_max,
                          restart=args.restart, relative_residual=args.rel, minimum_residual=1e-12)
    for _ in range(args.warmup):
        one_step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    stats = [one_step() for _ in range(args.steps)]
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    ctx.set_state(present, m1, m2)
    v = torch.rand(ctx.n_dofs, dtype=torch.float64, device=dev)
    y = torch.empty_like(v)
    ctx.jacobian_apply(v, y)
    ctx.timing(True)
    for _ in range(args.jv_reps):
        ctx.jacobian_apply(v, y)
    jv_ms, jv_n = ctx.timing_get(1)
    ctx.timing(False)
    N, nc = ctx.n_dofs, prob.mesh["n_cells"]
    # algorithmic bytes of one J.v (the sibling-group bricks on the pencil kernel, the other leaves on the
    # per-cell kernel, both writing element vectors summed per node): v and u (8N each), node maps
    # (4 B x 2 x 27 per cell), the cell box (48 B), the element vectors (8 B x 4 x 27)
    B = 16 * N + 4 * nc * 54 + 48 * nc + 8 * nc * 4 * 27
    ms = jv_ms / max(jv_n, 1)
    its_per_s = args.steps / el
    lev = [int(v_) for v_ in np.bincount(prob.mesh["cell_level"])]
    out = {
        "metric": "nonlinear iters/sec (3D lid-driven cavity, adapted octree, Q%d-Q%d, BDF2)" % (args.k, args.kp),
        "value": its_per_s, "unit": "nonlinear_iters/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": 1e3 * el / args.steps, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "f64", "data": "synthetic (smooth lid-driven profile, prm-style boundary values)",
        "config": {"workload": "cavity on an adapted octree: base %d^3, %d lid/edge refinement levels "
                               "(hanging-node constraints), nu %g, BDF2 dt %g" % (args.n, args.octree_steps, args.nu, args.dt),
                   "n_dofs": N, "n_cells": nc, "cells_per_level": lev,
                   "linear_solver": ("GMRES(%d)+GMG V(%d,%d) on the refinement hierarchy (%d levels, %s smoothing), rel %g"
                                     % (args.restart, args.mg_smooth[0], args.mg_smooth[1], len(prob.levels),
                                        "multicolor ILU(0)" if args.oct_smoother == "ilu" else
                                        "multicolor ILU(0) below the finest, damped-Jacobi FP32 brick J.v on it"
                                        if args.oct_smoother == "ilu-coarse" else
                                        ("damped-Jacobi, FP32 brick J.v" if args.mg_precision == "f32" else "damped-Jacobi FP64"),
                                        args.rel))
                   if mg else "GMRES(%d)+ILU(0) multicolor, rel %g" % (args.restart, args.rel)},
        "mdof_per_s": N * its_per_s / 1e6,
        "linear_iterations_per_step": float(np.mean([s_["linear_iterations"] for s_ in stats])),
        "forest_bricks": ctx.forest_bricks(),
        "roofline": {"bound": "hbm", "kernel": "gls_pencil_kernel<double,MODE_JVQ> (sibling-group bricks) + "
                                               "%s (other leaves) + k_gather_ev" % cell_jv_kernel_name(2),
                     "achieved": B / (ms * 1e-3) / 1e9,
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": B / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, "traffic": None,
                     "algorithmic_bytes_per_launch": B, "launch_ms": ms},
    }
    print(json.dumps(out))


def spawn_ranks(n):
    """Launcher-less N-rank run: start N fresh processes of this script with the torch.distributed.run
    environment (this parent never imports torch or touches the GPU), forward their output, and return
    the exit status: the first failing rank's code (the others are then terminated), else 0 after
    re-printing rank 0's JSON line as the only line on stdout."""
    import socket
    import subprocess
    import threading
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    procs, lines = [], []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), GLS_BENCH_SPAWNED="1")
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      stdout=subprocess.PIPE, text=True))

    def pump(r, f):  # keep rank 0's JSON line; everything else goes on to stderr
        for line in f:
            if r == 0 and line.lstrip().startswith("{"):
                lines.append(line)
            else:
                sys.stderr.write(line)
    ths = [threading.Thread(target=pump, args=(r, p.stdout), daemon=True) for r, p in enumerate(procs)]
    for th in ths:
        th.start()
    rc = 0
    while True:
        st = [p.poll() for p in procs]  # every rank polled (not short-circuited), so failures are seen
        if all(x is not None for x in st):
            break
        bad = [x for x in st if x not in (None, 0)]
        if bad:
            rc = bad[0]
            break
        time.sleep(0.2)
    if rc:
        sys.stderr.write("bench.py: a rank exited with status %d; terminating the others\n" % rc)
        for p in procs:
            if p.poll() is None:
                p.terminate()
        for p in procs:
            try:
                p.wait(timeout=20)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
    for th in ths:
        th.join(timeout=10)
    rc = rc or next((p.returncode for p in procs if p.returncode), 0)
    if rc:
        return rc if rc > 0 else 1
    if not lines:
        sys.stderr.write("bench.py: rank 0 printed no result line\n")
        return 1
    sys.stdout.write(lines[-1])
    sys.stdout.flush()
    return 0


def preflight_agreement(dist, ctl, world, failed, late):
    """The ranks' pre-flight outcomes, agreed over the gloo control group `ctl` (created with a timeout), never
    over the data-path transport that a failed rank may have left inside a collective. failed: this rank's
    pre-flight raised or missed the tolerance; late: it raised after the transport's first collective.
    Returns "ok"; "fallback" when no rank can be stuck in the native transport (every failure came before its
    first collective, or every rank failed); "abort" when a rank failed after the first collective while
    another did not, or a peer never reached the agreement (the control group's timeout)."""
    import torch
    t = torch.tensor([float(bool(failed)), float(bool(failed) and bool(late))], dtype=torch.float64)
    try:
        dist.all_reduce(t, group=ctl)
    except Exception as e:  # noqa: BLE001 -- a peer is stuck in the data-path transport
        sys.stderr.write("bench.py: pre-flight agreement failed (%r): a rank did not reach it\n" % (e,))
        return "abort"
    nfail, nlate = t.tolist()
    if nfail == 0:
        return "ok"
    if nlate == 0 or nfail == world:
        return "fallback"
    return "abort"


def preflight(args, rank, world, dev, dist, stage=None):
    """N-rank residual and J.v of a 16^3 cavity (the bench's boundary data, state and scheme; the same
    transport as the timed run) against a single-rank context of the whole mesh on rank 0. Returns the
    max relative difference (every rank gets rank 0's number). stage["s"] becomes "collective" when the
    transport's first collective (the communicator's creation) starts."""
    import torch

    import softx_2020_200_amd as sx
    from softx_2020_200_amd.dist import DistributedProblem, local_vector, owned_global_dofs
    from softx_2020_200_amd.problem import build_context, dirichlet_from_bcs
    n = 16
    mesh = sx.hyper_cube(3, n, args.k, args.kp, -1.0, 1.0)
    bcs = [("noslip", b, None) for b in (0, 1, 2, 4, 5)] + [("function", 3, (1.0, 0.0, 0.0))]
    mask, dd, dv = dirichlet_from_bcs(mesh, n, -1.0, 1.0, True, bcs)
    nv = mesh["n_vnodes"]
    u = smooth_state(mesh, n, 3, dd, dv, 0.0)
    u2 = smooth_state(mesh, n, 3, dd, dv, 0.3)
    v = np.random.default_rng(20200200).uniform(-1.0, 1.0, len(u))
    if stage is not None:
        stage["s"] = "collective"
    dp = DistributedProblem(mesh, rank, world, dev, viscosity=args.nu, vnode_mask=mask, dirichlet=(dd, dv),
                            backend=args.dist_backend, impl=args.dist_impl)
    dist.barrier()  # first collective before any batched P2P (NCCL requirement)
    if os.environ.get("GLS_BENCH_FAIL_NATIVE_PREFLIGHT") == "late%d" % rank and args.dist_impl == "native":
        raise RuntimeError("GLS_BENCH_FAIL_NATIVE_PREFLIGHT (after the first collective)")
    loc = lambda g: torch.from_numpy(local_vector(dp.plan, g, nv)).to(dev)  # noqa: E731
    dp.ctx.set_time(args.scheme, (args.dt,) * 4)
    dp.ctx.set_state(loc(u), loc(u), loc(u2))
    r = dp.ctx.residual().cpu().numpy()
    jv = dp.ctx.jacobian_apply(loc(v)).cpu().numpy()
    li, gi = owned_global_dofs(dp.plan, nv)
    parts = [None] * world
    dist.all_gather_object(parts, (gi, r[li], jv[li]))
    err = torch.zeros(1, dtype=torch.float64)
    if rank == 0:
        R, J = np.full(len(u), np.nan), np.full(len(u), np.nan)
        for g_, r_, j_ in parts:
            R[g_], J[g_] = r_, j_
        one = build_context(mesh, viscosity=args.nu, vnode_mask=mask)
        one.set_dirichlet(dd, dv)
        one.set_time(args.scheme, (args.dt,) * 4)
        t = lambda a: torch.from_numpy(a).to(dev)  # noqa: E731
        one.set_state(t(u), t(u), t(u2))
        r1 = one.residual().cpu().numpy()
        j1 = one.jacobian_apply(t(v)).cpu().numpy()
        one.close()
        e = max(np.abs(R - r1).max() / np.abs(r1).max(), np.abs(J - j1).max() / np.abs(j1).max())
        err[0] = e if np.isfinite(e) else np.inf  # a DoF no rank owns leaves a NaN
    if args.dist_backend == "nccl":
        err = err.to(dev)
    dist.broadcast(err, 0)
    dp.ctx.close()
    return float(err.item())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--workload", default="cavity", choices=["cavity", "cylinder3d", "taylorcouette3d", "octree"],
                    help="cavity: the BASELINE metric (configs[1] / [2]); cylinder3d: configs[4]'s adaptive-path "
                         "problem on one GPU (per-cell mapped kernels + ILU-GMRES)")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--cells", dest="n", type=int, default=128, help="cells per direction")
    ap.add_argument("--k", type=int, default=2)
    ap.add_argument("--kp", type=int, default=2)
    ap.add_argument("--nu", type=float, default=0.01)
    ap.add_argument("--scheme", default="bdf2", choices=["bdf2", "steady"],
                    help="bdf2 (configs[2], the metric) or steady (configs[1]: Q1 64^3, nu = 1)")
    ap.add_argument("--dt", type=float, default=0.01)
    ap.add_argument("--lin-max", type=int, default=200)
    ap.add_argument("--restart", type=int, default=30)
    ap.add_argument("--ilu-fill", type=int, default=0, help="cylinder3d: ILU level of fill (0: multicolor order)")
    ap.add_argument("--cyl-refine", type=int, default=0, help="cylinder3d: global refinements of the mesh")
    ap.add_argument("--cyl-precond", default="ilu", choices=["ilu", "hmg"],
                    help="cylinder3d: ILU(fill) or the multigrid on the refinement hierarchy (needs --cyl-refine)")
    ap.add_argument("--oct-smoother", default="jacobi", choices=["jacobi", "ilu", "ilu-coarse"],
                    help="octree --precond mg: level smoother (damped Jacobi with FP32 brick J.v, or multicolor ILU(0))")
    ap.add_argument("--cyl-smoother", default="ilu", choices=["ilu", "jacobi", "ilu-coarse"],
                    help="cylinder3d --cyl-precond hmg: level smoother (ILU(0) V(1,1) or damped Jacobi V(2,2))")
    ap.add_argument("--mg-coarse-sweeps-cyl", type=int, default=10,
                    help="cylinder3d --cyl-precond hmg: ILU sweeps on the base (coarsest) mesh")
    ap.add_argument("--cyl-plevel", type=int, default=1,
                    help="cylinder3d / taylorcouette3d --cyl-precond hmg: 1 = a Q1-Q1 p-level below the base mesh "
                         "(gls_fe_space_mg_transfer's p-level pair), solved by the dense LU")
    ap.add_argument("--cyl-sweeps", type=int, nargs=2, default=None, metavar=("PRE", "POST"),
                    help="--cyl-precond hmg: pre / post smoothing sweeps per level (default: ILU 0 1 on taylorcouette3d, "
                         "1 1 on cylinder3d; Jacobi 2 2)")
    ap.add_argument("--cyl-hp", type=int, default=0,
                    help="--cyl-precond hmg: 1 = p first (Q2-Q1 fine -> Q1-Q1 on the fine mesh -> the Q1-Q1 refinement "
                         "hierarchy, exact LU at the bottom)")
    ap.add_argument("--mg-omega-cyl", type=float, default=0.6, help="hmg: damped-Jacobi weight")
    ap.add_argument("--direct-max", type=int, default=40000,
                    help="hmg: the coarsest level is factored (dense LU) up to this many DoFs, else smoothed")
    ap.add_argument("--rel", type=float, default=1e-4)
    ap.add_argument("--octree-steps", type=int, default=3, help="octree: lid / edge refinement levels")
    ap.add_argument("--precond", default="mg", choices=["mg", "jacobi", "ilu"],
                    help="GMRES right preconditioner: geometric multigrid V-cycle (default) or Jacobi")
    ap.add_argument("--mg-coarsest", type=int, default=0,
                    help="cells per direction of the coarsest level (0: 2 on one GPU -- exact LU solve of its "
                         "500 DoFs --, 4 with Jacobi sweeps across ranks)")
    ap.add_argument("--mg-fine-sweeps", type=int, nargs=2, default=None, metavar=("PRE", "POST"),
                    help="sweeps on the finest level (default: --mg-smooth)")
    ap.add_argument("--mg-coarse-level-sweeps", type=int, default=2,
                    help="pre = post sweeps on the level above an exact coarsest solve")
    ap.add_argument("--mg-smooth", type=int, nargs=2, default=(1, 1), metavar=("PRE", "POST"),
                    help="damped-Jacobi sweeps before / after the coarse correction")
    ap.add_argument("--mg-omega", type=float, default=0.9)
    ap.add_argument("--mg-coarse-sweeps", type=int, default=100)
    ap.add_argument("--mg-coarse-omega", type=float, default=0.7, help="0 = --mg-omega")
    ap.add_argument("--mg-coarse-direct", type=int, default=0,
                    help="coarsest level: 0 auto (exact solve on one GPU when <= 2048 DoFs), 1 exact (LU above 2048), -1 Jacobi sweeps")
    ap.add_argument("--mg-operator", default="oseen", choices=["oseen", "newton"],
                    help="operator of the V-cycle's FP32 smoothing J.v: the Oseen (Picard) linearization (default; "
                         "gls_mg_params.smoother_operator = 1) or Newton's Jacobian; the outer GMRES operator is the "
                         "exact FP64 Jacobian either way")
    ap.add_argument("--mg-precision", default="f32", choices=["f32", "f64"],
                    help="arithmetic of the V-cycle's J.v (f32: FP32 linearization + FP32 sweeps; the outer "
                         "GMRES operator, Newton residual and all vectors stay FP64)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--cpu-full-1core", action="store_true", help="with --cpu-full: also the 1-thread Newton")
    ap.add_argument("--cpu-full", action="store_true",
                    help="cpu_baseline = a complete CPU Newton iteration on the full workload (the job threads; "
                         "minutes at configs[1]); default: the bounded extrapolated sample")
    ap.add_argument("--jv-reps", type=int, default=10, help="extra back-to-back J.v launches timed for the roofline")
    ap.add_argument("--no-pmc", action="store_true",
                    help="skip the live rocprofv3 --pmc traffic passes (roofline.traffic then replays the committed "
                         "summary, labelled)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl = RCCL over xGMI (default); gloo stages through the host (testing on one GPU)")
    ap.add_argument("--dist-impl", default="native", choices=["torch", "native"],
                    help="ghost exchange / reductions: the library's own RCCL communicator (default; gls_dist_attach_rccl: "
                         "ncclSend/ncclRecv/ncclAllReduce on the context stream, ghost import overlapped with the "
                         "interior bricks) or torch.distributed callbacks (host-synchronous; the gloo tests)")
    args = ap.parse_args()
    # GLS_BENCH_FAIL_NATIVE_PREFLIGHT (test hooks): "1" -- the native transport's pre-flight raises on every rank
    # before its first collective, so the fallback to the torch.distributed transport runs (on one GPU with gloo);
    # "late<r>" -- rank r raises after the first collective, so the run aborts instead of falling back
    fail_env = os.environ.get("GLS_BENCH_FAIL_NATIVE_PREFLIGHT", "")
    fail_native = fail_env == "1" or fail_env.startswith("late")
    if args.dist_backend == "gloo" and not fail_native:  # host-staged testing transport: no RCCL communicator
        args.dist_impl = "torch"
    env_world = os.environ.get("WORLD_SIZE")
    if args.gpus < 1:
        sys.exit("bench.py: --gpus must be >= 1")
    if env_world is not None and int(env_world) != args.gpus:
        sys.stderr.write("bench.py: WORLD_SIZE=%s but --gpus %d: launch one rank per GPU (torch.distributed.run "
                         "--nproc-per-node %d ... --gpus %d) or run without a launcher\n"
                         % (env_world, args.gpus, args.gpus, args.gpus))
        sys.exit(1)
    if env_world is None and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus))
    if args.workload in ("cylinder3d", "taylorcouette3d", "octree") and args.gpus > 1:
        sys.exit("bench.py: --workload %s runs on one GPU" % args.workload)
    if args.workload in ("cylinder3d", "taylorcouette3d", "octree"):
        import torch
        torch.cuda.set_device(0)
        return bench_octree(args) if args.workload == "octree" else bench_cylinder3d(args)

    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0")) % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")

    def barrier():
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()

    devices, rccl_ranks, pre_err = 1, None, None
    if dist is not None:
        props = torch.cuda.get_device_properties(local)
        ids = [None] * world
        dist.all_gather_object(ids, str(getattr(props, "uuid", None) or "%s:%d" % (os.uname().nodename, local)))
        devices = len(set(ids))
        from datetime import timedelta
        ctl = dist.new_group(backend="gloo", timeout=timedelta(seconds=180))  # control plane of the pre-flight
        stage = {"s": "local"}
        try:
            if fail_env == "1" and args.dist_impl == "native":
                raise RuntimeError("GLS_BENCH_FAIL_NATIVE_PREFLIGHT")
            pre_err = preflight(args, rank, world, torch.device("cuda", local), dist, stage)
            failed = not pre_err <= 1e-12
        except Exception as e:  # noqa: BLE001 -- reported, and the ranks agree on it below
            sys.stderr.write("bench.py: rank %d pre-flight with the %s transport raised (%s stage): %r\n"
                             % (rank, args.dist_impl, stage["s"], e))
            pre_err, failed = float("nan"), True
        verdict = preflight_agreement(dist, ctl, world, failed, stage["s"] == "collective" and pre_err != pre_err)
        if verdict == "abort":
            sys.stderr.write("bench.py: rank %d: pre-flight failed after the transport's first collective; no fallback "
                             "(a peer may be inside a collective)\n" % rank)
            sys.stderr.flush()
            os._exit(4)
        if verdict == "fallback" and args.dist_impl == "native":
            from softx_2020_200_amd.dist import drop_rccl
            drop_rccl()
            # the in-library RCCL transport failed its check on some rank: the timed run takes torch.distributed's
            # RCCL (callbacks) instead, after the same pre-flight, and the line says so
            if rank == 0:
                sys.stderr.write("bench.py: in-library RCCL pre-flight failed (%s); falling back to the torch.distributed "
                                 "transport\n" % pre_err)
            args.dist_impl, args.dist_impl_fallback = "torch", "native pre-flight failed (%s)" % pre_err
            pre_err = preflight(args, rank, world, torch.device("cuda", local), dist)
        if not pre_err <= 1e-12:
            if rank == 0:
                sys.stderr.write("bench.py: pre-flight FAILED: %d-rank residual / J.v differ from one rank by %.3e "
                                 "(16^3 cavity, %s transport)\n" % (world, pre_err, args.dist_impl))
            dist.destroy_process_group()
            sys.exit(3)
        if args.dist_impl == "native":
            from softx_2020_200_amd.dist import rccl_comm, rccl_info
            rccl_ranks = rccl_info(rccl_comm(rank, world))[1]

    from softx_2020_200_amd.problem import CavityProblem
    if args.mg_coarsest == 0:
        args.mg_coarsest = 2
    # N > 1 with the exact coarsest solve: the distributed levels stop at 4^3 (whole bricks per rank), and
    # below them every rank runs the one-GPU cycle's remainder on a replica of the 4^3 level (2 + 2
    # sweeps, exact LU on 2^3; gls_mg_set_coarse_replica): the same V-cycle as N = 1
    replica = world > 1 and args.precond == "mg" and args.mg_coarsest == 2 and args.mg_coarse_direct >= 0
    lsweeps = {-2: (args.mg_coarse_level_sweeps,) * 2} if world == 1 and args.mg_coarse_direct >= 0 else {}
    if args.mg_fine_sweeps:
        lsweeps[0] = tuple(args.mg_fine_sweeps)
    t_setup = time.perf_counter()
    dev = torch.device("cuda", local)
    ts = (args.dt,) * 4
    if world == 1:
        prob = CavityProblem(dim=3, n=args.n, k=args.k, kp=args.kp, viscosity=args.nu,
                             multigrid=args.precond == "mg", mg_coarsest=args.mg_coarsest,
                             pre_smooth=args.mg_smooth[0], post_smooth=args.mg_smooth[1], omega=args.mg_omega,
                             coarse_sweeps=args.mg_coarse_sweeps, coarse_omega=args.mg_coarse_omega,
                             mixed_precision=args.mg_precision == "f32", coarse_direct=args.mg_coarse_direct,
                             level_sweeps=lsweeps, smoother_operator=int(args.mg_operator == "oseen"))
        ctx = prob.ctx
        mesh = prob.mesh
        N = N_global = ctx.n_dofs
        m1_h = smooth_state(prob.mesh, args.n, 3, prob.dir_dofs, prob.dir_vals, 0.0)
        m2_h = smooth_state(prob.mesh, args.n, 3, prob.dir_dofs, prob.dir_vals, 0.3)
    else:
        import softx_2020_200_amd as sx
        from softx_2020_200_amd.dist import DistributedProblem, local_vector
        from softx_2020_200_amd.problem import dirichlet_from_bcs
        mesh = sx.hyper_cube(3, args.n, args.k, args.kp, -1.0, 1.0)
        bcs = [("noslip", b, None) for b in (0, 1, 2, 4, 5)] + [("function", 3, (1.0, 0.0, 0.0))]
        mask, ddofs, dvals = dirichlet_from_bcs(mesh, args.n, -1.0, 1.0, True, bcs)
        dp = DistributedProblem(mesh, rank, world, dev, viscosity=args.nu, vnode_mask=mask, dirichlet=(ddofs, dvals),
                                backend=args.dist_backend, impl=args.dist_impl)
        ctx = dp.ctx
        if args.precond == "mg":  # the same V-cycle on nested per-rank boxes (RCCL ghosts per level)
            from softx_2020_200_amd.dist import attach_distributed_multigrid, multigrid_levels
            lv, m_last = [dp], args.n
            for m in multigrid_levels(args.n, world, 4 if replica else args.mg_coarsest):
                m_last = m
                mm = sx.hyper_cube(3, m, args.k, args.kp, -1.0, 1.0)
                mk, dd, dv = dirichlet_from_bcs(mm, m, -1.0, 1.0, True, bcs)
                lv.append(DistributedProblem(mm, rank, world, dev, viscosity=args.nu, vnode_mask=mk,
                                             dirichlet=(dd, dv), backend=args.dist_backend, impl=args.dist_impl))
            rep = None
            if replica:  # the 4^3 level's whole mesh on every rank, with the one-GPU cycle below it
                rep = CavityProblem(dim=3, n=m_last, k=args.k,
                                    kp=args.kp, viscosity=args.nu, multigrid=True, mg_coarsest=2,
                                    pre_smooth=args.mg_coarse_level_sweeps, post_smooth=args.mg_coarse_level_sweeps,
                                    omega=args.mg_omega, coarse_sweeps=args.mg_coarse_sweeps,
                                    coarse_omega=args.mg_coarse_omega, mixed_precision=args.mg_precision == "f32",
                                    coarse_direct=args.mg_coarse_direct,
                                    smoother_operator=int(args.mg_operator == "oseen"))
            attach_distributed_multigrid(lv, replica=rep, pre_smooth=args.mg_smooth[0], post_smooth=args.mg_smooth[1],
                                         omega=args.mg_omega, coarse_sweeps=args.mg_coarse_sweeps,
                                         coarse_omega=args.mg_coarse_omega,
                                         mixed_precision=args.mg_precision == "f32",
                                         coarse_direct=-1 if replica else args.mg_coarse_direct,
                                         smoother_operator=int(args.mg_operator == "oseen"))
        N = ctx.n_dofs
        N_global = 3 * mesh["n_vnodes"] + mesh["n_pnodes"]
        m1_h = local_vector(dp.plan, smooth_state(mesh, args.n, 3, ddofs, dvals, 0.0), mesh["n_vnodes"])
        m2_h = local_vector(dp.plan, smooth_state(mesh, args.n, 3, ddofs, dvals, 0.3), mesh["n_vnodes"])
    ctx.set_time(args.scheme, ts)
    if dist is not None:
        dist.barrier()  # first collective before any batched P2P (NCCL requirement)
    m1 = torch.from_numpy(m1_h).to(dev)
    m2 = torch.from_numpy(m2_h).to(dev)
    del m1_h, m2_h
    present = m1.clone()
    t_setup = time.perf_counter() - t_setup

    def one_step():
        present.copy_(m1)
        return ctx.newton(present, m1, m2, tolerance=1e-30, max_iterations=1, lin_max_iterations=args.lin_max,
                          restart=args.restart, relative_residual=args.rel, minimum_residual=1e-14)

    for _ in range(args.warmup):
        one_step()
    barrier()
    t0 = time.perf_counter()
    stats = [one_step() for _ in range(args.steps)]  # per-launch event timing off in the timed region
    barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    # per-kernel breakdown: one extra, instrumented step (HIP events around every launch)
    ctx.timing(True)
    tb0 = time.perf_counter()
    one_step()
    torch.cuda.synchronize()
    elapsed_instr = time.perf_counter() - tb0
    jv_ms, jv_n = ctx.timing_get(1)
    res_ms, res_n = ctx.timing_get(0)
    dg_ms, dg_n = ctx.timing_get(2)
    lin_ms, lin_n = ctx.timing_get(3)
    f32_ms, f32_n = ctx.timing_get(4)
    sl_ms, sl_n = ctx.timing_get(5)
    ctx.timing(False)
    # dedicated back-to-back J.v launches on the same state for a clean per-launch duration
    ctx.set_state(present, m1, m2)
    v = torch.rand(N, dtype=torch.float64, device=dev)
    y = torch.empty_like(v)
    ctx.jacobian_apply(v, y)
    ctx.timing(True)
    for _ in range(args.jv_reps):
        ctx.jacobian_apply(v, y)
    jv2_ms, jv2_n = ctx.timing_get(1)
    sl2_ms, sl2_n = ctx.timing_get(5)
    ctx.timing(False)

    t_max = elapsed
    if dist is not None:
        tt = torch.tensor([elapsed], dtype=torch.float64)
        tt = tt.to(dev) if args.dist_backend == "nccl" else tt
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        t_max = float(tt.item())

    lin_its = [s["linear_iterations"] for s in stats]
    nres = [s["residual_evaluations"] for s in stats]
    its_per_s = args.steps / t_max  # the whole job advances one Newton iteration per step
    n_cells = mesh["n_cells"]
    nv = mesh["n_vnodes"]
    nvdofs = 3 * nv
    # algorithmic bytes of one J.v launch (this build's layout): v, Jv, u (8N each),
    # 2 history velocity vectors (BDF2), cell->node int32 indices, per-cell geometry (4 doubles),
    # velocity constraint mask (1 B/node)
    nvl = (args.k + 1) ** 3
    n_cells_rank = n_cells // world
    nv_rank = (N // 4) if world > 1 else nv
    k_hist = 2 if args.scheme == "bdf2" else 0  # history vectors the scheme reads
    B_jv = 8 * N * 3 + 8 * k_hist * 3 * nv_rank + 4 * n_cells_rank * nvl * (1 if args.kp == args.k else 2) + \
        32 * n_cells_rank + nv_rank
    jv_launch_ms = jv2_ms / max(jv2_n, 1)
    # the brick kernel writes per-brick surface slabs; the deterministic node sum (k_slab_sum) that
    # turns them into y is part of the same J.v, so its time is charged to the J.v's bytes too
    slab_launch_ms = sl2_ms / max(jv2_n, 1)
    op_ms = jv_launch_ms + slab_launch_ms
    achieved = B_jv / (op_ms * 1e-3) / 1e9
    pencil = os.environ.get("GLS_PENCIL", "1") != "0"
    pencil_jv = pencil and args.k == 2  # the Q2 brick J.v runs in the pencil dataflow (gls_brick_pencil.hip)
    # dense-contraction FLOP count of the kernel as written (per cell, Q2-Q2 3D): see DESIGN.md §4
    out = {
        "metric": "nonlinear iters/sec (3D cavity Q%d %d^3 %s)" % (args.k, args.n, args.scheme.upper()),
        "value": its_per_s,
        "unit": "nonlinear_iters/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": 1e3 * t_max / args.steps,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (smooth cavity-like %s, lid/wall Dirichlet values)" % (
            "BDF2 history" if args.scheme == "bdf2" else "state"),
        "config": {"workload": "3D lid-driven cavity Q%d-Q%d %d^3 %s%s"
                               % (args.k, args.kp, args.n, "transient BDF2" if args.scheme == "bdf2" else "steady",
                                  {(2, 128, "bdf2"): " (BASELINE configs[2])",
                                   (1, 64, "steady"): " (BASELINE configs[1])"}.get((args.k, args.n, args.scheme), "")),
                   "n_dofs": N_global, "n_cells": n_cells, "viscosity": args.nu, "dt": args.dt,
                   "linear_solver": "GMRES(%d)+%s, rel %.0e, max %d" % (
                       args.restart, "GMG V(%d,%d)-cycle to %d^3 (%s; %s %s smoothing J.v)" % (
                           tuple(args.mg_smooth) + (args.mg_coarsest, "exact LU" if (-2 in lsweeps or replica)
                                                    else "%d Jacobi sweeps" % args.mg_coarse_sweeps,
                                                    args.mg_precision.upper(),
                                                    "Oseen" if args.mg_operator == "oseen" else "Newton"))
                       if args.precond == "mg" else "Jacobi",
                       args.rel, args.lin_max),
                   "parallelism": ("domain decomposition x%d (%s)" % (world, "in-library RCCL P2P ghosts" if args.dist_impl == "native"
                                                                     else "torch.distributed %s ghosts" % args.dist_backend))
                   if world > 1 else "single"},
        "mdof_per_s": N_global * its_per_s / 1e6,
        "devices": devices, "rccl_ranks": rccl_ranks, "preflight_relerr": pre_err,
        "dist_impl": args.dist_impl if world > 1 else None,
        "dist_impl_fallback": getattr(args, "dist_impl_fallback", None),
        "linear_iterations_per_step": float(np.mean(lin_its)),
        "residual_evaluations_per_step": float(np.mean(nres)),
        "kernel_ms": {"jacobian_apply": jv_ms / max(jv_n, 1), "residual": res_ms / max(res_n, 1),
                      "diagonal": dg_ms / max(dg_n, 1), "jv_linearization": lin_ms / max(lin_n, 1),
                      "smoother_jv_f32": f32_ms / max(f32_n, 1), "slab_sum": sl_ms / max(sl_n, 1),
                      "source": "one extra instrumented step after the timed region (HIP events per launch)",
                      "note": ("diagonal = the Newton step's fused residual + linearization + Jacobian-diagonal launch "
                               "(assemble_matrix_and_rhs, gls_residual_and_diagonal); residual = the line search's"
                               if pencil_jv and world == 1 else ""),
                      "instrumented_step_ms": 1e3 * elapsed_instr,
                      "launches_per_step": {"jacobian_apply": jv_n, "residual": res_n, "diagonal": dg_n,
                                            "jv_linearization": lin_n, "smoother_jv_f32": f32_n, "slab_sum": sl_n},
                      "share_of_step": {"jacobian_apply": jv_ms / (1e3 * elapsed_instr),
                                        "residual": res_ms / (1e3 * elapsed_instr),
                                        "diagonal": dg_ms / (1e3 * elapsed_instr),
                                        "jv_linearization": lin_ms / (1e3 * elapsed_instr),
                                        "smoother_jv_f32": f32_ms / (1e3 * elapsed_instr),
                                        "slab_sum": sl_ms / (1e3 * elapsed_instr)}},
        "roofline": {"bound": "hbm", "kernel": ("gls_pencil_kernel<double,MODE_JVQ> + slab sum" if pencil_jv else
                                                "gls_brick_kernel<%d,MODE_JVQ> + k_slab_sum" % args.k) if ctx.uses_brick_kernels
                     else cell_jv_kernel_name(args.kp) if args.k == 2
                     else "gls_cell_kernel<3,%d,%d,%d,MODE_JV>" % (args.k, args.kp, args.k + 1), "achieved": achieved,
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                     "traffic": None, "algorithmic_bytes_per_launch": B_jv, "launch_ms": op_ms,
                     "launch_ms_by_kernel": {"gls_pencil_kernel" if pencil_jv else "gls_brick_kernel": jv_launch_ms,
                                             "k_slab_sum": slab_launch_ms}},
        "setup_s": t_setup,
    }
    # the whole Newton iteration against the HBM roof: algorithmic bytes of every operator / vector pass of the
    # step (model, step_bytes_model) over the measured step time
    if world == 1 and ctx.uses_brick_kernels and args.precond == "mg" and args.scheme == "bdf2":
        bs, parts = step_bytes_model(args.n, args.k, float(np.mean(lin_its)), float(np.mean(nres)) - 1.0, f32_n)
        ach = bs / (t_max / args.steps) / 1e9
        out["step_roofline"] = {"bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                "frac": ach / HBM_PEAK_GBS, "algorithmic_bytes_per_step": bs,
                                "bytes_by_part": parts, "ms_per_step": 1e3 * t_max / args.steps,
                                "model": "SURVEY §8d per-operator formulas x the step's measured counts (GMRES "
                                         "iterations, line-search residuals, fine smoother launches); kernel time "
                                         "and PMC bytes per class: profiles/r05_step_budget.txt"}
    # measured HBM traffic of the same kernel: live PMC passes (child rocprofv3 runs over tools/jv_bench.py),
    # else the committed summary, labelled as replayed
    tr, tr_src = None, None
    if world == 1 and args.n == 128 and args.k == 2 and args.kp == 2 and ctx.uses_brick_kernels and pencil:
        if not args.no_pmc:
            try:
                del v, y
                torch.cuda.empty_cache()
                tr = live_pmc_traffic(args.n, args.k, N_global)
                tr_src = ("MEASURED in this run: rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE (separate passes) over "
                          "tools/jv_bench.py %d, FETCH_SIZE x %.2f + WRITE_SIZE x %.2f (k_copy calibration of the same "
                          "run)" % (args.n, tr[1], tr[2]))
            except Exception as e:  # noqa: BLE001 (report, fall back)
                tr_src = "live PMC failed (%s: %s); " % (type(e).__name__, str(e)[:120])
        if tr is None:
            tr = pmc_traffic(os.path.join(ROOT, "profiles", PMC_TRAFFIC_FILE), 4, N_global)
            if tr is not None:
                tr_src = (tr_src or "") + ("REPLAYED from the committed profiles/%s (FETCH_SIZE x %.2f + WRITE_SIZE x "
                                           "%.2f), not measured in this run" % (PMC_TRAFFIC_FILE, tr[1], tr[2]))
    model_path = os.path.join(ROOT, "profiles", LDS_MODEL_FILE)
    if world == 1 and args.k == 2 and args.kp == 2 and ctx.uses_brick_kernels and pencil and os.path.exists(model_path):
        # the LDS and VALU issue floors of the pencil J.v from a STATIC model of its compiled instruction
        # stream (tools/lds_model.py: LDS instructions priced conflict-free by MI355X_MICROARCH.md §LDS,
        # FP64 VALU at 4 cycles per wave instruction), not a measurement; the commit it was derived from
        # is in the file
        import hashlib
        mdl = json.load(open(model_path))
        src = os.path.join(ROOT, mdl.get("source", "softx_2020_200_amd/csrc/gls_brick_pencil.hip"))
        stale = mdl.get("source_sha256") != hashlib.sha256(open(src, "rb").read()).hexdigest()
        km = next(v for k_, v in mdl["kernels"].items() if "gls_pencil_kernelIdLi4ELb0" in k_)
        waves_per_cu = -(-(n_cells // 8) // 3) * 4 / 256
        lds_ms = waves_per_cu * km["lds_cycles_per_wave"] / 2.4e9 * 1e3  # the CU's LDS pipe at 2400 MHz
        valu_ms = waves_per_cu / 4 * (4 * km["valu_f64"] + 2 * km["valu_other"]) / 2.4e9 * 1e3  # per SIMD
        out["roofline"]["lds"] = {"kernel": "gls_pencil_kernel<double,MODE_JVQ>", "model": "static",
                                  "lds_cycles_per_wave": km["lds_cycles_per_wave"], "waves_per_cu": waves_per_cu,
                                  "floor_ms_at_2400MHz": lds_ms, "valu_floor_ms_at_2400MHz": valu_ms,
                                  "launch_ms": jv_launch_ms, "frac": lds_ms / jv_launch_ms,
                                  "source": "profiles/%s (%s)" % (LDS_MODEL_FILE, mdl.get("commit")),
                                  "stale": stale,
                                  "stale_note": "the kernel source changed since the model was made: rerun "
                                                "tools/lds_model.py" if stale else "model made from this source"}
    if tr is not None:
        out["roofline"]["traffic"] = tr[0]
        out["roofline"]["traffic_source"] = (tr_src + "; includes the per-quadrature-point linearization stream "
                                             "(16 doubles/q) the cached J.v reads instead of re-deriving u, grad u, "
                                             "tau, R_s")
    elif tr_src:
        out["roofline"]["traffic_source"] = tr_src
    if rank == 0 and world == 1 and not args.no_cpu and args.cpu_full:
        # the reference's CPU path measured end to end on this very workload (1 Newton iteration)
        threads, cores_note = cpu_threads()
        full = cpu_newton(args.k, args.kp, args.n, args.nu, args.scheme, args.dt, threads)
        # the 1-thread leg only on request (--cpu-full-1core): at Q1 64^3 it is ~5 min of host time
        full1 = cpu_newton(args.k, args.kp, args.n, args.nu, args.scheme, args.dt, 1) if args.cpu_full_1core else None
        out["cpu_baseline"] = {
            "value": 1.0 / full["seconds"], "unit": "nonlinear_iters/s", "cores": threads, "cores_note": cores_note,
            "kind": "port",
            "value_1core": 1.0 / full1["seconds"] if full1 else None, "cpu": _cpu_model(), "host_cpus_visible": os.cpu_count(),
            "affinity": len(os.sched_getaffinity(0)),
            "sample": ("MEASURED: one complete Newton iteration of the reference's CPU path on the full workload "
                       "(%d DoFs, same synthetic state): oracle/gls_oracle.c assembly of the CSR system (%d nnz) on %d "
                       "OpenMP threads, ILU(0) setup, GMRES(30)+ILU(0) to rel 1e-4 (%d iterations), alpha line "
                       "search (%d residual); sparsity pattern (setup_dofs) %.1f s not counted"
                       % (full["n_dofs"], full["nnz"], threads, full["gmres_its"], full["line_search_rhs"],
                          full["t_pattern"])),
            "seconds_per_iter": {key: full[key] for key in ("t_assemble", "t_ilu", "t_gmres", "t_linesearch", "seconds")},
            "seconds_per_iter_1core": {key: full1[key] for key in ("t_assemble", "t_ilu", "t_gmres", "t_linesearch",
                                                                   "seconds")} if full1 else None,
        }
    elif rank == 0 and world == 1 and not args.no_cpu:
        # the OpenMP threads this process may use (OMP_NUM_THREADS; on the GPU box the job's CPU share)
        threads, cores_note = cpu_threads()
        cb = cpu_baseline(args.k, args.kp, args.nu, args.cpu_seconds, threads)
        per_cell = {key: cb[key][1] / cb[key][0] for key in ("matrix", "rhs", "matrix_1core", "rhs_1core")}
        L_ = float(np.mean(nres)) - 1.0    # line-search residuals per Newton step (GPU run's count)
        m_ = float(np.mean(lin_its))       # GMRES iterations per Newton step (GPU run's count)
        nnz_s, n_s, t_spmv_s = cb["spmv"]
        nnz_full = nnz_s / n_s * N_global  # same stencil per row (boundary rows make it a lower bound)
        t_spmv = t_spmv_s * nnz_full / nnz_s / threads   # SpMV scaled linearly over the threads (upper bound on the rate)
        t_prec = t_spmv                    # ILU(0) forward + backward substitution ~ one SpMV (ILU setup excluded)
        t_orth = sum(2 * (j + 2) for j in range(int(round(m_)))) * 8.0 * N_global / (cb["copy_gbs"] * 1e9)
        def t_iter(pc, spmv_scale=1.0):
            return n_cells * (pc[0] + L_ * pc[1]) + m_ * (t_spmv + t_prec) * spmv_scale + t_orth
        t_all = t_iter((per_cell["matrix"], per_cell["rhs"]))
        t_one = t_iter((per_cell["matrix_1core"], per_cell["rhs_1core"]), spmv_scale=threads)
        out["cpu_baseline"] = {
            "value": 1.0 / t_all, "unit": "nonlinear_iters/s", "cores": threads, "cores_note": cores_note, "kind": "port",
            "value_1core": 1.0 / t_one,
            "cpu": _cpu_model(), "host_cpus_visible": os.cpu_count(), "affinity": len(os.sched_getaffinity(0)),
            "sample": ("EXTRAPOLATED from measured samples to one Newton step of the GPU run (m = %.1f GMRES its, "
                       "L = %.1f line-search residuals) on %d Q%d-Q%d cells: oracle/gls_oracle.c with reference-cell "
                       "tables (FEValues-style) -- element matrix+rhs %d cells in %.1f s, rhs-only %d cells in %.1f s "
                       "(%d OpenMP threads; 1 thread: %d / %d cells in %.1f / %.1f s); CSR SpMV %.0f nnz (Q2 10^3 "
                       "cavity, scipy, 1 thread) in %.3f s scaled to %.3g nnz and %d threads; ILU(0) apply = 1 SpMV; "
                       "GMRES orthogonalisation at %.1f GB/s host copy bandwidth; ILU setup and sparsity-pattern "
                       "setup excluded (the reference's CSR for this size, ~%.0f GB, cannot be formed here)"
                       % (m_, L_, n_cells, args.k, args.kp, cb["matrix"][0], cb["matrix"][1], cb["rhs"][0], cb["rhs"][1],
                          threads, cb["matrix_1core"][0], cb["rhs_1core"][0], cb["matrix_1core"][1], cb["rhs_1core"][1],
                          nnz_s, t_spmv_s, nnz_full, threads, cb["copy_gbs"], nnz_full * 12 / 1e9)),
            "seconds_per_iter": {"assembly_matrix": n_cells * per_cell["matrix"], "assembly_rhs": n_cells * L_ * per_cell["rhs"],
                                 "spmv_and_ilu_apply": m_ * (t_spmv + t_prec), "orthogonalisation": t_orth,
                                 "total": t_all, "total_1core": t_one},
        }
        # cross-check: a complete CPU Newton iteration measured end to end on a smaller cube
        ns_ = 12 if args.k == 2 else 32
        sm = cpu_newton(args.k, args.kp, ns_, args.nu, args.scheme, args.dt, threads)
        out["cpu_baseline"]["measured_newton_small"] = {
            "cells": "%d^3" % ns_, "n_dofs": sm["n_dofs"], "seconds": sm["seconds"], "gmres_its": sm["gmres_its"],
            "threads": threads, "mdof_per_s": sm["n_dofs"] / sm["seconds"] / 1e6,
            "note": "complete Newton iteration (CSR assembly, ILU(0), GMRES(30)+ILU(0) to rel 1e-4, line search), measured; "
                    "its Mdof/s exceeds what the full size reaches (GMRES iterations grow with the mesh)"}
    if rank == 0:
        print(json.dumps(out))
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
