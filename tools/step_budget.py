"""Per-Newton-step budget of the configs[2] bench by kernel class (tooling, not product code).

Inputs: a rocprofv3 --kernel-trace CSV of `bench.py` (Q2-Q2 n^3 BDF2) and, optionally, the counter CSVs of two
separate `rocprofv3 --pmc FETCH_SIZE` / `--pmc WRITE_SIZE` runs of `bench.py --steps 1 --warmup 0`.
A Newton step starts at the fused residual + linearization + diagonal launch (gls_pencil_kernel<double, 5>,
assemble_matrix_and_rhs); the budget is taken over the last complete step before the final one (the
bench's instrumented step) in each file.

Per class: launches, ms, ALGORITHMIC bytes (the SURVEY §8d operator formulas at the launch's level size:
B_Jv for every J.v -- FP64 outer operator and FP32 smoother, the slab sums folded into their J.v --,
B_res (+ 8N for the diagonal) for the residual launches, (M+1) / (M+2) vectors for the Gram-Schmidt
multi-dot / multi-axpy passes; transfers, injections and vector updates at their vectors' sizes) and the
PMC bytes (FETCH_SIZE x 2 and WRITE_SIZE x 1: gfx950's half-counted streaming reads, MI355X_MICROARCH.md
"HBM", the k_copy calibration of profiles/r04_pmc_traffic_pencil_128_final2.txt).

Usage: python tools/step_budget.py TRACE_CSV [FETCH_CSV WRITE_CSV] [--n 128] [--json OUT]"""
import argparse
import collections
import csv
import json
import math
import re

FETCH_CORR, WRITE_CORR = 2.0, 1.0


def level_of_cells(cells):
    return int(round(cells ** (1.0 / 3.0)))


def sizes(n):
    nv = (2 * n + 1) ** 3
    return dict(n=n, cells=n ** 3, nv=nv, N=4 * nv)


def b_jv(n, k_hist=2):
    s = sizes(n)
    return 8 * s["N"] * 3 + 8 * k_hist * 3 * s["nv"] + 4 * s["cells"] * 27 + 32 * s["cells"] + s["nv"]


def b_res(n, k_hist=2):
    s = sizes(n)
    return 8 * s["N"] * 2 + 8 * k_hist * 3 * s["nv"] + 4 * s["cells"] * 27 + 32 * s["cells"]


def classify(name, blocks, threads, n_fine):
    """(class, level n, algorithmic bytes) of one launch"""
    nm = name.replace("(anonymous namespace)::", "")
    Nf = sizes(n_fine)["N"]
    if "gls_pencil_kernel" in nm or "gls_pencil_pair_kernel" in nm or "gls_brick_kernel" in nm:
        pair = "pair_kernel" in nm
        cells = blocks * 24  # 3 bricks per workgroup (both pencil kernels)
        n = level_of_cells(cells)
        while n > 1 and n ** 3 > cells:
            n -= 1
        n = 2 ** int(round(math.log2(max(n, 1))))
        if "<double, 5" in nm:
            return "RESLIN (residual + linearization + diagonal)", n, b_res(n) + 8 * sizes(n)["N"]
        if "<double, 0" in nm:
            return "residual (line search)", n, b_res(n)
        if "<double, 3" in nm:
            return "linearization + diagonal (coarse levels)", n, b_res(n) + 8 * sizes(n)["N"]
        if "<double, 4" in nm:
            return ("J.v FP64 (GMRES operator)" if n == n_fine else "J.v FP64 (other level)"), n, b_jv(n)
        if "<float, 4" in nm or pair:
            return ("smoother J.v FP32 fine" if n == n_fine else "smoother J.v FP32 coarse levels"), n, b_jv(n)
        return "brick kernel (other)", n, 0
    if "k_slab_sum" in nm:
        return "slab sums", None, 0  # folded into their J.v's algorithmic bytes (the J.v's y write)
    m = re.search(r"k_multidot(?:16)?<(\d+)", nm)
    if m:
        return "GMRES orthogonalisation", None, (int(m.group(1)) + 1) * 8 * Nf
    m = re.search(r"k_multiaxpy(?:_dot)?(?:16)?<(\d+)", nm)
    if m:
        return "GMRES orthogonalisation", None, (int(m.group(1)) + 2) * 8 * Nf
    if "transfer" in nm or "k_inject" in nm or "box" in nm:
        return "MG transfers", None, None
    if "jacobi" in nm:
        return "MG Jacobi updates", None, None
    if "rocsolver" in nm or "rocblas" in nm or "Cijk" in nm or "gemv" in nm:
        return "coarse LU (rocSOLVER / rocBLAS)", None, None
    return "vector ops / misc", None, None


def step_window(rows, key):
    starts = [i for i, r in enumerate(rows) if "gls_pencil_kernel<double, 5" in r["Kernel_Name"]]
    if len(starts) < 2:
        raise SystemExit("need two RESLIN launches in %s" % key)
    return starts[-2], starts[-1]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("pmc", nargs="*")
    ap.add_argument("--n", type=int, default=128)
    ap.add_argument("--json")
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
    i0, i1 = step_window(rows, a.trace)
    t_step = (int(rows[i1]["Start_Timestamp"]) - int(rows[i0]["Start_Timestamp"])) * 1e-6
    cls = collections.OrderedDict()
    busy = 0.0
    for r in rows[i0:i1]:
        blocks = int(r["Grid_Size_X"]) // max(int(r["Workgroup_Size_X"]), 1)
        c, _, b = classify(r["Kernel_Name"], blocks, int(r["Workgroup_Size_X"]), a.n)
        d = cls.setdefault(c, dict(launches=0, ms=0.0, alg_bytes=0.0, alg_known=True, pmc_bytes=0.0))
        d["launches"] += 1
        t = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6
        d["ms"] += t
        busy += t
        if b is None:
            d["alg_known"] = False
        else:
            d["alg_bytes"] += b
    # PMC: FETCH_SIZE / WRITE_SIZE per dispatch (KB), same step window in dispatch order
    for path in a.pmc:
        prow = [r for r in csv.DictReader(open(path))]
        ctr = prow[0]["Counter_Name"]
        corr = FETCH_CORR if "FETCH" in ctr else WRITE_CORR
        prow.sort(key=lambda r: int(r["Dispatch_Id"]))
        j0, j1 = step_window(prow, path)
        for r in prow[j0:j1]:
            blocks = int(r["Grid_Size"]) // max(int(r["Workgroup_Size"]), 1)
            c, _, _ = classify(r["Kernel_Name"], blocks, int(r["Workgroup_Size"]), a.n)
            if c in cls:
                cls[c]["pmc_bytes"] += float(r["Counter_Value"]) * 1024.0 * corr
    for d in cls.values():  # unmodelled small kernels: their PMC bytes stand in for the algorithmic ones
        if not d["alg_known"]:
            d["alg_bytes"] = d["pmc_bytes"] if a.pmc else 0.0
    tot_alg = sum(d["alg_bytes"] for d in cls.values())
    tot_pmc = sum(d["pmc_bytes"] for d in cls.values())
    print("Newton step (last complete one): %.2f ms wall, %.2f ms kernel busy" % (t_step, busy))
    print("%-48s %6s %9s %7s %10s %10s %9s %9s" % ("class", "launch", "ms", "share", "alg GB", "PMC GB", "alg TB/s",
                                                "PMC TB/s"))
    for c, d in sorted(cls.items(), key=lambda x: -x[1]["ms"]):
        print("%-48s %6d %9.3f %6.1f%% %10.3f %10.3f %9.2f %9.2f%s" % (
            c, d["launches"], d["ms"], 100 * d["ms"] / t_step, d["alg_bytes"] / 1e9, d["pmc_bytes"] / 1e9,
            d["alg_bytes"] / (d["ms"] * 1e-3) / 1e12 if d["ms"] else 0, d["pmc_bytes"] / (d["ms"] * 1e-3) / 1e12 if d["ms"] else 0,
            "" if d["alg_known"] else "  (alg = PMC)"))
    print("%-48s %6s %9.3f %7s %10.3f %10.3f %9.2f %9.2f" % ("TOTAL (step wall time)", "", t_step, "", tot_alg / 1e9, tot_pmc / 1e9,
                                                           tot_alg / (t_step * 1e-3) / 1e12, tot_pmc / (t_step * 1e-3) / 1e12))
    print("HBM roof fraction over the step: algorithmic %.3f, PMC %.3f (8 TB/s)" % (
        tot_alg / (t_step * 1e-3) / 8e12, tot_pmc / (t_step * 1e-3) / 8e12))
    if a.json:
        json.dump(dict(step_ms=t_step, busy_ms=busy, classes=cls, alg_bytes=tot_alg, pmc_bytes=tot_pmc,
                       frac_alg=tot_alg / (t_step * 1e-3) / 8e12, frac_pmc=tot_pmc / (t_step * 1e-3) / 8e12),
                  open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
