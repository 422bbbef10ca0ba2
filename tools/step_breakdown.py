"""Per-Newton-step kernel time by category from a rocprofv3 kernel trace of bench.py: the steps are
delimited by the residual launches (gls_brick_kernel<k, 0, double>: 2 per step); reports the last
complete step. Usage: python tools/step_breakdown.py <run_kernel_trace.csv>"""
import collections
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
res = [i for i, r in enumerate(rows) if "gls_brick_kernel<2, 0, double>" in r["Kernel_Name"]]
# a step starts with the first residual of a pair (assemble_matrix_and_rhs), the next pair starts the next step
starts = res[::2]
a, b = starts[-3], starts[-2]
cat = collections.OrderedDict()


def kind(n, grid):
    if "gls_brick_kernel<2, 4, double>" in n:
        return "J.v FP64 (fine)"
    if "gls_brick_kernel<2, 4, float>" in n:
        return "smoother J.v FP32 (fine)" if grid >= 2097152 // 8 * 256 else "smoother J.v FP32 (coarse levels)"
    if "gls_brick_kernel<2, 0" in n:
        return "residual"
    if "gls_brick_kernel<2, 3" in n:
        return "linearization+diag"
    if "k_slab_sum<double" in n:
        return "slab sum FP64"
    if "k_slab_sum<float" in n:
        return "slab sum FP32 (smoother)" if grid >= 1000000 else "slab sum FP32 (coarse levels)"
    if "multiaxpy" in n or "multidot" in n:
        return "GMRES orthogonalization"
    if "transfer" in n or "inject" in n or "box" in n:
        return "MG transfers"
    if "jacobi" in n:
        return "MG jacobi update"
    return "other vector / misc"


tot = 0.0
for r in rows[a:b]:
    t = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6
    k = kind(r["Kernel_Name"], int(r["Grid_Size_X"]))
    c = cat.setdefault(k, [0.0, 0])
    c[0] += t
    c[1] += 1
    tot += t
wall = (int(rows[b]["Start_Timestamp"]) - int(rows[a]["Start_Timestamp"])) * 1e-6
print("step wall %.2f ms, kernel time %.2f ms, launches %d" % (wall, tot, b - a))
for k, (t, n) in sorted(cat.items(), key=lambda kv: -kv[1][0]):
    print("  %-36s %8.2f ms  %5d launches  %5.1f%%" % (k, t, n, 100 * t / wall))
