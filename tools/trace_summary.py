"""Per (kernel, grid) totals from a rocprofv3 kernel trace: python tools/trace_summary.py DIR [filter] [top]"""
import collections
import csv
import glob
import sys

d = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
top = int(sys.argv[3]) if len(sys.argv) > 3 else 40
f = glob.glob(d + "/**/*kernel_trace.csv", recursive=True)[0]
agg = collections.defaultdict(lambda: [0, 0.0])
for r in csv.DictReader(open(f)):
    if flt not in r["Kernel_Name"]:
        continue
    key = (r["Kernel_Name"].replace("(anonymous namespace)::", "")[:60], r["Grid_Size_X"], r["Grid_Size_Y"])
    agg[key][0] += 1
    agg[key][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
tot = sum(v[1] for v in agg.values())
for k, v in sorted(agg.items(), key=lambda x: -x[1][1])[:top]:
    print("%-60s %9s %4s %6d %9.3f ms avg %.4f" % (k[0], k[1], k[2], v[0], v[1], v[1] / v[0]))
print("total %.3f ms" % tot)
