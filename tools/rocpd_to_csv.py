"""rocprofv3's SQLite output (run_results.db, the default format) -> the kernel-trace CSV columns
tools/step_budget.py reads (Kernel_Name, Start_Timestamp, End_Timestamp, Grid_Size_X, Workgroup_Size_X, ...).
Tooling, not product code.  Usage: python tools/rocpd_to_csv.py RESULTS_DB OUT_CSV"""
import csv
import sqlite3
import subprocess
import sys


def main():
    db, out = sys.argv[1], sys.argv[2]
    cur = sqlite3.connect(db).cursor()
    names = dict(cur.execute("select id, kernel_name from rocpd_info_kernel_symbol"))
    # demangled names (the CSV output's form): c++filt over the symbols without their ".kd" suffix
    keys = list(names)
    raw = [names[k][:-3] if names[k].endswith(".kd") else names[k] for k in keys]
    try:
        dem = subprocess.run(["c++filt"], input="\n".join(raw), capture_output=True, text=True, check=True).stdout.split("\n")
        names = {k: d for k, d in zip(keys, dem)}
    except (OSError, subprocess.CalledProcessError):
        pass
    rows = cur.execute("select kernel_id, dispatch_id, start, end, grid_size_x, workgroup_size_x, grid_size_y, "
                       "private_segment_size, group_segment_size from rocpd_kernel_dispatch order by start").fetchall()
    with open(out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Kernel_Name", "Dispatch_Id", "Start_Timestamp", "End_Timestamp", "Grid_Size_X", "Workgroup_Size_X",
                    "Grid_Size_Y", "Private_Segment_Size", "Group_Segment_Size"])
        for kid, did, t0, t1, gx, wx, gy, ps, gs in rows:
            w.writerow([names.get(kid, str(kid)), did, t0, t1, gx, wx, gy, ps, gs])
    print("%d dispatches -> %s" % (len(rows), out))


if __name__ == "__main__":
    main()
