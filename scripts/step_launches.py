"""Longest individual kernel launches of ONE steady-state step (rocprofv3 kernel trace).

usage: python scripts/step_launches.py gpurun_out/prof_q/hip_kernel_trace.csv|run_results.db [top=40] [filter-regex]"""
import csv
import re
import sys


def _load(path):
    """kernel_trace.csv (rocprofv3 --output-format csv) or the rocpd SQLite database (its default)."""
    if path.endswith(".db"):
        import sqlite3
        q = ("select name, start, end, grid_x, grid_y, workgroup_x from kernels order by start")
        keys = ("Kernel_Name", "Start_Timestamp", "End_Timestamp", "Grid_Size_X", "Grid_Size_Y", "Workgroup_Size_X")
        return [dict(zip(keys, map(str, r))) for r in sqlite3.connect(path).execute(q)]
    return list(csv.DictReader(open(path)))


rows = sorted(_load(sys.argv[1]), key=lambda r: int(r["Start_Timestamp"]))
top = int(sys.argv[2]) if len(sys.argv) > 2 else 40
flt = re.compile(sys.argv[3]) if len(sys.argv) > 3 else None
idx = [i for i, r in enumerate(rows) if "adam_kernel" in r["Kernel_Name"]]
step = rows[idx[-2] + 1:idx[-1] + 1]
out = []
for i, r in enumerate(step):
    n = re.sub(r"\((?!\)).*", "", r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", ""))
    if flt and not flt.search(n):
        continue
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    wg = int(r["Workgroup_Size_X"])
    out.append((d, i, n, int(r["Grid_Size_X"]) // wg, int(r["Grid_Size_Y"]), wg))
print(f"{sum(o[0] for o in out) / 1e3:.3f} ms in {len(out)} launches")
for d, i, n, gx, gy, wg in sorted(out, reverse=True)[:top]:
    print(f"{d:8.1f}us #{i:3d} {n[:58]:58s} blocks={gx}x{gy} wg={wg}")
