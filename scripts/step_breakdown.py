"""Per-kernel breakdown of ONE steady-state training step from a rocprofv3 kernel trace.

usage: python scripts/step_breakdown.py gpurun_out/prof_q/hip_kernel_trace.csv|run_results.db [marker=adam_kernel]
The step is the span between the last two launches of the marker kernel (one per optimizer step)."""
import collections
import csv
import re
import sys

path = sys.argv[1]
marker = sys.argv[2] if len(sys.argv) > 2 else "adam_kernel"
if path.endswith(".db"):  # the rocpd SQLite database (rocprofv3's default output)
    import sqlite3
    keys = ("Kernel_Name", "Start_Timestamp", "End_Timestamp")
    rows = [dict(zip(keys, map(str, r))) for r in sqlite3.connect(path).execute("select name, start, end from kernels")]
else:
    rows = list(csv.DictReader(open(path)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
a, b = idx[-2], idx[-1]
step = rows[a + 1:b + 1]
busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in step)
span = int(step[-1]["End_Timestamp"]) - int(rows[a]["End_Timestamp"])
agg = collections.defaultdict(lambda: [0, 0])
for r in step:
    name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
    name = re.sub(r"\((?!\)).*", "", name) or r["Kernel_Name"]
    name = name[:70]
    agg[name][0] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    agg[name][1] += 1
print(f"step span {span / 1e6:.3f} ms, kernel busy {busy / 1e6:.3f} ms, launches {len(step)}")
for k, (t, n) in sorted(agg.items(), key=lambda kv: -kv[1][0]):
    print(f"{t / 1e6:8.3f} ms {n:5d}x  {k}")

# per stream (queue): union of busy intervals, time it runs alone, and its top kernels - the compute stream's
# busy union is the critical chain; side-stream time that overlaps it is concurrency, not step time
qkey = next((k for k in ("Stream_Id", "Queue_Id") if step and k in step[0]), None)
if qkey is not None:
    def union(iv):
        iv = sorted(iv)
        tot, cs, ce = 0, None, None
        for s, e in iv:
            if cs is None or s > ce:
                if cs is not None:
                    tot += ce - cs
                cs, ce = s, e
            else:
                ce = max(ce, e)
        return tot + (ce - cs if cs is not None else 0)
    byq = collections.defaultdict(list)
    for r in step:
        byq[r[qkey]].append(r)
    allu = union([(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in step])
    print(f"\nper {qkey}: busy union of all streams {allu / 1e6:.3f} ms")
    for q, rs in sorted(byq.items(), key=lambda kv: -len(kv[1])):
        iv = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rs]
        others = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in step if r[qkey] != q]
        alone = allu - union(others)
        print(f"  {qkey} {q}: {len(rs)} launches, busy union {union(iv) / 1e6:.3f} ms, alone {alone / 1e6:.3f} ms")
        qa = collections.defaultdict(lambda: [0, 0])
        for r in rs:
            name = re.sub(r"\((?!\)).*", "", r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", ""))[:64]
            qa[name][0] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            qa[name][1] += 1
        for k, (t, n) in sorted(qa.items(), key=lambda kv: -kv[1][0])[:12]:
            print(f"    {t / 1e6:8.3f} ms {n:5d}x  {k}")
