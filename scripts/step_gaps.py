"""Per-queue busy time and idle gaps of the last full training step in a rocprofv3 kernel trace
(step = kernels between the last two adam_kernel launches): python scripts/step_gaps.py hip_kernel_trace.csv"""
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
adams = [i for i, r in enumerate(rows) if "adam_kernel" in r["Kernel_Name"] and "tick" not in r["Kernel_Name"]]
i0, i1 = adams[-2], adams[-1]
step = rows[i0+1:i1+1]
t0 = int(rows[i0]["End_Timestamp"]); t1 = int(rows[i1]["End_Timestamp"])
print(f"step {((t1-t0)/1e3):.1f} us, {len(step)} kernels")
byq = collections.defaultdict(list)
for r in step: byq[r["Queue_Id"]].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:60]))
for q, ks in byq.items():
    busy = sum(e-s for s, e, _ in ks)
    # union busy
    ks.sort(); u=0; cs, ce = ks[0][0], ks[0][1]
    gaps=[]
    for s, e, n in ks[1:]:
        if s > ce: u += ce-cs; gaps.append((s-ce, n)); cs, ce = s, e
        else: ce = max(ce, e)
    u += ce-cs
    gaps.sort(reverse=True)
    print(f"queue {q}: {len(ks)} kernels, busy(union) {u/1e3:.1f} us, gaps total {sum(g for g,_ in gaps)/1e3:.1f} us; largest gaps:")
    for g, n in gaps[:8]: print(f"     {g/1e3:7.1f} us before {n}")
# union over all queues
allk = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in step)
u=0; cs, ce = allk[0]
for s,e in allk[1:]:
    if s > ce: u += ce-cs; cs, ce = s, e
    else: ce = max(ce, e)
u += ce-cs
print(f"any-queue busy {u/1e3:.1f} us of {(t1-t0)/1e3:.1f}")
