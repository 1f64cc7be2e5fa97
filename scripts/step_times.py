"""Per-step wall spans from a rocprofv3 kernel trace, and what the slowest step spent its time on.

usage: python scripts/step_times.py gpurun_out/prof_x/hip_kernel_trace.csv [marker=adam_kernel]
A step is the span between consecutive launches of the marker kernel (one per optimizer step).  For the
slowest step it prints the longest kernels and the longest idle gaps (no kernel on any queue), which
tells a slow kernel (a bad tuning choice, an index overflow) from host / allocator stalls (gaps)."""
import csv
import re
import sys

path = sys.argv[1]
marker = sys.argv[2] if len(sys.argv) > 2 else "adam_kernel"
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]


def short(name):
    name = name.replace("(anonymous namespace)::", "").replace("void ", "")
    return (re.sub(r"\((?!\)).*", "", name) or name)[:80]


spans = []
for a, b in zip(idx, idx[1:]):
    spans.append((int(rows[b]["End_Timestamp"]) - int(rows[a]["End_Timestamp"]), a, b))
print("step spans (ms): " + " ".join(f"{s / 1e6:.1f}" for s, _, _ in spans))
if not spans:
    sys.exit(0)
s, a, b = max(spans)
step = rows[a + 1:b + 1]
print(f"slowest step: {s / 1e6:.3f} ms, {len(step)} kernels")
for r in sorted(step, key=lambda r: int(r["Start_Timestamp"]) - int(r["End_Timestamp"]))[:12]:
    d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    print(f"  {d / 1e3:10.1f} us  {short(r['Kernel_Name'])}")
gaps = []
end = int(rows[a]["End_Timestamp"])
for r in step:
    st = int(r["Start_Timestamp"])
    if st > end:
        gaps.append((st - end, short(r["Kernel_Name"])))
    end = max(end, int(r["End_Timestamp"]))
print(f"idle gaps: {sum(g for g, _ in gaps) / 1e6:.3f} ms total; largest:")
for g, k in sorted(gaps, reverse=True)[:8]:
    print(f"  {g / 1e3:10.1f} us before {k}")
