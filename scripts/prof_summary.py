"""Markdown summary of a rocprofv3 --stats kernel CSV: python scripts/prof_summary.py STATS.csv STEPS TITLE"""
import csv
import sys

path, steps, title = sys.argv[1], float(sys.argv[2]), sys.argv[3]
rows = list(csv.DictReader(open(path)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"# {title}\n")
print(f"Total kernel time {tot / 1e6:.1f} ms over {steps:g} profiled steps (incl. warmup/autotune launches).\n")
print("| total ms | % | calls | avg us | kernel |\n|---|---|---|---|---|")
for r in rows[:30]:
    t = float(r["TotalDurationNs"])
    print(f"| {t / 1e6:.3f} | {100 * t / tot:.1f} | {r['Calls']} | {float(r['AverageNs']) / 1e3:.1f} | `{r['Name'][:100]}` |")
