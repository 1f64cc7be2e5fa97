set -o pipefail
# round 6: headline with the re-tuned find-db, and a kernel trace of its step (per-launch durations, the tail)
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=r15h
timeout -k 10 300 python bench.py --warmup 8 --steps 20 > gpurun_out/${T}_bench.log 2>&1 || { tail -5 gpurun_out/${T}_bench.log; exit 1; }
grep -h '^{"metric' gpurun_out/${T}_bench.log | cut -c1-160
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_prof -o hip -- python3 bench.py --warmup 6 --steps 3 > gpurun_out/${T}_prof.log 2>&1 || { tail -5 gpurun_out/${T}_prof.log; exit 1; }
f=$(find gpurun_out/${T}_prof -name "*kernel_trace.csv" | head -1)
python scripts/step_breakdown.py $f > gpurun_out/${T}_step_breakdown.txt || exit 1
python scripts/step_launches.py $f 400 > gpurun_out/${T}_step_launches.txt || exit 1
python - "$f" > gpurun_out/${T}_step_tail.txt <<'PY'
import csv, sys, re
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "adam_kernel" in r["Kernel_Name"] and "tick" not in r["Kernel_Name"]]
st = rows[idx[-2] + 1: idx[-1] + 1]
t0 = int(rows[idx[-2]]["End_Timestamp"])
st.sort(key=lambda r: int(r["End_Timestamp"]))
print("last 30 kernels of the step by end time (us from the previous Adam's end): start end dur queue name grid")
for r in st[-30:]:
    s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
    n = re.sub(r"\((?!\)).*", "", r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", ""))[:70]
    print(f"{s/1e3:9.1f} {e/1e3:9.1f} {(e-s)/1e3:7.1f} q{r.get('Queue_Id', '?'):>3} {n} grid={r.get('Grid_Size_X','?')}")
PY
rm -f $f
head -3 gpurun_out/${T}_step_breakdown.txt; tail -12 gpurun_out/${T}_step_tail.txt
