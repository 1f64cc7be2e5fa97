#!/bin/bash
# headline at the new default batch (1024, find-db seeded), b512 control, reference stack at 1024, and a
# kernel-stats profile of the b1536 slowdown
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
export TMPDIR=/tmp
( while true; do sleep 30; date +%s >> gpurun_out/r4h_ticks.txt; done ) & TICK=$!
trap 'kill $TICK' EXIT
run() { local tag=$1; shift; timeout -k 10 600 python bench.py "$@" > gpurun_out/r4h_$tag.log 2>&1 || { tail -5 gpurun_out/r4h_$tag.log; return 1; }
        echo "$tag $(grep -h metric gpurun_out/r4h_$tag.log | cut -c80-150) $(grep -h 'peak memory' gpurun_out/r4h_$tag.log | cut -c20-)"; }
run d1 || exit 1
run d2 || exit 1
run b512 --batch 512 || exit 1
run torch1024 --batch 1024 --compute torch --steps 20 --warmup 5 || exit 1
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_b1536 -o hip -- python3 bench.py --batch 1536 --steps 2 --warmup 3 > gpurun_out/r4h_prof_b1536.log 2>&1; echo "prof rc=$?"
python - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/prof_b1536/hip_kernel_stats.csv")))
rows.sort(key=lambda r: -int(r["TotalDurationNs"]))
for r in rows[:15]:
    print(f'{int(r["TotalDurationNs"])/1e6:9.1f} ms {int(r["Calls"]):5d}x max {int(r["MaxNs"])/1e3:9.1f} us  {r["Name"][:110]}')
PY
