set -o pipefail
# Inception-v3 b128 run-to-run spread: are shapes timed at run time (per-process picks)?
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --model inceptionv3 --image-size 299 --batch 128 --steps 20 --warmup 8 > gpurun_out/r16o_run.log 2>&1 || { tail -5 gpurun_out/r16o_run.log; exit 1; }
  echo "run $i: $(grep -h '^{"metric' gpurun_out/r16o_run.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"])') | $(grep -h 'timed at run time\|allocator events' gpurun_out/r16o_run.log | cut -c1-160 | tr '\n' ' ')" | tee -a gpurun_out/r16o_spread.txt
done
