set -o pipefail
# whole-step graph replay above the auto threshold (per-GPU batch <= 64) on the final build: Inception-v3 b128 / b256, EfficientNet-B0 b256, ResNet-50 b128
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
out=gpurun_out/r17j_graph_ab.txt; : > $out
for cfg in "--model inceptionv3 --image-size 299 --batch 128" "--model inceptionv3 --image-size 299 --batch 256" "--model efficientnet-b0 --batch 256" "--batch 128"; do
  for r in 1 2; do for gph in off on; do
    timeout -k 10 300 python bench.py $cfg --graph $gph --steps 20 --warmup 8 > gpurun_out/r17j_run.log 2>&1 || { tail -5 gpurun_out/r17j_run.log; exit 1; }
    echo "$cfg --graph $gph round $r: $(grep -h '^{"metric' gpurun_out/r17j_run.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" | tee -a $out
  done; done
done
