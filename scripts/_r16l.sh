set -o pipefail
# BASELINE config 5 measured: bench.py --dtype fp8 (MX-FP8 forward convs, bf16 backward) against bf16, ResNet-50 b1024
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
out=gpurun_out/r16l_fp8_ab.txt; : > $out
for r in 1 2; do for d in bf16 fp8; do
  timeout -k 10 400 python bench.py --dtype $d --steps 20 --warmup 8 > gpurun_out/r16l_run.log 2>&1 || { tail -20 gpurun_out/r16l_run.log; exit 1; }
  echo "round $r | --dtype $d | $(grep -h '^{"metric' gpurun_out/r16l_run.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["dtype"], d["config"]["final_loss"])')" | tee -a $out
done; done
