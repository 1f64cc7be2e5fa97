#!/bin/bash
# host-overhead cuts (C++ side-stream fork for wgrad, memoised conv geometry): GPU suite, host profile, benches
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3j_pytest_gpu.log 2>&1; rc=$?; tail -2 gpurun_out/r3j_pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/r3j_pytest_gpu.log | head; exit $rc; }
timeout -k 10 300 python -u scripts/host_fn_prof.py inceptionv3 299 128 > gpurun_out/r3j_host_fn_inception.txt 2>&1 || exit 1
grep -v Warning gpurun_out/r3j_host_fn_inception.txt | grep -A12 "host "
for m in "inceptionv3 128 299" "resnet50 512 224" "efficientnet-b0 256 224" "inceptionv3 128 299"; do
  set -- $m
  timeout -k 10 300 python bench.py --model $1 --batch $2 --image-size $3 --steps 20 --warmup 8 > gpurun_out/r3j_$1.log 2>&1 || { tail -5 gpurun_out/r3j_$1.log; exit 1; }
  echo "$1 $(tail -1 gpurun_out/r3j_$1.log | grep -o '"value": [0-9.]*') $(grep -o 'host enqueue [0-9.]* ms' gpurun_out/r3j_$1.log)"
done
