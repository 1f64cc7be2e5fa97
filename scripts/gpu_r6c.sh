#!/bin/bash
# Round 3 call r6c: the whole GPU suite + smoke after the halo kernel / test fixes, the headline bench and
# the reference's default config (Inception-v3 @299, b4 / b32) with --graph auto.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
export TMPDIR=/tmp
( while true; do sleep 30; date +%s >> gpurun_out/r6c_ticks.txt; done ) & TICK=$!
trap 'kill $TICK' EXIT
b() { local tag=$1; shift; timeout -k 10 400 python bench.py "$@" > gpurun_out/r6c_$tag.log 2>&1 || { tail -5 gpurun_out/r6c_$tag.log; return 1; }
      echo "$tag $(grep -h '^{"metric' gpurun_out/r6c_$tag.log | cut -c80-150)"; }
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 400 --timeout-method thread > gpurun_out/r6c_pytest_gpu.log 2>&1; rc=$?
tail -15 gpurun_out/r6c_pytest_gpu.log | grep -v "^frame"
case $rc in 0|1) ;; *) echo "gpu suite rc=$rc"; exit 1;; esac
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6c_smoke.log 2>&1 || { tail -5 gpurun_out/r6c_smoke.log; exit 1; }
tail -1 gpurun_out/r6c_smoke.log
b device --warmup 8 --steps 20 || exit 1
b incep_b4 --model inceptionv3 --image-size 299 --batch 4 --warmup 10 --steps 60 || exit 1
b incep_b32 --model inceptionv3 --image-size 299 --batch 32 --warmup 10 --steps 60 || exit 1
b incep_b64 --model inceptionv3 --image-size 299 --batch 64 --warmup 10 --steps 40 || exit 1
b incep_b64_eager --model inceptionv3 --image-size 299 --batch 64 --warmup 10 --steps 40 --graph off || exit 1
