#!/bin/bash
# Round 3 call g: the reference's default config at small batch (Inception-v3 @299, per-GPU batch 4 and 32:
# eager / HIP-graph replay / reference stack), the host data path, SyncBN peer tests, and a 2-rank one-GPU
# rehearsal of the N > 1 bench fields (gloo: functional, not a scaling number).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
export TMPDIR=/tmp
( while true; do sleep 30; date +%s >> gpurun_out/r5g_ticks.txt; done ) & TICK=$!
trap 'kill $TICK' EXIT
b() { local tag=$1; shift; timeout -k 10 400 python bench.py "$@" > gpurun_out/r5g_$tag.log 2>&1 || { tail -5 gpurun_out/r5g_$tag.log; return 1; }
      echo "$tag $(grep -h '^{"metric' gpurun_out/r5g_$tag.log | cut -c80-150)"; }
# the full GPU suite and the driver's smoke step first (assertion failures are recorded; a timeout / crash ends it)
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 400 --timeout-method thread > gpurun_out/r5g_pytest_gpu.log 2>&1; rc=$?
tail -5 gpurun_out/r5g_pytest_gpu.log
case $rc in 0|1) ;; *) echo "gpu suite rc=$rc"; exit 1;; esac
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5g_smoke.log 2>&1 || { tail -5 gpurun_out/r5g_smoke.log; exit 1; }
tail -2 gpurun_out/r5g_smoke.log
# the new 1-stage 128 x 128 variants (8 waves: cfg 18 / 19; lean 4-wave at occupancy 4: cfg 20) against cfg 1
for shape in 128,128,3,1,1,28 256,256,3,1,1,14 64,64,3,1,1,56 512,512,3,1,1,7; do
  for c in 1 18 19 20; do
    timeout -k 10 120 python3 scripts/conv_probe.py --batch 1024 --iters 10 --op fwd --shape $shape --cfg $c 2>&1 | grep -h " us " || exit 1
  done
  for c in 1 18 20; do
    timeout -k 10 120 python3 scripts/conv_probe.py --batch 1024 --iters 10 --op dgrad --shape $shape --cfg $c 2>&1 | grep -h " us " || exit 1
  done
done | tee gpurun_out/r5g_cfg_probe.txt
# kernel-trace breakdown of the default headline step (XA on, run-ahead throttle, retuned find-db if present)
DB=""; [ -f tuning/mi355x_find_db_r5e.json ] && DB="--tune-db tuning/mi355x_find_db_r5e.json"
timeout -k 10 500 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r5g_prof -o hip -- \
  python3 bench.py --warmup 6 --steps 3 $DB > gpurun_out/r5g_prof.log 2>&1 || { tail -5 gpurun_out/r5g_prof.log; exit 1; }
python scripts/step_breakdown.py gpurun_out/r5g_prof/hip_kernel_trace.csv > gpurun_out/r5g_step_breakdown.txt
python scripts/step_gaps.py gpurun_out/r5g_prof/hip_kernel_trace.csv > gpurun_out/r5g_gaps.txt
rm -f gpurun_out/r5g_prof/hip_kernel_trace.csv
head -30 gpurun_out/r5g_step_breakdown.txt; head -3 gpurun_out/r5g_gaps.txt
b host --warmup 8 --steps 20 --data host $DB || exit 1
b device --warmup 8 --steps 20 $DB || exit 1
for bs in 4 32; do
  b incep_b${bs}_eager --model inceptionv3 --image-size 299 --batch $bs --warmup 10 --steps 60 || exit 1
  b incep_b${bs}_graph --model inceptionv3 --image-size 299 --batch $bs --warmup 10 --steps 60 --graph on || exit 1
  b incep_b${bs}_torch --model inceptionv3 --image-size 299 --batch $bs --warmup 10 --steps 60 --compute torch || exit 1
done
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_peer.py \
  > gpurun_out/r5g_pytest_peer.log 2>&1 || { tail -30 gpurun_out/r5g_pytest_peer.log; exit 1; }
tail -1 gpurun_out/r5g_pytest_peer.log
DRY=1 NS="2" SYNCBN="on" BUCKETS="32" COMMS="fp32" REF=0 BACKEND=gloo BATCH=64 STEPS=6 WARMUP=3 TIMEOUT=300 \
  OUT=gpurun_out/r5g_sweep_dry.jsonl bash scripts/scale_sweep.sh || exit 1
