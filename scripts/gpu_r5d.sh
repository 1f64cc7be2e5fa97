#!/bin/bash
# Round 3 call d: fused BN-backward (XA) and BN-apply (XF) tests, headline A/B + kernel-trace
# breakdown, learning-parity tests, b1536 memory diagnosis, SyncBN peer tests (incl. fatal timeout), host
# data path, Inception small batch (eager / graph / reference stack), and a 2-rank one-GPU rehearsal of the
# N>1 bench fields (gloo: functional, not a scaling number).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
export TMPDIR=/tmp
( while true; do sleep 30; date +%s >> gpurun_out/r5d_ticks.txt; done ) & TICK=$!
trap 'kill $TICK' EXIT
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_hip_ops.py \
  -k "fused or shadow or dense or large_mean or conv_bn_act or stem or defers" > gpurun_out/r5d_pytest_xa.log 2>&1 || { tail -40 gpurun_out/r5d_pytest_xa.log; exit 1; }
tail -2 gpurun_out/r5d_pytest_xa.log
b() { local tag=$1; shift; timeout -k 10 400 python bench.py "$@" > gpurun_out/r5d_$tag.log 2>&1 || { tail -5 gpurun_out/r5d_$tag.log; return 1; }
      echo "$tag $(grep -h '^{"metric' gpurun_out/r5d_$tag.log | cut -c80-170)"; }
# round-2 path (no fusion) / BN-backward fused (XA) / + BN-apply fused (XF, the default)
IMGCLS_BN_XA=0 IMGCLS_BN_XF=0 b xa0 --warmup 8 --steps 20 || exit 1
IMGCLS_BN_XF=0 b xa1 --warmup 8 --steps 20 || exit 1
b xaxf --warmup 8 --steps 20 || exit 1
timeout -k 10 500 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r5d_prof -o hip -- \
  python3 bench.py --warmup 6 --steps 3 > gpurun_out/r5d_prof.log 2>&1 || { tail -5 gpurun_out/r5d_prof.log; exit 1; }
python scripts/step_breakdown.py gpurun_out/r5d_prof/hip_kernel_trace.csv > gpurun_out/r5d_step_breakdown.txt
python scripts/step_gaps.py gpurun_out/r5d_prof/hip_kernel_trace.csv > gpurun_out/r5d_gaps.txt
rm -f gpurun_out/r5d_prof/hip_kernel_trace.csv
head -24 gpurun_out/r5d_step_breakdown.txt; head -3 gpurun_out/r5d_gaps.txt
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 400 --timeout-method thread tests/test_gpu_learning.py \
  > gpurun_out/r5d_pytest_learning.log 2>&1 || { tail -40 gpurun_out/r5d_pytest_learning.log; exit 1; }
grep -h "hip loss" gpurun_out/r5d_pytest_learning.log; tail -1 gpurun_out/r5d_pytest_learning.log
b b1536 --batch 1536 --warmup 12 --steps 10 || exit 1
grep -h -e "memory" gpurun_out/r5d_b1536.log | cut -c1-220
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_peer.py \
  > gpurun_out/r5d_pytest_peer.log 2>&1 || { tail -30 gpurun_out/r5d_pytest_peer.log; exit 1; }
tail -1 gpurun_out/r5d_pytest_peer.log
b host --warmup 8 --steps 20 --data host || exit 1
b incep_b4_eager --model inceptionv3 --image-size 299 --batch 4 --warmup 10 --steps 50 || exit 1
b incep_b4_graph --model inceptionv3 --image-size 299 --batch 4 --warmup 10 --steps 50 --graph on || exit 1
b incep_b4_torch --model inceptionv3 --image-size 299 --batch 4 --warmup 10 --steps 50 --compute torch || exit 1
b incep_b32_eager --model inceptionv3 --image-size 299 --batch 32 --warmup 10 --steps 30 || exit 1
b incep_b32_graph --model inceptionv3 --image-size 299 --batch 32 --warmup 10 --steps 30 --graph on || exit 1
b incep_b32_torch --model inceptionv3 --image-size 299 --batch 32 --warmup 10 --steps 30 --compute torch || exit 1
DRY=1 NS="2" SYNCBN="on" BUCKETS="32" COMMS="fp32" REF=0 BACKEND=gloo BATCH=64 STEPS=6 WARMUP=3 TIMEOUT=300 \
  OUT=gpurun_out/r5d_sweep_dry.jsonl bash scripts/scale_sweep.sh || exit 1
