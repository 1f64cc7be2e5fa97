#!/bin/bash
# Round 3 call f: the host run-ahead throttle (Trainer._throttle) against the allocator growth measured in
# r5d (44 GiB allocated, 286 GiB reserved, 1.6 s steps with XA): headline A/B (throttle off / on) for the
# three fusion levels, b1536 / b2048, then the learning-parity tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
export TMPDIR=/tmp
( while true; do sleep 30; date +%s >> gpurun_out/r5f_ticks.txt; done ) & TICK=$!
trap 'kill $TICK' EXIT
b() { local tag=$1; shift; timeout -k 10 400 python bench.py "$@" > gpurun_out/r5f_$tag.log 2>&1 || { tail -5 gpurun_out/r5f_$tag.log; return 1; }
      echo "$tag $(grep -h '^{"metric' gpurun_out/r5f_$tag.log | cut -c80-150) $(grep -h 'peak memory' gpurun_out/r5f_$tag.log | cut -c17-200)"; }
IMGCLS_BN_XA=0 IMGCLS_BN_XF=0 b plain --warmup 8 --steps 20 || exit 1
IMGCLS_BN_XF=0 b xa --warmup 8 --steps 20 || exit 1
b xaxf --warmup 8 --steps 20 || exit 1
IMGCLS_XA_MAX_REP=1000000 IMGCLS_XF_MAX_REP=1000000 b xaxf_ungated --warmup 8 --steps 20 || exit 1
IMGCLS_XA_MAX_REP=1 IMGCLS_XF_MAX_REP=1 b xaxf_rep1 --warmup 8 --steps 20 || exit 1
IMGCLS_XA_MAX_REP=4 IMGCLS_XF_MAX_REP=4 b xaxf_rep4 --warmup 8 --steps 20 || exit 1
IMGCLS_MAX_INFLIGHT_STEPS=0 b xaxf_unthrottled --warmup 8 --steps 20 || exit 1
b xaxf_b1536 --batch 1536 --warmup 8 --steps 15 || exit 1
b xaxf_b2048 --batch 2048 --warmup 8 --steps 10 || exit 1
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 400 --timeout-method thread tests/test_gpu_learning.py \
  > gpurun_out/r5f_pytest_learning.log 2>&1 || { grep -h "hip loss" gpurun_out/r5f_pytest_learning.log; tail -30 gpurun_out/r5f_pytest_learning.log; exit 1; }
grep -h "hip loss" gpurun_out/r5f_pytest_learning.log; tail -1 gpurun_out/r5f_pytest_learning.log
