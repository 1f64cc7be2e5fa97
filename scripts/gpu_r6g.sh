#!/bin/bash
# Round 3 call r6g: find-db refresh for the fused (XA) launches, which the round-2 db does not list (tuned
# live in every run): three seeded runs each save their choices; XA replication gate 1 / 4 vs the default 2.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/r6g
export TMPDIR=/tmp
b() { local tag=$1; shift; timeout -k 10 400 python bench.py "$@" > gpurun_out/r6g/$tag.log 2>&1 || { tail -3 gpurun_out/r6g/$tag.log; return 1; }
      echo "$tag $(grep -h '^{"metric' gpurun_out/r6g/$tag.log | cut -c80-150)"; }
for i in 1 2 3; do
  b tune$i --warmup 8 --steps 20 --tune-save gpurun_out/r6g/db$i.json || exit 1
done
for i in 1 2 3; do
  b check$i --warmup 8 --steps 20 --tune-db gpurun_out/r6g/db$i.json || exit 1
done
IMGCLS_XA_MAX_REP=1 b xarep1 --warmup 8 --steps 20 || exit 1
IMGCLS_XA_MAX_REP=4 b xarep4 --warmup 8 --steps 20 || exit 1
IMGCLS_XA_MAX_REP=8 b xarep8 --warmup 8 --steps 20 || exit 1
IMGCLS_MAX_INFLIGHT_STEPS=3 b inflight3 --warmup 8 --steps 20 || exit 1
