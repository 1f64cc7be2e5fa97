#!/bin/bash
# Round 3 call r6h: how much the weight-gradient side stream slows the compute stream (diagnostic: the step
# with the wgrad GEMMs skipped, and with them serialised on the compute stream).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/r6h
export TMPDIR=/tmp
b() { local tag=$1; shift; timeout -k 10 400 python bench.py "$@" > gpurun_out/r6h/$tag.log 2>&1 || { tail -3 gpurun_out/r6h/$tag.log; return 1; }
      echo "$tag $(grep -h '^{"metric' gpurun_out/r6h/$tag.log | grep -o '"ms_per_step": [0-9.]*')"; }
b default --warmup 8 --steps 20 || exit 1
IMGCLS_DIAG_SKIP_WGRAD=1 b skip_wgrad --warmup 8 --steps 20 || exit 1
IMGCLS_WGRAD_STREAM=0 b one_stream --warmup 8 --steps 20 || exit 1
