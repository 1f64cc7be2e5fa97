#!/bin/bash
# per-GPU batch 1024 for the headline: three tuning runs seeded from the b512 find-db (each saves its
# choices), larger batches probed, and the reference stack (torch DDP + MIOpen, bf16 autocast) at 1024
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
run() { local tag=$1; shift; timeout -k 10 500 python bench.py "$@" > gpurun_out/r4g_$tag.log 2>&1 || { tail -5 gpurun_out/r4g_$tag.log; return 1; }
        echo "$tag $(grep -h metric gpurun_out/r4g_$tag.log | cut -c80-140) $(grep -h 'peak memory' gpurun_out/r4g_$tag.log | cut -c20-)"; }
for i in 1 2 3; do run tune$i --batch 1024 --warmup 12 --tune-save gpurun_out/r4g_db_b1024_$i.json || exit 1; done
run b1536 --batch 1536 --warmup 12 || exit 1
run b2048 --batch 2048 --warmup 12 || exit 1
run torch1024 --batch 1024 --compute torch --steps 20 --warmup 5 || exit 1
