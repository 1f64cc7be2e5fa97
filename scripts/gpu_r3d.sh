#!/bin/bash
# per-candidate times (incl. stream-K tails) on the 14x14 / 7x7 ResNet-50 shapes at batch 512
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
timeout -k 10 300 python -u benchmarks/conv_bench.py --batch 512 --tune-log --only 0,3,4,5,9,12,13,19,20,21 > gpurun_out/r3d_conv_bench_sk.txt 2>&1 || exit $?
tail -60 gpurun_out/r3d_conv_bench_sk.txt
