#!/bin/bash
# 3-stage 256x128 / 128x256 tiles: plain-GEMM table, retuned bench x2
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/db
timeout -k 10 300 python benchmarks/gemm_ref.py --all > gpurun_out/r2r_gemm_ref.txt 2>&1 || { tail -20 gpurun_out/r2r_gemm_ref.txt; exit 1; }
grep -v "^      " gpurun_out/r2r_gemm_ref.txt | grep M=
for r in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 8 --tune-db none --tune-save gpurun_out/db/r2r_$r.json > gpurun_out/r2r_bench_$r.log 2>&1 || exit $?
  echo "tuned $r $(tail -1 gpurun_out/r2r_bench_$r.log | grep -o '"value": [0-9.]*')"
done
