#!/bin/bash
# setprio (T5) conv variants: plain-GEMM table, per-shape tuner candidate log, retuned bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/db
timeout -k 10 300 python benchmarks/gemm_ref.py --all > gpurun_out/r2o_gemm_ref.txt 2>&1 || { tail -20 gpurun_out/r2o_gemm_ref.txt; exit 1; }
grep -v "^      " gpurun_out/r2o_gemm_ref.txt | grep M=
timeout -k 10 400 python benchmarks/conv_bench.py --batch 512 --tune-log > gpurun_out/r2o_conv_bench.txt 2>&1 || { tail -20 gpurun_out/r2o_conv_bench.txt; exit 1; }
for r in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 8 --tune-db none --tune-save gpurun_out/db/r2o_$r.json > gpurun_out/r2o_bench_$r.log 2>&1 || exit $?
  echo "tuned $r $(tail -1 gpurun_out/r2o_bench_$r.log | grep -o '"value": [0-9.]*')"
done
