#!/bin/bash
# quad-gather max-pool backward: GPU tests, rocprofv3 kernel stats of the ResNet-50 b512 step, benches
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; ROOT="$(pwd)"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && tail -2 gpurun_out/pytest_gpu.log &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/prof_r1g" -o hip -- python3 "$ROOT/bench.py" --steps 5 --warmup 2 > gpurun_out/prof_r1g.log 2>&1 && tail -1 gpurun_out/prof_r1g.log &&
timeout -k 10 400 python bench.py > gpurun_out/bench_a.log 2>&1 && tail -1 gpurun_out/bench_a.log &&
timeout -k 10 400 python bench.py --model inceptionv3 --batch 128 --image-size 299 > gpurun_out/bench_inc.log 2>&1 && tail -1 gpurun_out/bench_inc.log &&
timeout -k 10 400 python bench.py > gpurun_out/bench_b.log 2>&1 && tail -1 gpurun_out/bench_b.log
