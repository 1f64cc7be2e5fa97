set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_hip_ops.py -k "pool" -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_pool.log 2>&1 && tail -2 gpurun_out/pytest_pool.log &&
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && tail -2 gpurun_out/pytest_gpu.log &&
timeout -k 10 300 python benchmarks/bn_bench.py --batch 256 > gpurun_out/bn_bench3.txt 2>&1 &&
timeout -k 10 400 python bench.py --steps 20 --warmup 8 > gpurun_out/bench_r50.log 2>&1 && tail -1 gpurun_out/bench_r50.log &&
timeout -k 10 400 python bench.py --batch 256 --steps 20 --warmup 8 > gpurun_out/bench_r50_256.log 2>&1 && tail -1 gpurun_out/bench_r50_256.log &&
timeout -k 10 400 python bench.py --model inceptionv3 --image-size 299 --batch 128 --steps 20 --warmup 8 > gpurun_out/bench_inc.log 2>&1 && tail -1 gpurun_out/bench_inc.log
