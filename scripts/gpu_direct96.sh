set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_hip_ops.py -x -q -m gpu -k "direct" --timeout 120 --timeout-method thread > gpurun_out/pytest_direct.log 2>&1; rc=$?; tail -1 gpurun_out/pytest_direct.log; [ $rc -eq 0 ] || { grep -E "^E|FAILED" gpurun_out/pytest_direct.log | head; exit 1; }
bash scripts/gpu_tune_var.sh "--model inceptionv3 --image-size 299 --batch 128 --steps 30 --warmup 10" 3
