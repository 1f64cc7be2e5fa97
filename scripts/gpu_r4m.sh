#!/bin/bash
# end-of-session check: train.py CLI on the GPU (2 short epochs + resume from latest), GPU suite, smoke,
# and the driver's bench command line
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
( while true; do sleep 30; date +%s >> gpurun_out/r4m_ticks.txt; done ) & TICK=$!
trap 'kill $TICK' EXIT
T="--synthetic --model resnet50 --image-size 64 --batchsize 32 --synthetic-train-size 512 --synthetic-val-size 64 --num-workers 0 --no-progress --ckpt-dir /tmp/ck_r4m --val-batchsize 16 --latest-every 1"
timeout -k 10 300 python train.py $T --epochs 2 --resume none > gpurun_out/r4m_train.log 2>&1 || { tail -20 gpurun_out/r4m_train.log; exit 1; }
grep -E "Validation|Epoch|saved|improved" gpurun_out/r4m_train.log | tail -6
timeout -k 10 300 python train.py $T --epochs 3 --resume latest > gpurun_out/r4m_resume.log 2>&1 || { tail -20 gpurun_out/r4m_resume.log; exit 1; }
grep -E "Validation|resum|Resum|epoch" gpurun_out/r4m_resume.log | tail -6
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4m_pytest.log 2>&1 || { grep -E "FAILED|Error" gpurun_out/r4m_pytest.log | head; exit 1; }
grep -E "passed|failed" gpurun_out/r4m_pytest.log | tail -1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4m_smoke.log 2>&1 && tail -1 gpurun_out/r4m_smoke.log || exit 1
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r4m_bench.log 2>&1 && grep -h metric gpurun_out/r4m_bench.log | cut -c1-260
