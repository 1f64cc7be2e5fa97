#!/bin/bash
# Round 3 call e: per-GEMM roofline of a ResNet-50 b1024 step (XA + XF on), Inception deferral tests,
# and PMC counter passes on the top conv shapes (scripts/conv_probe.py), one counter set per run.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
export TMPDIR=/tmp
( while true; do sleep 30; date +%s >> gpurun_out/r5e_ticks.txt; done ) & TICK=$!
trap 'kill $TICK' EXIT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_hip_ops.py -k "defers or apply_fused or large_mean" \
  > gpurun_out/r5e_pytest_xf.log 2>&1 || { tail -30 gpurun_out/r5e_pytest_xf.log; exit 1; }
tail -1 gpurun_out/r5e_pytest_xf.log

timeout -k 10 600 python scripts/conv_roofline.py 1024 2300 6.0 > gpurun_out/r5e_conv_roofline_b1024.txt 2>&1 || { tail -20 gpurun_out/r5e_conv_roofline_b1024.txt; exit 1; }
sed -n '8,40p' gpurun_out/r5e_conv_roofline_b1024.txt
P="python3 scripts/conv_probe.py --batch 1024 --iters 10"
for spec in "fwd 128,128,3,1,1,28 1" "fwd 64,64,3,1,1,56 0" "fwd 256,256,3,1,1,14 1" "fwd 256,256,3,1,1,14 4" "dgrad 128,512,1,1,0,28 1"; do
  set -- $spec
  tag="r5e_pmc_$1_$(echo $2 | tr , _)_c$3"
  timeout -k 10 120 $P --op $1 --shape $2 --cfg $3 > gpurun_out/$tag.time 2>&1 || { cat gpurun_out/$tag.time; exit 1; }
  cat gpurun_out/$tag.time
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS \
    --output-format csv -d gpurun_out/${tag}_a -o p -- $P --op $1 --shape $2 --cfg $3 > gpurun_out/${tag}_a.log 2>&1 || { tail -5 gpurun_out/${tag}_a.log; exit 1; }
  timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE FETCH_SIZE \
    --output-format csv -d gpurun_out/${tag}_b -o p -- $P --op $1 --shape $2 --cfg $3 > gpurun_out/${tag}_b.log 2>&1 || { tail -5 gpurun_out/${tag}_b.log; exit 1; }
done

# re-tune every shape (the 256 x 128 configurations are new) and bench the fresh choices
timeout -k 10 600 python bench.py --tune-db none --tune-save gpurun_out/r5e_find_db.json --warmup 8 --steps 20 > gpurun_out/r5e_retune.log 2>&1 || { tail -5 gpurun_out/r5e_retune.log; exit 1; }
grep -h '^{"metric' gpurun_out/r5e_retune.log | cut -c80-150
timeout -k 10 400 python bench.py --tune-db gpurun_out/r5e_find_db.json --warmup 8 --steps 20 > gpurun_out/r5e_retuned_bench.log 2>&1 || { tail -5 gpurun_out/r5e_retuned_bench.log; exit 1; }
grep -h '^{"metric' gpurun_out/r5e_retuned_bench.log | cut -c80-150
# learning parity last (its EfficientNet reference run faulted the GPU once in MIOpen's fp32 channels-last
# backward; the fp32 reference now runs NCHW)
# (an assertion failure here is recorded and the run goes on; a timeout / crash ends it)
timeout -k 10 900 python -u -m pytest -v -s --timeout 400 --timeout-method thread tests/test_gpu_learning.py \
  > gpurun_out/r5e_pytest_learning.log 2>&1; rc=$?
grep -h "hip loss" gpurun_out/r5e_pytest_learning.log; tail -1 gpurun_out/r5e_pytest_learning.log
case $rc in 0|1) ;; *) echo "learning tests rc=$rc"; exit 1;; esac
