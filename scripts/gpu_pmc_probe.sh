#!/bin/bash
# PMC counters of single conv kernels (benchmarks/kernel_probe.py), one rocprofv3 pass per counter group
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > gpurun_out/pmc/counters_list.txt 2>&1 || true
PROBES=("--shape 0 --mode fwd --cfg 5" "--shape 0 --mode fwd --cfg 1" "--shape 0 --mode wgrad --wblocks 512 --wstages 1" "--shape 6 --mode fwd --cfg 1")
GROUPS_=("SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
         "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_WAVES SQ_INSTS_MFMA TCC_HIT_sum TCC_MISS_sum")
for i in 0 1 2 3; do
  timeout -k 10 120 python benchmarks/kernel_probe.py ${PROBES[$i]} --iters 20 >> gpurun_out/pmc/timing.txt 2>&1 || exit $?
  for j in 0 1; do
    timeout -s KILL 90 rocprofv3 --pmc ${GROUPS_[$j]} --output-format csv -d gpurun_out/pmc/p${i}_$j -o pmc -- python3 benchmarks/kernel_probe.py ${PROBES[$i]} --iters 3 > gpurun_out/pmc/p${i}_$j.log 2>&1; rc=$?
    echo "probe $i group $j rc=$rc"
    [ $rc -eq 0 ] || { tail -5 gpurun_out/pmc/p${i}_$j.log; exit $rc; }
  done
done
cat gpurun_out/pmc/timing.txt | grep shape
