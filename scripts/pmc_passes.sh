#!/bin/bash
# Two rocprofv3 counter passes (each its own run: rocprofv3 does not split counters over passes) over one
# short probe command; outputs gpurun_out/<tag>_a|_b/p_counter_collection.csv for scripts/pmc_summary.py.
#   bash scripts/pmc_passes.sh <tag> python3 scripts/gemm_probe.py --kernel deep0 --iters 5
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
tag=$1; shift
A="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
B="SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
for pass in a b; do
  if [ $pass = a ]; then C=$A; else C=$B; fi
  timeout -s KILL 90 rocprofv3 --pmc $C -d gpurun_out/${tag}_$pass -o p --output-format csv -- "$@" \
    > gpurun_out/${tag}_$pass.log 2>&1 || { echo "pmc pass $pass failed"; tail -3 gpurun_out/${tag}_$pass.log; exit 1; }
  f=$(find gpurun_out/${tag}_$pass -name "p_counter_collection.csv" | head -1)
  if [ -n "$f" ] && [ "$f" != "gpurun_out/${tag}_$pass/p_counter_collection.csv" ]; then mv "$f" gpurun_out/${tag}_$pass/p_counter_collection.csv; fi
done
