#!/bin/bash
# PMC counters for the wgrad kernels of one shape (CONV_ONLY index into benchmarks/conv_bench.py R50)
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"; mkdir -p gpurun_out/pmcw
export TMPDIR=/tmp
ONLY="${CONV_ONLY:-0}"
fatal() { case "$1" in 124|134|137|139) echo "fatal rc=$1 at $2"; exit "$1";; esac; }
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" \
           "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SALU SQ_BUSY_CYCLES FETCH_SIZE"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $grp --output-format csv -d "$ROOT/gpurun_out/pmcw/p$i" -o pmc -- python3 "$ROOT/benchmarks/conv_bench.py" --batch 512 --only $ONLY --iters 3 > gpurun_out/pmcw/p$i.log 2>&1; rc=$?
  echo "pmc$i rc=$rc"; fatal $rc pmc$i
  [ $rc -eq 0 ] || exit 1
done
