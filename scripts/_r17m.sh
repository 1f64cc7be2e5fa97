set -o pipefail
# Where the timed-region hipMallocs of Inception-v3 b128 come from: per-stream pools after 8 warmup + 10 steps.
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python scripts/alloc_trace.py --warmup 8 --steps 10 > gpurun_out/r17m_alloc_trace.txt 2>&1 || { tail -5 gpurun_out/r17m_alloc_trace.txt; exit 1; }
timeout -k 10 300 python scripts/alloc_trace.py --warmup 8 --steps 30 > gpurun_out/r17m_alloc_trace30.txt 2>&1 || { tail -5 gpurun_out/r17m_alloc_trace30.txt; exit 1; }
cat gpurun_out/r17m_alloc_trace.txt gpurun_out/r17m_alloc_trace30.txt | grep -v Warning
