set -o pipefail
# Inception-v3 b128: host time per op-layer function (forward and the autograd thread's backward)
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python scripts/host_fn_prof.py inceptionv3 299 128 > gpurun_out/r16j_host_fn_prof.txt 2>&1 || { tail -20 gpurun_out/r16j_host_fn_prof.txt; exit 1; }
head -45 gpurun_out/r16j_host_fn_prof.txt
