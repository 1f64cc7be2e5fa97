#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/host_fn_prof.py inceptionv3 299 128 > gpurun_out/r3i_host_fn_inception.txt 2>&1 || { tail gpurun_out/r3i_host_fn_inception.txt; exit 1; }
grep -v Warning gpurun_out/r3i_host_fn_inception.txt | tail -45
