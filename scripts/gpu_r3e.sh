#!/bin/bash
# host-side (Python) profile of an Inception-v3 b128 and an EfficientNet-B0 b256 step (host-bound models)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/host_prof.py 128 inceptionv3 299 > gpurun_out/r3e_host_inception.txt 2>&1 || exit $?
timeout -k 10 300 python -u scripts/host_prof.py 256 efficientnet-b0 224 > gpurun_out/r3e_host_effb0.txt 2>&1 || exit $?
head -60 gpurun_out/r3e_host_inception.txt
