#!/bin/bash
# isolated weight-gradient candidate timings incl. the 64 / 128 x 256 tiles (no-spill build)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/wgrad_tile_probe.py > gpurun_out/r4d_wgrad_tiles.txt 2>&1; rc=$?; cat gpurun_out/r4d_wgrad_tiles.txt | grep -v Warning; exit $rc
