#!/bin/bash
# whole-step HIP graph replay speed: single-stream vs side-stream capture, CLR graph env knobs
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
run() {  # tag, env..., -- model batch size
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --model inceptionv3 --batch 128 --image-size 299 --steps 20 --warmup 8 --graph on > gpurun_out/r3g_$tag.log 2>&1 || { tail -3 gpurun_out/r3g_$tag.log; return 1; }
  echo "inception $tag $(tail -1 gpurun_out/r3g_$tag.log | grep -o '"value": [0-9.]*')"
}
run side0 IMGCLS_GRAPH_SIDE=0 || exit 1
run side1 IMGCLS_GRAPH_SIDE=1 || exit 1
run side0_pkt1 IMGCLS_GRAPH_SIDE=0 DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 || exit 1
run side0_pkt0 IMGCLS_GRAPH_SIDE=0 DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 || exit 1
run side0_devkarg IMGCLS_GRAPH_SIDE=0 HIP_FORCE_DEV_KERNARG=1 || exit 1
IMGCLS_GRAPH_SIDE=0 timeout -k 10 300 python bench.py --steps 20 --warmup 8 --graph on > gpurun_out/r3g_r50_side0.log 2>&1 && echo "r50 side0 $(tail -1 gpurun_out/r3g_r50_side0.log | grep -o '"value": [0-9.]*')"
