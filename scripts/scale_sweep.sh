#!/bin/bash
# Scaling sweep for an 8-GPU MI355X node (SURVEY 6 protocol; reference train.py:124,128: DDP + SyncBN).
#
#   N in {1,2,4,8} x SyncBN {on,off} x bucket MiB {8,16,32,64} x gradient transport {fp32,bf16}
#   x gradient backend {pg (ProcessGroupNCCL), rccl (our C++ communicator)},
#   plus the reference stack (torch DDP + nn.SyncBatchNorm + bf16 autocast, --compute torch) at each N.
#   The reference's own default launch: MODEL=inceptionv3 IMAGE_SIZE=299 BATCH=4 (graph replay at that batch;
#   with BACKENDS=rccl the bucket collectives sit inside the captured graph).
#
# Every run is one bench.py JSON line (rank 0) appended to $OUT; at N > 1 the line carries the
# all-reduce timeline (ms_first_bucket_before_bwd_end, ms_side_stream_tail, ms_comm_wait), the bucket
# layout, and the SyncBN checks (peer_errors, syncbn_running_stats_equal_across_ranks).
#
#   bash scripts/scale_sweep.sh                 # full sweep (8 GPUs)
#   NS="1 2" SYNCBN="on" BUCKETS="32" COMMS="fp32" bash scripts/scale_sweep.sh     # a slice
#   DRY=1 NS="2 4" BACKEND=gloo BATCH=64 bash scripts/scale_sweep.sh              # one-GPU functional rehearsal
#
# Env: NS, SYNCBN, BUCKETS, COMMS, BACKENDS (default "pg rccl"), MODEL / IMAGE_SIZE (default resnet50 / 224),
# BATCH (per GPU, default 1024), STEPS, WARMUP, REF (1: also the
# reference stack), BACKEND (auto | gloo), DRY (1: ranks share GPU 0 - functional only, not a scaling
# number), OUT (default gpurun_out/scale_sweep.jsonl), TIMEOUT (seconds per run), EXTRA (more bench.py flags:
# EXTRA="--device cpu" with BACKEND=gloo rehearses the sweep's plumbing on the CPU, tests/test_distributed.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
NS=${NS:-"1 2 4 8"}
SYNCBN=${SYNCBN:-"on off"}
BUCKETS=${BUCKETS:-"8 16 32 64"}
COMMS=${COMMS:-"fp32 bf16"}
BACKENDS=${BACKENDS:-"pg rccl"}
MODEL=${MODEL:-resnet50}
IMAGE_SIZE=${IMAGE_SIZE:-224}
BATCH=${BATCH:-1024}
STEPS=${STEPS:-20}
WARMUP=${WARMUP:-8}
REF=${REF:-1}
BACKEND=${BACKEND:-auto}
TIMEOUT=${TIMEOUT:-900}
OUT=${OUT:-gpurun_out/scale_sweep.jsonl}
mkdir -p "$(dirname "$OUT")" gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0

run() {  # run N tag args...
  local n=$1 tag=$2; shift 2
  local log="gpurun_out/sweep_${tag}.log"
  local env=()
  if [ "${DRY:-0}" = "1" ]; then env=(env HIP_VISIBLE_DEVICES=0); fi
  if [ "$n" = "1" ]; then
    "${env[@]}" timeout -k 10 "$TIMEOUT" python bench.py --gpus 1 --model "$MODEL" --image-size "$IMAGE_SIZE" \
      --batch "$BATCH" --steps "$STEPS" --warmup "$WARMUP" --dist-backend "$BACKEND" $EXTRA "$@" > "$log" 2>&1
  else
    "${env[@]}" timeout -k 10 "$TIMEOUT" python -m torch.distributed.run --nnodes=1 --nproc-per-node "$n" \
      --master-addr 127.0.0.1 --master-port $((29500 + RANDOM % 2000)) bench.py --gpus "$n" --model "$MODEL" \
      --image-size "$IMAGE_SIZE" --batch "$BATCH" --steps "$STEPS" --warmup "$WARMUP" --dist-backend "$BACKEND" \
      $EXTRA "$@" > "$log" 2>&1
  fi
  local rc=$?
  local line
  line=$(grep -h '^{"metric"' "$log" | tail -1)
  if [ $rc -ne 0 ] || [ -z "$line" ]; then
    echo "{\"tag\": \"$tag\", \"rc\": $rc, \"error\": \"see $log\"}" >> "$OUT"
    echo "$tag FAILED rc=$rc ($log)"
    return $rc
  fi
  echo "{\"tag\": \"$tag\", \"dry\": ${DRY:-0}, \"run\": $line}" >> "$OUT"
  echo "$tag $(echo "$line" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], "img/s", d["ms_per_step"], "ms/step", {k: d[k] for k in d if k.startswith("ms_") and k != "ms_per_step"})')"
}

for n in $NS; do
  for sb in $SYNCBN; do
    for bk in $BUCKETS; do
      for cm in $COMMS; do
        for be in $BACKENDS; do
          run "$n" "${MODEL}_n${n}_sb${sb}_b${bk}_${cm}_${be}" --sync-bn "$sb" --bucket-mb "$bk" --comm-dtype "$cm" \
            --comm-backend "$be" || exit 1
          [ "$n" = "1" ] && break 4  # N=1: no gradient collectives, no SyncBN exchange - one run suffices
        done
      done
    done
  done
  if [ "$REF" = "1" ]; then
    run "$n" "${MODEL}_n${n}_reference_stack" --compute torch --sync-bn on || exit 1
  fi
done
echo "results: $OUT"
