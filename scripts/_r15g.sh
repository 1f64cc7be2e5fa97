set -o pipefail
# round 6: labelled per-GEMM roofline (which kernel each launch ran), corrected byte rooflines of EfficientNet-B0
# b1024 and Inception-v3 b128, and a fresh find-db tuning of the headline config
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=r15g
timeout -k 10 300 python scripts/conv_roofline.py 1024 > gpurun_out/${T}_conv_roofline.txt 2>&1 || { tail -5 gpurun_out/${T}_conv_roofline.txt; exit 1; }
grep -A4 "conv GEMM launches" gpurun_out/${T}_conv_roofline.txt
bp() { local tag=$1; shift
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 240 rocprofv3 --pmc $c -d gpurun_out/${T}_${tag}_$c -o p --output-format csv -- python3 bench.py "$@" \
      > gpurun_out/${T}_${tag}_$c.log 2>&1 || { tail -5 gpurun_out/${T}_${tag}_$c.log; return 1; }
    f=$(find gpurun_out/${T}_${tag}_$c -name p_counter_collection.csv | head -1)
    [ "$f" = "gpurun_out/${T}_${tag}_$c/p_counter_collection.csv" ] || mv "$f" gpurun_out/${T}_${tag}_$c/p_counter_collection.csv
  done
  python scripts/byte_roofline.py gpurun_out/${T}_${tag}_FETCH_SIZE gpurun_out/${T}_${tag}_WRITE_SIZE > gpurun_out/${T}_${tag}_byte_roofline.txt || return 1
  head -12 gpurun_out/${T}_${tag}_byte_roofline.txt; }
bp effb0 --model efficientnet-b0 --batch 1024 --warmup 3 --steps 2 || exit 1
bp incep --model inceptionv3 --image-size 299 --batch 128 --warmup 3 --steps 2 || exit 1
TAG=${T}_retune RUNS=2 ARGS="--batch 1024" bash scripts/retune_model.sh || exit 1
