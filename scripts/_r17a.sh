set -o pipefail
# final build: Inception-v3 b128 byte roofline (merged heads, one-launch small BNs) and ResNet-50 b1024 byte roofline
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=r17a
bp() { local tag=$1; shift
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 240 rocprofv3 --pmc $c -d gpurun_out/${T}_${tag}_$c -o p --output-format csv -- python3 bench.py "$@" \
      > gpurun_out/${T}_${tag}_$c.log 2>&1 || { tail -5 gpurun_out/${T}_${tag}_$c.log; return 1; }
    f=$(find gpurun_out/${T}_${tag}_$c -name p_counter_collection.csv | head -1)
    [ "$f" = "gpurun_out/${T}_${tag}_$c/p_counter_collection.csv" ] || mv "$f" gpurun_out/${T}_${tag}_$c/p_counter_collection.csv
  done
  python scripts/byte_roofline.py gpurun_out/${T}_${tag}_FETCH_SIZE gpurun_out/${T}_${tag}_WRITE_SIZE > gpurun_out/${T}_${tag}_byte_roofline.txt || return 1
  rm -rf gpurun_out/${T}_${tag}_FETCH_SIZE gpurun_out/${T}_${tag}_WRITE_SIZE
  head -12 gpurun_out/${T}_${tag}_byte_roofline.txt; }
bp incep --model inceptionv3 --image-size 299 --batch 128 --warmup 3 --steps 2 || exit 1
bp r50 --batch 1024 --warmup 3 --steps 2 || exit 1
