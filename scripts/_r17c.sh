set -o pipefail
# one-launch BN kernels with the first rows loaded before the partial-row reduce: numerics, the b128 byte roofline
# (bn_fin_* ms / TB/s against r17a), and bench numbers against the r17b defaults on this build
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_hip_blocks.py -x -q --timeout 120 --timeout-method thread -k "inception or bn_fin" > gpurun_out/r17c_pytest.log 2>&1 || { tail -30 gpurun_out/r17c_pytest.log; exit 1; }
tail -1 gpurun_out/r17c_pytest.log
T=r17c
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $c -d gpurun_out/${T}_incep_$c -o p --output-format csv -- python3 bench.py --model inceptionv3 --image-size 299 --batch 128 --warmup 3 --steps 2 > gpurun_out/${T}_incep_$c.log 2>&1 || { tail -5 gpurun_out/${T}_incep_$c.log; exit 1; }
  f=$(find gpurun_out/${T}_incep_$c -name p_counter_collection.csv | head -1)
  [ "$f" = "gpurun_out/${T}_incep_$c/p_counter_collection.csv" ] || mv "$f" gpurun_out/${T}_incep_$c/p_counter_collection.csv
done
python scripts/byte_roofline.py gpurun_out/${T}_incep_FETCH_SIZE gpurun_out/${T}_incep_WRITE_SIZE > gpurun_out/${T}_incep_byte_roofline.txt || exit 1
rm -rf gpurun_out/${T}_incep_FETCH_SIZE gpurun_out/${T}_incep_WRITE_SIZE
head -4 gpurun_out/${T}_incep_byte_roofline.txt; grep "bn_fin" gpurun_out/${T}_incep_byte_roofline.txt
for cfg in "--batch 256" "--batch 4 --steps 50 --warmup 10" "--batch 32 --steps 30 --warmup 8"; do
  for r in 1 2; do timeout -k 10 300 python bench.py --model inceptionv3 --image-size 299 $cfg > gpurun_out/${T}_run.log 2>&1 || { tail -5 gpurun_out/${T}_run.log; exit 1; }
    echo "$cfg round $r: $(grep -h '^{"metric' gpurun_out/${T}_run.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" | tee -a gpurun_out/${T}_bench.txt; done
done
