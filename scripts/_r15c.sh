set -o pipefail
# FETCH_SIZE calibration, current-build ResNet-50 b1024 byte roofline, allocator steady state across models,
# and the changed GPU tests (round 6)
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=r15c
hipcc -O3 --offload-arch=gfx950 scripts/probes/fetch_calib.hip -o /tmp/fetch_calib || exit 1
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 60 rocprofv3 --pmc $c -d gpurun_out/${T}_calib_$c -o p --output-format csv -- /tmp/fetch_calib \
    > gpurun_out/${T}_calib_$c.log 2>&1 || { tail -5 gpurun_out/${T}_calib_$c.log; exit 1; }
done
python - <<'PY'
import csv, glob
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    f = glob.glob(f"gpurun_out/r15c_calib_{c}/**/p_counter_collection.csv", recursive=True)[0]
    for r in csv.DictReader(open(f)):
        print(c, r["Kernel_Name"].split("(")[0], f"{float(r['Counter_Value']) * 1024 / 2**30:.3f} GiB counted of 1 GiB moved")
PY
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_extents.py tests/test_gpu_graph_rccl.py "tests/test_hip_blocks.py::test_deferred_downsample_bn" > gpurun_out/${T}_pytest.log 2>&1; rc=$?
grep -E "passed|failed" gpurun_out/${T}_pytest.log | tail -2
[ $rc -eq 0 ] || exit 1
b() { local tag=$1; shift; timeout -k 10 400 python bench.py "$@" > gpurun_out/${T}_$tag.log 2>&1 || { tail -3 gpurun_out/${T}_$tag.log; return 1; }
      echo "$tag $(grep -h '^{"metric' gpurun_out/${T}_$tag.log | grep -o '"value": [0-9.]*\|"timed_device_[a-z]*": [0-9]*' | tr '\n' ' ')"; }
b resnet50_b1024 --batch 1024 --warmup 8 --steps 20 || exit 1
b incep_b128 --model inceptionv3 --image-size 299 --batch 128 --warmup 8 --steps 20 || exit 1
b effb3_b128 --model efficientnet-b3 --image-size 300 --batch 128 --warmup 8 --steps 20 || exit 1
b effb0_b1024 --model efficientnet-b0 --batch 1024 --warmup 8 --steps 20 || exit 1
A="--batch 1024 --warmup 3 --steps 2"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $c -d gpurun_out/${T}_r50_$c -o p --output-format csv -- python3 bench.py $A \
    > gpurun_out/${T}_r50_$c.log 2>&1 || { tail -5 gpurun_out/${T}_r50_$c.log; exit 1; }
  f=$(find gpurun_out/${T}_r50_$c -name p_counter_collection.csv | head -1); mv "$f" gpurun_out/${T}_r50_$c/p_counter_collection.csv
done
python scripts/byte_roofline.py gpurun_out/${T}_r50_FETCH_SIZE gpurun_out/${T}_r50_WRITE_SIZE > gpurun_out/${T}_r50_byte_roofline.txt || exit 1
head -14 gpurun_out/${T}_r50_byte_roofline.txt
