set -o pipefail
# Final round-6 build: conv FLOP/byte roofline and PMC passes over a ResNet-50 b1024 step (compare r15a, the
# round-6 starting point), and PMC passes over an Inception-v3 b128 step.
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=r17k
timeout -k 10 300 python scripts/conv_roofline.py 1024 > gpurun_out/${T}_conv_roofline.txt 2>&1 || { tail -5 gpurun_out/${T}_conv_roofline.txt; exit 1; }
grep -A4 "conv GEMM launches" gpurun_out/${T}_conv_roofline.txt
bash scripts/pmc_passes.sh ${T}_pmc python3 bench.py --steps 2 --warmup 2 || exit 1
python scripts/pmc_summary.py gpurun_out/${T}_pmc_a gpurun_out/${T}_pmc_b > gpurun_out/${T}_pmc_summary.txt
head -12 gpurun_out/${T}_pmc_summary.txt
bash scripts/pmc_passes.sh ${T}_incpmc python3 bench.py --model inceptionv3 --image-size 299 --batch 128 --steps 2 --warmup 2 || exit 1
python scripts/pmc_summary.py gpurun_out/${T}_incpmc_a gpurun_out/${T}_incpmc_b > gpurun_out/${T}_incpmc_summary.txt
head -12 gpurun_out/${T}_incpmc_summary.txt
