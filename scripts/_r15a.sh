set -o pipefail
# Round-6 starting point: current-build per-GEMM roofline, PMC passes over a
# ResNet-50 b1024 step, our main loop (no epilogue) vs hipBLASLt on the 1x1 GEMMs, and the headline bench.
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=r15a
timeout -k 10 300 python bench.py --warmup 8 --steps 20 > gpurun_out/${T}_bench.log 2>&1 || { tail -5 gpurun_out/${T}_bench.log; exit 1; }
grep -h '^{"metric' gpurun_out/${T}_bench.log | cut -c1-120
timeout -k 10 300 python scripts/conv_roofline.py 1024 > gpurun_out/${T}_conv_roofline.txt 2>&1 || { tail -5 gpurun_out/${T}_conv_roofline.txt; exit 1; }
grep -A4 "conv GEMM launches" gpurun_out/${T}_conv_roofline.txt
timeout -k 10 300 python benchmarks/gemm_ref.py --batch 1024 > gpurun_out/${T}_gemm_ref.txt 2>&1 || { tail -5 gpurun_out/${T}_gemm_ref.txt; exit 1; }
bash scripts/pmc_passes.sh ${T}_pmc python3 bench.py --steps 2 --warmup 2 || exit 1
python scripts/pmc_summary.py gpurun_out/${T}_pmc_a gpurun_out/${T}_pmc_b > gpurun_out/${T}_pmc_summary.txt
head -30 gpurun_out/${T}_pmc_summary.txt
