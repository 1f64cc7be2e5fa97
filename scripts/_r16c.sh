set -o pipefail
# ResNet-50 learning test: is the HIP (deterministic) trajectory unchanged by the round-6 knobs, and how much does the fp32 side vary
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for e in "-" "IMGCLS_BN_FIN=0 IMGCLS_BN_FIN_BWD=0 IMGCLS_POOL_BN_REDUCE=0 IMGCLS_WGRAD_ATOMIC_PIX=0" "-"; do
  envs=(); [ "$e" != "-" ] && read -ra envs <<< "$e"
  env "${envs[@]}" timeout -k 10 300 python -u -m pytest tests/test_gpu_learning.py -x -q -s --timeout 280 --timeout-method thread -k "resnet50" > gpurun_out/r16c_run.log 2>&1; rc=$?
  echo "== $e rc=$rc"; grep -E "hip loss|gaps|passed|failed" gpurun_out/r16c_run.log | cut -c1-200
  case $rc in 0|1) ;; *) exit 1;; esac
done
