set -o pipefail
# which fused path makes a --deterministic ResNet-50 run irreproducible (ResNet-18 is bitwise reproducible)
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for e in "-" "IMGCLS_STEM_XA=0" "IMGCLS_DS_FUSE=0" "IMGCLS_RES_DEFER=0" "IMGCLS_XA_OUT=0" "IMGCLS_FUSED_BWD=0" "IMGCLS_BN_XA=0" "IMGCLS_FUSE_BN_BWD=0" "IMGCLS_WGRAD_STREAM=0"; do
  envs=(); [ "$e" != "-" ] && read -ra envs <<< "$e"
  echo "== $e: $(env "${envs[@]}" timeout -k 10 200 python scripts/det_check.py resnet50 96 30 32 2>&1 | grep 'bitwise' )" | tee -a gpurun_out/r16d_det.txt || exit 1
done
