set -o pipefail
# ResNet-50 b1024 with every training BN on the one-launch kernels (IMGCLS_BN_FIN_MAX unbounded), 256 / 1024 / 4096 row blocks
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=r17g_r50 ROUNDS=2 bash scripts/ab_env.sh "-" "IMGCLS_BN_FIN_MAX=2147483647" "IMGCLS_BN_FIN_MAX=2147483647 IMGCLS_BN_FIN_BLOCKS=1024" "IMGCLS_BN_FIN_MAX=2147483647 IMGCLS_BN_FIN_BLOCKS=4096" || exit 1
