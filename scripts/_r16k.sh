set -o pipefail
# fused BN-backward operand map on more replication (IMGCLS_XA_MAX_REP: 3x3 producers take XA above 2), ResNet-50 b1024
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=r16k_xarep ROUNDS=2 bash scripts/ab_env.sh "-" "IMGCLS_XA_MAX_REP=9" "IMGCLS_XA_MAX_REP=18" || exit 1
