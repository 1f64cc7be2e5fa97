set -o pipefail
# Final GPU check after the find-db gained the zoo configs: suite, smoke, headline, Inception b4, step breakdown.
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=r17q bash scripts/gpu_check.sh || exit 1
