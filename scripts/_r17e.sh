set -o pipefail
# final build: GPU check (suite, smoke, headline, Inception b4, step breakdown), then the model zoo
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=r17e bash scripts/gpu_check.sh || exit 1
TAG=r17f bash scripts/bench_models.sh || exit 1
