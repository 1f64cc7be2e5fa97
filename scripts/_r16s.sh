set -o pipefail
# Inception-v3 b128 host time per function: merged sibling heads vs the per-branch path
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for e in IMGCLS_SIBLINGS=0 IMGCLS_SIBLINGS=1; do
  env $e timeout -k 10 400 python scripts/host_fn_prof.py inceptionv3 299 128 > gpurun_out/r16s_host_$e.txt 2>&1 || { tail -20 gpurun_out/r16s_host_$e.txt; exit 1; }
  echo "== $e"; grep -A25 "^host" gpurun_out/r16s_host_$e.txt
done
