set -o pipefail
# 64 x 256 weight-gradient tile (stages 16): numerics, then a fresh ResNet-50 b1024 tuning run A/B'd against the shipped db
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_hip_ops.py -x -q --timeout 120 --timeout-method thread -k "wgrad_ring_variants or stem_xa or conv_bn_act_pool" > gpurun_out/r15y_pytest.log 2>&1 || { tail -30 gpurun_out/r15y_pytest.log; exit 1; }
tail -1 gpurun_out/r15y_pytest.log
TAG=r15y_retune RUNS=1 ARGS="--batch 1024" bash scripts/retune_model.sh || exit 1
grep -h "Co=64 Ntot=256\|64, 256" gpurun_out/r15y_retune_1.log | head -5
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/r15y_retune_fresh_1.json"))
w = d.get("wgrad", d)
hits = [(k, v) for k, v in (w.items() if isinstance(w, dict) else []) if "16" in str(v)]
print("wgrad entries choosing stages 16:", len(hits), hits[:4])
PY
