"""Stream-race detection: deterministic training steps digest bitwise the same with every kernel
serialised (AMD_SERIALIZE_KERNEL=3) as with the side / comm / copy streams running concurrently
(scripts/race_check.py).  A missing stream wait would make the concurrent digest differ."""
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _digest(serialize: bool, model: str) -> str:
    env = dict(os.environ)
    env.pop("AMD_SERIALIZE_KERNEL", None)
    if serialize:
        env["AMD_SERIALIZE_KERNEL"] = "3"
    env["MASTER_ADDR"] = "127.0.0.1"
    with socket.socket() as s:  # the pytest process may already hold its own rendezvous port
        s.bind(("127.0.0.1", 0))
        env["MASTER_PORT"] = str(s.getsockname()[1])
    # fixed kernel choices in both processes (the per-shape tuner times candidates, and serialised timings
    # could pick other kernels - another fp32 summation order, not a race)
    env.update(IMGCLS_CONV_STAGES="1", IMGCLS_WGRAD_STAGES="2", IMGCLS_WGRAD_BLOCKS="256", IMGCLS_DIRECT_CONV="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "race_check.py"), "--model", model,
                        "--steps", "3"], capture_output=True, text=True, env=env, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("race_check")][-1]
    return line.split()[-1]


@pytest.mark.parametrize("model", ["resnet18"])
def test_serialized_equals_concurrent(model):
    assert _digest(False, model) == _digest(True, model)
