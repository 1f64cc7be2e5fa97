"""Kernel-choice find-db (ops/hip.py save_tuning / load_tuning, bench.py --tune-db): round trip, entries
naming configurations this build lacks are skipped, existing choices win, the committed file parses."""
import json
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture
def hip():
    try:
        from pytorch_imageclassification_distributed_amd.ops import hip as h
    except Exception as e:  # noqa: BLE001  (no extension built)
        pytest.skip(f"extension not importable: {e}")
    keep = (dict(h._STAGES_TUNED), dict(h._WGRAD_TUNED))
    h._STAGES_TUNED.clear()
    h._WGRAD_TUNED.clear()
    yield h
    h._STAGES_TUNED.clear()
    h._WGRAD_TUNED.clear()
    h._STAGES_TUNED.update(keep[0])
    h._WGRAD_TUNED.update(keep[1])


def test_round_trip(hip, tmp_path):
    k1 = ((1024, 64, 576, 64, 8, 8, 8, 8, 1, 576, 8, 8, 1, 0, 0, 64, 0), 64, (-1, -1, -1, 0, 0, 0, 1, 1, 1),
          (-1, 0, 1) * 3, True, False, False, False, False, 0, False, True)
    k2 = k1[:1] + (128,) + k1[2:]
    hip._STAGES_TUNED[k1] = (0, 0, 1)
    hip._STAGES_TUNED[k2] = (0, 0, hip.DIRECT_BASE + 3)
    wk = (2, 64, 8, 8, 64, 3, 3, 1, 1, 1, 1, (256, 512), (1, 2))
    hip._WGRAD_TUNED[wk] = (512, 1)
    path = str(tmp_path / "db.json")
    assert hip.save_tuning(path) == 3
    hip._STAGES_TUNED.clear()
    hip._WGRAD_TUNED.clear()
    assert hip.load_tuning(path) == 3
    assert hip._STAGES_TUNED[k1] == (0, 0, 1) and hip._STAGES_TUNED[k2] == (0, 0, hip.DIRECT_BASE + 3)
    assert hip._WGRAD_TUNED[wk] == (512, 1)


def test_invalid_and_existing_entries(hip, tmp_path):
    k = ((64, 64, 64, 64, 1, 1, 1, 1, 1, 64, 1, 1, 1, 0, 0, 64, 0), 64, (0,), (0,), False, False, False, False,
         False, 0, False, True)
    db = {"conv": [[repr(k), [0, 0, 999]], [repr(k[:1] + (32,) + k[2:]), [0, 0, 0]], ["not python", [0, 0, 0]]],
          "wgrad": [["(1, 2)", [512, 99]]]}
    path = tmp_path / "db.json"
    path.write_text(json.dumps(db))
    hip._STAGES_TUNED[k[:1] + (32,) + k[2:]] = (0, 0, 2)
    assert hip.load_tuning(str(path)) == 0  # bad index, existing key, unparsable key, bad wgrad variant
    assert hip._STAGES_TUNED[k[:1] + (32,) + k[2:]] == (0, 0, 2)
    assert hip.load_tuning(str(tmp_path / "missing.json")) == 0


def test_committed_db_parses(hip):
    # every committed entry names a configuration this build has: none is dropped on load (pointwise entries,
    # cfg >= PW_BASE, used to fall into the deep-kernel range check and were skipped)
    path = os.path.join(ROOT, "tuning", "mi355x_find_db.json")
    with open(path) as f:
        db = json.load(f)
    assert hip.load_tuning(path) == len(db["conv"]) + len(db["wgrad"]) > 100


def test_round_trip_every_kernel_family(hip, tmp_path):
    base = ((1024, 64, 64, 64, 8, 8, 8, 8, 1, 64, 8, 8, 1, 0, 0, 64, 0), 64, (0,), (0,), False, False, False,
            False, False, 0, False, True)
    cfgs = [(0, 0, 0), (0, 0, hip.DIRECT_BASE + 5), (3, 128, hip.HALO_BASE), (0, 0, hip.DEEP_BASE),
            (0, 0, hip.PW_BASE + len(hip.conv_pw_cfgs()) - 1)]
    for i, v in enumerate(cfgs):
        hip._STAGES_TUNED[base[:1] + (16 * (i + 1),) + base[2:]] = v
    path = str(tmp_path / "db.json")
    assert hip.save_tuning(path) == len(cfgs)
    hip._STAGES_TUNED.clear()
    assert hip.load_tuning(path) == len(cfgs)
    assert sorted(hip._STAGES_TUNED.values()) == sorted(cfgs)


def test_diagnostic_and_disabled_families_rejected(hip, tmp_path, monkeypatch):
    """A stale or hand-edited db cannot select the deep kernel's diagnostic variants (var & 6: wrong results
    by design) or its untuned 32x32 form (var & 256), and a family switched off by its flag (IMGCLS_DEEP=0,
    IMGCLS_PW=0, ...) is not served from the db either - the same filters the tuner applies."""
    base = ((1024, 64, 64, 64, 8, 8, 8, 8, 1, 64, 8, 8, 1, 0, 0, 64, 0), 64, (0,), (0,), False, False, False,
            False, False, 0, False, True)
    deep = hip.conv_deep_cfgs()
    bad = [i for i, c in enumerate(deep) if c[4] & (6 | 256)]
    good = [i for i, c in enumerate(deep) if not c[4] & (6 | 256)]
    assert bad and good
    db = {"conv": [[repr(base[:1] + (16 * (j + 1),) + base[2:]), [0, 0, hip.DEEP_BASE + i]]
                   for j, i in enumerate(bad + good[:1])], "wgrad": []}
    path = tmp_path / "db.json"
    path.write_text(json.dumps(db))
    assert hip.load_tuning(str(path)) == 1
    assert list(hip._STAGES_TUNED.values()) == [(0, 0, hip.DEEP_BASE + good[0])]
    hip._STAGES_TUNED.clear()
    from pytorch_imageclassification_distributed_amd.ops._hip import gemm
    monkeypatch.setattr(gemm, "DEEP_CONV", False)
    assert hip.load_tuning(str(path)) == 0
