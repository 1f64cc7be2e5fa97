"""End-to-end train.py on CPU (BASELINE config 1): loop semantics, checkpoint layout, resume."""
import os

import pytest
import torch

import train
from pytorch_imageclassification_distributed_amd.utils import load_checkpoint

ARGS = ["--synthetic", "--model", "resnet18", "--image-size", "32", "--device", "cpu", "--batchsize", "16",
        "--num-workers", "0", "--synthetic-train-size", "96", "--synthetic-val-size", "32", "--lr", "2e-3",
        "--no-progress", "--val-batchsize", "8"]


def test_train_checkpoint_and_resume(tmp_path, capsys):
    ck = str(tmp_path)
    hist = train.main(ARGS + ["--epochs", "3", "--ckpt-dir", ck, "--resume", "none"])
    out = capsys.readouterr().out
    assert "Validation Accuracy" in out and "Model improved to" in out
    assert len(hist) == 3
    assert hist[-1]["train_loss"] < hist[0]["train_loss"]
    d = os.path.join(ck, "resnet18")
    best, latest = os.path.join(d, "best_model"), os.path.join(d, "latest_model")
    assert os.path.exists(best) and os.path.exists(latest)
    b = load_checkpoint(best)
    assert {"epoch", "best_score", "state_dict"} <= set(b)
    assert "module.encoder.conv1.weight" in b["state_dict"]
    assert "module.encoder.fc.6.bias" in b["state_dict"]
    lt = load_checkpoint(latest)
    assert lt["epoch"] == 0  # latest saved at epochs 0, 5, 10, ...
    assert {"optimizer", "scheduler", "rng"} <= set(lt)
    # resume from best (reference default) honours the stored epoch
    hist2 = train.main(ARGS + ["--epochs", "4", "--ckpt-dir", ck, "--resume", "best"])
    out = capsys.readouterr().out
    assert "Loading Checkpoint from best_model" in out
    assert [h["epoch"] for h in hist2] == list(range(b["epoch"] + 1, 4))


def test_lr_schedule_multistep(tmp_path):
    hist = train.main(ARGS + ["--epochs", "3", "--ckpt-dir", str(tmp_path), "--resume", "none",
                              "--milestones", "1", "2", "--gamma", "0.5", "--steps-per-epoch", "1",
                              "--val-steps", "1"])
    # lr recorded after scheduler.step(): 2e-3 halves at epoch-count 1 and 2
    assert [h["lr"] for h in hist] == pytest.approx([1e-3, 5e-4, 5e-4])


def test_inception_aux_loss_path(tmp_path):
    # the aux head (avgpool 5x5/3 -> 5x5 conv) needs the full 299 resolution (Mixed_6e at 17x17)
    hist = train.main(["--synthetic", "--model", "inceptionv3", "--image-size", "299", "--device", "cpu",
                       "--batchsize", "2", "--num-workers", "0", "--synthetic-train-size", "4",
                       "--synthetic-val-size", "2", "--no-progress", "--epochs", "1", "--ckpt-dir", str(tmp_path),
                       "--resume", "none", "--val-batchsize", "2"])
    assert torch.isfinite(torch.tensor(hist[0]["train_loss"]))


def test_step_timers_metrics_and_profiler(tmp_path):
    """--step-timers writes per-phase step timing + throughput to the JSONL metrics file;
    --profile-steps writes a torch.profiler chrome trace containing the phase ranges."""
    import json
    metrics = tmp_path / "m.jsonl"
    prof = tmp_path / "prof"
    train.main(ARGS + ["--epochs", "1", "--ckpt-dir", str(tmp_path), "--resume", "none", "--steps-per-epoch", "5",
                       "--val-steps", "1", "--step-timers", "--log-interval", "2", "--metrics-file", str(metrics),
                       "--profile-steps", "2", "--profile-start", "1", "--profile-dir", str(prof)])
    recs = [json.loads(line) for line in metrics.read_text().splitlines()]
    steps = [r for r in recs if r["kind"] == "step"]
    assert len(steps) == 2 and [r["step"] for r in steps] == [2, 4]
    for r in steps:
        assert r["images_per_sec"] > 0
        assert {"ms_forward", "ms_backward", "ms_comm_wait", "ms_optimizer", "ms_data"} <= set(r)
        assert r["ms_forward"] > 0 and r["ms_backward"] > 0
    assert [r for r in recs if r["kind"] == "epoch"]
    trace = json.loads((prof / "trace_rank0.json").read_text())
    names = {e.get("name") for e in trace.get("traceEvents", [])}
    assert {"imgcls::forward", "imgcls::backward", "imgcls::optimizer"} <= names


def test_full_resume_continues_the_run(tmp_path):
    """SURVEY 5.4 full resume: ``latest_model`` carries optimizer, scheduler, RNG and sampler epoch, so
    'train 1 epoch, stop, resume, train 1 more' reproduces the uninterrupted 2-epoch run."""
    common = ARGS + ["--latest-every", "1", "--steps-per-epoch", "3", "--val-steps", "1"]
    full = train.main(common + ["--epochs", "2", "--ckpt-dir", str(tmp_path / "a"), "--resume", "none"])
    train.main(common + ["--epochs", "1", "--ckpt-dir", str(tmp_path / "b"), "--resume", "none"])
    lt = load_checkpoint(str(tmp_path / "b" / "resnet18" / "latest_model"))
    assert lt["sampler_epoch"] == 0 and isinstance(lt["rng"]["numpy"], dict)
    rest = train.main(common + ["--epochs", "2", "--ckpt-dir", str(tmp_path / "b"), "--resume", "latest"])
    assert [h["epoch"] for h in rest] == [1]
    assert rest[0]["train_loss"] == pytest.approx(full[1]["train_loss"], rel=1e-4)
    assert rest[0]["lr"] == full[1]["lr"]


def test_rng_state_roundtrip():
    import random

    import numpy as np

    from pytorch_imageclassification_distributed_amd.utils import restore_rng_state
    from pytorch_imageclassification_distributed_amd.utils.checkpoint import _rng_state
    torch.manual_seed(3)
    np.random.seed(4)
    random.seed(5)
    st = _rng_state()
    a = (torch.rand(3), np.random.rand(3), random.random(), np.random.randn())
    torch.rand(7), np.random.rand(5), random.random()
    restore_rng_state(st)
    b = (torch.rand(3), np.random.rand(3), random.random(), np.random.randn())
    assert torch.equal(a[0], b[0]) and np.array_equal(a[1], b[1]) and a[2] == b[2] and a[3] == b[3]


def test_step_throttle_bounds_steps_in_flight(monkeypatch):
    """Trainer._throttle waits on the oldest step's end event once MAX_INFLIGHT_STEPS are enqueued (the guard
    against the allocator growth of an unbounded host run-ahead, docs/DESIGN.md)."""
    import collections
    import types

    from pytorch_imageclassification_distributed_amd.engine import trainer as tm

    waited = []

    class Ev:
        def __init__(self, i):
            self.i = i

        def synchronize(self):
            waited.append(self.i)

    monkeypatch.setattr(tm, "MAX_INFLIGHT_STEPS", 2)
    fake = types.SimpleNamespace(dev=types.SimpleNamespace(type="cuda"), _inflight=collections.deque(),
                                 _auto_inflight=None, _steps_enqueued=0)
    fake._inflight_limit = lambda: tm.Trainer._inflight_limit(fake)
    for i in range(5):
        tm.Trainer._throttle(fake)
        assert len(fake._inflight) < 2
        fake._inflight.append(Ev(i))  # what _step_enqueued records after the step
    assert waited == [0, 1, 2]
    monkeypatch.setattr(tm, "MAX_INFLIGHT_STEPS", 0)  # 0: unbounded, never waits
    tm.Trainer._throttle(fake)
    assert waited == [0, 1, 2]
    # unset (-1): 2 while the first steps tune, then the memory-based choice (3 for a small step)
    monkeypatch.setattr(tm, "MAX_INFLIGHT_STEPS", -1)
    assert tm.Trainer._inflight_limit(fake) == 2
    fake._steps_enqueued, fake._auto_inflight = 5, 3
    assert tm.Trainer._inflight_limit(fake) == 3


def test_hip_graph_auto_mode():
    """--hip-graph on / off / auto: auto replays the step as a graph at a per-GPU batch of at most
    GRAPH_AUTO_MAX_BATCH (where replay measured faster than eager dispatch), at any world size (N > 1: the
    Trainer also needs the peer SyncBN transport or SyncBN off, ``Trainer.graph_capable``); the bare flag
    still means on."""
    from pytorch_imageclassification_distributed_amd.engine.config import (GRAPH_AUTO_MAX_BATCH, build_parser,
                                                                           hip_graph_enabled)
    p = build_parser()
    a = p.parse_args(["--batchsize", "4"])
    assert a.hip_graph == "auto" and hip_graph_enabled(a, 1) and hip_graph_enabled(a, 2)
    a = p.parse_args(["--batchsize", str(GRAPH_AUTO_MAX_BATCH + 1)])
    assert not hip_graph_enabled(a, 1)
    a = p.parse_args(["--batchsize", "512", "--hip-graph"])
    assert a.hip_graph == "on" and hip_graph_enabled(a, 1)
    a = p.parse_args(["--batchsize", "4", "--hip-graph", "off"])
    assert not hip_graph_enabled(a, 1)
