"""train.py end to end on the GPU through Trainer.fit() - the reference loop, not a hand-rolled one.

Reference: train.py:132-188 (epoch driver: train -> scheduler -> validate -> best / latest checkpoints) and
train.py:137-153 (resume).  The HIP path runs every kernel (forward, weighted CE, backward, fused Adam, the
eval path with the reference BN momentum) on synthetic CIFAR-style data with a class signal (SyntheticImage-
Dataset).  On the CPU (torch, fp32) the same configuration reaches 55-86 % validation accuracy over 8 epochs
at 64 x 64 (3 epochs stay at 27-43 %: the reference-momentum running statistics lag), so the bar is the best
validation accuracy, as the reference keeps it (best_model).
"""
import os

import pytest
import torch

import train
from pytorch_imageclassification_distributed_amd.utils import load_checkpoint

pytestmark = pytest.mark.gpu

ARGS = ["--synthetic", "--model", "resnet18", "--image-size", "64", "--batchsize", "64", "--lr", "5e-4",
        "--synthetic-train-size", "1024", "--synthetic-val-size", "128", "--val-batchsize", "64", "--no-progress",
        "--num-workers", "0", "--latest-every", "1"]


def test_train_py_fit_checkpoints_and_resume(tmp_path, capsys):
    ck = str(tmp_path)
    hist = train.main(ARGS + ["--epochs", "8", "--ckpt-dir", ck, "--resume", "none"])
    out = capsys.readouterr().out
    assert out.count("Validation Accuracy") == 8 and "Model improved to" in out
    assert len(hist) == 8 and all(torch.isfinite(torch.tensor(h["train_loss"])) for h in hist)
    assert hist[-1]["train_loss"] < hist[0]["train_loss"]
    best = max(h["val_acc"] for h in hist)
    assert best > 50.0, [h["val_acc"] for h in hist]  # 7 classes: chance is 14 %
    d = os.path.join(ck, "resnet18")
    b = load_checkpoint(os.path.join(d, "best_model"))
    lt = load_checkpoint(os.path.join(d, "latest_model"))
    assert b["best_score"] == pytest.approx(best)
    for c in (b, lt):
        assert "module.encoder.conv1.weight" in c["state_dict"] and "module.encoder.fc.6.bias" in c["state_dict"]
    assert lt["epoch"] == 7 and len(lt["rng_ranks"]) == 1 and {"optimizer", "scheduler"} <= set(lt)
    # resume from latest: continues at epoch 8 with the saved optimizer / scheduler / random streams
    hist2 = train.main(ARGS + ["--epochs", "9", "--ckpt-dir", ck, "--resume", "latest"])
    out = capsys.readouterr().out
    assert "Loading Checkpoint from latest_model" in out
    assert [h["epoch"] for h in hist2] == [8]
    assert hist2[0]["train_loss"] < hist[0]["train_loss"]
