"""Checkpoint save / resume with the reference's on-disk layout.

Reference layout (train.py:132-188): ``dtmodel/cp/<name>/{best_model,latest_model}``
written by rank 0 with ``torch.save({'epoch', 'best_score', 'state_dict'})``
where ``state_dict`` keys carry DDP's ``module.`` prefix
(``module.encoder.<torchvision names>``).

Kept: paths, file names, the three keys, the ``module.`` prefix, best-on-
improvement and latest-every-5-epochs cadence.  Fixed:
* the directory is created (A10);
* ``latest_model`` additionally stores ``optimizer``, ``scheduler``, ``rng`` and
  ``sampler_epoch`` as *extra* keys (A9), and ``rng_ranks`` - every rank's random
  streams (gathered to rank 0), so a resumed multi-rank run draws per-rank dropout /
  drop-connect masks as the uninterrupted one would;
* resume honours the stored epoch, can pick ``latest`` or ``best`` (A11), and
  accepts keys with or without the ``module.`` prefix (partial key match as the
  reference does, train.py:143-147);
* writes go to a temp file + ``os.replace`` so a crash never leaves a torn file;
* loading uses ``weights_only=True`` (no code execution from checkpoint files).
"""
from __future__ import annotations

import os
import random

import numpy as np
import torch

BEST = "best_model"
LATEST = "latest_model"


def ckpt_dir(root: str, name: str) -> str:
    return os.path.join(root, name)


def ddp_state_dict(model: torch.nn.Module) -> dict:
    """state_dict with the reference's DDP key prefix ``module.``."""
    return {"module." + k: v.detach().cpu() for k, v in model.state_dict().items()}


def _rng_state() -> dict:
    """Every random stream the trainer draws from, in forms ``torch.load(weights_only=True)`` accepts
    (tensors, lists, ints, floats): torch CPU / current CUDA device, numpy's MT19937 and Python's."""
    np_st = np.random.get_state()
    py_st = random.getstate()
    st = {"torch": torch.get_rng_state(),
          "numpy": {"keys": np_st[1].tolist(), "pos": int(np_st[2]), "has_gauss": int(np_st[3]),
                    "cached_gaussian": float(np_st[4])},
          "python": {"version": int(py_st[0]), "state": list(py_st[1]),
                     "gauss_next": None if py_st[2] is None else float(py_st[2])}}
    if torch.cuda.is_available() and torch.cuda.is_initialized():
        st["cuda"] = torch.cuda.get_rng_state()
    return st


def gather_rng_states() -> list:
    """Every rank's ``_rng_state()`` on every rank (collective when a process group with > 1 rank exists)."""
    import torch.distributed as dist
    mine = _rng_state()
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return [mine]
    box = [None] * dist.get_world_size()
    dist.all_gather_object(box, mine)
    return box


def restore_rank_rng(ck: dict, rank: int, world: int) -> str:
    """Restore this rank's random streams from a checkpoint: its own entry of ``rng_ranks`` when the run has
    the same world size, else the single ``rng`` entry (rank 0's - every rank then draws the same masks).
    Returns which one was used."""
    ranks = ck.get("rng_ranks")
    if isinstance(ranks, list) and len(ranks) == world:
        restore_rng_state(ranks[rank])
        return "rank"
    if "rng" in ck:
        restore_rng_state(ck["rng"])
        return "shared"
    return "none"


def restore_rng_state(st: dict) -> None:
    """Inverse of ``_rng_state`` (resume).  Older checkpoints that stored only the key arrays restore
    what they have."""
    if "torch" in st:
        torch.set_rng_state(st["torch"])
    if "cuda" in st and torch.cuda.is_available():
        torch.cuda.set_rng_state(st["cuda"])
    npst = st.get("numpy")
    if isinstance(npst, dict):
        np.random.set_state(("MT19937", np.asarray(npst["keys"], dtype=np.uint32), npst["pos"],
                             npst["has_gauss"], npst["cached_gaussian"]))
    pyst = st.get("python")
    if isinstance(pyst, dict):
        random.setstate((pyst["version"], tuple(pyst["state"]), pyst["gauss_next"]))


def save_checkpoint(path: str, model, epoch: int, best_score: float, optimizer=None,
                    scheduler=None, extra: dict | None = None, rng_ranks: list | None = None) -> None:
    os.makedirs(os.path.dirname(path), exist_ok=True)
    payload = {"epoch": epoch, "best_score": float(best_score), "state_dict": ddp_state_dict(model)}
    if optimizer is not None:
        payload["optimizer"] = optimizer.state_dict()
    if scheduler is not None:
        payload["scheduler"] = scheduler.state_dict()
    payload["rng"] = _rng_state()
    if rng_ranks is not None:
        payload["rng_ranks"] = rng_ranks
    payload["sampler_epoch"] = epoch
    if extra:
        payload.update(extra)
    tmp = path + ".tmp"
    torch.save(payload, tmp)
    os.replace(tmp, path)


def load_checkpoint(path: str) -> dict:
    return torch.load(path, map_location="cpu", weights_only=True)


def load_model_state(model, loaded: dict) -> tuple[int, int]:
    """Partial key-matched load (reference train.py:142-148).  Returns (#matched, #model keys)."""
    sd = model.state_dict()
    norm = {}
    for k, v in loaded.items():
        norm[k[len("module."):] if k.startswith("module.") else k] = v
    matched = 0
    for k in sd:
        if k in norm and norm[k].shape == sd[k].shape:
            sd[k] = norm[k]
            matched += 1
    model.load_state_dict(sd)
    return matched, len(sd)


def resolve_resume(root: str, name: str, mode: str) -> str | None:
    """mode: 'auto' (latest, else best), 'latest', 'best', 'none', or an explicit path."""
    if mode in (None, "none"):
        return None
    d = ckpt_dir(root, name)
    if mode == "auto":
        for f in (LATEST, BEST):
            p = os.path.join(d, f)
            if os.path.exists(p):
                return p
        return None
    if mode in ("latest", "best"):
        p = os.path.join(d, LATEST if mode == "latest" else BEST)
        return p if os.path.exists(p) else None
    return mode if os.path.exists(mode) else None
