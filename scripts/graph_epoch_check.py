"""Per-step losses of Trainer.fit()'s epoch loop with HIP-graph replay, around the epoch boundary (diagnostic).

    python scripts/graph_epoch_check.py [--epochs 3] [--latest] [--no-val] [--graph on|off] [--det]

Runs the same epoch driver as Trainer.fit (train_epoch -> scheduler -> empty_cache -> val_epoch -> checkpoint
saves) but prints every step's loss, so a corruption that starts at an epoch boundary shows where.
"""
from __future__ import annotations

import argparse
import os
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from pytorch_imageclassification_distributed_amd.engine import Trainer, build_parser  # noqa: E402
from pytorch_imageclassification_distributed_amd.parallel import init_distributed  # noqa: E402
from pytorch_imageclassification_distributed_amd.utils import LATEST, save_checkpoint  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--epochs", type=int, default=3)
    ap.add_argument("--latest", action="store_true")
    ap.add_argument("--optim-state", action="store_true", help="only call optimizer.state_dict() at epoch end")
    ap.add_argument("--no-val", action="store_true")
    ap.add_argument("--graph", default="on")
    ap.add_argument("--det", action="store_true")
    ap.add_argument("--memtrace", action="store_true",
                    help="record allocator history; list blocks alive at capture start that are freed before epoch 1")
    a = ap.parse_args()
    if a.memtrace:
        torch.cuda.memory._record_memory_history(max_entries=2_000_000, stacks="python")
    args = ["--synthetic", "--model", "resnet18", "--image-size", "64", "--batchsize", "64", "--lr", "5e-4",
            "--synthetic-train-size", "1024", "--synthetic-val-size", "128", "--val-batchsize", "64",
            "--no-progress", "--num-workers", "0", "--resume", "none", "--hip-graph", a.graph,
            "--ckpt-dir", tempfile.mkdtemp()] + (["--deterministic"] if a.det else [])
    targs = build_parser().parse_args(args)
    ctx = init_distributed(device="cuda")
    tr = Trainer(targs, ctx)
    marks = {}
    if a.memtrace:
        orig_capture = tr.capture_step

        def traced_capture(images, labels):
            marks["c0"] = len(torch.cuda.memory._snapshot()["device_traces"][0])
            orig_capture(images, labels)
            marks["c1"] = len(torch.cuda.memory._snapshot()["device_traces"][0])
        tr.capture_step = traced_capture

    def report_frees():
        tr_ = torch.cuda.memory._snapshot()["device_traces"][0]
        c0, c1 = marks["c0"], marks["c1"]
        alive = {}
        for i, e in enumerate(tr_[:c0]):
            if e["action"] == "alloc":
                alive[e["addr"]] = e
            elif e["action"] == "free_requested":
                alive.pop(e["addr"], None)

        def where(fr):
            fr = [f for f in fr if f["filename"].endswith(".py") and "-packages" not in f["filename"]]
            return " <- ".join(f"{os.path.basename(f['filename'])}:{f['line']}:{f['name']}" for f in fr[:4])
        print(f"  memtrace: {len(alive)} blocks alive at capture start; trace {c0}..{c1}..{len(tr_)}", flush=True)
        for i, e in enumerate(tr_[c0:], start=c0):
            if e["action"] == "free_requested" and e["addr"] in alive:
                al = alive.pop(e["addr"])
                phase = "DURING CAPTURE" if i < c1 else "after capture"
                print(f"    freed {phase}: {al['size']} B @ {al['addr']:#x} stream {al.get('stream')}\n"
                      f"      alloc: {where(al.get('frames', []))}\n      free : {where(e.get('frames', []))}",
                      flush=True)
    def sums():
        torch.cuda.synchronize()
        out = {}
        out["params"] = sum(float(p.detach().double().abs().sum()) for p in tr.model.parameters())
        out["bufs"] = sum(float(b.detach().double().abs().sum()) for n, b in tr.model.named_buffers() if "running" in n)
        m = v = 0.0
        for st in tr.optimizer.state.values():
            if "exp_avg" in st:
                m += float(st["exp_avg"].double().abs().sum())
                v += float(st["exp_avg_sq"].double().abs().sum())
        out["m"], out["v"] = m, v
        from pytorch_imageclassification_distributed_amd.ops import hip
        out["shadows"] = sum(float(e.t.double().abs().sum()) for e in hip._SHADOWS.values())
        out["tt"] = sum(float(e.tt.double().abs().sum()) for e in hip._SHADOWS.values() if e.tt is not None)
        w = hip.ws(tr.dev)
        out["stats(=0)"] = float(w.stats.double().abs().sum())
        out["parts(=0)"] = sum(float(b.double().abs().sum()) for b in w.parts)
        out["nparts"] = len(w.parts)
        out["wgrad_ws"] = sum(float(b.double().abs().nansum()) for b in hip._WGRAD_WS.values())
        out["n_wgrad_ws"] = len(hip._WGRAD_WS)
        return out

    def bad_grads(tag):
        torch.cuda.synchronize()
        rows = []
        for n, p in tr.model.named_parameters():
            g = p.grad
            if g is None:
                continue
            mx = float(g.detach().float().abs().max())
            rows.append((n, mx, tuple(p.shape)))
        bad = [r for r in rows if not (r[1] < 1e3)]
        print(f"  {tag}: {len(bad)}/{len(rows)} grads with |g|max >= 1e3 or non-finite; "
              f"max finite {max((r[1] for r in rows if r[1] < 1e3), default=0):.3g}", flush=True)
        for n, mx, shp in bad[:12]:
            print(f"    {n} {shp} {mx:.3g}", flush=True)

    def diff(tag, a_, b_):
        ch = [k for k in a_ if a_[k] != b_[k]]
        print(f"  {tag}: changed {ch}" + "".join(f" {k} {a_[k]:.6g}->{b_[k]:.6g}" for k in ch), flush=True)

    for epoch in range(a.epochs):
        tr.train_sampler.set_epoch(epoch)
        tr.net.train()
        losses = []
        for i, b in enumerate(tr._loader(tr.train_loader)):
            if i == 0 and epoch > 0:
                if a.memtrace and epoch == 1:
                    report_frees()
                sa = sums()
            loss = tr._epoch_step(b["image"].to(tr.dev, non_blocking=True), b["label"].to(tr.dev, non_blocking=True), i)
            losses.append(float(loss.item()))
            if i == 0 and epoch > 0:
                diff("first step", sa, sums())
                bad_grads("first step grads")
            if i == 15 and epoch == 0:
                bad_grads("last step grads (epoch 0)")
        print(f"epoch {epoch} graph={tr._graph is not None}: " + " ".join(f"{v:.3g}" for v in losses), flush=True)
        s0 = sums()
        tr.scheduler.step()
        torch.cuda.empty_cache()
        if not a.no_val:
            print(f"  val {tr.val_epoch(epoch):.1f}", flush=True)
        s1 = sums()
        diff("val", s0, s1)
        if a.latest:
            save_checkpoint(tr.ckpt_path(LATEST), tr.model, epoch, 0.0, tr.optimizer, tr.scheduler)
        elif a.optim_state:
            tr.optimizer.state_dict()
        s2 = sums()
        diff("save", s1, s2)


if __name__ == "__main__":
    main()
