"""Per-GEMM roofline of the convolutions in one ResNet-50 training step.

Every implicit-GEMM launch of a steady-state step (forward, data-gradient phases, weight-gradient) is
timed with HIP events around it (synchronising, so the numbers are per-launch, not overlapped), and
compared with its roofline time max(FLOP / PEAK_TF, bytes / PEAK_BW).  Sorted by time lost to the
roofline: the top rows are where kernel work pays most.

    python scripts/conv_roofline.py [batch=256] [peak_tf=2300] [peak_tbps=6.0] [model=resnet50] [image_size]
"""
import collections
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from pytorch_imageclassification_distributed_amd.data import DeviceSyntheticLoader
from pytorch_imageclassification_distributed_amd.engine import Trainer, build_parser
from pytorch_imageclassification_distributed_amd.ops import hip
from pytorch_imageclassification_distributed_amd.parallel import init_distributed

B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
PEAK_TF = float(sys.argv[2]) if len(sys.argv) > 2 else 2300.0
PEAK_BW = float(sys.argv[3]) if len(sys.argv) > 3 else 6.0
MODEL = sys.argv[4] if len(sys.argv) > 4 else "resnet50"
SIZE = int(sys.argv[5]) if len(sys.argv) > 5 else 224
REC = []
ON = [False]

_orig_gemm, _orig_wg = hip._conv_gemm, hip._wgrad_launch


def _timed(kind, fn, flop, nbytes, desc):
    if not ON[0]:
        return fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record()
    r = fn()
    b.record()
    b.synchronize()
    REC.append((kind, desc, a.elapsed_time(b) * 1e3, flop, nbytes))
    return r


def _kernel_label(geo, out, stats, bias, addend, bwd, dh, dw, kw):
    """The kernel the tuner picked for this launch (the same key as gemm._conv_gemm builds)."""
    from pytorch_imageclassification_distributed_amd.ops._hip import gemm as G
    xa, xf, y2 = kw.get("xa"), kw.get("xf"), kw.get("y2")
    key = (tuple(geo), out.shape[1], tuple(dh), tuple(dw), stats is not None, bias is not None,
           addend is not None, bwd[0] is not None, bwd[1] is not None, bwd[4], False,
           G.DIRECT_CONV) + ((True,) if xa is not None else ()) + (("xf",) if xf is not None else ()) + \
        (("y2",) if y2 is not None else ())
    cfg = G._STAGES_TUNED.get(key)
    if cfg is None:
        return "?"
    c = cfg[2]
    tag = "+xa" if xa is not None else "+xf" if xf is not None else ""
    if c >= G.PW_BASE:
        return f"pw{c - G.PW_BASE}{tag}"
    if c >= G.DEEP_BASE:
        t = G.conv_deep_cfgs()[c - G.DEEP_BASE]
        return f"deep{t[0]}x{t[1]}v{t[4]}{tag}"
    if c >= G.HALO_BASE:
        return f"halo{c - G.HALO_BASE}{tag}"
    if c >= G.DIRECT_BASE:
        return f"direct{c - G.DIRECT_BASE}{tag}"
    if c >= 0:
        t = G.conv_cfgs()[c]
        return f"glds{t[0]}x{t[1]}/{t[2]}x{t[3]}/s{t[4]}{tag}"
    return f"auto{tag}"


def gemm(A, B_, out, stats, bias, geo, dh, dw, tb, zero, addend=None, bwd=(None,) * 4 + (0, 1), **kw):
    m, n, k = geo[0], geo[1], geo[2]
    xa = kw.get("xa")
    kind = "dgrad" if (bwd[0] is not None or addend is not None or xa is not None or geo[12] > 1 or geo[13]
                       or geo[14]) else "fwd"
    nb = 2 * (A.numel() + B_.numel() + m * n) + (2 * m * n if addend is not None else 0) + \
        (4 * m * n if bwd[0] is not None else 0) + (2 * A.numel() if xa is not None else 0) + \
        (2 * A.numel() if (xa is not None and len(xa) > 2 and xa[2] is not None) else 0)  # XA_OUT writes dY
    r = _timed(kind, lambda: _orig_gemm(A, B_, out, stats, bias, geo, dh, dw, tb, zero, addend, bwd, **kw),
               2.0 * m * n * k, nb, f"M={m} N={n} K={k} CA={geo[3]}")
    if ON[0]:
        REC[-1] = REC[-1][:2] + REC[-1][2:] + (_kernel_label(geo, out, stats, bias, addend, bwd, dh, dw, kw),)
    return r


def wgrad(dy, x, out, g, m, ntot, kps, splits, stages=2, side=None, **kw):
    # timed on the current stream (the side-stream fork would escape the events); the in-step overlap
    # is not part of a per-launch roofline
    nb = 2 * (dy.numel() + x.numel()) + 4 * out.numel() * splits + (2 * dy.numel() if kw.get("xa") is not None else 0)
    if not ON[0]:
        return _orig_wg(dy, x, out, g, m, ntot, kps, splits, stages, side=side, **kw)
    return _timed("wgrad", lambda: _orig_wg(dy, x, out, g, m, ntot, kps, splits, stages, **kw), 2.0 * m * g.Co * ntot, nb,
                  f"Co={g.Co} Ntot={ntot} Mpix={m} splits={splits} st={stages}")


hip._conv_gemm, hip._wgrad_launch = gemm, wgrad

ctx = init_distributed(device="cuda")
targs = build_parser().parse_args(["--synthetic", "--model", MODEL, "--image-size", str(SIZE), "--batchsize", str(B), "--num-classes", "7",
                                   "--num-workers", "0", "--synthetic-train-size", "8", "--synthetic-val-size", "8",
                                   "--no-sync-bn", "--lr", "1e-4"])
tr = Trainer(targs, ctx)
_db = os.environ.get("IMGCLS_TUNE_DB", os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                   "tuning", "mi355x_find_db.json"))
if _db != "none" and os.path.exists(_db):
    print(f"{hip.load_tuning(_db)} kernel choices from {_db}")
tr.net.train()
batches = list(iter(DeviceSyntheticLoader(B, 7, SIZE, ctx.device, steps=2, ring=2, seed=1)))
for i in range(4):
    tr.train_step(batches[i % 2]["image"], batches[i % 2]["label"])
torch.cuda.synchronize()
ON[0] = True
tr.train_step(batches[0]["image"], batches[0]["label"])
ON[0] = False
torch.cuda.synchronize()

tot = collections.defaultdict(lambda: [0.0, 0.0])
rows = []
for kind, desc, us, flop, nb, *lab in REC:
    roof = max(flop / (PEAK_TF * 1e12), nb / (PEAK_BW * 1e12)) * 1e6
    rows.append((us - roof, kind, desc + (f"  [{lab[0]}]" if lab else ""), us, roof, flop / us / 1e6, nb / us / 1e6))
    tot[kind][0] += us
    tot[kind][1] += roof
print(f"batch {B}: {len(REC)} conv GEMM launches; roofline at {PEAK_TF:.0f} TF/s, {PEAK_BW:.1f} TB/s")
for k, (t, r) in tot.items():
    print(f"  {k:6s} {t / 1e3:7.3f} ms measured  {r / 1e3:7.3f} ms roofline")
print(f"{'lost_us':>8} {'kind':6} {'us':>8} {'roof_us':>8} {'TF/s':>6} {'TB/s':>5}  shape")
for lost, kind, desc, us, roof, tf, tb in sorted(rows, reverse=True):
    print(f"{lost:8.1f} {kind:6} {us:8.1f} {roof:8.1f} {tf:6.0f} {tb:5.2f}  {desc}")
