"""A/B of the weight-gradient kernels on ResNet-50 b1024 shapes, one process: the tuner's pick without
the prefetch-depth-2 kernel (stages 13-15, csrc/wgrad_deep.hip) vs with it.  B=<batch> python scripts/wgrad_ab.py"""
import os, sys, statistics, torch, torch.nn as nn
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
from pytorch_imageclassification_distributed_amd.ops import hip
from pytorch_imageclassification_distributed_amd.ops._hip import gemm
SHAPES = ["512,512,3,1,1,7", "256,256,3,1,1,14", "128,128,3,1,1,28", "64,64,3,1,1,56", "256,256,3,2,1,28",
          "1024,256,1,1,0,14", "256,1024,1,1,0,14", "512,2048,1,1,0,7", "2048,512,1,1,0,7", "128,512,1,1,0,28",
          "512,128,1,1,0,28", "256,64,1,1,0,56", "64,256,1,1,0,56"]
dev = torch.device("cuda"); torch.manual_seed(0)
B = int(os.environ.get("B", "1024"))
for shape in SHAPES:
    cin, cout, k, s, p, h = (int(v) for v in shape.split(","))
    conv = nn.Conv2d(cin, cout, k, s, p, bias=False).to(dev).to(memory_format=torch.channels_last)
    x = torch.randn(B, cin, h, h, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    hip.ensure_channels_last_weight(conv)
    g = hip.conv_geom(x, conv)
    y = hip.conv_forward_raw(x, conv.weight, g)
    dy = torch.randn_like(y)
    m, ntot = g.N * g.OH * g.OW, g.T * cin
    flops = 2.0 * m * cout * ntot
    res = {}
    for arm, deep in (("old", False), ("new", True)):
        gemm.WGRAD_DEEP = deep
        gemm._WGRAD_TUNED.clear()
        kps, splits, st = gemm._wgrad_plan(g, dy, x, m, ntot)
        out = torch.zeros(cout * ntot, device=dev)
        ts = []
        for r in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                gemm._wgrad_launch(dy, x, out, g, m, ntot, kps, splits, st)
            e1.record(); torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) / 10 * 1e3)
        res[arm] = (statistics.median(ts), st, splits)
    o, n = res["old"], res["new"]
    times = gemm.WGRAD_TUNE_LOG[-1][3]  # the "new" arm's tuning: best time per stages value
    per = {}
    for (cand, st), ms in times.items():
        if st not in per or ms < per[st][0]:
            per[st] = (ms, cand)
    print("   per stages (us, blocks): " + "  ".join(f"{st}:{ms * 1e3:.0f}/{c}" for st, (ms, c) in sorted(per.items())))
    print(f"{shape:20s} old {o[0]:7.1f} us (st {o[1]:2d}, {o[2]:4d} splits, {flops / o[0] / 1e6:5.0f} TF) | "
          f"new {n[0]:7.1f} us (st {n[1]:2d}, {n[2]:4d} splits, {flops / n[0] / 1e6:5.0f} TF) | {o[0] / n[0]:.2f}x", flush=True)
