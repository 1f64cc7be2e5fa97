"""Per-class HBM byte roofline of ONE training step from two rocprofv3 counter passes.

    rocprofv3 --pmc FETCH_SIZE -d <dir_fetch> -o p --output-format csv -- python3 bench.py ...
    rocprofv3 --pmc WRITE_SIZE -d <dir_write> -o p --output-format csv -- python3 bench.py ...
    python scripts/byte_roofline.py <dir_fetch> <dir_write> [peak_tbps=6.0] [fetch_scale=2.0]

``fetch_scale`` multiplies FETCH_SIZE: on gfx950 the counter reports half the bytes of 16-B-per-lane streaming
reads, global loads and LDS-DMA alike (MI355X_MICROARCH.md §HBM; calibrated on known byte counts by
scripts/probes/fetch_calib.hip, profiles/r15c_fetch_calibration.txt), which is how every kernel here reads its
tensors.  Round-5 byte rooflines (r13a, r13f) used the raw counter: their read bytes are half the real ones.

The step is the span between the last two ``adam_kernel`` dispatches of each pass (counter runs serialise
the kernels, so each dispatch's time is its own, without the side-stream overlap of a real step).  Bytes
are the TCC (L2) <-> HBM traffic of the dispatch (FETCH_SIZE + WRITE_SIZE, KiB); the roofline time of a
class is its bytes at ``peak_tbps``.  Classes are named after the pass kinds of docs/DESIGN.md.
"""
import collections
import csv
import os
import re
import sys

CLASSES = [  # first match wins
    ("depthwise", r"^dw_|dw_dgrad|dw_wgrad"),
    ("SE (squeeze-excite)", r"^se_|spatial_reduce|scale_rows"),
    ("BN apply (+act)", r"bn_apply|bn_act"),
    ("BN backward elementwise", r"bn_bwd_elemt"),
    ("BN statistics / reduces", r"bn_stats|bn_bwd_reduce|bn_reduce|bn_partials"),
    ("conv GEMM fwd/dgrad", r"conv_gemm|conv_deep|conv_fused_bwd|direct_conv|stem|halo"),
    ("conv wgrad (+reduce)", r"wgrad"),
    ("head / loss / optimizer", r"sgemm|colsum|ce_|adam|weight_t|mlp|gap|avgpool|pool"),
]


def _short(k):
    k = k.replace("void ", "").replace("(anonymous namespace)::", "")
    return re.sub(r"\((?!\)).*", "", k)[:64]


def _step(path):
    rows = list(csv.DictReader(open(os.path.join(path, "p_counter_collection.csv"))))
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    idx = [i for i, r in enumerate(rows) if "adam_kernel" in r["Kernel_Name"]]
    if len(idx) < 2:
        raise SystemExit(f"{path}: fewer than two optimizer steps")
    return rows[idx[-2] + 1:idx[-1] + 1]


def main():
    fetch, write = _step(sys.argv[1]), _step(sys.argv[2])
    peak_bw = float(sys.argv[3]) if len(sys.argv) > 3 else 6.0
    fscale = float(sys.argv[4]) if len(sys.argv) > 4 else 2.0
    if len(fetch) != len(write):
        raise SystemExit("the two passes ran different kernel sequences")
    # the per-shape tuner may pick another tile for a shape the find-db does not list: pair dispatches by
    # position (same layer) and report how many differ
    diff = sum(f["Kernel_Name"] != w["Kernel_Name"] for f, w in zip(fetch, write))
    if diff:
        print(f"({diff} of {len(fetch)} dispatches ran a different kernel variant in the WRITE_SIZE pass; "
              f"paired by position, named after the FETCH_SIZE pass)")
    per = collections.defaultdict(lambda: [0.0, 0.0, 0])  # kernel -> [us, bytes, launches]
    for f, w in zip(fetch, write):
        k = _short(f["Kernel_Name"])
        us = (int(f["End_Timestamp"]) - int(f["Start_Timestamp"])) / 1e3
        nb = (fscale * float(f["Counter_Value"]) + float(w["Counter_Value"])) * 1024.0
        per[k][0] += us
        per[k][1] += nb
        per[k][2] += 1
    cls = collections.defaultdict(lambda: [0.0, 0.0, 0])
    owner = {}
    for k, (us, nb, n) in per.items():
        c = next((name for name, rx in CLASSES if re.search(rx, k)), "other")
        owner[k] = c
        cls[c][0] += us
        cls[c][1] += nb
        cls[c][2] += n
    tot_us = sum(v[0] for v in per.values())
    tot_b = sum(v[1] for v in per.values())
    print(f"(FETCH_SIZE x {fscale:g}: gfx950 counts half the bytes of 16-B streaming reads)")
    print(f"one step, kernels serialised: {tot_us / 1e3:.2f} ms, {tot_b / 1e9:.2f} GB HBM traffic "
          f"({tot_b / tot_us / 1e6:.2f} TB/s mean); roofline at {peak_bw:.1f} TB/s = {tot_b / peak_bw / 1e9:.2f} ms")
    print(f"{'class':28s} {'ms':>7s} {'GB':>7s} {'TB/s':>5s} {'roof_ms':>7s} {'x_roof':>6s} {'launch':>6s}")
    for c, (us, nb, n) in sorted(cls.items(), key=lambda kv: -kv[1][0]):
        roof = nb / peak_bw / 1e9
        print(f"{c:28s} {us / 1e3:7.2f} {nb / 1e9:7.2f} {nb / us / 1e6:5.2f} {roof:7.2f} {us / 1e3 / max(roof, 1e-9):6.2f} {n:6d}")
    print()
    print(f"{'kernel':64s} {'class':24s} {'ms':>6s} {'GB':>6s} {'TB/s':>5s} {'n':>4s}")
    for k, (us, nb, n) in sorted(per.items(), key=lambda kv: -kv[1][0])[:40]:
        print(f"{k:64s} {owner[k][:24]:24s} {us / 1e3:6.2f} {nb / 1e9:6.2f} {nb / us / 1e6:5.2f} {n:4d}")


if __name__ == "__main__":
    main()
