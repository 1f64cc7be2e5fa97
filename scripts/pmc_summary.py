"""Summarise rocprofv3 --pmc CSV passes of scripts/conv_probe.py runs (one directory per counter pass).

    python scripts/pmc_summary.py gpurun_out/r5e_pmc_*_a gpurun_out/r5e_pmc_*_b

Per conv kernel: MFMA utilisation (SQ_VALU_MFMA_BUSY_CYCLES over SIMD-cycles = GRBM_GUI_ACTIVE / 8 XCDs x 1024
SIMDs), the wave-cycle split (parked on waitcnt / barrier, issue-stalled, issuing), VALU and LDS instructions
per wave, LDS bank-conflict share.  Means over the dispatches of the kernel.
"""
import collections
import csv
import os
import sys

runs = collections.defaultdict(dict)  # (probe tag, kernel) -> counter -> mean
for d in sys.argv[1:]:
    f = os.path.join(d, "p_counter_collection.csv")
    if not os.path.exists(f):
        continue
    tag = os.path.basename(d)[:-2]
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if not any(t in k for t in ("glds_kernel", "direct_conv", "direct64", "deep_kernel", "Cijk", "conv_pw", "wgrad", "fused_bwd", "bn_apply", "bn_bwd", "stem")):
            continue
        kn = k.replace("void ", "", 1).replace("(anonymous namespace)::", "").split("(")[0]
        acc[kn][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for kn, cs in acc.items():
        runs[(tag, kn)].update({c: sum(v) / len(v) for c, v in cs.items()})
        runs[(tag, kn)]["kernel"] = kn
for (tag, _kn), c in sorted(runs.items()):
    simd_cycles = c.get("GRBM_GUI_ACTIVE", 0) / 8 * 1024
    wc = c.get("SQ_WAVE_CYCLES", 0) or 1
    waves = c.get("SQ_WAVES", 0) or 1
    print(f"{tag}: {c.get('kernel', '?')[:90]}")
    if simd_cycles:
        print(f"  MFMA busy {100 * c.get('SQ_VALU_MFMA_BUSY_CYCLES', 0) / simd_cycles:5.1f} % of SIMD-cycles")
    print(f"  wave-cycles: parked (waitcnt / barrier) {100 * c.get('SQ_WAIT_ANY', 0) / wc:4.1f} %, issue-stalled "
          f"{100 * c.get('SQ_WAIT_INST_ANY', 0) / wc:4.1f} % (LDS issue {100 * c.get('SQ_WAIT_INST_LDS', 0) / wc:4.1f} %), "
          f"issuing {100 * c.get('SQ_ACTIVE_INST_ANY', 0) / wc:4.1f} %")
    print(f"  per wave: {c.get('SQ_INSTS_VALU', 0) / waves:7.0f} VALU, {c.get('SQ_INSTS_LDS', 0) / waves:6.0f} LDS instructions; "
          f"LDS bank-conflict cycles {100 * c.get('SQ_LDS_BANK_CONFLICT', 0) / max(c.get('SQ_LDS_IDX_ACTIVE', 1), 1):4.1f} % of LDS-active")
