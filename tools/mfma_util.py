"""MFMA utilisation per kernel from a rocprofv3 counter pass (tools/gpu_measure.sh) joined with the
kernel-trace averages of the same workload.

Counters (one pass: 2 SQ + 1 GRBM): SQ_INSTS_VALU_MFMA_MOPS_<T> (MFMA math ops / 512 per dispatch,
summed over the chip), SQ_VALU_MFMA_BUSY_CYCLES (cycles any MFMA was busy, summed over SIMDs),
GRBM_GUI_ACTIVE (GPU-active cycles of the dispatch).  Per kernel:
  flops / launch  = MOPS * 512
  TFLOP/s         = flops / (kernel-trace average duration)   (counter passes serialise dispatches,
                                                              so their own durations are not used)
  frac_of_peak    = TFLOP/s / dense peak (bf16 2.5 PF, fp32 MFMA 157.3 TF: MI355X_MICROARCH.md)
  mfma_busy       = BUSY_CYCLES / (1024 SIMDs * 2.4 GHz * kernel-trace duration): the share of the
                    launch's SIMD-cycles the matrix cores were busy (rocprofv3's MfmaUtil divides by
                    GRBM_GUI_ACTIVE, which on gfx950 sums the 8 XCDs and includes the counter
                    pass's serialisation, so it is not used)
usage: python tools/mfma_util.py <counter dir> <kernel_stats.csv> <out.json> [bf16|fp32 [model]]
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

PEAK_TFLOPS = {"bf16": 2500.0, "fp32": 157.3}
SIMDS = 256 * 4
CLOCK_HZ = 2.4e9


def short(name):
    m = re.search(r"(k_[A-Za-z0-9_]+)(<[^>(]*>)?", name)
    return (m.group(1) + (m.group(2) or "")) if m else name[:60]


def main(root, stats_csv, out, dtype="bf16", model=None):
    mops_name = "SQ_INSTS_VALU_MFMA_MOPS_" + ("BF16" if dtype == "bf16" else "F32")
    vals = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            vals[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    dur = {}
    for r in csv.DictReader(open(stats_csv)):
        dur[short(r["Name"])] = float(r["AverageNs"])
    res = {"_workload": {"dtype": dtype}}
    if model:  # a non-headline row (bench.py --model)
        res["_workload"]["model"] = model
    for k, c in vals.items():
        mops = c.get(mops_name, [])
        split = False
        if dtype == "fp32" and (not mops or sum(mops) == 0) and sum(c.get("SQ_INSTS_VALU_MFMA_MOPS_BF16", [])) > 0:
            # fp32 parity mode's split tiles (csrc/g32.h DSSM_G32_SPLIT): six bf16 partial products per
            # fp32 product on the bf16 matrix cores
            mops, split = c["SQ_INSTS_VALU_MFMA_MOPS_BF16"], True
        if not mops or sum(mops) == 0:
            continue
        n = len(mops)
        flops = 512.0 * sum(mops) / n
        busy = sum(c.get("SQ_VALU_MFMA_BUSY_CYCLES", [0])) / max(len(c.get("SQ_VALU_MFMA_BUSY_CYCLES", [])), 1)
        gui = sum(c.get("GRBM_GUI_ACTIVE", [0])) / max(len(c.get("GRBM_GUI_ACTIVE", [])), 1)
        e = {"launches": n, "flops_per_launch": int(flops), "mfma_busy_cycles": int(busy),
             "grbm_gui_active": int(gui)}
        if k in dur:
            tf = flops / (dur[k] * 1e-9) / 1e12
            e.update({"avg_us": round(dur[k] / 1e3, 2), "mfma_busy": round(busy / (SIMDS * CLOCK_HZ * dur[k] * 1e-9), 4)})
            if split:  # executed bf16 rate against the bf16 peak; the fp32 products (1 per 6) against fp32's
                e.update({"split_bf16x6": True, "bf16_tflops_executed": round(tf, 2), "bf16_peak_tflops": PEAK_TFLOPS["bf16"],
                          "bf16_frac_of_peak": round(tf / PEAK_TFLOPS["bf16"], 5), "tflops": round(tf / 6, 2),
                          "peak_tflops": PEAK_TFLOPS["fp32"], "frac_of_peak": round(tf / 6 / PEAK_TFLOPS["fp32"], 5)})
            else:
                e.update({"tflops": round(tf, 2), "peak_tflops": PEAK_TFLOPS[dtype],
                          "frac_of_peak": round(tf / PEAK_TFLOPS[dtype], 5)})
        res[k] = e
    json.dump(res, open(out, "w"), indent=1, sort_keys=True)
    for k, v in sorted(res.items()):
        if k != "_workload":
            print(f"{k:40s} {v}")


if __name__ == "__main__":
    main(*sys.argv[1:])
