"""Summarise a rocprofv3 kernel trace: per-kernel average duration and one step's launch sequence
(durations and gaps).  Usage: python tools/kstats.py gpurun_out/prof/run_kernel_trace.csv"""
import csv
import sys
from collections import defaultdict


def short(name):
    n = name.replace("dssm::(anonymous namespace)::", "").replace("void ", "").split("(")[0]
    return n[:48]


def main(path, tail=16):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    agg = defaultdict(list)
    for r in rows:
        agg[short(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000)
    for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        print(f"{k:50s} n={len(v):5d} avg={sum(v) / len(v):8.2f} us")
    print("--- last launches (duration, gap before) ---")
    prev = None
    for r in rows[-tail:]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gap = (s - prev) / 1000 if prev else 0.0
        print(f"{short(r['Kernel_Name']):50s} {(e - s) / 1000:8.2f} {gap:7.2f}")
        prev = e


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 16)
