"""One step's kernel timeline (start / end relative to the step's first launch, duration) from a
rocprofv3 kernel trace: the launches between the last-but-`back` and last-but-`back-1` occurrences of
a marker kernel.  Usage: python tools/step_timeline.py run_kernel_trace.csv [marker] [back]"""
import csv
import sys


def short(n):
    return n.replace("dssm::(anonymous namespace)::", "").replace("void ", "").split("(")[0][:40]


def main(path, marker="k_loss_finalize", back=3):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
    a, b = idx[-back], idx[-back + 1]
    t0 = int(rows[a]["Start_Timestamp"])
    for r in rows[a:b + 1]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        print(f"{short(r['Kernel_Name']):42s} start {(s - t0) / 1000:8.2f} end {(e - t0) / 1000:8.2f} "
              f"dur {(e - s) / 1000:7.2f}")


if __name__ == "__main__":
    main(sys.argv[1], *(sys.argv[2:3]), *(int(x) for x in sys.argv[3:4]))
