"""Inter-kernel gaps at the start and end of the timed region of a bench kernel trace
(rocprofv3 --kernel-trace csv): the region is the last run of kernels holding `steps` Adam launches."""
import csv
import re
import sys

path, steps = sys.argv[1], int(sys.argv[2])
rows = list(csv.DictReader(open(path)))
ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), (re.findall(r"k_\w+|__amd\w+|\w+Functor", r["Kernel_Name"]) or ["?"])[0])
            for r in rows)
adam = [i for i, k in enumerate(ks) if "adam" in k[2]]
end = adam[-1]
start = adam[-steps] - 10
seg = ks[start:end + 1]
gaps = [(seg[i + 1][0] - seg[i][1]) / 1e3 for i in range(len(seg) - 1)]
print(f"steps={steps} span={(seg[-1][1] - seg[0][0]) / 1e3:.1f}us gaps_sum={sum(g for g in gaps if g > 0):.1f}us")
print(" head:", [(seg[i + 1][2], round(gaps[i], 1)) for i in range(8)])
print(" tail:", [(seg[i + 1][2], round(gaps[i], 1)) for i in range(len(gaps) - 8, len(gaps))])
big = [(i, round(g, 1)) for i, g in enumerate(gaps) if g > 3]
print(" gaps>3us at node:", big[:20], "of", len(gaps))
