"""Timeline of one data-parallel step from a rocprofv3 kernel trace (--kernel-trace csv): the kernels
between the last two k_adam_step launches that advance... simply the last `n` kernels of the run,
printed in start order with their start offset, duration and the idle gap before them."""
import csv
import re
import sys

path, n = sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 60
rows = list(csv.DictReader(open(path)))
ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
             (re.findall(r"k_\w+|__amd\w+|\w+Functor|\w+Kernel\w*", r["Kernel_Name"]) or [r["Kernel_Name"][:30]])[0],
             r.get("Queue_Id", r.get("Stream_Id", "?")))
            for r in rows)
seg = ks[-n:]
t0 = seg[0][0]
busy_end = seg[0][0]
for s, e, name, q in seg:
    gap = (s - busy_end) / 1e3
    print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:7.1f}  gap {gap:6.1f}  q{q}  {name}")
    busy_end = max(busy_end, e)
print(f"span {(seg[-1][1] - t0) / 1e3:.1f} us")
