"""Per-kernel HBM bytes per launch from the tools/gpu_pmc.sh counter passes.

FETCH_SIZE / WRITE_SIZE are rocprofv3 derived counters in KiB per dispatch.  gfx950 correction
(MI355X_MICROARCH.md, HBM): FETCH_SIZE reports half the bytes of 16-B/lane streaming reads, so it
is doubled; WRITE_SIZE is exact for 16-B/lane stores and float atomics.
usage: python tools/pmc_traffic.py gpurun_out/pmc profiles/r02_traffic.json [dtype columns feed [model]]
The workload the counters were collected on (default bf16 zipf device: bench.py's defaults) is
recorded as "_workload"; bench.py attaches the traffic only to a line of the same workload.
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def short(name):
    m = re.search(r"(k_[A-Za-z0-9_]+)(<[^>(]*>)?", name)
    return (m.group(1) + (m.group(2) or "")) if m else name[:60]


def collect(root, counter):
    vals = defaultdict(list)
    for f in glob.glob(os.path.join(root, counter, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") != counter:
                continue
            vals[short(r["Kernel_Name"])].append(float(r["Counter_Value"]))
    return vals


def main(root, out, dtype="bf16", columns="zipf", feed="device", model=None):
    fetch, write = collect(root, "FETCH_SIZE"), collect(root, "WRITE_SIZE")
    res = {}
    for k in sorted(set(fetch) | set(write)):
        f = sum(fetch.get(k, [0])) / max(len(fetch.get(k, [])), 1)
        w = sum(write.get(k, [0])) / max(len(write.get(k, [])), 1)
        res[k] = {"fetch_kib_raw": round(f, 1), "write_kib": round(w, 1),
                  "hbm_bytes": int(round((2 * f + w) * 1024)),
                  "launches": max(len(fetch.get(k, [])), len(write.get(k, [])))}
    res["_workload"] = {"dtype": dtype, "columns": columns, "feed": feed}
    if model:  # a non-headline row (bench.py --model): bench.py reads it only for that model
        res["_workload"]["model"] = model
    json.dump(res, open(out, "w"), indent=1, sort_keys=True)
    for k, v in sorted(((k, v) for k, v in res.items() if k != "_workload"), key=lambda kv: -kv[1]["hbm_bytes"]):
        print(f"{v['hbm_bytes'] / 1e6:10.2f} MB  {k}")


if __name__ == "__main__":
    main(*sys.argv[1:])
