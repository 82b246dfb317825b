"""Per-ICP-iteration SQ counters of one lone-frame kernel (rocprofv3 --pmc csv directories of
tools/frame_probe.py, one or more passes): dispatches in order, grouped by their position in the
20-iteration frame, per wave."""
import csv
import glob
import sys
from collections import defaultdict

import numpy as np

kernel, iters = sys.argv[1], 20
per = defaultdict(lambda: defaultdict(float))
for d in sys.argv[2:]:
    rows = defaultdict(dict)
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if kernel + "<" not in r.get("Kernel_Name", "") and kernel + "(" not in r.get("Kernel_Name", ""):
                continue
            rows[int(r["Dispatch_Id"])][r["Counter_Name"]] = rows[int(r["Dispatch_Id"])].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    for k, did in enumerate(sorted(rows)):
        for n, v in rows[did].items():
            per[k][n] = v
names = sorted({n for c in per.values() for n in c})
n = len(per) // iters * iters
print(f"{kernel}: {len(per)} dispatches; per wave, median over frames, by iteration")
print("iter " + " ".join(f"{c[3:]:>14s}" for c in names))
for it in range(iters):
    ks = [k for k in range(it, n, iters)]
    vals = []
    for c in names:
        v = np.median([per[k].get(c, 0.0) / max(per[k].get("SQ_WAVES", 1.0), 1.0) if c != "SQ_WAVES" else per[k].get(c, 0.0) for k in ks])
        vals.append(v)
    print(f"{it:4d} " + " ".join(f"{v:14.1f}" for v in vals))
