"""Per-ICP-iteration medians of the projection / solve kernels from a rocprofv3 kernel trace of a
one-pair-in-flight config-B run (launches come in groups of `iters` per pair, in stream order)."""
import collections
import csv
import sys

import numpy as np

path = sys.argv[1]
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 20
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
d = collections.defaultdict(list)
keys = ("k_knn_wave", "k_knn_qwave", "k_finish", "k_solve_first", "k_resid_fused", "k_resid_hist", "k_find_bins", "k_collect",
        "k_solve_final", "k_solve_small", "k_project_lane")
for r in rows:
    n = r["Kernel_Name"]
    for k in keys:
        if k + "<" in n or k + "(" in n:
            d[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k in keys:
    if not d[k]:
        continue
    a = np.array(d[k])
    m = len(a) // iters * iters
    if m and k in ("k_knn_wave", "k_knn_qwave", "k_finish"):
        med = np.median(a[:m].reshape(-1, iters), 0)
        print(f"{k:16s} sum/pair {med.sum():8.1f} us  per iter {np.round(med).astype(int).tolist()}")
    else:
        print(f"{k:16s} median {np.median(a):7.1f} us  n {len(a)}")
