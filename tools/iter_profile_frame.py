"""Per-ICP-iteration medians of the lone-frame kernels (k_knn_qwave[_f], k_finish_q, k_finish_slab,
k_project_lane, k_solve_small) from a rocprofv3 kernel trace of tools/frame_probe.py (20 iterations
per frame, launches in stream order)."""
import collections
import csv
import sys

import numpy as np

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 20
keys = ("k_knn_qwave", "k_knn_qwave_f", "k_finish_q", "k_finish_slab", "k_fallback_slab", "k_project_lane", "k_solve_small")
d = collections.defaultdict(list)
gaps = []
prev_end = None
for r in rows:
    n = r["Kernel_Name"]
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    for k in keys:
        if k + "<" in n or k + "(" in n:
            d[k].append((e - s) / 1e3)
    if prev_end is not None and s > prev_end:
        gaps.append((s - prev_end) / 1e3)
    prev_end = e
for k in keys:
    a = np.array(d[k])
    m = len(a) // iters * iters
    if m:
        med = np.median(a[:m].reshape(-1, iters), 0)
        print(f"{k:15s} sum/frame {med.sum():8.1f} us  per iter {np.round(med).astype(int).tolist()}")
if gaps:
    g = np.array(gaps)
    print(f"inter-kernel gaps: median {np.median(g):.1f} us, p90 {np.percentile(g, 90):.1f} us over {len(g)} launches")
