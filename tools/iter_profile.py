"""Per-ICP-iteration medians of the projection / solve kernels from a rocprofv3 kernel trace of a
one-pair-in-flight config-B run (stream order; an iteration ends at its k_finish).  The traversal of an
iteration is every k_knn_wave* launch since the previous k_finish: the one-pass k_knn_wave (iteration
0), or, from round 6, the reuse-decision launch k_knn_wave_m<KL, 1> + the compacted walk <KL, 2>
(listed separately as prep / walk)."""
import collections
import csv
import re
import sys

import numpy as np

path = sys.argv[1]
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 20
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))


def dur(r):
    return (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3


per_iter = collections.defaultdict(list)      # kind -> one value per iteration, in order
cur = collections.defaultdict(float)
single = collections.defaultdict(list)
for r in rows:
    n = r["Kernel_Name"]
    if re.search(r"k_knn_wave_m<\d+, 1>", n):
        cur["prep"] += dur(r)
        cur["k_knn_wave"] += dur(r)
    elif re.search(r"k_knn_wave_m<\d+, 2>", n):
        cur["walk"] += dur(r)
        cur["k_knn_wave"] += dur(r)
    elif "k_knn_wave<" in n or "k_knn_wave(" in n:
        cur["k_knn_wave"] += dur(r)
    elif "k_finish<" in n or "k_finish(" in n:
        for k in ("k_knn_wave", "prep", "walk"):
            per_iter[k].append(cur.get(k, 0.0))
        per_iter["k_finish"].append(dur(r))
        cur.clear()
    else:
        for k in ("k_solve_first", "k_resid_fused", "k_resid_hist", "k_find_bins", "k_collect", "k_solve_final",
                  "k_solve_small", "k_project_lane"):
            if k + "<" in n or k + "(" in n:
                single[k].append(dur(r))
for k in ("k_knn_wave", "prep", "walk", "k_finish"):
    a = np.array(per_iter.get(k, []))
    m = len(a) // iters * iters
    if not m:
        continue
    med = np.median(a[:m].reshape(-1, iters), 0)
    print(f"{k:16s} sum/pair {med.sum():8.1f} us  per iter {np.round(med).astype(int).tolist()}")
for k, v in single.items():
    print(f"{k:16s} median {np.median(v):7.1f} us  n {len(v)}")
