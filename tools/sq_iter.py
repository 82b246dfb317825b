"""Per-ICP-iteration SQ counters of k_knn_wave / k_finish from a rocprofv3 --pmc csv directory
(tools/gpu_sq_iter.sh): the dispatches of each kernel in order, iteration = index mod 20."""
import csv, glob, sys
from collections import defaultdict
rows = []
for f in glob.glob(f"{sys.argv[1]}/**/*counter_collection.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 20
disp = defaultdict(lambda: defaultdict(float))   # (kernel, dispatch id) -> counter -> value
for r in rows:
    name = r.get("Kernel_Name", "")
    k = "k_knn_wave" if "k_knn_wave" in name else ("k_finish" if "k_finish" in name else None)
    if not k:
        continue
    disp[(k, int(r["Dispatch_Id"]))][r["Counter_Name"]] += float(r["Counter_Value"])
for k in ("k_knn_wave", "k_finish"):
    ids = sorted(d for kk, d in disp if kk == k)
    by = defaultdict(list)
    for i, d in enumerate(ids):
        by[i % iters].append(disp[(k, d)])
    print(f"{k}: {len(ids)} dispatches")
    tot = defaultdict(float)
    for it in range(iters):
        c = by.get(it, [])
        if not c:
            continue
        avg = {n: sum(x.get(n, 0.0) for x in c) / len(c) for n in c[0]}
        w = max(avg.get("SQ_WAVES", 1.0), 1.0)
        for n, v in avg.items():
            tot[n] += v
        print(f"  it {it:2d} waves {w:6.0f} valu/wave {avg.get('SQ_INSTS_VALU', 0) / w:8.0f} salu/wave {avg.get('SQ_INSTS_SALU', 0) / w:7.0f} "
              f"lds/wave {avg.get('SQ_INSTS_LDS', 0) / w:6.0f} smem/wave {avg.get('SQ_INSTS_SMEM', 0) / w:5.0f} "
              f"wavecyc/wave {avg.get('SQ_WAVE_CYCLES', 0) / w:8.0f} wait {avg.get('SQ_WAIT_ANY', 0) / max(avg.get('SQ_WAVE_CYCLES', 1), 1):.2f} "
              f"valu {avg.get('SQ_INSTS_VALU', 0) / 1e6:7.2f}M")
    print(f"  total per pair: valu {tot['SQ_INSTS_VALU'] / 1e6:.1f}M salu {tot['SQ_INSTS_SALU'] / 1e6:.1f}M lds {tot['SQ_INSTS_LDS'] / 1e6:.2f}M")
