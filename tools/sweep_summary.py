import csv, glob, json, pathlib
for d in sorted(glob.glob("gpurun_out/sweep/*/")):
    name = pathlib.Path(d).name
    kt = pathlib.Path(d) / "run_kernel_trace.csv"
    if not kt.exists():
        continue
    rows = sorted((r for r in csv.DictReader(open(kt)) if "k_knn_wave" in r["Kernel_Name"]), key=lambda r: int(r["Start_Timestamp"]))
    us = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows][-20:]
    b = json.loads(open(f"gpurun_out/sweep/{name}.json").read().strip().splitlines()[-1])
    print(f"{name:12s} {b['value']:6.2f} pairs/s sum {sum(us)/1e3:6.2f} ms:", [round(x) for x in us])
