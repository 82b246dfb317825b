"""Per-dispatch and per-wave averages of SQ counters from rocprofv3 --pmc csv directories (one or more
passes of the same command, tools/gpu_sq4.sh), per kernel name (templates collapsed to the base name)."""
import csv
import glob
import re
import sys
from collections import defaultdict

vals = defaultdict(lambda: defaultdict(list))    # kernel -> counter -> per-dispatch values
for d in sys.argv[1:]:
    per = defaultdict(lambda: defaultdict(float))
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            name = re.sub(r"<.*", "", r.get("Kernel_Name", "")).split("::")[-1].split("(")[0].strip()
            per[(name, r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    for (name, _), c in per.items():
        for n, v in c.items():
            vals[name][n].append(v)
for name, c in sorted(vals.items()):
    avg = {n: sum(v) / len(v) for n, v in c.items()}
    waves = max(avg.get("SQ_WAVES", 1.0), 1.0)
    n_disp = max(len(v) for v in c.values())
    print(f"{name}: {n_disp} dispatches")
    for n in sorted(avg):
        print(f"  {n:22s} per dispatch {avg[n]:14.1f}   per wave {avg[n] / waves:12.1f}")
    wc = avg.get("SQ_WAVE_CYCLES")
    if wc:
        for n in ("SQ_WAIT_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_ANY"):
            if n in avg:
                print(f"  {n} / SQ_WAVE_CYCLES = {avg[n] / wc:.3f}")
