"""Summarize gpurun_out/: test tail, bench JSON essentials, PMC averages per dispatch."""
import collections, csv, glob, json, pathlib, sys
out = pathlib.Path(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out")
t = out / "gpu_tests.log"
if t.exists():
    print("tests:", t.read_text().strip().splitlines()[-1])
b = out / "bench.json"
if b.exists() and b.read_text().strip():
    d = json.loads(b.read_text().strip().splitlines()[-1])
    r = d["roofline"]
    print(f"bench: {d['value']:.2f} pairs/s, {d['ms_per_step']:.2f} ms/pair, proj {r['avg_launch_ms']:.3f} ms/launch, "
          f"achieved {r['achieved']:.1f} GB/s ({100*r['frac']:.2f}%), breakdown {json.dumps({k: round(v, 3) for k, v in d['breakdown_ms_per_pair'].items()})}")
    if d.get("traversal_per_launch"):
        print("   traversal/launch:", {k: round(v) for k, v in d["traversal_per_launch"].items()})
    if d.get("cpu_baseline"):
        print(f"   cpu {d['cpu_baseline']['value']:.4f} pairs/s → speedup {d['value'] / d['cpu_baseline']['value']:.0f}x")
for f in sorted(glob.glob(str(out / "pmc" / "*" / "run_counter_collection.csv"))):
    agg = collections.defaultdict(list)
    for row in csv.DictReader(open(f)):
        agg[row["Counter_Name"]].append(float(row["Counter_Value"]))
    waves = sum(agg.get("SQ_WAVES", [1])) / max(len(agg.get("SQ_WAVES", [1])), 1)
    print(pathlib.Path(f).parent.name, {k: f"{sum(v)/len(v):.4g}" + (f" ({sum(v)/len(v)/waves:.4g}/wave)" if k.startswith("SQ_INSTS") else "") for k, v in agg.items()})
