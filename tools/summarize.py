"""Summarize gpurun_out/: test tail, bench JSON essentials, PMC averages per dispatch."""
import collections, csv, glob, json, pathlib, re, sys


def kname(n):
    m = re.search(r'(k_\w+(<\d+>)?|__amd\w+|DeviceRadixSort\w*|\w+Kernel\w*)', n)
    return m.group(1) if m else n[:40]

out = pathlib.Path(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out")
t = out / "gpu_tests.log"
if t.exists():
    print("tests:", t.read_text().strip().splitlines()[-1])
for b in [out / "bench.json", out / "bench1.json"]:
  if b.exists() and b.read_text().strip():
    d = json.loads(b.read_text().strip().splitlines()[-1])
    r = d["roofline"]
    print(f"bench: {d['value']:.2f} pairs/s, {d['ms_per_step']:.2f} ms/pair, proj {r['avg_launch_ms']:.3f} ms/launch, "
          f"achieved {r['achieved']:.1f} GB/s ({100*r['frac']:.2f}%), breakdown {json.dumps({k: round(v, 3) for k, v in d['breakdown_ms_per_pair'].items()})}")
    if d.get("traversal_per_launch"):
        print("   traversal/launch:", {k: round(v) for k, v in d["traversal_per_launch"].items()})
    if d.get("cpu_baseline"):
        print(f"   cpu {d['cpu_baseline']['value']:.4f} pairs/s → speedup {d['value'] / d['cpu_baseline']['value']:.0f}x")
for f in sorted(glob.glob(str(out / "kt" / "**" / "*kernel_stats.csv"), recursive=True)):
    rows = list(csv.DictReader(open(f)))
    print("kernel stats:", f)
    for r in rows[:14]:
        print(f"   {kname(r['Name']):40s} calls {r['Calls']:>6s} avg {float(r['AverageNs'])/1e3:9.1f} us  {float(r['Percentage']):5.1f}%")
for f in sorted(glob.glob(str(out / "pmc" / "*" / "run_counter_collection.csv"))):
    byk = collections.defaultdict(lambda: collections.defaultdict(list))
    for row in csv.DictReader(open(f)):
        byk[kname(row["Kernel_Name"])][row["Counter_Name"]].append(float(row["Counter_Value"]))
    for kn, agg in byk.items():
        waves = sum(agg.get("SQ_WAVES", [1])) / max(len(agg.get("SQ_WAVES", [1])), 1)
        print(pathlib.Path(f).parent.name, kn, {k: f"{sum(v)/len(v):.4g}" + (f" ({sum(v)/len(v)/waves:.4g}/wave)" if k.startswith("SQ_INSTS") else "") for k, v in agg.items()})

kt = out / "kt" / "run_kernel_trace.csv"
if kt.exists():
    rows = [r for r in csv.DictReader(open(kt)) if "k_knn_wave" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
    if len(d) >= 20:
        print("k_knn_wave per-iteration us (last frame):", [round(x) for x in d[-20:]])
