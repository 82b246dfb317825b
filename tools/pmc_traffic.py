"""HBM traffic per projection launch from the PMC passes of tools/measure_round.sh.

traffic = 2·FETCH_SIZE + WRITE_SIZE (MI355X_MICROARCH.md § HBM: on gfx950 FETCH_SIZE reports ½ of
the bytes of wide coalesced reads; WRITE_SIZE is exact for 16-B stores), per launch of
k_knn_wave + k_finish, averaged over the dispatches of the PMC runs.  rocprofv3 reports both
counters in KB.  Writes profiles/pmc_traffic.json (read by bench.py) and a copy next to the round's
profiles.
usage: python tools/pmc_traffic.py gpurun_out/measure profiles/<round_tag>
"""
import collections, csv, json, pathlib, sys

src = pathlib.Path(sys.argv[1])
dst = pathlib.Path(sys.argv[2])
per = {}
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    f = next((src / f"pmc_{c}").rglob("*counter_collection.csv"))
    acc = collections.defaultdict(list)
    for row in csv.DictReader(open(f)):
        k = "k_knn_wave" if "k_knn_wave" in row["Kernel_Name"] else "k_finish"
        acc[k].append(float(row["Counter_Value"]) * 1024.0)
    per[c] = {k: sum(v) / len(v) for k, v in acc.items()}
jf = src / "pmc_FETCH_SIZE.json"
jf = jf if jf.exists() else src / "pmc_FETCH_SIZE.out"
bench = json.loads(jf.read_text().strip().splitlines()[-1])
kern = {k: 2 * per["FETCH_SIZE"].get(k, 0.0) + per["WRITE_SIZE"].get(k, 0.0) for k in ("k_knn_wave", "k_finish")}
out = {
    "queries": bench["config"]["queries"],
    "iters": bench["config"]["icp_iterations"],
    "bytes_per_launch": sum(kern.values()),
    "per_kernel_bytes": kern,
    "fetch_size_bytes_raw": per["FETCH_SIZE"],
    "write_size_bytes": per["WRITE_SIZE"],
    "formula": "2*FETCH_SIZE + WRITE_SIZE (KB->bytes), per launch, k_knn_wave + k_finish",
}
dst.mkdir(parents=True, exist_ok=True)
(dst / "pmc_traffic.json").write_text(json.dumps(out, indent=1))
pathlib.Path("profiles/pmc_traffic.json").write_text(json.dumps(out, indent=1))
print(json.dumps(out, indent=1))
