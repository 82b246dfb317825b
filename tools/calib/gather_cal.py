"""FETCH_SIZE / WRITE_SIZE calibration from tools/calib/gather_cal (run under two separate rocprofv3
--pmc passes).  usage: python tools/calib/gather_cal.py <out_dir>  where out_dir holds
fetch/ (rocprofv3 -d of the FETCH_SIZE pass), write/ (WRITE_SIZE pass) and fetch.out (the program's
stdout of the FETCH pass: one line per launch, in launch order).
Writes <out_dir>/gather_cal.json: per (pattern, table) the counted bytes per known byte (the last two
of three repetitions: the first warms the caches), the achieved rate, and the factors the traffic
figure uses (MI355X_MICROARCH.md §HBM: counted × factor = bytes)."""
import collections
import csv
import json
import pathlib
import sys

d = pathlib.Path(sys.argv[1])


def counters(sub, name):
    f = next((d / sub).rglob("*counter_collection.csv"))
    per = collections.defaultdict(float)
    for r in csv.DictReader(open(f)):
        if "k_gather" in r["Kernel_Name"] and r["Counter_Name"] == name:
            per[int(r["Dispatch_Id"])] += float(r["Counter_Value"]) * 1024.0     # KB → bytes
    return [per[k] for k in sorted(per)]


lines = [l.split() for l in (d / "fetch.out").read_text().splitlines() if l.strip()]
fetch = counters("fetch", "FETCH_SIZE")
write = counters("write", "WRITE_SIZE")
assert len(fetch) == len(lines) == len(write), (len(fetch), len(lines), len(write))
acc = collections.defaultdict(list)
for k, (ln, fb, wb) in enumerate(zip(lines, fetch, write)):
    pat, tb, rows, rd, wr, ms = ln[0], int(ln[1]), float(ln[2]), float(ln[3]), float(ln[4]), float(ln[5])
    acc[(pat, tb)].append(dict(fetch=fb, write=wb, read_bytes=rd, write_bytes=wr, ms=ms))
out = {"note": "counted FETCH_SIZE bytes per byte the kernel reads (known by construction); factor = 1 / that "
               "(bytes = counted x factor). reps 2-3 of 3 (rep 1 warms). Table 512 MiB: beyond the 256-MiB "
               "Infinity Cache; 40 MB: config B's Morton-map size, Infinity-Cache resident.", "patterns": {}}
for (pat, tb), reps in sorted(acc.items()):
    use = reps[1:] if len(reps) > 1 else reps
    f = sum(r["fetch"] for r in use) / len(use)
    w = sum(r["write"] for r in use) / len(use)
    rd = use[0]["read_bytes"]
    wr = use[0]["write_bytes"]
    ms = sum(r["ms"] for r in use) / len(use)
    out["patterns"][f"{pat}_{tb >> 20}MiB"] = {
        "known_read_bytes": rd, "fetch_size_bytes": f, "counted_per_read_byte": f / rd, "factor": rd / f if f else None,
        "known_write_bytes": wr, "write_size_bytes": w, "write_counted_per_byte": w / wr,
        "ms": ms, "requested_GBps": rd / (ms / 1e3) / 1e9, "counted_GBps": f / (ms / 1e3) / 1e9}
p = out["patterns"]
# the factors the projection traffic uses: wide streaming (the guide's x2) and the 16-B gather of a
# 40-MB map (config B's map stays in the Infinity Cache)
out["factor_stream"] = p["stream_512MiB"]["factor"]
out["factor_gather16_map40MB"] = p["rand16_40MiB"]["factor"]
out["factor_gather16_hbm"] = p["rand16_512MiB"]["factor"]
(d / "gather_cal.json").write_text(json.dumps(out, indent=1))
for k, v in p.items():
    print(f"{k:18s} counted/read {v['counted_per_read_byte']:.3f}  write {v['write_counted_per_byte']:.3f}  "
          f"{v['ms']:.3f} ms  req {v['requested_GBps']:.0f} GB/s  counted {v['counted_GBps']:.0f} GB/s")
print(json.dumps({k: out[k] for k in out if k.startswith("factor")}))
