#!/bin/bash
# FETCH_SIZE / WRITE_SIZE of k_knn_wave and k_finish per launch for each VARIANTS entry ("base" or
# NAME=VALUE[+...]), one pair in flight, one --pmc pass per counter (outputs under
# gpurun_out/${OUT:-fab}/); prints MB per launch (FETCH reported ×2 per the gfx950 correction).
set -u
O=gpurun_out/${OUT:-fab}
mkdir -p $O
export TMPDIR=/tmp
B="python3 bench.py --steps 2 --warmup 1 --no-cpu --no-verify --inflight 1 --no-fuse --latency-pairs 3 --busy-steps 0"
for v in ${VARIANTS:-base}; do
  envs=""; [ "$v" = base ] || envs="${v//+/ }"
  for e in $envs; do export "$e"; done
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 240 rocprofv3 --kernel-trace --kernel-include-regex 'k_knn_wave|k_finish' --output-format csv \
        --pmc $c -d $O/${v}_$c -o run -- $B > $O/${v}_$c.json 2> $O/${v}_$c.err
    rc=$?; [ $rc -eq 0 ] || { echo "pmc $v $c rc=$rc"; exit $rc; }
  done
  for e in $envs; do unset "${e%%=*}"; done
  python3 - "$O" "$v" <<'PY'
import collections, csv, glob, sys
o, v = sys.argv[1], sys.argv[2]
res = {}
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    acc = collections.defaultdict(list)
    for f in glob.glob(f"{o}/{v}_{c}/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            k = "k_knn_wave" if "k_knn_wave" in row["Kernel_Name"] else "k_finish"
            acc[k].append(float(row["Counter_Value"]) * 1024.0)
    res[c] = {k: sum(x) / len(x) for k, x in acc.items()}
t = {k: 2 * res["FETCH_SIZE"].get(k, 0) + res["WRITE_SIZE"].get(k, 0) for k in ("k_knn_wave", "k_finish")}
print(v, "MB/launch: knn %.1f finish %.1f total %.1f (fetch raw knn %.1f finish %.1f)" % (
    t["k_knn_wave"] / 1e6, t["k_finish"] / 1e6, sum(t.values()) / 1e6,
    res["FETCH_SIZE"].get("k_knn_wave", 0) / 1e6, res["FETCH_SIZE"].get("k_finish", 0) / 1e6))
PY
done
echo done
