"""GPU busy time (union of kernel intervals) and per-category kernel time over the last `window`
seconds of a rocprofv3 kernel trace (the timed steps), for reading where a pipelined run spends the GPU."""
import csv
import re
import sys
from collections import defaultdict

path = sys.argv[1]
window = float(sys.argv[2]) if len(sys.argv) > 2 else 0.0
rows = list(csv.DictReader(open(path)))
iv = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows]
iv.sort()
t_end = max(e for _, e, _ in iv)
t0 = t_end - int(window * 1e9) if window > 0 else iv[0][0]
iv = [x for x in iv if x[0] >= t0]
busy, cur_s, cur_e = 0, None, None
for s, e, _ in iv:
    if cur_e is None or s > cur_e:
        if cur_e is not None:
            busy += cur_e - cur_s
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
busy += cur_e - cur_s
span = t_end - iv[0][0]
print(f"span {span/1e6:.2f} ms  busy(union) {busy/1e6:.2f} ms  ({100*busy/span:.1f} %)  kernels {len(iv)}")
cat = defaultdict(lambda: [0, 0])
for s, e, n in iv:
    n = re.sub(r"imlsgpu::\(anonymous namespace\)::", "", n)
    n = re.sub(r"^void ", "", n).split("(")[0].split("<")[0]
    if "rocprim" in n:
        n = "rocprim"
    cat[n][0] += e - s
    cat[n][1] += 1
for n, (t, c) in sorted(cat.items(), key=lambda x: -x[1][0])[:25]:
    print(f"  {n:32s} {t/1e6:9.2f} ms  {c:6d} calls  {t/c/1e3:8.1f} us")
# the largest idle gaps between consecutive busy intervals, with the kernels on either side
if len(sys.argv) > 3:
    ngap = int(sys.argv[3])
    gaps, cur_e, last = [], None, None
    for s, e, n in iv:
        if cur_e is not None and s > cur_e:
            gaps.append((s - cur_e, last, n, cur_e))
        if cur_e is None or e > cur_e:
            cur_e, last = e, n
    short = lambda n: re.sub(r"^void ", "", re.sub(r"imlsgpu::\(anonymous namespace\)::", "", n)).split("(")[0][:40]
    tot = sum(g[0] for g in gaps)
    print(f"idle gaps: {len(gaps)}, total {tot/1e6:.2f} ms; largest:")
    for g, a, b, t in sorted(gaps, reverse=True)[:ngap]:
        print(f"  {g/1e6:8.3f} ms at +{(t - iv[0][0])/1e6:9.2f} ms  after {short(a):40s} before {short(b)}")
