"""Roofline fraction of the projection step recomputed from a rocprofv3 kernel trace of the bench
command itself: the union of the busy intervals of the projection kernels
(k_knn_wave[_b] / k_knn_qwave[_b] + k_finish[_b] + k_project_lane[_b]) over the TIMED steps and over
the bench's HIP-event busy pass, against the bench JSON's own algorithmic bytes per step.

    python tools/trace_frac.py <kernel_trace.csv> <bench.json> [--warmup W] [--steps K] [--busy-steps S]

The batched launches (`_b` kernels) run only in the warm-up, timed, stats and busy-pass steps, in that
order (the verify / latency probes use the single-frame kernels), launch_groups × iterations
traversal launches per step; the timed launches are therefore the traversal launches
[W·L, (W+K)·L) by start time and the busy pass the last S·L."""
import argparse
import csv
import gzip
import json
import re

HBM_PEAK_GBS = 8000.0


def union(iv):
    iv = sorted(iv)
    busy, cs, ce = 0, None, None
    for s, e in iv:
        if ce is None or s > ce:
            if ce is not None:
                busy += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    return busy + (ce - cs if ce is not None else 0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("bench")
    ap.add_argument("--warmup", type=int, default=None)
    ap.add_argument("--steps", type=int, default=None)
    ap.add_argument("--busy-steps", type=int, default=5)
    a = ap.parse_args()
    b = json.loads(open(a.bench).read().strip().splitlines()[-1])
    W = a.warmup if a.warmup is not None else b["warmup"]
    K = a.steps if a.steps is not None else b["steps"]
    L = b["config"]["launch_groups"] * b["config"]["icp_iterations"]
    bps = b["roofline"]["algorithmic_bytes_per_step"]
    rows = list(csv.DictReader(gzip.open(a.trace, "rt") if a.trace.endswith(".gz") else open(a.trace)))
    knn, proj = [], []
    for r in rows:
        n = r["Kernel_Name"]
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if not re.search(r"k_(knn_wave|knn_qwave|finish|project_lane)_(b|mb)\b", n):   # full or reduced name
            continue
        proj.append((s, e, n))
        # one marker per traversal: the one-pass launch, or (round 6, later iterations) the reuse-
        # decision launch k_knn_wave_mb<KL, 1> — its compacted walk <KL, 2> is projection time only
        if re.search(r"k_knn_(wave|qwave)_b\b", n) or re.search(r"k_knn_wave_mb<\d+, ?1>", n):
            knn.append((s, e))
    knn.sort()
    proj.sort()
    # one traversal launch per (group, iteration): qwave and wave variants of one launch sequence
    # never both run for B / stream (the auto choice is per batch), so index the traversal launches
    total = len(knn)
    expect = (W + K + 1 + a.busy_steps) * L
    out = {"trace": a.trace, "launches_per_step": L, "traversal_launches": total, "expected": expect}

    def window(i0, i1, nsteps):
        t0 = knn[i0][0]
        t1 = knn[i1][0] if i1 < total else None
        iv = [(s, e) for s, e, _ in proj if s >= t0 and (t1 is None or s < t1)]
        # the window ends with the last projection kernel that started before the next phase
        end = max(e for _, e in iv)
        busy = union(iv) / 1e6   # ms
        span = (end - t0) / 1e6
        ach = nsteps * bps / (busy / 1e3) / 1e9
        return {"steps": nsteps, "span_ms": span, "projection_busy_ms": busy,
                "busy_ms_per_step": busy / nsteps, "achieved_GBps": ach, "frac": ach / HBM_PEAK_GBS}

    out["timed"] = window(W * L, (W + K) * L, K)
    out["timed"]["bench_ms_per_step"] = b["ms_per_step"]
    if a.busy_steps > 0 and total >= a.busy_steps * L:
        out["busy_pass"] = window(total - a.busy_steps * L, total, a.busy_steps)
        out["busy_pass"]["bench_frac"] = b["roofline"].get("frac")
        out["busy_pass"]["bench_busy_ms_per_step"] = b["roofline"].get("busy_projection_ms_per_step")
        out["busy_pass"]["frac_ratio_trace_vs_bench"] = out["busy_pass"]["frac"] / b["roofline"]["frac"]
    out["timed"]["frac_ratio_trace_vs_bench"] = out["timed"]["frac"] / b["roofline"]["frac"]
    if total != expect:
        out["warning"] = f"{total} traversal launches, expected {expect}: phase boundaries are approximate"
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
