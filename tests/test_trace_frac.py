"""tools/trace_frac.py: the roofline fraction recomputed from a kernel trace (CPU, synthetic trace).

Two launch sequences overlap; the busy time is the union of their projection intervals, phases are
split by traversal-launch index (warm-up, timed, stats, busy pass), and single-frame kernels (the
verify / latency probes) are ignored."""
import csv
import gzip
import json
import pathlib
import subprocess
import sys

ROOT = pathlib.Path(__file__).resolve().parents[1]


def _write_trace(path, rows):
    op = gzip.open if str(path).endswith(".gz") else open
    with op(path, "wt", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Kernel_Name", "Start_Timestamp", "End_Timestamp"])
        w.writerows(rows)


def test_trace_frac_union_and_phases(tmp_path):
    # 2 groups × 1 iteration = L = 2 traversal launches per step; warmup 1, timed 2, stats 1, busy 1
    W, K, S, L = 1, 2, 1, 2
    rows, t = [], 0
    for step in range(W + K + 1 + S):
        # two sequences overlapping: knn 0-100 / 50-150, finish 100-120 / 150-170 (ns, +offset)
        for g, off in ((0, 0), (1, 50)):
            rows.append(("k_knn_wave_b", t + off, t + off + 100))
            rows.append(("k_finish_b", t + off + 100, t + off + 120))
        if step == W + K - 1:
            rows.append(("k_knn_wave", t + 1000, t + 5000))     # single-frame probe: ignored
        t += 10_000
    _write_trace(tmp_path / "t.csv.gz", rows)
    bps = 1e6                                                  # algorithmic bytes per step
    bench = {"warmup": W, "steps": K, "ms_per_step": 0.01,
             "config": {"launch_groups": 2, "icp_iterations": 1},
             "roofline": {"algorithmic_bytes_per_step": bps, "frac": 0.5, "busy_projection_ms_per_step": 1.7e-4}}
    (tmp_path / "b.json").write_text(json.dumps(bench) + "\n")
    out = subprocess.run([sys.executable, str(ROOT / "tools" / "trace_frac.py"), str(tmp_path / "t.csv.gz"),
                          str(tmp_path / "b.json"), "--busy-steps", str(S)], capture_output=True, text=True, check=True)
    r = json.loads(out.stdout)
    assert r["traversal_launches"] == r["expected"] == (W + K + 1 + S) * L
    # each step: union of [0,120) and [50,170) = 170 ns busy
    assert abs(r["timed"]["busy_ms_per_step"] - 170e-6) < 1e-12
    assert abs(r["busy_pass"]["busy_ms_per_step"] - 170e-6) < 1e-12
    want_frac = bps / 170e-9 / 1e9 / 8000.0
    assert abs(r["timed"]["frac"] / want_frac - 1) < 1e-9
    assert r["timed"]["steps"] == K and r["busy_pass"]["steps"] == S
