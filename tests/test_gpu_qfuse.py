"""The lone-small-frame exact stage: fused into the wave-per-query traversal (k_knn_qwave_f, the
default), as its own launch (k_finish_q, IMLS_QFUSE=0) and lane per query (k_finish, IMLS_QFINISH=0)
must give the same frame bit for bit: the correspondences are the same, and k_solve_small forms the
pass-1 normal equations from the rows in one fixed order whichever kernel produced them.  With every
3rd query uncertified (IMLS_FORCE_FALLBACK) the fused path builds those queries' exact lists in the
wave (exact_wave_list) while the other two defer them to the fallback launch (k_project_lane's
search): the same correspondences, so the same poses; frames registered back to back in one
context also check the deferred-query counter's reset.  One path is also compared with the CPU
oracle (imls_icp.cpp:496-745 restated in oracle/imls_oracle.cpp)."""
import pathlib

import numpy as np
import pytest

import oracle_ctypes as oc
from planetary_lidar_odometry_amd import config, imls_icp

pytestmark = pytest.mark.gpu
GOLDEN = pathlib.Path(__file__).resolve().parent / "golden"

PATHS = {
    "fused": {"IMLS_QFUSE": "1", "IMLS_QFINISH": "1"},
    "finish_q": {"IMLS_QFUSE": "0", "IMLS_QFINISH": "1"},
    "lane_finish": {"IMLS_QFUSE": "1", "IMLS_QFINISH": "0"},
}


def _run(ctx, p, env, force, monkeypatch):
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    if force:
        monkeypatch.setenv("IMLS_FORCE_FALLBACK", "3")
    else:
        monkeypatch.delenv("IMLS_FORCE_FALLBACK", raising=False)
    ctx.set_params(p)                  # KParams are read when params are set
    ctx.enable_stats(True)
    r = ctx.register_frame()
    r["stats"] = ctx.traversal_stats()
    return r


@pytest.mark.parametrize("name", ["vlp16_pair", "planetary_pair"])
def test_exact_stage_paths_bit_identical(name, monkeypatch):
    g = dict(np.load(GOLDEN / f"{name}.npz"))
    src, tgt = np.ascontiguousarray(g["src"]), np.ascontiguousarray(g["tgt"])
    monkeypatch.setenv("IMLS_QWAVE", "-1")          # auto: wave per query for these ≤ 2000-query frames
    p = config.bench_params(10)
    runs = {}
    with imls_icp.ImlsContext(p) as ctx:
        ctx.set_target(np.ascontiguousarray(tgt.T))
        ctx.set_source(np.ascontiguousarray(src.T))
        for force in (False, True):
            for path, env in PATHS.items():
                runs[(path, force)] = _run(ctx, p, env, force, monkeypatch)
    ref = runs[("fused", False)]
    for key, r in runs.items():
        assert r["iters"] == ref["iters"] and r["status"] == ref["status"], key
        dp = np.abs(r["pose"] - ref["pose"]).max()
        assert dp == 0, (key, dp)
        for ta, tb in zip(r["trace"], ref["trace"]):
            assert ta.n_valid == tb.n_valid and ta.n_kept == tb.n_kept, key
            assert list(ta.reject) == list(tb.reject), key
            dd = np.abs(np.array(ta.delta) - np.array(tb.delta)).max()
            assert dd == 0, (key, dd)
    for path in PATHS:
        assert runs[(path, True)]["stats"]["uncertified"] > 0.3 * len(src[0]), (path, runs[(path, True)]["stats"])
    want = oc.register_frame(src, tgt, p)
    assert ref["iters"] == want["iters"] and ref["status"] == want["status"]
    for tg, tw in zip(ref["trace"], want["trace"]):
        assert tg.n_valid == tw.n_valid
        assert list(tg.reject) == list(tw.reject)
    assert np.abs(ref["pose"] - want["pose"]).max() < 1e-6
