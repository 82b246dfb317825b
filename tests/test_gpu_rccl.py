"""RCCL on the MI355X: the one collective north_star names (the pose all-gather of config D,
laser_odometry.cpp:652-655 per sequence) run through bench.py's own distributed path.

A fresh child process is started before anything touches the GPU in it, with the environment
`torch.distributed.run --nproc-per-node 1` gives bench.py (RANK=0 WORLD_SIZE=1 LOCAL_RANK=0,
MASTER_ADDR=127.0.0.1): bench.dist_setup initialises an nccl (= RCCL) process group, 16 stream
sequences register 3 timed steps through StreamRunner / Pipeline, and bench.exchange_poses gathers
the tagged relative poses over RCCL.  The gathered records and every sequence's trajectory must be
bit-equal to sequences.chain_per_sequence of the local results.
"""
import json
import os
import pathlib
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = pathlib.Path(__file__).resolve().parent.parent


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def test_rccl_pose_exchange_world1():
    env = dict(os.environ, RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", LOCAL_WORLD_SIZE="1",
               MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run([sys.executable, "-u", str(ROOT / "tests" / "helpers" / "rccl_pose_exchange.py")],
                       env=env, capture_output=True, text=True, timeout=240, cwd=str(ROOT))
    assert r.returncode == 0, (r.returncode, r.stdout[-2000:], r.stderr[-4000:])
    line = [l for l in r.stdout.splitlines() if l.startswith("{")][-1]
    out = json.loads(line)
    print(out)
    assert out["backend"] == "nccl" and out["world"] == 1
    assert out["records_equal"] and out["trajectories_equal"]
    assert out["results"] == 48 and out["sequences"] == 16
