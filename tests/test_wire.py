"""Wire formats (saver.cpp:135-319): the PointXYZINormal PointCloud2 of
publishPointCloud / pcl::toROSMsg and the DataPoints PointCloud2 of libPointMatcherToRosMsg /
rosMsgToLibPointMatcherCloud.  The C++ header (include/imls_wire.hpp, compiled here by g++) and the
Python mirror must produce the same field tables and bytes on the same data; round trips; the DP
reader's by-position field reads; the in-place strided view the C ABI takes.  The layouts are the
reference's own code (no third-party semantics involved), so these are pinned by construction."""
import pathlib
import subprocess

import numpy as np
import pytest

from planetary_lidar_odometry_amd import synth, wire

ROOT = pathlib.Path(__file__).resolve().parents[1]


@pytest.fixture(scope="module")
def cpp_out():
    subprocess.run(["make", "-C", str(ROOT / "tests" / "cpp"), "wire_check"], check=True, capture_output=True)
    out = subprocess.run([str(ROOT / "tests" / "cpp" / "wire_check")], check=True, capture_output=True, text=True).stdout
    lines = out.splitlines()

    def line(prefix):
        hit = [ln for ln in lines if ln.startswith(prefix)]
        assert len(hit) == 1, (prefix, lines)
        return hit[0]
    return line


def _records(n=37):
    rec = np.array([[(i * 13 + k * 7) * 0.125 - 3.0 for k in range(12)] for i in range(n)], np.float32)
    return rec.view(synth.POINT_DTYPE).reshape(n)


def _dp(n=37):
    feat = np.array([[(i * 3 + r) * 0.5 - 1.0 for r in range(3)] + [1.0] for i in range(n)], np.float32)
    desc = np.array([[i * 22 + r for r in range(22)] for i in range(n)], np.float32) * np.float32(0.01)   # float math, as C++
    times = (np.arange(n, dtype=np.float32) * np.float32(0.1)).reshape(n, 1)
    return wire.DPCloud([("x", 1), ("y", 1), ("z", 1), ("pad", 1)], list(wire.DP_DESCRIPTOR_LABELS), [("time", 1)],
                        feat, desc, times)


def _fields(m):
    return "".join(f"{f.name}:{f.offset}:{f.datatype}:{f.count}," for f in m.fields)


def test_xyzinormal_matches_cpp(cpp_out):
    m = wire.xyzinormal_to_msg(_records(), "velodyne", 12.5)
    assert cpp_out("xyzinormal step") == f"xyzinormal step=48 width=37 fields={_fields(m)} fnv={wire.fnv1a(m.data)}"
    # pcl's PointXYZINormal offsets: x y z at 0/4/8, normals at 16/20/24, intensity 32, curvature 36
    assert [(f.name, f.offset) for f in m.fields] == [("x", 0), ("y", 4), ("z", 8), ("intensity", 32), ("normal_x", 16),
                                                     ("normal_y", 20), ("normal_z", 24), ("curvature", 36)]
    assert cpp_out("strided") == "strided ok=1 n=37 stride=12 xyz_off=0 nrm_off=16"


def test_xyzinormal_roundtrip_and_view():
    c = _records()
    m = wire.xyzinormal_to_msg(c)
    back = wire.xyzinormal_from_msg(m)
    for f in ("x", "y", "z", "intensity", "normal_x", "normal_y", "normal_z", "curvature"):
        assert np.array_equal(back[f], c[f])
    buf, xo, no, n, stride = wire.strided_view(m)
    assert (xo, no, n, stride) == (0, 16, 37, 12)
    f = buf.view("<f4").reshape(n, stride)
    assert np.array_equal(f[:, 0], c["x"]) and np.array_equal(f[:, 4], c["normal_x"])
    # a message whose normals are not consecutive has no strided view; fromROSMsg still reads it
    m2 = wire.PointCloud2(width=m.width, fields=[wire.PointField("x", 0), wire.PointField("y", 4), wire.PointField("z", 8),
                                                 wire.PointField("normal_x", 16), wire.PointField("normal_y", 24),
                                                 wire.PointField("normal_z", 20)],
                          point_step=48, row_step=48 * m.width, data=m.data)
    assert wire.strided_view(m2) is None
    assert np.array_equal(wire.xyzinormal_from_msg(m2)["normal_y"], c["normal_z"])


def test_dp_matches_cpp(cpp_out):
    m = wire.dp_to_msg(_dp(), "map", 3.25)
    assert m.point_step == 4 * (3 + 22 + 1)
    assert cpp_out("dp step") == f"dp step=104 width=37 fields={_fields(m)} fnv={wire.fnv1a(m.data)}"


def test_dp_roundtrip_and_by_position_reads(cpp_out):
    dp = _dp()
    m = wire.dp_to_msg(dp)
    q = wire.dp_from_msg(m)
    assert np.array_equal(q.features[:, :3], dp.features[:, :3]) and np.all(q.features[:, 3] == 1)
    assert np.array_equal(q.descriptors, dp.descriptors) and np.all(q.times == 0)
    # swapped table entries are read by position, as rosMsgToLibPointMatcherCloud does
    m.fields[3], m.fields[4] = m.fields[4], m.fields[3]
    s = wire.dp_from_msg(m)
    assert np.array_equal(s.descriptors[:, 0], dp.descriptors[:, 1]) and np.array_equal(s.descriptors[:, 1], dp.descriptors[:, 0])
    assert cpp_out("dp swapped").endswith(f"fnv={wire.fnv1a(np.ascontiguousarray(s.descriptors).tobytes())}")
    assert wire.dp_from_msg(wire.PointCloud2()) is None and cpp_out("dp empty") == "dp empty=0"


def test_cpp_roundtrips(cpp_out):
    assert cpp_out("xyzinormal roundtrip") == "xyzinormal roundtrip=1"
    assert cpp_out("dp roundtrip") == "dp roundtrip=1"


def test_malformed_messages_rejected(cpp_out):
    """Truncated data or a field past point_step: the C++ readers return false (no out-of-bounds
    host read), the Python mirror raises."""
    assert cpp_out("malformed") == "malformed xyzinormal_short=0 xyzinormal_offset=0 dp_short=0 dp_offset=0"
    m = wire.xyzinormal_to_msg(_records())
    m.data = m.data[:-1]
    with pytest.raises(Exception):
        wire.xyzinormal_from_msg(m)
