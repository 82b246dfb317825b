"""GPU: frames handed over in the reference's wire format — PointCloud2 messages of
pcl::PointXYZINormal (publishPointCloud, saver.cpp:308-319) — go into the C ABI in place (strided
view of the message's data buffer: xyz at +0, normals at +16, stride 12 floats) and register
exactly as the same clouds given as arrays; a message with a non-consecutive field layout is
unpacked by name (pcl::fromROSMsg) and registers the same too."""
import numpy as np
import pytest

from planetary_lidar_odometry_amd import config, imls_icp, synth, wire

pytestmark = pytest.mark.gpu


def test_register_from_pointcloud2():
    q = synth.make_pairs(1, "vlp16", map_scans=1, scene_seed=8, traj_seed=2008, noise_seed=1008)[0]
    src = synth.fps_subsample(q.source, 1500, seed=3)
    p = config.bench_params(6)
    with imls_icp.ImlsContext(p) as c:
        c.set_target(q.target)
        c.set_source(src)
        ref = c.register_frame()
        c.map_clear()
        c.map_push(wire.xyzinormal_to_msg(q.target, "velodyne", 1.0))
        c.set_source(wire.xyzinormal_to_msg(src, "velodyne", 1.0), count=False)
        r = c.register_frame()
        assert np.array_equal(r["pose"], ref["pose"]) and r["iters"] == ref["iters"]
        # an interleaved layout (x nx y ny z nz): no strided view, unpacked by name
        names = ("x", "normal_x", "y", "normal_y", "z", "normal_z")
        rec = np.zeros(src.size, np.dtype([(k, "<f4") for k in names]))
        for k in names:
            rec[k] = src[k]
        m = wire.PointCloud2(width=src.size, fields=[wire.PointField(k, 4 * j) for j, k in enumerate(names)],
                             point_step=24, row_step=24 * src.size, data=rec.tobytes())
        assert wire.strided_view(m) is None
        c.set_source(m)
        assert np.array_equal(c.register_frame()["pose"], ref["pose"])
