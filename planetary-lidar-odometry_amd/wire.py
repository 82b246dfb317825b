"""Wire formats around the registration path — the Python mirror of
include/imls_wire.hpp (the C++ host side):

* sensor_msgs/PointCloud2 of pcl::PointXYZINormal (publishPointCloud → pcl::toROSMsg,
  saver.cpp:308-319; read back by pcl::fromROSMsg): 8 FLOAT32 fields in PCL's registration order,
  point_step 48, the 48-byte records as they are — synth.POINT_DTYPE is that record, so a message's
  data buffer is the strided cloud the C ABI takes, in place (``strided_view``).
* libpointmatcher DataPoints as PointCloud2 (libPointMatcherToRosMsg / rosMsgToLibPointMatcherCloud,
  saver.cpp:135-306): x, y, z (no pad row), the descriptor labels with their spans (the 22-float
  layout), "time" when present.  The reader keeps the reference's by-position field reads.

DataPoints matrices are column-major in Eigen (column = point); here they are (n, rows) arrays.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

from .synth import POINT_DTYPE

INT8, UINT8, INT16, UINT16, INT32, UINT32, FLOAT32, FLOAT64 = range(1, 9)


@dataclass
class PointField:
    name: str
    offset: int
    datatype: int = FLOAT32
    count: int = 1


@dataclass
class PointCloud2:
    frame_id: str = ""
    stamp: float = 0.0
    height: int = 1
    width: int = 0
    fields: list = field(default_factory=list)
    is_bigendian: bool = False
    point_step: int = 0
    row_step: int = 0
    data: bytes = b""
    is_dense: bool = True


# ---- pcl::PointXYZINormal ----------------------------------------------------------------------
XYZINORMAL_STEP = 48


def xyzinormal_fields():
    """The field table pcl::toROSMsg emits for PointXYZINormal."""
    return [PointField("x", 0), PointField("y", 4), PointField("z", 8), PointField("intensity", 32),
            PointField("normal_x", 16), PointField("normal_y", 20), PointField("normal_z", 24),
            PointField("curvature", 36)]


def xyzinormal_to_msg(cloud: np.ndarray, frame_id: str = "", stamp: float = 0.0) -> PointCloud2:
    """pcl::toROSMsg of a PointXYZINormal cloud (synth.POINT_DTYPE records)."""
    a = np.ascontiguousarray(cloud, dtype=POINT_DTYPE)
    return PointCloud2(frame_id=frame_id, stamp=stamp, height=1, width=a.size, fields=xyzinormal_fields(),
                       point_step=XYZINORMAL_STEP, row_step=XYZINORMAL_STEP * a.size, data=a.tobytes())


def _field(m: PointCloud2, name: str):
    for f in m.fields:
        if f.name == name:
            return f
    return None


def strided_view(m: PointCloud2):
    """(records array backing the data, xyz byte offset, normal byte offset, n, stride in floats) when
    x y z and normal_x normal_y normal_z are consecutive aligned FLOAT32 fields (the C ABI's strided
    cloud, no copy); None otherwise."""
    fs = [_field(m, k) for k in ("x", "y", "z", "normal_x", "normal_y", "normal_z")]
    if any(f is None for f in fs) or m.is_bigendian or m.point_step % 4 or not m.data:
        return None
    if any(f.datatype != FLOAT32 or f.offset % 4 for f in fs):
        return None
    x, y, z, nx, ny, nz = fs
    if (y.offset, z.offset, ny.offset, nz.offset) != (x.offset + 4, x.offset + 8, nx.offset + 4, nx.offset + 8):
        return None
    if m.row_step != m.point_step * m.width:
        return None
    buf = np.frombuffer(m.data, dtype=np.uint8)
    return buf, x.offset, nx.offset, m.width * m.height, m.point_step // 4


def xyzinormal_from_msg(m: PointCloud2) -> np.ndarray:
    """pcl::fromROSMsg: fields matched by name (FLOAT32); a missing field stays 0."""
    n = m.width * m.height
    out = np.zeros(n, POINT_DTYPE)
    raw = np.frombuffer(m.data, dtype=np.uint8).reshape(n, m.point_step) if n else None
    for name in ("x", "y", "z", "intensity", "normal_x", "normal_y", "normal_z", "curvature"):
        f = _field(m, name)
        if f is None or f.datatype != FLOAT32 or n == 0:
            continue
        out[name] = raw[:, f.offset:f.offset + 4].copy().view("<f4").reshape(n)
    return out


# ---- libpointmatcher DataPoints ----------------------------------------------------------------
DP_DESCRIPTOR_LABELS = [("surfaceness", 1), ("curveness", 1), ("pointness", 1), ("normals", 3), ("tangents", 3),
                        ("labels", 1), ("sticks", 4), ("plates", 7), ("balls", 1)]
DP_DESCRIPTOR_ROWS = 22


@dataclass
class DPCloud:
    feature_labels: list            # [(text, span)], normally x y z pad
    descriptor_labels: list
    time_labels: list
    features: np.ndarray            # (n, feature rows) float32
    descriptors: np.ndarray         # (n, descriptor rows)
    times: np.ndarray               # (n, time rows)

    @property
    def n(self):
        return self.features.shape[0]


def dp_to_msg(dp: DPCloud, frame_id: str = "", stamp: float = 0.0) -> PointCloud2:
    """libPointMatcherToRosMsg (saver.cpp:135-221)."""
    fields, off = [], 0
    for text, span in dp.feature_labels:
        if text == "pad":
            continue
        fields.append(PointField(text, off, FLOAT32, span))
        off += 4 * span
    for text, span in dp.descriptor_labels:
        fields.append(PointField(text, off, FLOAT32, span))
        off += 4 * span
    tr = sum(s for _, s in dp.time_labels)
    if tr > 0:
        fields.append(PointField("time", off, FLOAT32, tr))
        off += 4 * tr
    n = dp.n
    parts = [np.ascontiguousarray(dp.features[:, :3], np.float32)]
    dr = 0
    for _, span in dp.descriptor_labels:
        parts.append(np.asarray(dp.descriptors[:, dr:dr + span], np.float32))
        dr += span
    if tr > 0:
        parts.append(np.asarray(dp.times[:, :tr], np.float32))
    rec = np.concatenate(parts, axis=1) if n else np.zeros((0, off // 4), np.float32)
    assert rec.shape[1] * 4 == off
    return PointCloud2(frame_id=frame_id, stamp=stamp, height=1, width=n, fields=fields, point_step=off,
                       row_step=off * n, data=np.ascontiguousarray(rec, "<f4").tobytes())


def dp_from_msg(m: PointCloud2):
    """rosMsgToLibPointMatcherCloud (saver.cpp:224-306): None (the empty DP()) for a message without
    fields; otherwise fields[0..11] read BY POSITION at their offsets into the fixed 22-descriptor
    layout, pad = 1, the one time row left 0.  (A message with fewer than 12 fields would make the
    reference read past its field vector; it is rejected here.)"""
    if not m.fields or len(m.fields) < 12:
        return None
    n = m.width * m.height
    raw = np.frombuffer(m.data, dtype=np.uint8).reshape(n, m.point_step) if n else np.zeros((0, m.point_step), np.uint8)

    def take(f, k):
        return raw[:, f.offset:f.offset + 4 * k].copy().view("<f4").reshape(n, k)

    feat = np.ones((n, 4), np.float32)
    for k in range(3):
        feat[:, k:k + 1] = take(m.fields[k], 1)
    desc = np.zeros((n, DP_DESCRIPTOR_ROWS), np.float32)
    row = 0
    for j, (_, span) in enumerate(DP_DESCRIPTOR_LABELS):
        desc[:, row:row + span] = take(m.fields[3 + j], span)
        row += span
    return DPCloud([("x", 1), ("y", 1), ("z", 1), ("pad", 1)], list(DP_DESCRIPTOR_LABELS), [("time", 1)],
                   feat, desc, np.zeros((n, 1), np.float32))


def fnv1a(data: bytes) -> int:
    """64-bit FNV-1a (tests compare the C++ and Python encoders' bytes through it)."""
    h = 0xcbf29ce484222325
    for b in data:
        h = ((h ^ b) * 0x100000001b3) & 0xFFFFFFFFFFFFFFFF
    return h
