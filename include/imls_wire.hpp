// imls_wire.hpp — the two wire formats on either side of the registration path,
// header-only, no ROS / PCL / libpointmatcher headers needed:
//
//  (1) sensor_msgs/PointCloud2 of pcl::PointXYZINormal — what scan_registration publishes as
//      /laser_cloud_filtered and /laser_cloud_flat (publishPointCloud, saver.cpp:308-319, i.e.
//      pcl::toROSMsg) and laser_odometry reads back with pcl::fromROSMsg.  Eight FLOAT32 fields in
//      PCL's registration order (x, y, z, intensity, normal_x, normal_y, normal_z, curvature) at the
//      48-byte record's offsets, point_step 48, the records' bytes as they are.  strided_view() turns
//      such a message into the strided cloud the C ABI takes (imls_set_target / imls_set_source /
//      imls_map_push: xyz at +0, normal at +16, stride 12 floats) without a copy.
//
//  (2) libpointmatcher DataPoints ("DP") as PointCloud2 — libPointMatcherToRosMsg and
//      rosMsgToLibPointMatcherCloud (saver.cpp:135-306), the tensor-voting clouds' format: the
//      features x, y, z (the homogeneous "pad" row is not sent), then every descriptor label with
//      its span (the 22-float layout surfaceness 1, curveness 1, pointness 1, normals 3, tangents 3,
//      labels 1, sticks 4, plates 7, balls 1), then "time" when the cloud has time rows; FLOAT32,
//      little endian, dense.  The reader keeps the reference's behaviour exactly: a message without
//      fields is an empty cloud; otherwise it reads fields[0..11] BY POSITION at their offsets into
//      the fixed 22-descriptor layout (the names are not looked at), and sets pad = 1.
//
// DataPoints matrices are Eigen column-major: column = point.  DPCloud keeps that: features[4·i + r],
// descriptors[rows·i + r], times[time_rows·i + r].
#pragma once
#include <cstddef>
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

namespace imls_wire {

enum : uint8_t { INT8 = 1, UINT8 = 2, INT16 = 3, UINT16 = 4, INT32 = 5, UINT32 = 6, FLOAT32 = 7, FLOAT64 = 8 };

struct PointField {
    std::string name;
    uint32_t offset = 0;
    uint8_t datatype = FLOAT32;
    uint32_t count = 1;
};

struct PointCloud2 {
    std::string frame_id;
    double stamp = 0.0;
    uint32_t height = 1, width = 0;
    std::vector<PointField> fields;
    bool is_bigendian = false;
    uint32_t point_step = 0, row_step = 0;
    std::vector<uint8_t> data;
    bool is_dense = true;
};

// ---- (1) pcl::PointXYZINormal ------------------------------------------------------------------
constexpr uint32_t kXYZINormalStep = 48;

// The field table pcl::toROSMsg emits for PointXYZINormal (POINT_CLOUD_REGISTER_POINT_STRUCT order).
inline std::vector<PointField> xyzinormal_fields() {
    return {{"x", 0, FLOAT32, 1},         {"y", 4, FLOAT32, 1},         {"z", 8, FLOAT32, 1},
            {"intensity", 32, FLOAT32, 1}, {"normal_x", 16, FLOAT32, 1}, {"normal_y", 20, FLOAT32, 1},
            {"normal_z", 24, FLOAT32, 1},  {"curvature", 36, FLOAT32, 1}};
}

// pcl::toROSMsg of n 48-byte PointXYZINormal records (publishPointCloud, saver.cpp:308-319).
inline PointCloud2 xyzinormal_to_msg(const void* records, size_t n, const std::string& frame_id, double stamp) {
    PointCloud2 m;
    m.frame_id = frame_id;
    m.stamp = stamp;
    m.height = 1;
    m.width = (uint32_t)n;
    m.fields = xyzinormal_fields();
    m.point_step = kXYZINormalStep;
    m.row_step = m.point_step * m.width;
    m.data.resize((size_t)m.row_step);
    if (n) std::memcpy(m.data.data(), records, (size_t)m.row_step);
    return m;
}

inline const PointField* find_field(const PointCloud2& m, const char* name) {
    for (const auto& f : m.fields)
        if (f.name == name) return &f;
    return nullptr;
}

// A message's points as the C ABI's strided cloud, in place: x, y, z and normal_x, normal_y,
// normal_z must be consecutive FLOAT32 fields, 4-byte aligned, point_step a multiple of 4, little
// endian.  Returns false otherwise (then unpack with xyzinormal_from_msg).
struct StridedCloud {
    const float* xyz = nullptr;
    const float* nrm = nullptr;
    size_t n = 0;
    size_t stride_floats = 0;
};
inline bool strided_view(const PointCloud2& m, StridedCloud* out) {
    const PointField *x = find_field(m, "x"), *y = find_field(m, "y"), *z = find_field(m, "z");
    const PointField *nx = find_field(m, "normal_x"), *ny = find_field(m, "normal_y"), *nz = find_field(m, "normal_z");
    if (!x || !y || !z || !nx || !ny || !nz || m.is_bigendian || m.point_step % 4 || m.data.empty()) return false;
    for (const PointField* f : {x, y, z, nx, ny, nz})
        if (f->datatype != FLOAT32 || f->offset % 4) return false;
    if (y->offset != x->offset + 4 || z->offset != x->offset + 8 || ny->offset != nx->offset + 4 || nz->offset != nx->offset + 8)
        return false;
    if ((reinterpret_cast<uintptr_t>(m.data.data()) % 4) || m.row_step != m.point_step * m.width) return false;
    out->xyz = reinterpret_cast<const float*>(m.data.data() + x->offset);
    out->nrm = reinterpret_cast<const float*>(m.data.data() + nx->offset);
    out->n = (size_t)m.width * m.height;
    out->stride_floats = m.point_step / 4;
    return true;
}

// A message holds n = width·height records of point_step bytes: its data must cover them.
inline bool msg_covers(const PointCloud2& m) {
    const size_t n = (size_t)m.width * m.height;
    return m.point_step == 0 ? n == 0 : m.data.size() / m.point_step >= n;
}

// pcl::fromROSMsg into 48-byte PointXYZINormal records (12 floats each): fields matched by name,
// FLOAT32 only; a field the message lacks stays 0.  Returns false (records untouched) for a
// malformed message: data shorter than width·height·point_step, or a field not inside point_step.
inline bool xyzinormal_from_msg(const PointCloud2& m, float* records) {
    static const char* names[8] = {"x", "y", "z", "intensity", "normal_x", "normal_y", "normal_z", "curvature"};
    static const uint32_t dst[8] = {0, 1, 2, 8, 4, 5, 6, 9};
    const size_t n = (size_t)m.width * m.height;
    if (!msg_covers(m)) return false;
    for (int k = 0; k < 8; ++k) {
        const PointField* f = find_field(m, names[k]);
        if (f && f->datatype == FLOAT32 && (size_t)f->offset + 4 > m.point_step) return false;
    }
    std::memset(records, 0, n * kXYZINormalStep);
    for (int k = 0; k < 8; ++k) {
        const PointField* f = find_field(m, names[k]);
        if (!f || f->datatype != FLOAT32) continue;
        for (size_t i = 0; i < n; ++i)
            std::memcpy(records + 12 * i + dst[k], m.data.data() + i * m.point_step + f->offset, 4);
    }
    return true;
}

// ---- (2) libpointmatcher DataPoints -----------------------------------------------------------
struct Label {
    std::string text;
    uint32_t span = 1;
};

// The descriptor labels rosMsgToLibPointMatcherCloud fills (saver.cpp:246-254): 22 rows.
inline std::vector<Label> dp_descriptor_labels() {
    return {{"surfaceness", 1}, {"curveness", 1}, {"pointness", 1}, {"normals", 3}, {"tangents", 3},
            {"labels", 1},      {"sticks", 4},    {"plates", 7},    {"balls", 1}};
}
constexpr uint32_t kDPDescriptorRows = 22;

struct DPCloud {
    std::vector<Label> feature_labels;     // normally x, y, z, pad
    std::vector<Label> descriptor_labels;
    std::vector<Label> time_labels;        // "time" or none
    size_t n = 0;
    std::vector<float> features;           // [n][feature rows]
    std::vector<float> descriptors;        // [n][descriptor rows]
    std::vector<float> times;              // [n][time rows]
    uint32_t feature_rows() const { uint32_t r = 0; for (auto& l : feature_labels) r += l.span; return r; }
    uint32_t descriptor_rows() const { uint32_t r = 0; for (auto& l : descriptor_labels) r += l.span; return r; }
    uint32_t time_rows() const { uint32_t r = 0; for (auto& l : time_labels) r += l.span; return r; }
};

// libPointMatcherToRosMsg (saver.cpp:135-221).
inline PointCloud2 dp_to_msg(const DPCloud& dp, const std::string& frame_id, double stamp) {
    PointCloud2 m;
    m.frame_id = frame_id;
    m.stamp = stamp;
    m.height = 1;
    m.width = (uint32_t)dp.n;
    m.is_bigendian = false;
    m.is_dense = true;
    uint32_t off = 0;
    for (const auto& l : dp.feature_labels) {
        if (l.text == "pad") continue;
        m.fields.push_back({l.text, off, FLOAT32, l.span});
        off += l.span * 4;
    }
    for (const auto& l : dp.descriptor_labels) {
        m.fields.push_back({l.text, off, FLOAT32, l.span});
        off += l.span * 4;
    }
    const uint32_t tr = dp.time_rows();
    if (tr > 0) {
        m.fields.push_back({"time", off, FLOAT32, tr});
        off += 4 * tr;
    }
    m.point_step = off;
    m.row_step = m.point_step * m.width;
    m.data.assign((size_t)m.row_step * m.height, 0);
    const uint32_t fr = dp.feature_rows(), dr = dp.descriptor_rows();
    for (size_t pt = 0; pt < dp.n; ++pt) {
        uint8_t* p = m.data.data() + pt * m.point_step;
        std::memcpy(p, &dp.features[pt * fr], 3 * 4);         // features.block<3,1>(0, pt)
        p += 3 * 4;
        size_t doff = 0;
        for (const auto& l : dp.descriptor_labels) {
            std::memcpy(p, &dp.descriptors[pt * dr + doff], l.span * 4);
            p += l.span * 4;
            doff += l.span;
        }
        if (tr > 0) std::memcpy(p, &dp.times[pt * tr], tr * 4);
    }
    return m;
}

// rosMsgToLibPointMatcherCloud (saver.cpp:224-306): fixed labels, fields read by position.
// Times are allocated (one "time" row) and left 0.  Returns false (empty cloud) for a message
// without fields, one with fewer than the 12 fields it reads, or a malformed one (see msg_covers).
inline bool dp_from_msg(const PointCloud2& m, DPCloud* dp) {
    *dp = DPCloud{};
    if (m.fields.empty()) return false;
    if (m.fields.size() < 12) return false;
    // malformed: data shorter than width·height·point_step, or a read past point_step
    static const uint32_t span_of[12] = {1, 1, 1, 1, 1, 1, 3, 3, 1, 4, 7, 1};
    if (!msg_covers(m)) return false;
    for (int k = 0; k < 12; ++k)
        if ((size_t)m.fields[k].offset + 4 * (size_t)span_of[k] > m.point_step) return false;
    dp->feature_labels = {{"x", 1}, {"y", 1}, {"z", 1}, {"pad", 1}};
    dp->descriptor_labels = dp_descriptor_labels();
    dp->time_labels = {{"time", 1}};
    dp->n = (size_t)m.width * m.height;
    dp->features.assign(dp->n * 4, 0.f);
    dp->descriptors.assign(dp->n * kDPDescriptorRows, 0.f);
    dp->times.assign(dp->n, 0.f);
    static const uint32_t drow[9] = {0, 1, 2, 3, 6, 9, 10, 14, 21};   // first row of each label
    static const uint32_t dspan[9] = {1, 1, 1, 3, 3, 1, 4, 7, 1};
    for (size_t pt = 0; pt < dp->n; ++pt) {
        const uint8_t* p = m.data.data() + pt * m.point_step;
        float* f = &dp->features[pt * 4];
        for (int k = 0; k < 3; ++k) std::memcpy(f + k, p + m.fields[k].offset, 4);
        f[3] = 1.f;                                            // padView.setConstant(1)
        float* d = &dp->descriptors[pt * kDPDescriptorRows];
        for (int k = 0; k < 9; ++k) std::memcpy(d + drow[k], p + m.fields[3 + k].offset, 4 * dspan[k]);
    }
    return true;
}

}  // namespace imls_wire
