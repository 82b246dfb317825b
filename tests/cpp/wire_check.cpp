// tests/cpp/wire_check — exercises include/imls_wire.hpp on deterministic data and prints the
// field tables, point steps and FNV-1a hashes of the encoded bytes; tests/test_wire.py compares
// them with the Python mirror (planetary-lidar-odometry_amd/wire.py) on the same data.
#include <cstdio>
#include <vector>

#include "imls_wire.hpp"

using namespace imls_wire;

static unsigned long long fnv1a(const uint8_t* p, size_t n) {
    unsigned long long h = 0xcbf29ce484222325ull;
    for (size_t i = 0; i < n; ++i) h = (h ^ p[i]) * 0x100000001b3ull;
    return h;
}
static void print_msg(const char* tag, const PointCloud2& m) {
    std::printf("%s step=%u width=%u fields=", tag, m.point_step, m.width);
    for (const auto& f : m.fields) std::printf("%s:%u:%u:%u,", f.name.c_str(), f.offset, (unsigned)f.datatype, f.count);
    std::printf(" fnv=%llu\n", fnv1a(m.data.data(), m.data.size()));
}

int main() {
    const size_t n = 37;
    std::vector<float> rec(n * 12);
    for (size_t i = 0; i < n; ++i)
        for (int k = 0; k < 12; ++k) rec[i * 12 + k] = (float)(i * 13 + k * 7) * 0.125f - 3.f;
    PointCloud2 m = xyzinormal_to_msg(rec.data(), n, "velodyne", 12.5);
    print_msg("xyzinormal", m);
    StridedCloud sc;
    const bool ok = strided_view(m, &sc);
    std::printf("strided ok=%d n=%zu stride=%zu xyz_off=%td nrm_off=%td\n", (int)ok, sc.n, sc.stride_floats,
                (const uint8_t*)sc.xyz - m.data.data(), (const uint8_t*)sc.nrm - m.data.data());
    std::vector<float> back(n * 12);
    xyzinormal_from_msg(m, back.data());
    bool same = true;   // the named fields come back; the pads are 0
    for (size_t i = 0; i < n; ++i)
        for (int k : {0, 1, 2, 4, 5, 6, 8, 9}) same = same && back[i * 12 + k] == rec[i * 12 + k];
    std::printf("xyzinormal roundtrip=%d\n", (int)same);

    DPCloud dp;
    dp.feature_labels = {{"x", 1}, {"y", 1}, {"z", 1}, {"pad", 1}};
    dp.descriptor_labels = dp_descriptor_labels();
    dp.time_labels = {{"time", 1}};
    dp.n = n;
    dp.features.resize(n * 4);
    dp.descriptors.resize(n * kDPDescriptorRows);
    dp.times.resize(n);
    for (size_t i = 0; i < n; ++i) {
        for (int r = 0; r < 3; ++r) dp.features[i * 4 + r] = (float)(i * 3 + r) * 0.5f - 1.f;
        dp.features[i * 4 + 3] = 1.f;
        for (uint32_t r = 0; r < kDPDescriptorRows; ++r) dp.descriptors[i * kDPDescriptorRows + r] = (float)(i * 22 + r) * 0.01f;
        dp.times[i] = (float)i * 0.1f;
    }
    PointCloud2 d = dp_to_msg(dp, "map", 3.25);
    print_msg("dp", d);
    DPCloud dq;
    const bool rok = dp_from_msg(d, &dq);
    bool dsame = rok && dq.n == n;
    for (size_t i = 0; dsame && i < n; ++i) {
        for (int r = 0; r < 3; ++r) dsame = dsame && dq.features[i * 4 + r] == dp.features[i * 4 + r];
        dsame = dsame && dq.features[i * 4 + 3] == 1.f && dq.times[i] == 0.f;
        for (uint32_t r = 0; r < kDPDescriptorRows; ++r)
            dsame = dsame && dq.descriptors[i * kDPDescriptorRows + r] == dp.descriptors[i * kDPDescriptorRows + r];
    }
    std::printf("dp roundtrip=%d\n", (int)dsame);
    // the reader goes by position: swap the first two descriptor fields' entries in the table
    PointCloud2 sw = d;
    std::swap(sw.fields[3], sw.fields[4]);
    DPCloud ds;
    dp_from_msg(sw, &ds);
    std::printf("dp swapped fnv=%llu\n", fnv1a((const uint8_t*)ds.descriptors.data(), ds.descriptors.size() * 4));
    PointCloud2 empty;
    DPCloud de;
    std::printf("dp empty=%d\n", (int)dp_from_msg(empty, &de));
    // malformed messages are rejected, never read out of bounds
    PointCloud2 shortm = m;
    shortm.data.resize(shortm.data.size() - 1);
    PointCloud2 badoff = m;
    badoff.fields[0].offset = badoff.point_step - 2;
    PointCloud2 dshort = d;
    dshort.data.resize(d.point_step * (n - 1));
    PointCloud2 doff = d;
    doff.fields[11].offset = doff.point_step;
    std::printf("malformed xyzinormal_short=%d xyzinormal_offset=%d dp_short=%d dp_offset=%d\n",
                (int)xyzinormal_from_msg(shortm, back.data()), (int)xyzinormal_from_msg(badoff, back.data()),
                (int)dp_from_msg(dshort, &de), (int)dp_from_msg(doff, &de));
    return 0;
}
