// type_swap.cpp — the reference's per-frame loop (laser_odometry.cpp:489-647) written against the
// type-swapped API of include/imls_icp_hip.hpp: `IMLSICPMatcher matcher;` → `IMLSICPMatcherHip`,
// the solver calls → `imls_hip::SolveMotionEstimationProblem*` with solver.h's argument lists.
// Only the types change; the loop body (transform in double stored as float, project, gate,
// getXYZ/getNormals, solve, rPose = Δ·rPose, convergence test) is the reference's shape.
// PCL / Eigen stand-ins are minimal local types (the adapter needs none of their headers).
//
// usage: type_swap <LS|RANSAC> <iterations> <src.bin> <tgt.bin>
//   *.bin: uint64 count, then count 48-byte PointXYZINormal records (common.h:17).
// prints: one line per iteration "iter <i> <n_valid>", then "iters <n>" and "pose <16 x %.17g>".
#include <array>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <memory>
#include <string>
#include <vector>

#include "imls_icp_hip.hpp"

struct PointXYZINormal {          // pcl::PointXYZINormal memory layout (48 B)
    float x, y, z, pad0;
    float normal_x, normal_y, normal_z, pad1;
    float intensity, curvature, pad2, pad3;
};
static_assert(sizeof(PointXYZINormal) == 48, "layout");
struct Cloud {                    // pcl::PointCloud<PointType> stand-in
    std::vector<PointXYZINormal> points;
    size_t size() const { return points.size(); }
    void push_back(const PointXYZINormal& p) { points.push_back(p); }
    void clear() { points.clear(); }
};
using CloudPtr = std::shared_ptr<Cloud>;
using Vector3d = std::array<double, 3>;
struct Matrix4d {                 // Eigen::Matrix4d stand-in (row/col access, product, identity)
    double m[16];
    double& operator()(int r, int c) { return m[r * 4 + c]; }
    double operator()(int r, int c) const { return m[r * 4 + c]; }
    void setIdentity() { for (int k = 0; k < 16; ++k) m[k] = (k % 5 == 0) ? 1.0 : 0.0; }
};
static Matrix4d mul(const Matrix4d& a, const Matrix4d& b) {   // Eigen 4x4 lazy product order
    Matrix4d r;
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) {
            double s = a(i, 0) * b(0, j);
            s = s + a(i, 1) * b(1, j);
            s = s + a(i, 2) * b(2, j);
            s = s + a(i, 3) * b(3, j);
            r(i, j) = s;
        }
    return r;
}
static void getXYZ(const CloudPtr& c, std::vector<Vector3d>& v) {      // common.h:51-63
    v.clear();
    for (auto& p : c->points) v.push_back({(double)p.x, (double)p.y, (double)p.z});
}
static void getNormals(const CloudPtr& c, std::vector<Vector3d>& v) {  // common.h:65-75
    v.clear();
    for (auto& p : c->points) v.push_back({(double)p.normal_x, (double)p.normal_y, (double)p.normal_z});
}
static CloudPtr load(const char* path) {
    FILE* f = std::fopen(path, "rb");
    if (!f) { std::perror(path); std::exit(2); }
    unsigned long long n = 0;
    if (std::fread(&n, 8, 1, f) != 1) std::exit(2);
    auto c = std::make_shared<Cloud>();
    c->points.resize(n);
    if (n && std::fread(c->points.data(), sizeof(PointXYZINormal), n, f) != n) std::exit(2);
    std::fclose(f);
    return c;
}

int main(int argc, char** argv) {
    if (argc != 5) { std::fprintf(stderr, "usage: type_swap <LS|RANSAC> <iterations> <src.bin> <tgt.bin>\n"); return 2; }
    const std::string solve_method = argv[1];
    const int iterations = std::atoi(argv[2]);
    CloudPtr flatCloud = load(argv[3]);
    CloudPtr accumulatedTargetCloud = load(argv[4]);
    const int correspond_number = 6;
    const double delta_dist_threshold = 0.001, delta_angle_threshold = 0.0001745353;
    const bool transform_normal = false;
    try {
        Matrix4d rPose;
        rPose.setIdentity();
        imls_hip::IMLSICPMatcherHip matcher;                                   // laser_odometry.cpp:489
        matcher.setSourcePointCloud(flatCloud);                                // 509
        matcher.setTargetPointCloud(accumulatedTargetCloud);                   // 510
        matcher.setParameters(iterations, 1.0, 3.0, 1.0, 0.8, false, true, false, 50, 0.2, 0.6, 10, 20, true, 30.0,
                              "");                                              // 514-518 (config.json values)
        int it = 0;
        for (int i = 0; i < iterations; i++) {                                 // 524
            CloudPtr in_cloud(new Cloud(*flatCloud));                          // 527
            for (size_t ix = 0; ix < flatCloud->size(); ix++) {
                const auto& q = flatCloud->points[ix];
                double now_pt[4];
                for (int r = 0; r < 4; ++r) {                                  // Eigen Matrix4d * Vector4d
                    double s = rPose(r, 0) * q.x;
                    s = s + rPose(r, 1) * q.y;
                    s = s + rPose(r, 2) * q.z;
                    s = s + rPose(r, 3) * 1.0;
                    now_pt[r] = s;
                }
                in_cloud->points[ix].x = now_pt[0];
                in_cloud->points[ix].y = now_pt[1];
                in_cloud->points[ix].z = now_pt[2];
                (void)transform_normal;
            }
            CloudPtr ref_cloud(new Cloud);
            matcher.ProjSourcePtToSurface(in_cloud, ref_cloud, "0", i);        // 559
            if ((int)in_cloud->size() < correspond_number || (int)ref_cloud->size() < correspond_number) break;   // 570-576
            std::printf("iter %d %zu\n", i, ref_cloud->size());
            std::vector<Vector3d> in_cloud_vec, ref_cloud_vec, ref_normal;
            getXYZ(in_cloud, in_cloud_vec);                                    // 595-599
            getXYZ(ref_cloud, ref_cloud_vec);
            getNormals(ref_cloud, ref_normal);
            Matrix4d deltaTrans;
            std::string timestamp = "0";
            bool flag = false;
            if (solve_method == "LS")                                          // dispatcher 195-203
                flag = imls_hip::SolveMotionEstimationProblemLS(in_cloud_vec, ref_cloud_vec, ref_normal, deltaTrans,
                                                                timestamp, 0.02);
            else if (solve_method == "RANSAC")                                 // dispatcher 204-229 (config.json values)
                flag = imls_hip::SolveMotionEstimationProblemRANSAC(in_cloud_vec, ref_cloud_vec, ref_normal, deltaTrans,
                                                                    timestamp, 5000, 0.8, 0.95, 0.648, "DRPM", 0.02,
                                                                    0.05, 0.02, 0.05);
            if (!flag) break;                                                  // 611-616
            rPose = mul(deltaTrans, rPose);                                    // 619
            ++it;
            const double deltaDist = std::sqrt(std::pow(deltaTrans(0, 3), 2) + std::pow(deltaTrans(1, 3), 2) +
                                               std::pow(deltaTrans(2, 3), 2));
            double cos_theta = (((deltaTrans(0, 0) + deltaTrans(1, 1)) + deltaTrans(2, 2)) - 1.0) / 2.0;
            cos_theta = std::min(1.0, std::max(cos_theta, -1.0));
            const double deltaAngle = std::acos(cos_theta);
            if (deltaDist < delta_dist_threshold && deltaAngle < delta_angle_threshold) break;   // 640-646
        }
        std::printf("iters %d\npose", it);
        for (int k = 0; k < 16; ++k) std::printf(" %.17g", rPose.m[k]);
        std::printf("\n");
    } catch (const std::exception& e) {
        std::fprintf(stderr, "type_swap: %s\n", e.what());
        return 1;
    }
    return 0;
}
