// imls_icp_hip.hpp — header-only C++ adapter that gives the HIP path the member signatures of the
// reference's IMLSICPMatcher (imls_icp.h:45-147) and the SolveMotionEstimationProblem* free
// functions (solver.h:77-139), so laser_odometry.cpp:489-616 becomes a type swap.
//
// Works with any PCL-shaped cloud: `CloudPtr` dereferences to a struct with `points`
// (contiguous vector of a point type that has x,y,z,normal_x,normal_y,normal_z fields, e.g.
// pcl::PointXYZINormal), `size()`, `push_back()`, `clear()`.  Needs only imls_gpu.h (no PCL,
// Eigen or ROS headers), so it also builds where those are absent.
#pragma once
#include <cmath>
#include <cstddef>
#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

#include "imls_gpu.h"

namespace imls_hip {

class IMLSICPMatcherHip {
public:
    // Replaces `IMLSICPMatcher matcher;` (laser_odometry.cpp:489).  params == nullptr → the
    // shipped config.json values with solve_method = LS.
    explicit IMLSICPMatcherHip(int device = 0, const imls_params* params = nullptr) {
        imls_params p;
        if (params) p = *params;
        else { imls_default_params(&p); p.solve_method = IMLS_SOLVE_LS; }
        params_ = p;
        ctx_ = imls_create(device, &p);
        if (!ctx_) throw std::runtime_error("imls_create failed: no MI355X visible (no CPU fallback)");
    }
    ~IMLSICPMatcherHip() { if (ctx_) imls_destroy(ctx_); }
    IMLSICPMatcherHip(const IMLSICPMatcherHip&) = delete;
    IMLSICPMatcherHip& operator=(const IMLSICPMatcherHip&) = delete;

    imls_ctx* context() const { return ctx_; }

    // imls_icp.h:62-66, same 16 parameters in the same order.
    void setParameters(int _iter, double _h, double _r, double _r_normal, double _r_proj, bool _useTensorVoting,
                       bool _isGetNormals, bool _useProjectedDistance, int _tensor_k, double _tensor_sigma,
                       double _tensor_distance_threshold, int _search_number_normal, int _search_number,
                       bool _normal_angle_constraint, double _angle_diff_threshold, const std::string& /*_output_dir*/) {
        imls_params p = params_;
        p.iterations = _iter; p.h = _h; p.r = _r; p.r_normal = _r_normal; p.r_proj = _r_proj;
        p.use_tensor_voting = _useTensorVoting; p.get_normals = _isGetNormals;
        p.use_projected_distance = _useProjectedDistance; p.tensor_k = _tensor_k; p.tensor_sigma = _tensor_sigma;
        p.tensor_distance_threshold = _tensor_distance_threshold; p.search_number_normal = _search_number_normal;
        p.search_number = _search_number; p.normal_angle_constraint = _normal_angle_constraint;
        p.angle_diff_threshold = _angle_diff_threshold;
        check(imls_set_params(ctx_, &p));
        params_ = p;
    }

    // imls_icp.cpp:74-78: the cloud is NaN-filtered in place, as the reference does.
    template <class CloudPtr>
    void setSourcePointCloud(CloudPtr cloud) {
        remove_nan(*cloud);
        if (cloud->size() == 0) return;
        const auto& p0 = cloud->points[0];
        check(imls_set_source(ctx_, &p0.x, &p0.normal_x, cloud->size(), stride(*cloud), nullptr, nullptr));
    }

    // imls_icp.cpp:80-103: NaN filter in place + index build on the GPU.
    template <class CloudPtr>
    void setTargetPointCloud(CloudPtr cloud) {
        remove_nan(*cloud);
        if (cloud->size() == 0) return;
        const auto& p0 = cloud->points[0];
        check(imls_set_target(ctx_, &p0.x, &p0.normal_x, cloud->size(), stride(*cloud), nullptr));
    }

    // imls_icp.cpp:496-745.  With pose == nullptr, `in_cloud` is taken as already transformed
    // (laser_odometry.cpp:527-549 does that) and uploaded as the source; with a pose, the source
    // set by setSourcePointCloud is transformed on the GPU.  Unmatched points are erased from
    // in_cloud (order kept); out_cloud receives y and the NN-1 normal per surviving point.
    template <class CloudPtr>
    void ProjSourcePtToSurface(CloudPtr& in_cloud, CloudPtr& out_cloud, const std::string& /*timestamp*/,
                               const int& /*i*/, const double* pose = nullptr) {
        static const double I[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
        out_cloud->clear();
        const size_t n = in_cloud->size();
        if (n == 0) return;
        if (!pose) {
            const auto& p0 = in_cloud->points[0];
            check(imls_set_source(ctx_, &p0.x, &p0.normal_x, n, stride(*in_cloud), nullptr, nullptr));
        }
        std::vector<float> x(3 * n), y(3 * n), nn(3 * n);
        std::vector<uint32_t> idx(n);
        size_t nv = 0;
        check(imls_project(ctx_, pose ? pose : I, x.data(), y.data(), nn.data(), idx.data(), &nv, reject_));
        auto& pts = in_cloud->points;
        using Pt = typename std::decay<decltype(pts[0])>::type;
        std::vector<Pt> kept;
        kept.reserve(nv);
        for (size_t k = 0; k < nv; ++k) {
            Pt s = pts[idx[k]];
            s.x = x[3 * k]; s.y = x[3 * k + 1]; s.z = x[3 * k + 2];
            kept.push_back(s);
            Pt t{};
            t.x = y[3 * k]; t.y = y[3 * k + 1]; t.z = y[3 * k + 2];
            t.normal_x = nn[3 * k]; t.normal_y = nn[3 * k + 1]; t.normal_z = nn[3 * k + 2];
            out_cloud->push_back(t);
        }
        pts.assign(kept.begin(), kept.end());
    }

    // plane_ICP_proj (laser_odometry.cpp:277-413): the same contract as ProjSourcePtToSurface
    // (in_cloud erased in order, out_cloud = y + NN-1 normal) with the plane_ICP parameters of
    // config.json (matching_method.plane_ICP: r, use_projected_distance {enabled, r_proj},
    // normal_angle_constraint {enabled, angle_diff_threshold}).  The reference's uninitialised
    // tree pointer (522) and by-value pointer (279) are not reproduced: the context owns the index.
    template <class CloudPtr>
    void planeICPProj(CloudPtr& in_cloud, CloudPtr& ref_cloud, double r, bool use_projected_distance, double r_proj,
                      bool normal_angle_constraint, double angle_diff_threshold, const double* pose = nullptr) {
        imls_params p = params_;
        p.matching_method = IMLS_MATCH_PLANE_ICP;
        p.picp_r = r;
        p.picp_use_projected_distance = use_projected_distance;
        p.picp_r_proj = r_proj;
        p.picp_normal_angle_constraint = normal_angle_constraint;
        p.picp_angle_diff_threshold = angle_diff_threshold;
        check(imls_set_params(ctx_, &p));
        ProjSourcePtToSurface(in_cloud, ref_cloud, std::string(), 0, pose);
        check(imls_set_params(ctx_, &params_));
    }

    // Fused laser_odometry.cpp:524-647 for the clouds already set; pose_out = rPose.
    int registerFrame(double pose_out[16], int* iters_run = nullptr, int* status = nullptr) {
        return imls_register_frame(ctx_, pose_out, iters_run, status, nullptr);
    }

    const uint64_t* rejectCounters() const { return reject_; }
    const imls_params& params() const { return params_; }

private:
    static void check(int rc) {
        if (rc != IMLS_OK) throw std::runtime_error("imls_gpu call failed with status " + std::to_string(rc));
    }
    template <class Cloud>
    static size_t stride(const Cloud& c) { return sizeof(c.points[0]) / sizeof(float); }
    template <class Cloud>
    static void remove_nan(Cloud& c) {
        auto& pts = c.points;
        size_t w = 0;
        for (size_t r = 0; r < pts.size(); ++r)
            if (std::isfinite(pts[r].x) && std::isfinite(pts[r].y) && std::isfinite(pts[r].z)) pts[w++] = pts[r];
        pts.resize(w);
    }

    imls_ctx* ctx_ = nullptr;
    imls_params params_{};
    uint64_t reject_[IMLS_NUM_REJ] = {0, 0, 0, 0, 0, 0};
};

namespace detail {
template <class V>
inline void flatten(const V& v, std::vector<double>& out) {
    out.resize(3 * v.size());
    for (size_t i = 0; i < v.size(); ++i) { out[3 * i] = v[i][0]; out[3 * i + 1] = v[i][1]; out[3 * i + 2] = v[i][2]; }
}
template <class M>
inline void to_matrix(const double D[16], M& m) { for (int r = 0; r < 4; ++r) for (int c = 0; c < 4; ++c) m(r, c) = D[r * 4 + c]; }
inline void to_matrix(const double D[16], double (&m)[16]) { for (int k = 0; k < 16; ++k) m[k] = D[k]; }
}  // namespace detail

// solver.cpp:74-166 — same arguments plus the context that owns the device.  Vec3List is
// std::vector<Eigen::Vector3d> (or any vector of 3-indexable doubles); Mat4 is Eigen::Matrix4d
// or double[16].
template <class Vec3List, class Mat4>
bool SolveMotionEstimationProblemLS(IMLSICPMatcherHip& m, const Vec3List& source_cloud, const Vec3List& ref_cloud,
                                    const Vec3List& ref_normals, Mat4& deltaTrans, const std::string& /*timestamp*/,
                                    const double threshold) {
    imls_params p = m.params();
    p.ls_threshold = threshold;
    p.solve_method = IMLS_SOLVE_LS;
    if (imls_set_params(m.context(), &p) != IMLS_OK) return false;
    std::vector<double> s, d, n;
    detail::flatten(source_cloud, s); detail::flatten(ref_cloud, d); detail::flatten(ref_normals, n);
    double D[16];
    int ok = 0;
    if (imls_solve_correspondences(m.context(), IMLS_SOLVE_LS, s.data(), d.data(), n.data(), nullptr,
                                   source_cloud.size(), D, &ok) != IMLS_OK) return false;
    detail::to_matrix(D, deltaTrans);
    return ok != 0;
}

// solver.cpp:168-220.
template <class Vec3List, class WVec, class Mat4>
bool SolveMotionEstimationProblemWeightedLS(IMLSICPMatcherHip& m, const Vec3List& source_cloud, const Vec3List& ref_cloud,
                                            const Vec3List& ref_normals, Mat4& deltaTrans, const WVec& weights,
                                            const std::string& /*timestamp*/) {
    std::vector<double> s, d, n, w(weights.size());
    detail::flatten(source_cloud, s); detail::flatten(ref_cloud, d); detail::flatten(ref_normals, n);
    for (size_t i = 0; i < w.size(); ++i) w[i] = weights[i];
    double D[16];
    int ok = 0;
    if (imls_solve_correspondences(m.context(), IMLS_SOLVE_WEIGHTED_LS, s.data(), d.data(), n.data(), w.data(),
                                   source_cloud.size(), D, &ok) != IMLS_OK) return false;
    detail::to_matrix(D, deltaTrans);
    return ok != 0;
}

// solver.cpp:222-385 (+ 486-603 for the DRPM final): same arguments; final_solve_method is
// config.json's string ("LS", "Weighted LS", "DRPM").  rand() is replayed on the device from
// the context's ransac_seed (glibc's default 1 unless set), re-seeded per call.
template <class Vec3List, class Mat4>
bool SolveMotionEstimationProblemRANSAC(IMLSICPMatcherHip& m, const Vec3List& source_cloud, const Vec3List& ref_cloud,
                                        const Vec3List& ref_normals, Mat4& deltaTrans, const std::string& /*timestamp*/,
                                        const int max_iterations, const double distance_threshold,
                                        const double min_inliers_percentage, const double huber_threshold,
                                        const std::string& final_solve_method, const double ls_threshold,
                                        const double drpm_threshold, const double drpm_stdev_points,
                                        const double drpm_stdev_normals) {
    imls_params p = m.params();
    p.solve_method = IMLS_SOLVE_RANSAC;
    p.ransac_max_iterations = max_iterations;
    p.ransac_distance_threshold = distance_threshold;
    p.ransac_min_inliers_percentage = min_inliers_percentage;
    p.ransac_huber_threshold = huber_threshold;
    if (final_solve_method == "LS") p.ransac_final_method = IMLS_FINAL_LS;
    else if (final_solve_method == "Weighted LS") p.ransac_final_method = IMLS_FINAL_WEIGHTED_LS;
    else if (final_solve_method == "DRPM") p.ransac_final_method = IMLS_FINAL_DRPM;
    else return false;   // solver.cpp:380-384: unknown final method → false
    p.ransac_ls_threshold = ls_threshold;
    p.drpm_threshold = drpm_threshold;
    p.drpm_stdev_points = drpm_stdev_points;
    p.drpm_stdev_normals = drpm_stdev_normals;
    if (imls_set_params(m.context(), &p) != IMLS_OK) return false;
    std::vector<double> s, d, n;
    detail::flatten(source_cloud, s); detail::flatten(ref_cloud, d); detail::flatten(ref_normals, n);
    double D[16];
    int ok = 0;
    const int rc = imls_solve_correspondences(m.context(), IMLS_SOLVE_RANSAC, s.data(), d.data(), n.data(), nullptr,
                                              source_cloud.size(), D, &ok);
    imls_set_params(m.context(), &m.params());
    if (rc != IMLS_OK) return false;
    detail::to_matrix(D, deltaTrans);
    return ok != 0;
}

}  // namespace imls_hip
