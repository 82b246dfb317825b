// imls_icp_hip.hpp — header-only C++ adapter that gives the HIP path the member signatures of the
// reference's IMLSICPMatcher (imls_icp.h:45-147) and the SolveMotionEstimationProblem* free
// functions with the argument lists of solver.h:84-139, so laser_odometry.cpp:489-616 becomes a
// type swap (`IMLSICPMatcher` → `imls_hip::IMLSICPMatcherHip`, the solver calls qualified with
// `imls_hip::` or brought in by `using namespace imls_hip;`).
//
// Works with any PCL-shaped cloud: `CloudPtr` dereferences to a struct with `points`
// (contiguous vector of a point type that has x,y,z,normal_x,normal_y,normal_z fields, e.g.
// pcl::PointXYZINormal), `size()`, `push_back()`, `clear()`; any list of 3-indexable doubles
// (std::vector<Eigen::Vector3d>) and any 4×4 with operator()(r, c) (Eigen::Matrix4d) or double[16].
// Needs only imls_gpu.h (no PCL, Eigen or ROS headers), so it also builds where those are absent.
//
// Contexts.  The reference constructs a fresh matcher per frame (laser_odometry.cpp:489) and calls
// free solver functions; both share one process-wide glibc rand() stream (RANSAC, common.cpp:49).
// Here every default-constructed matcher and every free solver function uses ONE context per host
// thread (`thread_context()`, created on first use on device 0 and destroyed at thread exit), so
// device buffers are reused across frames and the RANSAC rand() stream runs on across iterations
// and frames exactly as the reference's does on its single processData thread.
#pragma once
#include <cmath>
#include <cstddef>
#include <cstdint>
#include <stdexcept>
#include <string>
#include <type_traits>
#include <vector>

#include "imls_gpu.h"

namespace imls_hip {

namespace detail {
struct ThreadContext {
    imls_ctx* ctx = nullptr;
    ~ThreadContext() { if (ctx) imls_destroy(ctx); }
};
inline void check(int rc, imls_ctx* ctx = nullptr) {
    if (rc != IMLS_OK)
        throw std::runtime_error("imls_gpu call failed with status " + std::to_string(rc) + ": " +
                                 (ctx ? imls_last_error(ctx) : ""));
}
// shipped config.json values (imls_default_params) with the LS solver
inline imls_params default_ls_params() {
    imls_params p;
    imls_default_params(&p);
    p.solve_method = IMLS_SOLVE_LS;
    return p;
}
}  // namespace detail

// The calling thread's context (device 0, shipped parameters, LS).  Throws when no MI355X is
// visible: the GPU path has no CPU fallback.
inline imls_ctx* thread_context() {
    thread_local detail::ThreadContext tc;
    if (!tc.ctx) {
        const imls_params p = detail::default_ls_params();
        tc.ctx = imls_create(0, &p);
        if (!tc.ctx) throw std::runtime_error("imls_create failed: no MI355X visible (no CPU fallback)");
    }
    return tc.ctx;
}

class IMLSICPMatcherHip {
public:
    // Replaces `IMLSICPMatcher matcher;` (laser_odometry.cpp:489): binds the thread's context.
    IMLSICPMatcherHip() : ctx_(thread_context()), own_(false), params_(detail::default_ls_params()) {}
    // A matcher with its own context on `device` (params == nullptr → shipped values, LS).
    explicit IMLSICPMatcherHip(int device, const imls_params* params = nullptr)
        : params_(params ? *params : detail::default_ls_params()) {
        ctx_ = imls_create(device, &params_);
        if (!ctx_) throw std::runtime_error("imls_create failed: no MI355X visible (no CPU fallback)");
        own_ = true;
    }
    ~IMLSICPMatcherHip() { if (own_ && ctx_) imls_destroy(ctx_); }
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
        apply(p);
    }
    // Any other field (solver, FIFO length, plane_ICP, ...) at once.
    void setParams(const imls_params& p) { apply(p); }

    // imls_icp.cpp:74-78: the cloud is NaN-filtered in place, as the reference does.
    template <class CloudPtr>
    void setSourcePointCloud(CloudPtr cloud) {
        remove_nan(*cloud);
        if (cloud->size() == 0) return;
        const auto& p0 = cloud->points[0];
        detail::check(imls_set_source(ctx_, &p0.x, &p0.normal_x, cloud->size(), stride(*cloud), nullptr, nullptr), ctx_);
    }

    // imls_icp.cpp:80-103: NaN filter in place + index build on the GPU.
    template <class CloudPtr>
    void setTargetPointCloud(CloudPtr cloud) {
        remove_nan(*cloud);
        if (cloud->size() == 0) return;
        const auto& p0 = cloud->points[0];
        detail::check(imls_set_target(ctx_, &p0.x, &p0.normal_x, cloud->size(), stride(*cloud), nullptr), ctx_);
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
        detail::check(imls_set_params(ctx_, &params_), ctx_);
        if (!pose) {
            const auto& p0 = in_cloud->points[0];
            detail::check(imls_set_source(ctx_, &p0.x, &p0.normal_x, n, stride(*in_cloud), nullptr, nullptr), ctx_);
        }
        std::vector<float> x(3 * n), y(3 * n), nn(3 * n);
        std::vector<uint32_t> idx(n);
        size_t nv = 0;
        detail::check(imls_project(ctx_, pose ? pose : I, x.data(), y.data(), nn.data(), idx.data(), &nv, reject_), ctx_);
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
        const imls_params keep = params_;
        imls_params p = params_;
        p.matching_method = IMLS_MATCH_PLANE_ICP;
        p.picp_r = r;
        p.picp_use_projected_distance = use_projected_distance;
        p.picp_r_proj = r_proj;
        p.picp_normal_angle_constraint = normal_angle_constraint;
        p.picp_angle_diff_threshold = angle_diff_threshold;
        params_ = p;
        try {
            ProjSourcePtToSurface(in_cloud, ref_cloud, std::string(), 0, pose);
        } catch (...) {
            params_ = keep;
            throw;
        }
        params_ = keep;
    }

    // Fused laser_odometry.cpp:524-647 for the clouds already set; pose_out = rPose.
    int registerFrame(double pose_out[16], int* iters_run = nullptr, int* status = nullptr) {
        const int rc = imls_set_params(ctx_, &params_);
        if (rc != IMLS_OK) return rc;
        return imls_register_frame(ctx_, pose_out, iters_run, status, nullptr);
    }

    const uint64_t* rejectCounters() const { return reject_; }
    const imls_params& params() const { return params_; }

private:
    void apply(const imls_params& p) {
        detail::check(imls_set_params(ctx_, &p), ctx_);
        params_ = p;
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
    bool own_ = false;
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

// One solve on the thread's context with `p` (then the context's previous parameters restored).
template <class Vec3List, class Mat4>
inline bool solve(int32_t method, imls_params p, const Vec3List& s3, const Vec3List& d3, const Vec3List& n3,
                  const double* w, Mat4& deltaTrans) {
    imls_ctx* ctx = thread_context();
    std::vector<double> s, d, n;
    flatten(s3, s); flatten(d3, d); flatten(n3, n);
    double D[16];
    int ok = 0;
    if (imls_set_params(ctx, &p) != IMLS_OK) return false;
    const int rc = imls_solve_correspondences(ctx, method, s.data(), d.data(), n.data(), w, s3.size(), D, &ok);
    if (rc != IMLS_OK || !ok) return false;
    to_matrix(D, deltaTrans);
    return true;
}
inline imls_params thread_params() {
    // the thread context's current parameters are not readable through the ABI: start from the
    // shipped values; every solver argument the reference passes is applied on top
    return default_ls_params();
}
}  // namespace detail

// solver.cpp:74-166 (solver.h:84-90): same arguments.
template <class Vec3List, class Mat4>
bool SolveMotionEstimationProblemLS(Vec3List& source_cloud, Vec3List& ref_cloud, Vec3List& ref_normals,
                                    Mat4& deltaTrans, const std::string& /*timestamp*/, const double threshold) {
    imls_params p = detail::thread_params();
    p.solve_method = IMLS_SOLVE_LS;
    p.ls_threshold = threshold;
    return detail::solve(IMLS_SOLVE_LS, p, source_cloud, ref_cloud, ref_normals, nullptr, deltaTrans);
}

// solver.cpp:168-220 (solver.h:92-98): same arguments (weights: Eigen::VectorXd or any indexable).
template <class Vec3List, class Mat4, class WVec>
bool SolveMotionEstimationProblemWeightedLS(Vec3List& source_cloud, Vec3List& ref_cloud, Vec3List& ref_normals,
                                            Mat4& deltaTrans, const WVec& weights, const std::string& /*timestamp*/) {
    std::vector<double> w(source_cloud.size());
    for (size_t i = 0; i < w.size(); ++i) w[i] = weights[i];
    imls_params p = detail::thread_params();
    p.solve_method = IMLS_SOLVE_LS;
    return detail::solve(IMLS_SOLVE_WEIGHTED_LS, p, source_cloud, ref_cloud, ref_normals, w.data(), deltaTrans);
}

// solver.cpp:222-385 (+ 486-603 for the DRPM final) (solver.h:100-114): same arguments;
// final_solve_method is config.json's string ("LS", "Weighted LS", "DRPM"), anything else returns
// false like solver.cpp:380-384.  Hypotheses draw from the thread context's rand() stream, which
// runs on across calls (seeded once from ransac_seed = 1, glibc's default, like the reference's
// never-seeded process).
template <class Vec3List, class Mat4>
bool SolveMotionEstimationProblemRANSAC(Vec3List& source_cloud, Vec3List& ref_cloud, Vec3List& ref_normals,
                                        Mat4& deltaTrans, const std::string& /*timestamp*/, const int max_iterations,
                                        const double distance_threshold, const double min_inliers_percentage,
                                        const double huber_threshold, const std::string final_solve_method,
                                        const double ls_threshold, const double drpm_threshold,
                                        const double drpm_stdev_points, const double drpm_stdev_normals) {
    imls_params p = detail::thread_params();
    p.solve_method = IMLS_SOLVE_RANSAC;
    p.ransac_max_iterations = max_iterations;
    p.ransac_distance_threshold = distance_threshold;
    p.ransac_min_inliers_percentage = min_inliers_percentage;
    p.ransac_huber_threshold = huber_threshold;
    if (final_solve_method == "LS") p.ransac_final_method = IMLS_FINAL_LS;
    else if (final_solve_method == "Weighted LS") p.ransac_final_method = IMLS_FINAL_WEIGHTED_LS;
    else if (final_solve_method == "DRPM") p.ransac_final_method = IMLS_FINAL_DRPM;
    else return false;
    p.ransac_ls_threshold = ls_threshold;
    p.drpm_threshold = drpm_threshold;
    p.drpm_stdev_points = drpm_stdev_points;
    p.drpm_stdev_normals = drpm_stdev_normals;
    return detail::solve(IMLS_SOLVE_RANSAC, p, source_cloud, ref_cloud, ref_normals, nullptr, deltaTrans);
}

// solver.cpp:499-603 (solver.h:130-139): same arguments.
template <class Vec3List, class Mat4, class WVec>
bool SolveMotionEstimationProblemDRPM(Vec3List& source_cloud, Vec3List& ref_cloud, Vec3List& ref_normals,
                                      Mat4& deltaTrans, const WVec& weights, const std::string& /*timestamp*/,
                                      const double threshold, const double stdev_points, const double stdev_normals) {
    std::vector<double> w(source_cloud.size());
    for (size_t i = 0; i < w.size(); ++i) w[i] = weights[i];
    imls_params p = detail::thread_params();
    p.solve_method = IMLS_SOLVE_LS;
    p.drpm_threshold = threshold;
    p.drpm_stdev_points = stdev_points;
    p.drpm_stdev_normals = stdev_normals;
    return detail::solve(IMLS_SOLVE_DRPM, p, source_cloud, ref_cloud, ref_normals, w.data(), deltaTrans);
}

}  // namespace imls_hip
