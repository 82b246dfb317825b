/*
 * imls_oracle.h — CPU restatement of the reference IMLS-ICP path.  TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this library,
 * and only as the checker / the timed CPU baseline — never as the product path.
 *
 * PARITY STATUS: "parity unpinned" at the third-party boundaries.  The reference
 * (spirit-man/Planetary-LiDAR-Odometry) cannot be compiled here (no Eigen, libnabo, PCL, ROS,
 * libpointmatcher, Ceres, TEASER++, Boost) and ships no tests, fixtures or
 * golden vectors.  This file restates the reference source line by line (citations in
 * imls_oracle.cpp) and restates the published algorithms of the third-party pieces it calls:
 *   - libnabo (unpinned version) kNN: exact, radius-bounded (d² ≤ r²), sorted, unfound = +inf,
 *     self-match excluded unless ALLOW_SELF_MATCH (d² > DBL_EPSILON test);
 *   - Eigen ≥ 3.3.4 ColPivHouseholderQR (solve = basic solution), AngleAxis::toRotationMatrix,
 *     JacobiSVD polar factor, SelfAdjointEigenSolver;
 *   - Boost.Math 1.72 cdf(normal_distribution);  glibc rand() (TYPE_3 additive feedback).
 * It is pinned instead by (a) an independent numpy/scipy restatement (oracle/imls_np.py),
 * (b) analytic known-answer tests, (c) glibc rand() itself.
 */
#ifndef IMLS_ORACLE_H
#define IMLS_ORACLE_H
#include <stddef.h>
#include <stdint.h>
#include "../include/imls_gpu.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Clouds are SoA float32[6][n]: x[n], y[n], z[n], nx[n], ny[n], nz[n].  Non-finite-xyz points
 * are dropped first (imls_icp.cpp:58-78), so indices refer to the filtered clouds. */

/* kNN with libnabo semantics.  d2/idx: Q*K outputs, sorted ascending by (d², index); unfound
 * slots get d² = +inf, idx = -1. */
int oracle_knn(const float* tgt6, size_t M, const float* q3 /* [3][Q] */, size_t Q, int K,
               double max_radius, int allow_self_match, double* d2, int32_t* idx);

/* ProjSourcePtToSurface on the source transformed by `pose` (laser_odometry.cpp:527-549). */
int oracle_project(const float* src6, size_t N, const float* tgt6, size_t M, const double pose[16],
                   const imls_params* p, float* x_out, float* y_out, float* n_out,
                   uint32_t* src_index_out, size_t* n_valid, uint64_t reject[IMLS_NUM_REJ]);

/* solveMotionEstimationProblem on host double triples; method = imls_solve_method.
 * rand_state (nullable, int32[34]) carries the glibc rand() state across calls (Q15). */
int oracle_solve(int32_t method, const double* s, const double* d, const double* n,
                 const double* weights, size_t N, const imls_params* p, int32_t* rand_state,
                 double delta_out[16], int* ok);

/* One frame of laser_odometry.cpp:478-660.  corr (nullable) receives, for iteration `corr_iter`,
 * the correspondences as float32 [n_valid][9] (x, y, n). corr_capacity = N. */
int oracle_register_frame(const float* src6, size_t N, const float* tgt6, size_t M,
                          const imls_params* p, double pose_out[16], int* iters_run, int* status,
                          imls_iter_trace* trace, int corr_iter, float* corr, size_t* corr_n,
                          double* seconds_index, double* seconds_total);

/* Tensor voting (VoteForAny, imls_icp.cpp:171-296): per query point, the voted normal ("tangents",
 * flipped to +z) and whether its tensor is non-zero.  ten6: the target's input tensors, SoA
 * float32[6][M] (xx, xy, xz, yy, yz, zz), input order.  tensors (nullable): the summed tensors,
 * row-major [Q][9].  libpointmatcher decompose semantics are UNPINNED (see imls_oracle.cpp). */
int oracle_tv_normals(const float* tgt6, size_t M, const float* ten6, const float* q3, size_t Q,
                      const imls_params* p, double* nrm, int32_t* found, double* tensors);
/* oracle_project / oracle_register_frame with the target's tensors (use_tensor_voting). */
int oracle_project_tv(const float* src6, size_t N, const float* tgt6, size_t M, const float* ten6,
                      const double pose[16], const imls_params* p, float* x_out, float* y_out,
                      float* n_out, uint32_t* src_index_out, size_t* n_valid,
                      uint64_t reject[IMLS_NUM_REJ]);
int oracle_register_frame_tv(const float* src6, size_t N, const float* tgt6, size_t M,
                             const float* ten6, const imls_params* p, double pose_out[16],
                             int* iters_run, int* status, imls_iter_trace* trace, int corr_iter,
                             float* corr, size_t* corr_n, double* seconds_index,
                             double* seconds_total);

/* oracle_register_frame_tv with the RANSAC rand() stream carried in `rand_state` (nullable,
 * int32[34]; null = a fresh stream from p->ransac_seed), as the reference's process-wide rand(). */
int oracle_register_frame_rs(const float* src6, size_t N, const float* tgt6, size_t M,
                             const float* ten6, const imls_params* p, int32_t* rand_state,
                             double pose_out[16], int* iters_run, int* status,
                             imls_iter_trace* trace, int corr_iter, float* corr, size_t* corr_n,
                             double* seconds_index, double* seconds_total);

/* nowPose = prevLaserPose * rPose (laser_odometry.cpp:652) and one savePoseToFile line
 * (saver.cpp:46-54, Eigen quaternion + fixed/6) into buf; returns its length. */
void oracle_chain_pose(const double prev[16], const double rel[16], double out[16]);
int oracle_format_pose(const double pose[16], const char* timestamp, char* buf, size_t cap);
size_t oracle_format_matched(const float* x3, const float* y3, size_t n, char* buf, size_t cap);

/* CPU-baseline modes (bench.py only): threads of the per-query projection loop, and the
 * "faithful" container costs of the reference (AoS copy per iteration, erase per rejected point,
 * per-query heap vectors; identical results). */
void oracle_set_threads(int n);
void oracle_set_faithful(int on);

/* glibc rand() restated (common.cpp:49 consumes it).  Fills 34-word state for srand(seed). */
void oracle_rand_seed(int32_t* state, uint32_t seed);
int32_t oracle_rand_next(int32_t* state);

/* Eigen-style solve pieces exposed for the known-answer tests. */
int oracle_colpiv_qr_solve(const double* A /* rows×cols row-major */, int rows, int cols,
                           const double* b, double* x);
void oracle_delta_from_x(const double x[6], double delta[16]);
int oracle_sym_eig6(const double* H /* 6x6 */, double* evals, double* evecs /* col-major cols */);

#ifdef __cplusplus
}
#endif
#endif
