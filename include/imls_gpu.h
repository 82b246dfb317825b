/*
 * imls_gpu.h — C ABI of the MI355X-native IMLS-ICP registration path.
 *
 * This is the drop-in boundary for the reference's per-scan Matching → Solving loop
 * (spirit-man/Planetary-LiDAR-Odometry, laser_odometry.cpp:478-660).  Every entry point
 * replaces one reference interface; the citation is on each declaration.  The library
 * (libimls_gpu.so) is hand-written HIP for gfx950; there is NO CPU fallback: every compute
 * entry point returns IMLS_ERR_DEVICE when no MI355X is present.
 *
 * Conventions
 *   - Plain C types only; no C++ exceptions cross the ABI.  Status: 0 = OK, < 0 = error class
 *     (imls_status).  imls_last_error(ctx) returns a human-readable message.
 *   - Point inputs are float32 with an arbitrary stride in floats, so both the reference's
 *     48-byte pcl::PointXYZINormal AoS (xyz at float 0, normal at float 4, stride 12) and
 *     packed SoA/AoS layouts are accepted without a host copy by the caller.
 *   - The caller keeps ownership of every host buffer; the library copies in.
 *   - One context per host thread: a context is NOT thread-safe (the reference matcher is
 *     single-threaded too, laser_odometry.cpp:708).  A context owns its device buffers, its
 *     HIP stream and its spatial index.
 *   - 4x4 poses are row-major doubles: T[r*4 + c].
 */
#ifndef IMLS_GPU_H
#define IMLS_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define IMLS_GPU_ABI_VERSION 1

typedef enum imls_status {
    IMLS_OK = 0,
    IMLS_ERR_ARG = -1,          /* bad argument (null pointer, size, stride) */
    IMLS_ERR_DEVICE = -2,       /* no MI355X / HIP runtime error */
    IMLS_ERR_STATE = -3,        /* call order (e.g. project before set_target) */
    IMLS_ERR_UNSUPPORTED = -4,  /* method or option not built on the GPU path */
    IMLS_ERR_CAPACITY = -5      /* exceeds a compiled-in capacity */
} imls_status;

/* laser_odometry.matching_method.method (config.json; laser_odometry.cpp:487, 557-568) */
typedef enum imls_match_method {
    IMLS_MATCH_IMLS = 0,        /* "IMLS"      → IMLSICPMatcher::ProjSourcePtToSurface */
    IMLS_MATCH_PLANE_ICP = 1    /* "plane_ICP" → plane_ICP_proj (laser_odometry.cpp:277-413) */
} imls_match_method;

/* laser_odometry.solve_method.method (config.json; laser_odometry.cpp:173-275) */
typedef enum imls_solve_method {
    IMLS_SOLVE_LS = 0,          /* "LS"     → SolveMotionEstimationProblemLS (solver.cpp:74-166) */
    IMLS_SOLVE_RANSAC = 1,      /* "RANSAC" → SolveMotionEstimationProblemRANSAC (solver.cpp:222-385) */
    IMLS_SOLVE_WEIGHTED_LS = 2, /* "Weighted LS" (solver.cpp:168-220); unit weights when used directly */
    IMLS_SOLVE_DRPM = 3         /* SolveMotionEstimationProblemDRPM (solver.cpp:499-603) on caller rows:
                                   imls_solve_correspondences only (RANSAC's final, not a loop method) */
} imls_solve_method;

/* solve_method.RANSAC.final_solve_method (config.json; solver.cpp:368-384) */
typedef enum imls_final_method {
    IMLS_FINAL_LS = 0,
    IMLS_FINAL_WEIGHTED_LS = 1,
    IMLS_FINAL_DRPM = 2
} imls_final_method;

/* Per-frame outcome of imls_register_frame (laser_odometry.cpp:570-646). */
typedef enum imls_frame_status {
    IMLS_FRAME_MAX_ITERS = 0,   /* ran all `iterations` without meeting the convergence test */
    IMLS_FRAME_CONVERGED = 1,   /* ‖Δt‖ < delta_dist_threshold && angle(Δ) < delta_angle_threshold */
    IMLS_FRAME_TOO_FEW = 2,     /* correspondences < correspond_number → break, pose kept */
    IMLS_FRAME_SOLVE_FAILED = 3 /* solver returned false → break, pose kept */
} imls_frame_status;

/* Reject counters, same categories and order as ProjSourcePtToSurface
 * (imls_icp.cpp:506-511, printed at 736-744). */
enum {
    IMLS_REJ_NO_NORMAL = 0,
    IMLS_REJ_TOO_FAR = 1,
    IMLS_REJ_INVALID_NORMAL = 2,
    IMLS_REJ_NORMAL_CONSTRAINT = 3,
    IMLS_REJ_MLS_FAIL = 4,
    IMLS_REJ_NAN_INF_HEIGHT = 5,
    IMLS_NUM_REJ = 6
};

/*
 * All parameters of the path.  Field names follow the config.json key paths of the
 * reference (laser_odometry.*), read at laser_odometry.cpp:487-518, 570, 606, 640-641 and
 * 183-243.  imls_default_params() fills the values of the reference's shipped config.json.
 */
typedef struct imls_params {
    /* laser_odometry.matching_method */
    int32_t matching_method;          /* imls_match_method */
    int32_t correspond_number;        /* matching_method.correspond_number (6) */

    /* laser_odometry.matching_method.IMLS  (IMLSICPMatcher members, imls_icp.h:114-146) */
    double h;                         /* IMLS.h: NN-1 rejection radius (imls_icp.cpp:620) */
    double r;                         /* IMLS.r: kNN search radius (imls_icp.cpp:607, 375) */
    int32_t get_normals;              /* IMLS.get_normals.enabled */
    int32_t search_number_normal;     /* IMLS.get_normals.search_number_normal */
    double r_normal;                  /* IMLS.get_normals.r_normal */
    int32_t use_projected_distance;   /* IMLS.use_projected_distance.enabled */
    int32_t normal_angle_constraint;  /* IMLS.normal_angle_constraint.enabled */
    double r_proj;                    /* IMLS.use_projected_distance.r_proj */
    double angle_diff_threshold;      /* IMLS.normal_angle_constraint.angle_diff_threshold (deg) */
    int32_t search_number;            /* IMLS."IMLS function".search_number (K, ≤ 32) */
    int32_t use_tensor_voting;        /* IMLS.use_tensor_voting.enabled (with get_normals=false:
                                         VoteForAny normals; needs imls_set_target_tensors) */
    int32_t tensor_k;                 /* IMLS.use_tensor_voting.k (≤ 64 on the GPU path) */
    int32_t recompute_normal_count_mode; /* SURVEY Q1 switch: 0 = reference (libnabo knn() return
                                            value is a statistic → recompute path rejects), 1 = count */
    double tensor_sigma;
    double tensor_distance_threshold;

    /* laser_odometry.matching_method.plane_ICP (laser_odometry.cpp:295-299) */
    double picp_r;
    double picp_r_proj;
    double picp_angle_diff_threshold;
    int32_t picp_use_projected_distance;
    int32_t picp_normal_angle_constraint;

    /* laser_odometry.solve_method */
    int32_t solve_method;             /* imls_solve_method */
    int32_t iterations;               /* solve_method.iterations (30) */
    double delta_dist_threshold;      /* solve_method.delta_dist_threshold (1e-3 m) */
    double delta_angle_threshold;     /* solve_method.delta_angle_threshold (rad) */
    double ls_threshold;              /* solve_method.LS.threshold (0.02) */

    /* laser_odometry.solve_method.RANSAC (solver.cpp:222-385) */
    int32_t ransac_max_iterations;
    int32_t ransac_final_method;      /* imls_final_method */
    double ransac_distance_threshold;
    double ransac_min_inliers_percentage;
    double ransac_huber_threshold;
    double ransac_ls_threshold;
    double drpm_threshold;
    double drpm_stdev_points;
    double drpm_stdev_normals;
    uint32_t ransac_seed;             /* glibc rand() seed of the context's stream; 1 = the reference's
                                         unseeded process.  Applied at imls_create and whenever
                                         imls_set_params changes it; the stream then runs on across
                                         every RANSAC solve and frame (see imls_seed_rng) */

    /* laser_odometry */
    int32_t transform_normal;         /* laser_odometry.transform_normal (laser_odometry.cpp:541-548) */
    int32_t max_queue_size;           /* laser_odometry.max_queue_size (map FIFO length) */
    int32_t _reserved[4];
} imls_params;

/* Per-iteration record of imls_register_frame (the reference writes the same quantities to
 * imls_iter_results.txt and stdout: laser_odometry.cpp:579, 625; imls_icp.cpp:736-744). */
typedef struct imls_iter_trace {
    double delta[16];                 /* Δ of this iteration */
    double pose[16];                  /* rPose after `rPose = Δ·rPose` (laser_odometry.cpp:619) */
    uint64_t reject[IMLS_NUM_REJ];
    uint64_t n_valid;                 /* correspondences ("USED POINTS FINAL") */
    uint64_t n_kept;                  /* rows kept by the trimmed LS (LS path only) */
} imls_iter_trace;

typedef struct imls_ctx imls_ctx;

/* ---- lifecycle ------------------------------------------------------------------------- */
int imls_abi_version(void);
void imls_default_params(imls_params* p);
/* Replaces `IMLSICPMatcher matcher;` + setParameters (laser_odometry.cpp:489, 514-518;
 * imls_icp.cpp:9-30, 146-168).  Returns NULL on failure (no device). */
imls_ctx* imls_create(int device, const imls_params* p);
void imls_destroy(imls_ctx* ctx);
/* Replaces IMLSICPMatcher::setParameters (imls_icp.h:62-66). */
int imls_set_params(imls_ctx* ctx, const imls_params* p);
const char* imls_last_error(const imls_ctx* ctx);
/* Run every launch of the context on `stream` (a hipStream_t); NULL restores the context's own.
 * A device buffer the context outgrows is not freed at once: it is retired behind an event recorded
 * on every stream the context has used, and freed (or reused) once those events have passed — no
 * device-wide synchronisation, so other contexts and other GPU users of the process keep running.
 * The stream must stay valid until the context is destroyed or set to another stream. */
int imls_set_stream(imls_ctx* ctx, void* hip_stream);
int imls_synchronize(imls_ctx* ctx);

/* glibc rand() stream of the RANSAC solver.  The reference draws its hypotheses from the one
 * process-wide rand() stream (common.cpp:49 via solver.cpp:245-262; srand is never called, so it
 * starts from seed 1 and runs on across every ICP iteration and every frame).  A context keeps its
 * own device-resident copy of that stream and continues it across imls_solve,
 * imls_solve_correspondences and imls_register_frame exactly as the reference's sequential calls
 * consume it.  imls_seed_rng restarts it (= srand(seed)); imls_get_rng_state / imls_set_rng_state
 * (the glibc TYPE_3 state: 31 words, front index, rear index, 0) hand one stream from a context to
 * another, e.g. when a caller creates a fresh context per frame as the reference creates a fresh
 * matcher (laser_odometry.cpp:489).  Contexts used concurrently each run their own stream;
 * imls_register_batch restarts a context's stream from params.ransac_seed before every pair, so its
 * pairs are independent of the `streams` count and of the order they are given in.  imls_seed_rng
 * leaves params.ransac_seed unchanged (contexts seeded differently still batch together). */
int imls_seed_rng(imls_ctx* ctx, uint32_t seed);
int imls_get_rng_state(imls_ctx* ctx, int32_t state[34]);
int imls_set_rng_state(imls_ctx* ctx, const int32_t state[34]);

/* ---- clouds ---------------------------------------------------------------------------- */
/* Replaces IMLSICPMatcher::setTargetPointCloud (imls_icp.cpp:80-103): drops points with
 * non-finite xyz (RemoveNANandINFData, imls_icp.cpp:58-72), keeps order, builds the index.
 * xyz/nrm: host float pointers, element i at xyz + i*stride_floats (nrm likewise).
 * n_kept (nullable) receives the number of points after the NaN filter. */
int imls_set_target(imls_ctx* ctx, const float* xyz, const float* nrm, size_t n,
                    size_t stride_floats, size_t* n_kept);
/* Replaces IMLSICPMatcher::setSourcePointCloud (imls_icp.cpp:74-78). kept_index (nullable,
 * capacity n) receives the input index of every kept point, in order. */
int imls_set_source(imls_ctx* ctx, const float* xyz, const float* nrm, size_t n,
                    size_t stride_floats, size_t* n_kept, uint32_t* kept_index);
/* Same, for clouds already resident in device memory as SoA float32[6][n]
 * (x[], y[], z[], nx[], ny[], nz[]) — inputs stay in HBM, no PCIe in the hot loop.
 * Count-less mode (n_kept NULL, and no kept_index): the call returns at once; the index build runs
 * at the first use of the cloud (a registration, a projection, or all the frames of an
 * imls_register_frames batch together, in one launch sequence).  When d_soa6 is read depends only on
 * imls_set_defer: off (the default) — the NaN filter reads it on the context's stream right after
 * the call (the buffer may be rewritten by work ordered after the context's stream has passed the
 * call, e.g. after imls_synchronize or the next registration's result); on — the filter reads it at
 * the first use, so it must stay valid and unchanged until that first use has run (e.g. the
 * registration's result is collected).  Once filtered, the context works on its own copy.
 * Host-pointer calls copy their input at the call, so their buffers are free on return. */
int imls_set_target_device(imls_ctx* ctx, const float* d_soa6, size_t n, size_t* n_kept);
int imls_set_source_device(imls_ctx* ctx, const float* d_soa6, size_t n, size_t* n_kept);
/* Deferred reads of count-less device loads (see above): with it on, the NaN filters of the frames
 * of one imls_register_frames batch run together in three launches (a caller that loads hundreds of
 * small frames per batch).  Default off.  Applies to imls_set_target_device, imls_set_source_device
 * and imls_map_push_device (and to the owned upload buffers of the host-pointer forms). */
int imls_set_defer(imls_ctx* ctx, int on);

/* Map FIFO kept in HBM: replaces accumulateTargetCloud(newCloud, max_queue_size, ...)
 * (laser_odometry.cpp:116-136, called at 663-664) followed by the next frame's
 * setTargetPointCloud(accumulatedTargetCloud) (509-510; imls_icp.cpp:80-103).  The new filtered
 * scan (untransformed, as the reference keeps it) becomes the FIFO's newest entry; when the FIFO
 * then holds more than params.max_queue_size entries the oldest is dropped (once, like the
 * reference's `if`); the entries are concatenated oldest first on the device and the target index
 * is rebuilt over the concatenation (NaN filter included).  Only the new scan crosses PCIe: the
 * older ones stay resident.  n_map (nullable) receives the map size after the NaN filter.
 * imls_set_target replaces the index without touching the FIFO. */
int imls_map_push(imls_ctx* ctx, const float* xyz, const float* nrm, size_t n, size_t stride_floats,
                  size_t* n_map);
/* Device-resident scan (SoA6 floats in HBM).  With max_queue_size 1 the map is this scan alone and
 * is indexed in place (no FIFO copy): the buffer must then stay valid until the map's first use
 * (count-less with imls_set_defer on) or until the context's stream has passed the push; raising
 * max_queue_size afterwards needs a fresh push.  Larger FIFOs copy the scan into a FIFO slot. */
int imls_map_push_device(imls_ctx* ctx, const float* d_soa6, size_t n, size_t* n_map);
int imls_map_clear(imls_ctx* ctx);
/* FIFO entries and their total point count (before the NaN filter). */
int imls_map_size(imls_ctx* ctx, size_t* entries, size_t* points);

/* Tensor voting input (use_tensor_voting): the target's per-point input tensors T — what
 * VoteForAny's tv_input.encode(m_targetPointCloudDP, AWARE_TENSOR) produces (imls_icp.cpp:179,
 * 535; the DP cloud of setTargetPointCloudDP, 105-144).  n records of 6 floats (xx, xy, xz, yy,
 * yz, zz) at `stride_floats`, in the order of the last imls_set_target's points (n must equal
 * that call's n; records of points its NaN filter dropped are ignored).  Invalidated by the next
 * imls_set_target.  The _device form takes SoA float32[6][n] in device memory; after a count-less
 * (deferred) set_target it is read when the target is built (its first use), so it must stay valid
 * until then. */
int imls_set_target_tensors(imls_ctx* ctx, const float* tensors, size_t n, size_t stride_floats);
int imls_set_target_tensors_device(imls_ctx* ctx, const float* d_ten6, size_t n);
/* The reference's own tensor encoding of per-point PCA features (CustomTensorVoting::
 * myCustomFunctionWithEigen, scan_registration.cpp:358-381), host float arithmetic:
 * λ = |evals|, λ1 = max, λ3 = min, λ2 = Σλ − (λ1 + λ3); T = ((λ1−λ2)/k)·e1e1ᵀ +
 * (λ3/k)·(e1e1ᵀ + e2e2ᵀ), or I when not λ1 ≥ λ2 ≥ λ3.  evals: [n][3] (λ1, λ2, λ3 as
 * scan_registration.cpp:1204 stores them); evecs: [n][9], the 3×3 eigenvector matrix column-major
 * (1205-1207: e1 = largest, e2, e3 = normal); out: [n][6] as imls_set_target_tensors reads. */
void imls_tv_encode_pca(const float* evals, const float* evecs, size_t n, int32_t k, float* out);

/* ---- matching -------------------------------------------------------------------------- */
/* Replaces IMLSICPMatcher::ProjSourcePtToSurface (imls_icp.cpp:496-745) applied to the source
 * transformed by `pose` (laser_odometry.cpp:527-549).  Outputs (each nullable, capacity =
 * n_kept source points, float32 xyz triples) are compacted in SOURCE ORDER like the
 * reference's erase-based loop: x_out = transformed source point (in_cloud after the call),
 * y_out = its projection on the implicit surface, n_out = the NN-1 map normal (out_cloud);
 * src_index_out = index into the kept source cloud.  reject[6] in imls_icp.cpp:506-511 order. */
int imls_project(imls_ctx* ctx, const double pose[16], float* x_out, float* y_out, float* n_out,
                 uint32_t* src_index_out, size_t* n_valid, uint64_t reject[IMLS_NUM_REJ]);

/* ---- solving --------------------------------------------------------------------------- */
/* Replaces solveMotionEstimationProblem(solve_method, ...) (laser_odometry.cpp:173-275) on the
 * device-resident correspondences of the last imls_project.  *ok mirrors the bool return. */
int imls_solve(imls_ctx* ctx, double delta_out[16], int* ok);
/* Replaces SolveMotionEstimationProblemLS / WeightedLS / RANSAC / DRPM (solver.cpp:74-385,
 * 499-603) on host arrays of N double triples (s = source, d = target, n = target normal; weights
 * nullable = unit; LS uses params.ls_threshold, RANSAC the ransac_* fields and the context's rand()
 * stream, DRPM drpm_threshold / drpm_stdev_points / drpm_stdev_normals). */
int imls_solve_correspondences(imls_ctx* ctx, int32_t method, const double* s, const double* d,
                               const double* n, const double* weights, size_t N,
                               double delta_out[16], int* ok);

/* ---- fused registration ---------------------------------------------------------------- */
/* The device-resident equivalent of laser_odometry.cpp:478-660 for one frame: rPose = I, then
 * up to `iterations` × {transform, match, gate, solve, rPose = Δ·rPose, convergence test}, one
 * host synchronisation at the end.  trace (nullable) receives `iterations` records; only the
 * first *iters_run are meaningful. */
int imls_register_frame(imls_ctx* ctx, double pose_out[16], int* iters_run, int* status,
                        imls_iter_trace* trace);
/* Asynchronous form: enqueue on the context stream and return; collect with
 * imls_register_frame_result (which synchronises the stream). */
int imls_register_frame_async(imls_ctx* ctx);
int imls_register_frame_result(imls_ctx* ctx, double pose_out[16], int* iters_run, int* status,
                               imls_iter_trace* trace);
/* Per-iteration correspondences of imls_register_frame, for the reference's per-iteration outputs
 * (saveMatchedPointsToFile of in_cloud_vec / ref_cloud_vec into matched_points/<ts>_<i>.txt,
 * laser_odometry.cpp:621-623; saver.cpp:113-133).  While on, each iteration's correspondences are
 * kept on the device (48 B per source point per iteration); after the frame's result,
 * imls_captured_correspondences(iter) returns iteration `iter` (< iters_run of that frame) compacted in
 * source order exactly as imls_project does.  `cap` is the capacity of the caller's arrays in rows
 * (x/y/n: 3·cap floats, index: cap); *n_valid always receives the row count, and with every output
 * pointer NULL the call is a size query.  More rows than `cap` → IMLS_ERR_ARG, nothing written.
 * The capture stays readable across set_target / map_push (LaserOdometry writes the files after the
 * map has taken the new scan); a later set_source or a batched registration drops it
 * (IMLS_ERR_STATE until the next captured imls_register_frame). */
int imls_capture_correspondences(imls_ctx* ctx, int on);
int imls_captured_correspondences(imls_ctx* ctx, int iter, size_t cap, float* x_out, float* y_out, float* n_out,
                                  uint32_t* src_index_out, size_t* n_valid);

/* ---- many frames in one launch sequence (configs C/D: many sequences per GPU) ------------ */
/* Registers the frames already loaded into ctxs[0..n) (each by imls_set_target / imls_map_push +
 * imls_set_source, exactly as before imls_register_frame) in ONE launch sequence: every
 * per-iteration kernel is launched once for all n frames (grid y = frame), each frame at its own
 * pose, convergence flag and iteration count, so n small frames (the ≤ 2000-point flat clouds of a
 * KITTI stream) fill the GPU together.  Each frame's result, trace and iteration count are
 * bit-identical to imls_register_frame on its context (laser_odometry.cpp:478-660 per frame:
 * frames are independent, 484-485).  All contexts must be on one device with equal params; the
 * launches run on ctxs[0]'s stream after every context's pending uploads, and every context's later
 * work is ordered after them.  RANSAC / DRPM, tensor voting, the projected-distance rule and the
 * exact per-lane mode run one launch sequence per frame instead (same results, less overlap).
 * poses_out[16·k], iters_out[k], status_out[k], traces[k·iterations …] (each nullable) receive
 * frame k's result.  The _async form returns after enqueueing; imls_register_frames_result(ctxs[0],
 * …) synchronises and fills the outputs. */
int imls_register_frames(imls_ctx* const* ctxs, size_t n, double* poses_out, int32_t* iters_out,
                         int32_t* status_out, imls_iter_trace* traces);
int imls_register_frames_async(imls_ctx* const* ctxs, size_t n);
int imls_register_frames_result(imls_ctx* lead, double* poses_out, int32_t* iters_out,
                                int32_t* status_out, imls_iter_trace* traces);

/* ---- many independent pairs (configs C/D: a KITTI stream, many sequences per GPU) -------- */
/* Every frame's registration starts from rPose = I against the raw previous scan(s)
 * (laser_odometry.cpp:484-485, 116-136), so frames are independent: a batch keeps `streams`
 * contexts (1..256, one HIP stream each); pairs are taken in groups of that many, each group
 * uploaded and indexed (one context per pair) and then registered as ONE launch sequence
 * (imls_register_frames).  One batch per host thread. */
typedef struct imls_batch imls_batch;
typedef struct imls_pair_input {
    const float* src_xyz;             /* the flat (source) cloud, as imls_set_source */
    const float* src_nrm;
    size_t n_src;
    const float* tgt_xyz;             /* the accumulated map, as imls_set_target */
    const float* tgt_nrm;
    size_t n_tgt;
    size_t stride_floats;             /* stride of all four arrays */
} imls_pair_input;
imls_batch* imls_batch_create(int device, const imls_params* p, int32_t streams);
void imls_batch_destroy(imls_batch* b);
const char* imls_batch_last_error(const imls_batch* b);
/* Registers pairs[0..n_pairs) (each exactly as imls_set_target + imls_set_source +
 * imls_register_frame would on a context freshly seeded with params.ransac_seed); poses_out[16·i] (row-major), iters_out[i] and status_out[i]
 * (imls_frame_status; each nullable) receive pair i's result.  Returns the first error (the
 * message names the pair); the pairs in flight are drained before returning. */
int imls_register_batch(imls_batch* b, size_t n_pairs, const imls_pair_input* pairs, double* poses_out,
                        int32_t* iters_out, int32_t* status_out);

/* ---- upstream producer: front end (scan_registration.cpp:laserCloudHandler 809-1069) ---- */
/* Node parameters (scan_registration.cpp:1575-1581; the shipped launch file
 * planetary_slam_VLP_32.launch sets scan_line 64, minimum_range 2, maximum_range 150). */
typedef struct imls_front_params {
    int32_t n_scans;                /* scan_line: 16, 32 or 64 */
    float minimum_range;            /* removeClosedPointCloud thresholds (m) */
    float maximum_range;
    float scan_period;              /* scanPeriod = 0.1 (55) */
    int32_t is_dense;               /* the message's is_dense: pcl::removeNaNFromPointCloud copies a dense
                                       cloud unchanged (NaN points then meet the range test) */
} imls_front_params;
void imls_default_front_params(imls_front_params* p);    /* the launch file's values, is_dense 0 */
/* The raw sweep (pcl::PointXYZ records of the /velodyne_points message, in the driver's order:
 * x, y, z at xyz + i·stride_floats) → laserCloud: the NaN filter (862), the range filter
 * removeClosedPointCloud (87-115, 863), the ring assignment and relative time (898-1058), the
 * rings concatenated in ring order, each in input order (1064-1069).  out_xyzi: [n][4] = x, y, z,
 * intensity (= ring + scanPeriod·relTime, 1048); out_index (nullable): the input index of each
 * output point; ring_sizes: [n_scans] points per ring (the ring_sizes imls_ring_normals_pca takes;
 * scanStartInd / scanEndInd = prefix + 5 / prefix + size − 6, 1066-1068); *n_out = Σ ring sizes.
 * Capacity of the outputs: n points.  A sweep with no surviving point gives n_out = 0 (the
 * reference would index an empty cloud). */
int imls_scan_front_end(imls_ctx* ctx, const imls_front_params* p, const float* xyz, size_t stride_floats,
                        size_t n, float* out_xyzi, uint32_t* out_index, int32_t* ring_sizes, size_t* n_out);

/* ---- upstream producer: ring-neighbourhood PCA normals (scan_registration) ------------- */
/* scan_registration.compute_normal_method.pca + presample_method.geometric_features
 * (config.json; read at scan_registration.cpp:1140-1145, 1451, 1133).  imls_default_pca_params()
 * fills the shipped values. */
typedef struct imls_pca_params {
    int32_t window_size;            /* pca.window_size = 3 */
    int32_t iter_step;              /* pca.iter_step = 1 */
    float knn_distance_threshold;   /* pca.knn_distance_threshold = 10 (vs the SQUARED NN distance,
                                       which is what pcl::KdTreeFLANN::nearestKSearch returns) */
    int32_t neighbor_scan;          /* pca.neighbor_scan: 0 = "kdtree", 1 = "index" */
    float distance_threshold;       /* pca.plane_constraint.distance_threshold = 0.02 */
    float valid_points_threshold;   /* pca.plane_constraint.valid_points_threshold = 0.8 */
    int32_t use_all_points;         /* model.use_all_points = true */
    float planarity_threshold;      /* presample_method.geometric_features.planarity_threshold = 0.05 */
} imls_pca_params;
void imls_default_pca_params(imls_pca_params* p);

/* Output flags of imls_ring_normals_pca. */
enum {
    IMLS_PCA_PLANE_INVALID = 1,     /* failed checkPlaneValidity: eigenvalues (-1,-1,-1), normal = the
                                       largest-eigenvalue axis (scan_registration.cpp:215-218, 1182-1196) */
    IMLS_PCA_CANDIDATE = 2          /* presample candidate: planarity > threshold and not invalid
                                       (computeGeometricFeatures 321-326; erase 1481-1489) */
};

/* Replaces the point-cloud / "pca" branch of scan_registration.cpp's normal estimation
 * (1136-1229: computeNormalPCA 158-229 with findNearestPoint 117-136 and checkPlaneValidity
 * 138-156) followed by the geometric-features presample (computeGeometricFeatures 279-327, the
 * invalid-index erase 1481-1489).
 *   xyz: the ring-concatenated cloud `laserCloud` (1064-1069), point i at xyz + i*stride_floats;
 *   ring_sizes[n_rings]: points per scan line, in ring order (laserCloudScans[i].size()).
 * Outputs (capacity = the number of input points; each nullable) are the rows of
 * filteredLaserCloud / eigenvalues_matrix / eigenvectors_matrix in the reference's push order:
 *   index_out[r]  = filteredIndices (= scanStartInd[i] + j, which is 5 past the PCA centre j:
 *                   the reference's own offset, SURVEY Appendix B "Q-SR1"; the point's xyz,
 *                   intensity and curvature come from that index, 1210-1220);
 *   normal_out[3r] (flipped to +z), evals_out[3r] = (λ1, λ2, λ3) descending or (-1,-1,-1),
 *   evecs_out[9r] = the 3×3 eigenvector matrix column-major as 1205-1207 stores it,
 *   features_out[8r] = sum, omnivariance, eigenentropy, anisotropy, linearity, planarity,
 *                   surface variation, sphericity (279-319), flags_out[r] (IMLS_PCA_*).
 * counters[2] (nullable): pca_failure (1179), plane-check failures (1186; counted whether or
 * not use_all_points keeps them).  Requires n_rings ≤ 4096 and ring sizes ≤ 1<<20. */
int imls_ring_normals_pca(imls_ctx* ctx, const imls_pca_params* p, const float* xyz, size_t stride_floats,
                          const int32_t* ring_sizes, int32_t n_rings, uint32_t* index_out, float* normal_out,
                          float* evals_out, float* evecs_out, float* features_out, uint8_t* flags_out,
                          size_t* n_out, uint64_t counters[2]);

/* scan_registration.sample_method (config.json; samplePointCloud, scan_registration.cpp:761-806).
 * imls_default_sample_params() fills the shipped values of the chosen method. */
typedef enum imls_sample_method {
    IMLS_SAMPLE_NORMAL = 0,         /* "normal" — and "major_axis" on the first frame (783) */
    IMLS_SAMPLE_MAJOR_AXIS = 1      /* "major_axis" from the second frame on (791-801) */
} imls_sample_method;
typedef struct imls_sample_params {
    int32_t method;                 /* imls_sample_method */
    float r, r_proj;                /* major_axis.r = 0.5, major_axis.r_proj = 1.5 */
    int32_t max_total_points;       /* major_axis.max_total_points = 2000 */
    int32_t azimuth_bins, elevation_bins;            /* 8, 8 */
    int32_t min_points_per_bin, max_points_per_bin;  /* normal: 20, 100; major_axis: 20, 200 */
    int32_t sampling_strategy;      /* 0 = "FPS", 1 = "random" (normal: random; major_axis: FPS) */
    uint32_t shuffle_seed;          /* randomSampling's std::mt19937 seed: call k of one imls_sample_
                                       point_cloud uses shuffle_seed + k (the reference seeds each call
                                       from std::random_device, 571-572: not reproducible) */
    uint32_t rand_seed;             /* srand() seed of the glibc rand() stream farthestPointSampling
                                       draws its first index from (common.cpp:49); re-seeded per call
                                       (the reference's stream runs on across frames from seed 1) */
} imls_sample_params;
void imls_default_sample_params(imls_sample_params* p, int32_t method);

/* Replaces samplePointCloud for "normal" / "major_axis" (scan_registration.cpp:761-806):
 * computeSphericalHistogram (536-564) of the candidates' normals, then normalSampling (584-629) or
 * majorAxisSampling (631-759) — per-bin random subsets, the brute-force average distance to the
 * previous frame's cloud (679-701, on the GPU), bin weights, per-bin farthestPointSampling
 * (common.cpp:19-82, on the GPU) or random sampling.
 *   xyz/nrm: pcl_cloud (the filtered cloud), point i at xyz + i*stride_floats (nrm likewise);
 *   candidates[n_cand]: candidate_indices into it; last_xyz[m]: last_pcl_cloud (major_axis only).
 * sampled_out (capacity n_cand + azimuth_bins·elevation_bins) receives sampled_indices in the
 * reference's order; bin_weights_out (nullable, azimuth_bins·elevation_bins floats) the normalised
 * major_axis weights. */
int imls_sample_point_cloud(imls_ctx* ctx, const imls_sample_params* p, const float* xyz, const float* nrm,
                            size_t stride_floats, size_t n, const int32_t* candidates, size_t n_cand,
                            const float* last_xyz, size_t last_stride_floats, size_t m, int32_t* sampled_out,
                            size_t* n_sampled, float* bin_weights_out);

/* ---- runtime options ------------------------------------------------------------------- */
/* No reference equivalent: the documented tuning parameters and test hooks of the GPU path, per
 * context (the library reads no environment variable except IMLS_DEBUG_HOST, a host-side trace).
 * The defaults are the measured best; every value gives the same correspondences
 * and poses (the tests run each against the default).  Contexts registered together
 * (imls_register_frames) must share their options.  Returns IMLS_ERR_ARG for an unknown option or
 * an invalid value (the option is then unchanged). */
typedef enum imls_option {
    IMLS_OPT_TRAVERSAL = 0,            /* imls_traversal (default IMLS_TRAVERSAL_AUTO) */
    IMLS_OPT_LIST_REUSE = 1,           /* 1 (default): a query's neighbour list is reused without a
                                          traversal while its certificate holds (Verlet lists); 0 off */
    IMLS_OPT_TEMPORAL_SEED = 2,        /* 1 (default): iterations > 0 prefill the lists from the
                                          previous iteration's; 0: every iteration seeds afresh */
    IMLS_OPT_LEAF_SIZE = 3,            /* points per index leaf, a power of two in [4, 64] (default
                                          64); applies from the next index build */
    IMLS_OPT_FIRST_PACKET = 4,         /* queries per wave in the first ICP iteration(s) of a frame
                                          registered alone: 16, 32 (default) or 64 */
    IMLS_OPT_FIRST_PACKET_ITERS = 5,   /* ... for this many iterations (default 1) */
    IMLS_OPT_FIRST_PACKET_BATCHED = 6, /* ... in batched registrations too: 0 (default) or 1 */
    IMLS_OPT_TV_SKIN = 7,              /* tensor voting: a query's ball list is reused while it moved
                                          <= skin metres (default 0.03; 0 = walk every iteration) */
    IMLS_OPT_FORCE_FALLBACK = 8        /* test hook: every n-th query's list is treated as uncertified
                                          (resolved by the exact search); 0 off (default) */
} imls_option;
typedef enum imls_traversal {
    IMLS_TRAVERSAL_AUTO = 0,           /* one wave per query up to 16384 queries, packets above */
    IMLS_TRAVERSAL_PACKETS = 1,        /* packets of 64 Morton-coherent queries per wave */
    IMLS_TRAVERSAL_WAVE_PER_QUERY = 2, /* one wave per query */
    IMLS_TRAVERSAL_LANE = 3            /* reference mode: every query by the exact per-lane search */
} imls_traversal;
int imls_set_option(imls_ctx* ctx, int32_t option, double value);
int imls_get_option(imls_ctx* ctx, int32_t option, double* value);

/* ---- instrumentation ------------------------------------------------------------------- */
/* When enabled, HIP events bracket every launch of the projection kernel (on the stream it is
 * launched on); imls_kernel_timing returns the accumulated milliseconds and launch count since
 * the last reset.  kernel: 0 = projection (all its kernels), 1 = index build (all its kernels),
 * 2 = solve chain, 3 = k_knn_wave (packet traversal) alone, 4 = k_finish (exact stage) alone,
 * 5 = k_ring_pca (imls_ring_normals_pca), 6 = k_major_avg (imls_sample_point_cloud, major_axis),
 * 7 = imls_scan_front_end (all its kernels).  enable: 0 off, 1 every kind above (the members of
 * an imls_register_frames batch then build their indices one by one, each inside its events),
 * 2 light — only the projection (0) and solve-chain (2) events of the iterations, the launch
 * sequence otherwise unchanged (for timing a concurrent workload). */
int imls_enable_timing(imls_ctx* ctx, int enable);
/* Records a process-wide origin event on ctx's stream (and waits for it).  Afterwards every
 * harvested timing pair of every context on that device is also kept as an interval (start, end)
 * in ms since the origin: imls_timing_intervals copies up to `cap` of them (out[2k], out[2k+1]) and
 * returns their count in *n — the union over contexts is the busy time of concurrent work. */
int imls_timing_origin(imls_ctx* ctx);
int imls_timing_intervals(imls_ctx* ctx, int kernel, double* out, size_t cap, size_t* n);
/* Traversal / neighbour counters (imls_traversal_stats, and the sum_kq / nn_found fields of
 * imls_index_stats) are collected only while enabled (default off: they are device-scope atomics
 * onto a few shared words from every wave, ~60 µs per projection at config B). */
int imls_enable_stats(imls_ctx* ctx, int enable);
int imls_kernel_timing(imls_ctx* ctx, int kernel, double* total_ms, uint64_t* launches);
int imls_reset_timing(imls_ctx* ctx);
/* Sizes of the last built index (for roofline accounting): points, leaves, tree levels,
 * total neighbours visited in the last projection (Σ k_q), queries passing the NN/angle gates. */
int imls_index_stats(imls_ctx* ctx, uint64_t out[8]);
/* Counters accumulated since the last frame start / projection (diagnostics): Σ k_q, NN-1 found,
 * leaves visited (per wave), inner nodes visited (per wave), waves, uncertified queries re-run
 * exactly, lanes whose list was reused without a traversal (Verlet reuse), 0. */
int imls_traversal_stats(imls_ctx* ctx, uint64_t out[8]);

#ifdef __cplusplus
}
#endif
#endif /* IMLS_GPU_H */
