// api.hip — the C ABI of include/imls_gpu.h: context, uploads, and the fused per-frame loop.
//
// imls_register_frame is the device-resident form of laser_odometry.cpp:478-660: all
// `iterations` × {k_project, solve chain} launches are enqueued back to back on the context
// stream; convergence / too-few-correspondence exits are taken on the device (a `done` flag
// every later launch checks first), so the host synchronises once per frame.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <string>
#include <condition_variable>
#include <functional>
#include <thread>
#include <mutex>
#include <vector>
#include <unistd.h>

#include "internal.h"

// host → device copies of uploads on a per-context upload stream (upload_soa6); 0: on the context's
// stream, behind its running registrations (the round-4 behaviour, kept for same-box A/B builds)
#ifndef IMLS_UPLOAD_STREAM
#define IMLS_UPLOAD_STREAM 1
#endif

using namespace imlsgpu;

// ---- device buffers: retire instead of free (internal.h devbuf_grow) ------------------------------
namespace imlsgpu {
namespace {
struct Retired {
    void* p;
    size_t bytes;
    int device;
    std::vector<hipEvent_t> ev;       // one per stream that still had work when it was retired
};
std::mutex g_mem_mu;
struct StreamRef {
    hipStream_t s;
    int device, refs;
};
std::vector<StreamRef> g_streams;
std::vector<Retired> g_retired;

bool retired_ready(Retired& r) {
    for (size_t k = 0; k < r.ev.size(); ++k)
        if (hipEventQuery(r.ev[k]) != hipSuccess) return false;
    for (hipEvent_t e : r.ev) (void)hipEventDestroy(e);
    r.ev.clear();
    return true;
}
}  // namespace

void register_stream(hipStream_t s, int device) {
    if (!s) return;
    std::lock_guard<std::mutex> lk(g_mem_mu);
    for (auto& r : g_streams)
        if (r.s == s) { ++r.refs; return; }
    g_streams.push_back({s, device, 1});
}

void unregister_stream(hipStream_t s) {
    if (!s) return;
    std::lock_guard<std::mutex> lk(g_mem_mu);
    for (size_t k = 0; k < g_streams.size(); ++k)
        if (g_streams[k].s == s && --g_streams[k].refs == 0) {
            g_streams.erase(g_streams.begin() + (long)k);
            return;
        }
}

void devbuf_retire(DevBuf& b) {
    if (!b.p) return;
    int dev = 0;
    (void)hipGetDevice(&dev);
    std::lock_guard<std::mutex> lk(g_mem_mu);
    Retired r{b.p, b.bytes, dev, {}};
    for (const auto& sr : g_streams) {
        if (sr.device != dev || hipStreamQuery(sr.s) == hipSuccess) continue;   // idle: all its work has run
        hipEvent_t e = nullptr;
        if (hipEventCreateWithFlags(&e, hipEventDisableTiming) == hipSuccess && hipEventRecord(e, sr.s) == hipSuccess) {
            r.ev.push_back(e);
        } else {
            // no event to wait for (never expected): wait for that stream here instead
            if (e) (void)hipEventDestroy(e);
            (void)hipStreamSynchronize(sr.s);
        }
    }
    g_retired.push_back(std::move(r));
    b.p = nullptr;
    b.bytes = 0;
}

bool devbuf_grow(DevBuf& b, size_t bytes, size_t alloc) {
    if (b.bytes >= bytes) return true;
    devbuf_retire(b);
    alloc = std::max(alloc, bytes);
    int dev = 0;
    (void)hipGetDevice(&dev);
    {
        // a retired buffer whose readers have all finished: the smallest that fits, at most 4× the size
        std::lock_guard<std::mutex> lk(g_mem_mu);
        long best = -1;
        for (size_t k = 0; k < g_retired.size(); ++k) {
            Retired& r = g_retired[k];
            if (r.device != dev || r.bytes < alloc || r.bytes > 4 * alloc) continue;
            if (best >= 0 && r.bytes >= g_retired[(size_t)best].bytes) continue;
            if (retired_ready(r)) best = (long)k;
        }
        if (best >= 0) {
            b.p = g_retired[(size_t)best].p;
            b.bytes = g_retired[(size_t)best].bytes;
            g_retired.erase(g_retired.begin() + best);
            return true;
        }
    }
    if (hipMalloc(&b.p, alloc) != hipSuccess) {
        b.p = nullptr;
        return false;
    }
    b.bytes = alloc;
    return true;
}

void release_retired(int device) {
    std::lock_guard<std::mutex> lk(g_mem_mu);
    std::vector<Retired> keep;
    for (auto& r : g_retired) {
        if (r.device != device) { keep.push_back(std::move(r)); continue; }
        for (hipEvent_t e : r.ev) (void)hipEventDestroy(e);
        (void)hipFree(r.p);                                // teardown: hipFree waits for the device
    }
    g_retired.swap(keep);
}
}  // namespace imlsgpu

constexpr int kTimingKinds = 8;   // projection, index, solve chain, k_knn_wave, k_finish, k_ring_pca, k_major_avg, front end

// Runtime options of a context (imls_set_option; include/imls_gpu.h documents each): the validated
// tuning parameters and test hooks.  Nothing is read from the environment.
struct Options {
    int traversal = IMLS_TRAVERSAL_AUTO;
    int list_reuse = 1;
    int temporal_seed = 1;
    int leaf_size = 64;
    int first_packet = 32;
    int first_packet_iters = 1;
    int first_packet_batched = 0;
    double tv_skin = 0.03;
    int force_fallback = 0;
};

inline bool same_options(const Options& a, const Options& b) {
    return a.traversal == b.traversal && a.list_reuse == b.list_reuse && a.temporal_seed == b.temporal_seed &&
           a.leaf_size == b.leaf_size && a.first_packet == b.first_packet && a.first_packet_iters == b.first_packet_iters &&
           a.first_packet_batched == b.first_packet_batched && a.tv_skin == b.tv_skin && a.force_fallback == b.force_fallback;
}

struct imls_ctx {
    int device = 0;
    hipStream_t own = nullptr, stream = nullptr;
    imls_params P{};
    KParams kp{};
    std::string err;
    int B = 64;
    // target
    DevBuf tpt, tnr, mpt, nodes, tscratch, treescratch, permbuf, upload_t;
    int M = 0, Pl = 0, levels = 0;
    bool has_target = false;
    // source
    DevBuf spt, snr, sscratch, qperm, upload_s, skept;
    // map FIFO (accumulateTargetCloud, laser_odometry.cpp:116-136): the last max_queue_size filtered
    // scans, each SoA6 in its own slot, and their concatenation (oldest first) the index is built from
    // a FIFO entry: its raw SoA6 scan (the concatenation path), and for the incremental index its
    // filtered points (fpt / fnr, NaN filter at the push) and its sorted run (index.hip)
    struct MapSlot {
        DevBuf buf, fpt, fnr, run;
        size_t n = 0;
        bool ghost = false;
        int id = -1;                      // run id (incremental index)
        int nk = -1;                      // kept count after the NaN filter (−1: not read yet)
        bool sorted = false;              // run built under the current quantisation frame
    };
    std::deque<MapSlot> fifo;
    std::vector<MapSlot> slot_pool;       // freed slots, their buffers reused (no allocation per frame)
    // incremental FIFO index (max_queue_size 2..kMaxFifoRuns−1): each scan sorted once at its first
    // build under a quantisation frame fixed for the FIFO, the previous merged order kept across
    // registrations (finish_target → fifo_build)
    bool fifo_inc = false;                // the current / pending target is the FIFO's incremental index
    unsigned fifo_seq = 0;                // run ids: pushes mod kMaxFifoRuns
    int* h_fifo_cnt = nullptr;            // pinned [kMaxFifoRuns]: kept count of each run's filter
    unsigned* h_fifo_clamp = nullptr;     // pinned: points outside the frame at the last build
    DevBuf fifo_dev;                      // fq[4] | clamp counter
    bool fq_valid = false;
    std::vector<int> merged_ids;          // runs in the merged order, oldest first
    DevBuf mkey[2], mval[2];
    int mcur = 0, m_n = 0;
    DevBuf fscr;                          // FIFO build scratch
    hipEvent_t ev_fifo = nullptr;         // after the last incremental build (batch joins)
    DevBuf macc;
    size_t map_points = 0;                // Σ n over the FIFO (before the NaN filter)
    DevBuf fb;                            // deferred-query counts per k_finish block + their lists
    size_t fb_off = 64;                   // words: start of the lists in fb
    DevBuf lkeys;                         // leaf first Morton keys + quantisation (seed search)
    DevBuf rnr;                           // recomputed map normals (count mode), Morton order
    bool rnr_valid = false;
    int rnr_k = -1;
    double rnr_r = -1.0;
    DevBuf prevnn;                        // per-query neighbour lists carried between ICP iterations
    DevBuf tkept;                         // target: filtered index → input index (tensor upload)
    DevBuf mten, upload_ten;              // tensor voting: input tensors (Morton order) + upload staging
    DevBuf tvn;                           // tensor voting: per-source voted normal + found flag (double4)
    DevBuf pca_mem;                       // imls_ring_normals_pca scratch (upstream producer)
    DevBuf sample_mem;                    // imls_sample_point_cloud scratch
    DevBuf front_mem;                     // imls_scan_front_end scratch
    size_t n_target_in = 0;               // input size of the last set_target (tensor arrays match it)
    bool has_tensors = false;
    Options opt;                          // imls_set_option
    int lane_mode = 0;                    // opt.traversal == IMLS_TRAVERSAL_LANE
    int temporal_seed = 1;                // opt.temporal_seed
    int N = 0;
    bool has_source = false;
    // deferred index builds: set_target / map_push / set_source without a requested count only
    // enqueue the upload and the NaN filter; the rest of the build (which needs the kept count on
    // the host) runs at the first use (ensure_built), so many frames' filters overlap one wait
    int* h_cnt = nullptr;                 // pinned [4]: kept counts of the pending target / source
    hipEvent_t ev_tgt = nullptr, ev_src = nullptr;
    bool tgt_pending = false, src_pending = false;
    // deferred filters (no count requested): the NaN filter itself waits for the first use, reading
    // its input (an owned upload / FIFO buffer, or the caller's device scan) then — a batch runs all
    // its members' filters in one launch sequence (filter_batch)
    const float* tf_soa = nullptr;
    const float* sf_soa = nullptr;
    size_t tf_n = 0, sf_n = 0;
    bool tgt_filter_deferred = false, src_filter_deferred = false;
    bool defer = false;                   // imls_set_defer: count-less loads read their input at first use
    const float* ten_src = nullptr;       // tensors set while the target build was pending
    size_t ten_n = 0;
    bool ten_pending = false;
    int tgt_slot = -1;                    // timing event slot of the pending target build
    uint32_t* src_kept_out = nullptr;
    // pinned staging of host uploads (0: target / map scans, 1: source), reused once its copy ran
    float* h_stage[2] = {nullptr, nullptr};
    size_t stage_cap[2] = {0, 0};
    hipEvent_t ev_stage[2] = {nullptr, nullptr};
    // an upload of that kind whose NaN filter has not been consumed by a build yet (it may still be
    // reading its device buffer): the next upload's copy is then ordered behind it
    bool stage_pending[2] = {false, false};
    hipStream_t ustream = nullptr;        // host → device copies of uploads (upload_soa6)
    // correspondences + solver state
    DevBuf cs, cd, cn, solve_mem, trace_mem, stats, rows_d, pose_tmp;
    DevBuf ransac_mem, rng;               // RANSAC scratch + the glibc rand() state (34 words)
    int rng_seed_state[34] = {};          // host copy of the seeded state
    bool rng_dirty = true;                // upload rng_seed_state to the device before its next use
    int* h_rng = nullptr;                 // pinned source of that upload (rewritten after ev_rng)
    hipEvent_t ev_rng = nullptr;
    bool rng_init = false;                // seeded from params.ransac_seed (first imls_set_params)
    SolveState st{};
    int st_N = -1, trace_cap = 0;
    bool has_corr = false;
    // per-iteration correspondences of imls_register_frame (imls_capture_correspondences): slot it =
    // cs / cd / cn (float4 [N] each) after iteration it's projection
    bool capture = false;
    DevBuf cap_mem;
    int cap_iters = 0, cap_N = 0;
    int cap_run = -1;                     // iterations the captured frame ran (-1: result not collected yet)
    // async frame results
    imls_iter_trace* h_trace = nullptr;   // pinned
    double* h_misc = nullptr;             // pinned: pose[16], iters, status
    int pending_iters = 0;
    bool pending = false;
    // batched registration led by this context (imls_register_frames*): frame table, results
    PairDev* tab_h = nullptr;             // pinned [tab_cap]
    DevBuf tab_d, res_d;
    double* res_h = nullptr;              // pinned: [n][kResStride] results, then [n][iters] traces
    size_t res_h_bytes = 0;
    int tab_cap = 0;
    std::vector<imls_ctx*> members;       // frames of the pending batch (members[0] == this)
    std::vector<int> member_n;
    bool batch_pending = false, batch_fused = false, batch_traces = false;
    bool batch_member = false;            // part of a pending batch (as lead or member)
    hipEvent_t ev_batch = nullptr;
    // batched index builds of a batch's members (build_batch): scratch, job table, pinned staging
    DevBuf bscratch, btable;
    void* h_btable = nullptr;
    size_t h_btable_bytes = 0;
    DevBuf fscratch, ftable;              // batched filters (filter_batch)
    void* h_ftable = nullptr;
    size_t h_ftable_bytes = 0;
    hipEvent_t ev_build = nullptr;
    // traversal / neighbour counters (imls_traversal_stats): off by default — their per-wave
    // device-scope atomics onto a few shared words cost ~60 µs per projection at config B
    bool collect_stats = false;
    // timing: 0 off, 1 every launch kind (a batch's members then build one by one, each inside its
    // own events), 2 light — the projection / solve events of the iterations only (builds unchanged),
    // kept as intervals on a process-wide clock (imls_timing_intervals: busy time of concurrent work)
    int timing = 0;
    std::vector<std::pair<double, double>> iv[kTimingKinds];
    std::vector<hipEvent_t> ev;
    int ev_used = 0;
    std::vector<std::pair<int, int>> ev_pairs[kTimingKinds];
    double t_ms[kTimingKinds] = {};
    uint64_t t_n[kTimingKinds] = {};
};

namespace {

int fail(imls_ctx* c, int code, const std::string& m) {
    if (c) c->err = m;
    return code;
}

// Grow-only device buffers with 25 % headroom: per-frame sizes vary by a few percent.  A replaced
// buffer is retired, not freed (devbuf_grow below): no reallocation waits for the device.
bool grow(DevBuf& b, size_t bytes) { return devbuf_grow(b, bytes, bytes + bytes / 4 + 256); }

// grow keeping the first `keep` bytes (copied on stream s, a registered stream: the old buffer is
// retired behind the copy)
bool grow_keep(DevBuf& b, size_t bytes, size_t keep, hipStream_t s) {
    if (b.bytes >= bytes) return true;
    if (!b.p || keep == 0) return grow(b, bytes);
    DevBuf nb;
    if (!grow(nb, bytes)) return false;
    if (hipMemcpyAsync(nb.p, b.p, std::min(keep, b.bytes), hipMemcpyDeviceToDevice, s) != hipSuccess) {
        devbuf_retire(nb);
        return false;
    }
    devbuf_retire(b);
    b = nb;
    return true;
}

KParams make_kparams(const imls_params& p, const Options& o) {
    KParams k{};
    k.h2 = p.h * p.h;
    k.r2 = p.r * p.r;
    k.angle_thr_deg = p.angle_diff_threshold;
    k.K = p.search_number;
    k.angle_on = p.normal_angle_constraint ? 1 : 0;
    k.get_normals = p.get_normals ? 1 : 0;
    k.transform_normal = p.transform_normal ? 1 : 0;
    k.correspond_number = p.correspond_number;
    k.solve_method = p.solve_method;
    k.ls_threshold = p.ls_threshold;
    k.delta_dist = p.delta_dist_threshold;
    k.delta_angle = p.delta_angle_threshold;
    // get_normals=false in count mode reads normals recomputed from the map (normals.hip); in the
    // reference's own (dead, Q1) mode every candidate normal is ∞
    if (!p.get_normals && p.recompute_normal_count_mode) k.get_normals = 1;
    k.matcher = p.matching_method;
    // projected-distance gates: IMLS ‖p−x‖ < r_proj, proj < r (imls_icp.cpp:576); plane_ICP keeps the
    // reference's swapped gate ‖p−x‖ < r·r, proj < r_proj (laser_odometry.cpp:322)
    k.proj = p.use_projected_distance ? 1 : 0;
    k.gate_dist = p.r_proj;
    k.gate_proj = p.r;
    if (p.matching_method == IMLS_MATCH_PLANE_ICP) {
        k.proj = p.picp_use_projected_distance ? 1 : 0;
        k.gate_dist = p.picp_r * p.picp_r;
        k.gate_proj = p.picp_r_proj;
        // plane_ICP_proj (laser_odometry.cpp:295-299, 346-350): NN-1 within its own r and angle gate
        k.r2 = p.picp_r * p.picp_r;
        k.K = 1;
        k.angle_on = p.picp_normal_angle_constraint ? 1 : 0;
        k.angle_thr_deg = p.picp_angle_diff_threshold;
    }
    // traversal (imls_set_option, include/imls_gpu.h): −1 auto = one wave per query up to
    // kQwaveAutoN queries (the exact stage fused in for ≤ kSmallRows), packets above
    k.qwave = o.traversal == IMLS_TRAVERSAL_PACKETS ? 0 : o.traversal == IMLS_TRAVERSAL_WAVE_PER_QUERY ? 1 : -1;
    // one frame alone on the GPU (imls_register_frame): its first ICP iteration, where every lane
    // seeds, traverses in 32-query packets (the launch lasts as long as its slowest wave; measured
    // on config B, one pair: k_knn_wave 240 -> 229 us per launch, 8.35 -> 8.14 ms per pair).
    // Batched launches keep 64 (with 4 pairs in flight 32 measured 295 vs 305 pairs/s: the GPU is
    // then throughput-bound and the idle half-waves cost more than the shorter tail saves).
    k.packet = 64;
    k.pk_small = o.first_packet;
    k.pk_iters = o.first_packet_iters;
    k.pk_batch = o.first_packet_batched;
    // Verlet-list reuse (and the prefill certificate), both traversals (round 4: a lone 1949-query
    // frame 1.95 -> 1.84 ms with it on the wave-per-query traversal)
    k.reuse = o.list_reuse;
    k.force_fb = o.force_fallback;
    k.xcd = -1;   // auto: XCD-grouped frames for batches of ≥ 16 frames
    // tensor voting replaces the NN-1 normal only on the IMLS matcher's get_normals=false branch
    // (imls_icp.cpp:514, 630-644); the IMLS neighbours keep the recompute branch (404-434)
    k.tv = (p.use_tensor_voting && !p.get_normals && p.matching_method == IMLS_MATCH_IMLS) ? 1 : 0;
    k.tv_k = p.tensor_k;
    k.tv_sigma = p.tensor_sigma;
    k.tv_thr = p.tensor_distance_threshold;
    k.tv_skin = (float)o.tv_skin;
    k.cos_thr = std::cos(k.angle_thr_deg * M_PI / 180.0);
    return k;
}

int check_params(imls_ctx* c, const imls_params* p) {
    if (!p) return fail(c, IMLS_ERR_ARG, "null params");
    if (p->search_number < 1 || p->search_number > 32) return fail(c, IMLS_ERR_UNSUPPORTED, "search_number must be in [1, 32]");
    if (p->matching_method != IMLS_MATCH_IMLS && p->matching_method != IMLS_MATCH_PLANE_ICP)
        return fail(c, IMLS_ERR_ARG, "matching_method must be IMLS or plane_ICP");
    if (p->use_tensor_voting && !p->get_normals) {
        if (p->tensor_k < 1 || p->tensor_k > kTvMaxK) return fail(c, IMLS_ERR_UNSUPPORTED, "tensor_voting.k must be in [1, 64]");
        if (!(p->tensor_sigma > 0)) return fail(c, IMLS_ERR_ARG, "tensor_voting.sigma must be > 0");
    }
    if (!p->get_normals && p->recompute_normal_count_mode && (p->search_number_normal < 1 || p->search_number_normal > 32))
        return fail(c, IMLS_ERR_UNSUPPORTED, "search_number_normal must be in [1, 32]");
    if (p->solve_method != IMLS_SOLVE_LS && p->solve_method != IMLS_SOLVE_WEIGHTED_LS && p->solve_method != IMLS_SOLVE_RANSAC)
        return fail(c, IMLS_ERR_UNSUPPORTED, "solve_method must be LS, Weighted LS or RANSAC (Ceres/ICP/Teaser stay on the CPU path)");
    if (p->solve_method == IMLS_SOLVE_RANSAC) {
        if (p->ransac_final_method != IMLS_FINAL_LS && p->ransac_final_method != IMLS_FINAL_WEIGHTED_LS &&
            p->ransac_final_method != IMLS_FINAL_DRPM)
            return fail(c, IMLS_ERR_ARG, "RANSAC final_solve_method must be LS, Weighted LS or DRPM");
        if (p->ransac_max_iterations < 1) return fail(c, IMLS_ERR_ARG, "RANSAC max_iterations < 1");
        if (!(p->ransac_ls_threshold >= 0 && p->ransac_ls_threshold < 0.5))
            return fail(c, IMLS_ERR_ARG, "RANSAC LS threshold must be in [0, 0.5)");
    }
    if (p->iterations < 0) return fail(c, IMLS_ERR_ARG, "iterations < 0");
    if (!(p->ls_threshold >= 0 && p->ls_threshold < 0.5)) return fail(c, IMLS_ERR_ARG, "LS threshold must be in [0, 0.5)");
    return IMLS_OK;
}

// Per-N solver / correspondence buffers.
int ensure_solve(imls_ctx* c, int N) {
    if (c->st_N >= N && c->st.trace) return IMLS_OK;
    size_t n = (size_t)std::max(N, 1);
    n += n / 4 + 64;                      // headroom (see grow): the next frames' N differ a little
    // deferred (uncertified) queries: k_finish's wave w writes its count to word w and its queries,
    // in slot order, to the region fb_off + w·64 (project.hip finish_body, k_project_lane)
    const size_t nfb = (n + 63) / 64;
    c->fb_off = (nfb + 63) / 64 * 64;
    if (!grow(c->cs, n * 16) || !grow(c->cd, n * 16) || !grow(c->cn, n * 16) || !grow(c->fb, (c->fb_off + nfb * 64) * 4))
        return fail(c, IMLS_ERR_DEVICE, "hipMalloc (correspondences)");
    if (!grow(c->prevnn, prevnn_bytes((int)n))) return fail(c, IMLS_ERR_DEVICE, "hipMalloc (prevnn)");
    if (!grow(c->tvn, n * kTvBytesPerQuery)) return fail(c, IMLS_ERR_DEVICE, "hipMalloc (tvn)");
    const int pb = std::max(project_blocks((int)n), solve_blocks((int)n)) + 1;
    size_t bytes = 0;
    auto add = [&](size_t b) { size_t o = bytes; bytes += (b + 255) / 256 * 256; return o; };
    size_t o_pose = add(16 * 8), o_delta = add(16 * 8), o_x0 = add(8 * 8), o_done = add(16), o_status = add(16),
           o_iters = add(16), o_hist = add(kHistBins * 4), o_coarse = add(kHistBins / 256 * 4), o_cc = add(16), o_cl = add((size_t)kCandCap * 8),
           o_clr = add((size_t)kCandCap * 4), o_ch = add((size_t)kCandCap * 8), o_chr = add((size_t)kCandCap * 4),
           o_sel = add(16 * 4), o_p1 = add((size_t)pb * kNormEq * 8), o_p2 = add((size_t)pb * kNormEq * 8),
           o_keys = add(n * 8), o_trace1 = add(sizeof(imls_iter_trace));
    if (!grow(c->solve_mem, bytes)) return fail(c, IMLS_ERR_DEVICE, "hipMalloc (solver)");
    char* b = (char*)c->solve_mem.p;
    SolveState& s = c->st;
    s.pose = (double*)(b + o_pose);
    s.delta = (double*)(b + o_delta);
    s.x0 = (double*)(b + o_x0);
    s.done = (int*)(b + o_done);
    s.status = (int*)(b + o_status);
    s.iters = (int*)(b + o_iters);
    s.hist = (unsigned*)(b + o_hist);
    s.coarse = (unsigned*)(b + o_coarse);
    s.cand_count = (unsigned*)(b + o_cc);
    s.cand_lo = (unsigned long long*)(b + o_cl);
    s.cand_lo_row = (unsigned*)(b + o_clr);
    s.cand_hi = (unsigned long long*)(b + o_ch);
    s.cand_hi_row = (unsigned*)(b + o_chr);
    s.sel = (int*)(b + o_sel);
    s.partial1 = (double*)(b + o_p1);
    s.partial2 = (double*)(b + o_p2);
    s.keys = (double*)(b + o_keys);
    s.trace = (imls_iter_trace*)(b + o_trace1);
    s.partial_cap = pb;
    // the residual histogram is re-zeroed after each use (k_collect); it starts zero
    if (hipMemsetAsync(s.hist, 0, kHistBins * 4, c->stream) != hipSuccess ||
        hipMemsetAsync(s.coarse, 0, kHistBins / 256 * 4, c->stream) != hipSuccess)
        return fail(c, IMLS_ERR_DEVICE, "hipMemset (solver)");
    c->st_N = (int)n;
    return IMLS_OK;
}

RansacParams ransac_params(const imls_params& p) {
    RansacParams r;
    r.max_iterations = p.ransac_max_iterations;
    r.distance_threshold = p.ransac_distance_threshold;
    r.min_inliers_percentage = p.ransac_min_inliers_percentage;
    r.huber_threshold = p.ransac_huber_threshold;
    r.final_method = p.ransac_final_method;
    r.ls_threshold = p.ransac_ls_threshold;
    r.drpm_threshold = p.drpm_threshold;
    r.drpm_stdev_points = p.drpm_stdev_points;
    r.drpm_stdev_normals = p.drpm_stdev_normals;
    return r;
}

// The context's glibc rand() state lives on the device and runs on across every RANSAC solve and
// every frame, like the reference's one process-wide rand() stream (solver.cpp / common.cpp:49 never
// call srand).  It is seeded from params.ransac_seed at context creation, when imls_set_params
// changes ransac_seed, and by imls_seed_rng; imls_set_rng_state hands a stream from one context to
// the next.  Async on the context stream.
int sync_rng(imls_ctx* c) {
    if (!grow(c->rng, 34 * 4)) return fail(c, IMLS_ERR_DEVICE, "hipMalloc (rand state)");
    if (!c->rng_dirty) return IMLS_OK;
    // pinned source, rewritten only after its previous copy ran (ev_rng): no host wait on the stream
    // (a caller that reseeds before every frame keeps its frames in flight)
    if (!c->h_rng && hipHostMalloc((void**)&c->h_rng, 34 * 4) != hipSuccess) return fail(c, IMLS_ERR_DEVICE, "hipHostMalloc (rand state)");
    if (!c->ev_rng && hipEventCreateWithFlags(&c->ev_rng, hipEventDisableTiming) != hipSuccess)
        return fail(c, IMLS_ERR_DEVICE, "hipEventCreate (rand state)");
    if (hipEventSynchronize(c->ev_rng) != hipSuccess) return fail(c, IMLS_ERR_DEVICE, "rand state upload");
    std::memcpy(c->h_rng, c->rng_seed_state, 34 * 4);
    if (hipMemcpyAsync(c->rng.p, c->h_rng, 34 * 4, hipMemcpyHostToDevice, c->stream) != hipSuccess ||
        hipEventRecord(c->ev_rng, c->stream) != hipSuccess)
        return fail(c, IMLS_ERR_DEVICE, "rand state upload");
    c->rng_dirty = false;
    return IMLS_OK;
}

// RANSAC scratch for `rows` rows and the (persistent) rand() state.
int prepare_ransac(imls_ctx* c, int rows) {
    if (c->P.solve_method != IMLS_SOLVE_RANSAC) return IMLS_OK;
    if (!grow(c->ransac_mem, ransac_bytes(rows))) return fail(c, IMLS_ERR_DEVICE, "hipMalloc (RANSAC)");
    if (ransac_init_tables(c->device)) return fail(c, IMLS_ERR_DEVICE, "RANSAC rand() table upload");
    return sync_rng(c);
}

TreeView tree_view(imls_ctx* c);

// count mode: (re)compute the map normals once per (map, search_number_normal, r_normal)
int ensure_map_normals(imls_ctx* c) {
    if (c->P.get_normals || !c->P.recompute_normal_count_mode) return IMLS_OK;
    if (c->rnr_valid && c->rnr_k == c->P.search_number_normal && c->rnr_r == c->P.r_normal) return IMLS_OK;
    if (!grow(c->rnr, (size_t)std::max(c->M, 1) * 16)) return fail(c, IMLS_ERR_DEVICE, "hipMalloc (normals)");
    TreeView t = tree_view(c);
    if (launch_map_normals(c->stream, t, c->P.search_number_normal, c->P.r_normal, (float4*)c->rnr.p))
        return fail(c, IMLS_ERR_DEVICE, "map normal launch failed");
    c->rnr_valid = true;
    c->rnr_k = c->P.search_number_normal;
    c->rnr_r = c->P.r_normal;
    return IMLS_OK;
}

SolveLaunch solve_launch(imls_ctx* c, imls_iter_trace* tr, int update_pose) {
    SolveLaunch L{};
    L.N = c->N;
    L.blocks1 = project_blocks(c->N);
    L.kp = c->kp;
    L.cs = (const float4*)c->cs.p;
    L.cd = (const float4*)c->cd.p;
    L.cn = (const float4*)c->cn.p;
    L.st = c->st;
    L.tr = tr;
    L.update_pose = update_pose;
    L.scratch = c->ransac_mem.p;
    L.rng = (int*)c->rng.p;
    L.ransac = ransac_params(c->P);
    return L;
}

int ensure_trace(imls_ctx* c, int iters) {
    if (c->trace_cap >= iters && c->h_trace) return IMLS_OK;
    if (!grow(c->trace_mem, (size_t)std::max(iters, 1) * sizeof(imls_iter_trace))) return fail(c, IMLS_ERR_DEVICE, "hipMalloc (trace)");
    if (c->h_trace) (void)hipHostFree(c->h_trace);
    if (hipHostMalloc((void**)&c->h_trace, (size_t)std::max(iters, 1) * sizeof(imls_iter_trace)) != hipSuccess)
        return fail(c, IMLS_ERR_DEVICE, "hipHostMalloc (trace)");
    c->trace_cap = std::max(iters, 1);
    return IMLS_OK;
}

unsigned* fb_count(imls_ctx* c) { return (unsigned*)c->fb.p; }
unsigned long long* stats_ptr(imls_ctx* c) { return c->collect_stats ? (unsigned long long*)c->stats.p : nullptr; }
unsigned* fb_list(imls_ctx* c) { return (unsigned*)c->fb.p + c->fb_off; }

TreeView tree_view(imls_ctx* c) {
    TreeView t;
    t.mpt = (const float4*)c->mpt.p;
    t.mnr = t.mpt ? t.mpt + c->M : nullptr;
    if (!c->P.get_normals && c->P.recompute_normal_count_mode && c->rnr.p) t.mnr = (const float4*)c->rnr.p;
    t.ipos = t.mpt ? (const unsigned*)(t.mpt + 2 * (size_t)c->M) : nullptr;
    t.nodes = (const float4*)c->nodes.p;
    t.tpt = (const float4*)c->tpt.p;
    t.tnr = (const float4*)c->tnr.p;
    t.M = c->M;
    t.B = c->B;
    t.P = c->Pl;
    t.levels = c->levels;
    t.L = c->B > 0 ? (c->M + c->B - 1) / c->B : 0;
    t.lkeys = (const unsigned long long*)c->lkeys.p;
    t.qparams = c->lkeys.p ? (const float*)((const unsigned long long*)c->lkeys.p + t.L) : nullptr;
    t.mten = c->has_tensors ? (const float4*)c->mten.p : nullptr;
    t.tvn = (const double4*)c->tvn.p;
    return t;
}

int ev_pair(imls_ctx* c) {
    if (c->ev_used + 2 > (int)c->ev.size()) {
        for (int k = 0; k < 64; ++k) {
            hipEvent_t e;
            if (hipEventCreate(&e) != hipSuccess) return -1;
            c->ev.push_back(e);
        }
    }
    int i = c->ev_used;
    c->ev_used += 2;
    return i;
}

void timed_begin(imls_ctx* c, int kind, int& slot) {
    slot = -1;
    if (!c->timing) return;
    slot = ev_pair(c);
    if (slot >= 0) hipEventRecord(c->ev[slot], c->stream);
}
void timed_end(imls_ctx* c, int kind, int slot) {
    if (slot < 0) return;
    hipEventRecord(c->ev[slot + 1], c->stream);
    c->ev_pairs[kind].push_back({slot, slot + 1});
}
// Events around the two projection kernels (kinds 3 and 4): marks[0..2], or null when off.
hipEvent_t* project_marks(imls_ctx* c, hipEvent_t marks[3]) {
    if (!c->timing) return nullptr;
    const int a = ev_pair(c), b = ev_pair(c);
    if (a < 0 || b < 0) return nullptr;
    marks[0] = c->ev[a];
    marks[1] = c->ev[a + 1];
    marks[2] = c->ev[b];
    c->ev_pairs[3].push_back({a, a + 1});
    c->ev_pairs[4].push_back({a + 1, b});
    return marks;
}

// Process-wide origin of the timing intervals (imls_timing_origin): one clock per device for every
// context of that device, so the busy time of concurrent launch sequences is the union of their
// intervals.  One origin per device, created once and never destroyed while the process runs (a
// context on another device cannot pull an origin out from under this one); the mutex orders the
// origin's (re)recording against the comparisons in harvest_timing.
constexpr int kMaxDevices = 64;
std::mutex g_origin_mu;
hipEvent_t g_origin[kMaxDevices] = {};
bool g_origin_set[kMaxDevices] = {};
// intervals kept per context and launch kind until imls_reset_timing / imls_timing_origin (a cap:
// a caller that never resets keeps a bounded record, the oldest first)
constexpr size_t kMaxIntervals = (size_t)1 << 20;

void harvest_timing(imls_ctx* c) {
    std::lock_guard<std::mutex> lk(g_origin_mu);
    const bool dev_ok = c->device >= 0 && c->device < kMaxDevices;
    const bool iv = dev_ok && g_origin_set[c->device];
    for (int k = 0; k < kTimingKinds; ++k) {
        for (auto& pr : c->ev_pairs[k]) {
            float ms = 0;
            if (hipEventElapsedTime(&ms, c->ev[pr.first], c->ev[pr.second]) == hipSuccess) {
                c->t_ms[k] += ms;
                c->t_n[k] += 1;
                float a = 0, b = 0;
                if (iv && c->iv[k].size() < kMaxIntervals &&
                    hipEventElapsedTime(&a, g_origin[c->device], c->ev[pr.first]) == hipSuccess &&
                    hipEventElapsedTime(&b, g_origin[c->device], c->ev[pr.second]) == hipSuccess)
                    c->iv[k].push_back({a, b});
            }
        }
        c->ev_pairs[k].clear();
    }
    c->ev_used = 0;
}

// Persistent host workers for the upload packing: a scan of ~10^5 points is a strided gather of
// several MB, split over a few threads — created once per process, not per call (spawning 7
// std::threads per upload cost ~0.2 ms, more than the gather itself: round 3 measured 333 µs per
// 118k-point scan).  One job at a time (the mutex serialises contexts on other host threads).
class PackPool {
public:
    static PackPool& get() {
        static PackPool pool;
        return pool;
    }
    size_t width() const { return workers_.size() + 1; }
    // fn(i0, i1) over [0, n) in `parts` contiguous chunks (parts ≤ width()), the caller taking the first
    void run(size_t n, size_t parts, const std::function<void(size_t, size_t)>& fn) {
        parts = std::max<size_t>(1, std::min(parts, width()));
        // a forked child inherits the pool object but not its threads: pack serially there
        if (parts == 1 || n == 0 || getpid() != pid_) {
            fn(0, n);
            return;
        }
        std::lock_guard<std::mutex> job_lock(job_mu_);
        const size_t chunk = (n + parts - 1) / parts;
        {
            std::lock_guard<std::mutex> lk(mu_);
            fn_ = &fn;
            n_ = n;
            chunk_ = chunk;
            parts_ = parts;
            pending_ = parts - 1;
            pending_left_.store(parts - 1, std::memory_order_release);
            ++gen_;
        }
        gen_seen_.store(gen_, std::memory_order_release);
        cv_.notify_all();
        fn(0, std::min(n, chunk));
        // the helpers finish at about the caller's pace: poll briefly before sleeping on the cv
        const auto t0 = std::chrono::steady_clock::now();
        while (pending_left_.load(std::memory_order_acquire) != 0 &&
               std::chrono::steady_clock::now() - t0 < std::chrono::microseconds(spin_us_)) {
        }
        std::unique_lock<std::mutex> lk(mu_);
        done_cv_.wait(lk, [&] { return pending_ == 0; });
        fn_ = nullptr;
        last_job_ns_.store(now_ns(), std::memory_order_release);
    }

private:
    PackPool() {
        // the process's CPU share, at most kMaxHelpers helpers: the gather is bound by each core's
        // memory bandwidth (round 4: 118k 48-B records took ~90 µs on 8 threads)
        size_t hw = std::max<unsigned>(std::thread::hardware_concurrency(), 1u);
        if (const char* e = std::getenv("OMP_NUM_THREADS")) hw = std::min<size_t>(hw, (size_t)std::max(1, std::atoi(e)));
        size_t cap = kMaxHelpers;
        const size_t helpers = std::min<size_t>(cap, hw > 1 ? hw - 1 : 0);
        for (size_t k = 0; k < helpers; ++k) workers_.emplace_back([this, k] { loop(k + 1); });
    }
    ~PackPool() {
        {
            std::lock_guard<std::mutex> lk(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto& t : workers_) t.join();
    }
    void loop(size_t id) {
        uint64_t seen = 0;
        for (;;) {
            const std::function<void(size_t, size_t)>* fn;
            size_t i0, i1;
            bool mine;
            {
                // a job soon after the last one (frames back to back) starts without a wake-up: a
                // helper polls up to spin_us_ only while jobs come in bursts (the last one ended
                // < kBurstNs ago), so an idle pool sleeps at once instead of holding cores
                const auto t0 = std::chrono::steady_clock::now();
                const bool burst = now_ns() - last_job_ns_.load(std::memory_order_acquire) < kBurstNs;
                while (burst && gen_seen_.load(std::memory_order_acquire) == seen &&
                       std::chrono::steady_clock::now() - t0 < std::chrono::microseconds(spin_us_)) {
                }
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
                if (stop_) return;
                seen = gen_;
                mine = id < parts_;
                fn = fn_;
                i0 = std::min(n_, id * chunk_);
                i1 = std::min(n_, (id + 1) * chunk_);
            }
            if (!mine) continue;
            (*fn)(i0, i1);
            std::lock_guard<std::mutex> lk(mu_);
            pending_left_.fetch_sub(1, std::memory_order_release);
            if (--pending_ == 0) done_cv_.notify_one();
        }
    }
    std::vector<std::thread> workers_;
    std::mutex job_mu_, mu_;
    std::condition_variable cv_, done_cv_;
    const std::function<void(size_t, size_t)>* fn_ = nullptr;
    size_t n_ = 0, chunk_ = 0, parts_ = 0, pending_ = 0;
    static constexpr size_t kMaxHelpers = 15;
    std::atomic<uint64_t> gen_seen_{0};       // gen_, readable without the mutex (the helpers' poll)
    std::atomic<size_t> pending_left_{0};      // pending_, likewise (the caller's poll)
    static int64_t now_ns() {
        return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch()).count();
    }
    static constexpr int64_t kBurstNs = 2000000;   // 2 ms
    std::atomic<int64_t> last_job_ns_{0};
    const pid_t pid_ = getpid();
    int spin_us_ = 200;
    uint64_t gen_ = 0;
    bool stop_ = false;
};

// Pack a strided host cloud into SoA6 floats in pinned staging and upload asynchronously (no host
// wait: the staging buffer is reused only after its previous copy has run).  The reference's
// PointXYZINormal records (48 B: x y z pad | nx ny nz pad | intensity curvature pad pad, nrm =
// xyz + 4, stride 12 floats) take a record-at-a-time path (two 16-B loads per point).
int upload_soa6(imls_ctx* c, DevBuf& dst, const float* xyz, const float* nrm, size_t n, size_t stride, int which) {
    if (!xyz || !nrm || n == 0 || stride < 3) return fail(c, IMLS_ERR_ARG, "bad cloud pointer/size/stride");
    if (!c->ev_stage[which] && hipEventCreateWithFlags(&c->ev_stage[which], hipEventDisableTiming) != hipSuccess)
        return fail(c, IMLS_ERR_DEVICE, "hipEventCreate (staging)");
    if (hipEventSynchronize(c->ev_stage[which]) != hipSuccess) return fail(c, IMLS_ERR_DEVICE, "staging wait");
    if (c->stage_cap[which] < 6 * n) {
        if (c->h_stage[which]) (void)hipHostFree(c->h_stage[which]);
        c->h_stage[which] = nullptr;
        c->stage_cap[which] = 0;
        const size_t cap = 6 * n + 6 * n / 4 + 1024;
        if (hipHostMalloc((void**)&c->h_stage[which], cap * 4) != hipSuccess) return fail(c, IMLS_ERR_DEVICE, "hipHostMalloc (staging)");
        c->stage_cap[which] = cap;
    }
    float* h = c->h_stage[which];
    const bool rec48 = nrm == xyz + 4 && stride == 12 && (reinterpret_cast<uintptr_t>(xyz) & 15) == 0;
    const std::function<void(size_t, size_t)> pack = [=](size_t i0, size_t i1) {
        float *hx = h, *hy = h + n, *hz = h + 2 * n, *hnx = h + 3 * n, *hny = h + 4 * n, *hnz = h + 5 * n;
        if (rec48) {
            typedef float f4 __attribute__((ext_vector_type(4)));
            const f4* r = reinterpret_cast<const f4*>(xyz);
            for (size_t i = i0; i < i1; ++i) {
                const f4 p = r[3 * i], q = r[3 * i + 1];
                hx[i] = p.x; hy[i] = p.y; hz[i] = p.z;
                hnx[i] = q.x; hny[i] = q.y; hnz[i] = q.z;
            }
            return;
        }
        for (size_t i = i0; i < i1; ++i) {
            const float* p = xyz + i * stride;
            const float* q = nrm + i * stride;
            hx[i] = p[0]; hy[i] = p[1]; hz[i] = p[2];
            hnx[i] = q[0]; hny[i] = q[1]; hnz[i] = q[2];
        }
    };
    PackPool::get().run(n, n / 8192 + 1, pack);
    if (!grow(dst, 6 * n * 4)) return fail(c, IMLS_ERR_DEVICE, "hipMalloc (upload)");
    // the copy runs on the context's upload stream, not behind its running registrations: the
    // buffer's previous reader — the NaN filter of the last upload of this kind — has finished once a
    // build consumed its kept count (stage_pending false), else the copy is ordered after it on the
    // context's stream.  The context's stream waits for the copy (its filter reads the buffer).
    hipStream_t us = c->stream;
#if IMLS_UPLOAD_STREAM
    if (!c->stage_pending[which]) {
        if (!c->ustream) {
            if (hipStreamCreateWithFlags(&c->ustream, hipStreamNonBlocking) != hipSuccess)
                return fail(c, IMLS_ERR_DEVICE, "hipStreamCreate (upload)");
            register_stream(c->ustream, c->device);
        }
        us = c->ustream;
    }
#endif
    if (hipMemcpyAsync(dst.p, h, 6 * n * 4, hipMemcpyHostToDevice, us) != hipSuccess ||
        hipEventRecord(c->ev_stage[which], us) != hipSuccess ||
        (us != c->stream && hipStreamWaitEvent(c->stream, c->ev_stage[which], 0) != hipSuccess))
        return fail(c, IMLS_ERR_DEVICE, "upload failed");
    c->stage_pending[which] = true;
    return IMLS_OK;
}

int gather_tensors(imls_ctx* c, hipStream_t s, const float* d_ten6, size_t n);

int fifo_build(imls_ctx* c);

// Phase B of a pending target build (waits for its filter's kept count).
int finish_target(imls_ctx* c) {
    if (!c->tgt_pending) return IMLS_OK;
    c->tgt_pending = false;
    if (c->fifo_inc) return fifo_build(c);
    if (c->tgt_filter_deferred) {
        c->tgt_filter_deferred = false;
        if (int rc = filter_async(c->stream, c->tf_soa, c->tf_n, c->tpt, c->tnr, c->tscratch, (unsigned*)c->tkept.p,
                                  &c->h_cnt[0], c->err))
            return rc;
        if (hipEventRecord(c->ev_tgt, c->stream) != hipSuccess) return fail(c, IMLS_ERR_DEVICE, "event record");
    }
    if (hipEventSynchronize(c->ev_tgt) != hipSuccess) return fail(c, IMLS_ERR_DEVICE, "target filter failed");
    c->stage_pending[0] = false;
    c->M = c->h_cnt[0];
    int rc = build_target_tree(c->stream, c->M, c->B, c->lkeys, c->tpt, c->tnr, c->mpt, c->nodes, c->tscratch,
                               c->treescratch, c->permbuf, &c->Pl, &c->levels, c->err);
    timed_end(c, 1, c->tgt_slot);
    c->tgt_slot = -1;
    c->has_target = rc == IMLS_OK && c->M > 0;
    if (rc == IMLS_OK && c->ten_pending) {
        c->ten_pending = false;
        if (c->has_target) rc = gather_tensors(c, c->stream, c->ten_src, c->ten_n);
        else c->has_tensors = false;
    }
    return rc;
}

// Phase B of a pending source load.
int finish_source(imls_ctx* c) {
    if (!c->src_pending) return IMLS_OK;
    c->src_pending = false;
    if (c->src_filter_deferred) {
        c->src_filter_deferred = false;
        if (int rc = filter_async(c->stream, c->sf_soa, c->sf_n, c->spt, c->snr, c->sscratch, nullptr, &c->h_cnt[1], c->err))
            return rc;
        if (hipEventRecord(c->ev_src, c->stream) != hipSuccess) return fail(c, IMLS_ERR_DEVICE, "event record");
    }
    if (hipEventSynchronize(c->ev_src) != hipSuccess) return fail(c, IMLS_ERR_DEVICE, "source filter failed");
    c->stage_pending[1] = false;
    c->N = c->h_cnt[1];
    c->has_source = false;
    if (int rc = source_order(c->stream, c->N, c->spt, c->sscratch, c->qperm, c->err)) return rc;
    if (c->src_kept_out && c->N > 0 &&
        (hipMemcpyAsync(c->src_kept_out, c->skept.p, (size_t)c->N * 4, hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
         hipStreamSynchronize(c->stream) != hipSuccess))
        return fail(c, IMLS_ERR_DEVICE, "kept index download failed");
    c->src_kept_out = nullptr;
    c->has_source = c->N > 0;
    return ensure_solve(c, c->N);
}

int ensure_built(imls_ctx* c) {
    if (int rc = finish_target(c)) return rc;
    return finish_source(c);
}

// IMLS_DEBUG_HOST=1: host-time split of imls_register_frames_async on stderr (diagnostics only)
struct HostSplit {
    bool on = std::getenv("IMLS_DEBUG_HOST") != nullptr;
    std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now(), t = t0;
    char buf[512];
    int len = 0;
    void mark(const char* what) {
        if (!on) return;
        const auto now = std::chrono::steady_clock::now();
        len += std::snprintf(buf + len, sizeof(buf) - (size_t)len, " %s %.2f", what,
                             std::chrono::duration<double, std::milli>(now - t).count());
        t = now;
    }
    ~HostSplit() {
        if (on) std::fprintf(stderr, "[imls host ms]%s total %.2f\n", buf,
                             std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
    }
};

// The pending builds of a batch's members in ONE launch sequence on the lead's stream (index.hip
// build_batch: one radix sort for every frame's points): after each member's filter count (one
// host wait each, all filters already enqueued), the trees and source orders of all of them; the
// members' streams are then ordered after it.  Members with per-launch timing on keep their own
// build (its timing events are on their streams).
int batch_builds(imls_ctx* L, imls_ctx* const* ctxs, size_t n, bool fused, HostSplit* hs = nullptr) {
    bool any = false, timing = false;
    for (size_t k = 0; k < n; ++k) {
        any |= ctxs[k]->tgt_pending || ctxs[k]->src_pending;
        timing |= ctxs[k]->timing == 1;
    }
    if (!any) return IMLS_OK;
    // incremental FIFO targets (index.hip fifo_*): each member's own build on its stream (a merge of
    // sorted runs, not the batch's one radix sort), joined by the lead's stream
    for (size_t k = 0; k < n; ++k) {
        imls_ctx* c = ctxs[k];
        if (!c->tgt_pending || !c->fifo_inc) continue;
        if (int rc = finish_target(c)) return fail(L, rc, "context " + std::to_string(k) + ": " + c->err);
        if (c != L && c->has_target && hipStreamWaitEvent(L->stream, c->ev_fifo, 0) != hipSuccess)
            return fail(L, IMLS_ERR_DEVICE, "FIFO build join");
    }
    if (timing) {
        for (size_t k = 0; k < n; ++k)
            if (int rc = ensure_built(ctxs[k])) return fail(L, rc, "context " + std::to_string(k) + ": " + ctxs[k]->err);
        return IMLS_OK;
    }
    // the deferred NaN filters of every member: one launch sequence on the lead's stream, ordered
    // after each member's stream (its uploads), then one wait for all their counts
    {
        std::vector<FilterJob> fj;
        for (size_t k = 0; k < n; ++k) {
            imls_ctx* c = ctxs[k];
            // (a join only where the member's stream still has work: an idle stream's is done)
            if (c->tgt_pending && c->tgt_filter_deferred) {
                if (c != L && hipEventQuery(c->ev_tgt) != hipSuccess && hipStreamWaitEvent(L->stream, c->ev_tgt, 0) != hipSuccess)
                    return fail(L, IMLS_ERR_DEVICE, "filter join");
                if (!grow(c->tkept, c->tf_n * 4 + 16)) return fail(L, IMLS_ERR_DEVICE, "hipMalloc (kept)");
                fj.push_back(FilterJob{c->tf_soa, c->tf_n, &c->tpt, &c->tnr, (unsigned*)c->tkept.p, &c->h_cnt[0]});
                c->tgt_filter_deferred = false;
            }
            if (c->src_pending && c->src_filter_deferred) {
                if (c != L && hipEventQuery(c->ev_src) != hipSuccess && hipStreamWaitEvent(L->stream, c->ev_src, 0) != hipSuccess)
                    return fail(L, IMLS_ERR_DEVICE, "filter join");
                fj.push_back(FilterJob{c->sf_soa, c->sf_n, &c->spt, &c->snr, nullptr, &c->h_cnt[1]});
                c->src_filter_deferred = false;
            }
        }
        if (!fj.empty()) {
            const size_t tb = fj.size() * filter_job_bytes();
            if (L->h_ftable_bytes < tb) {
                if (L->h_ftable) (void)hipHostFree(L->h_ftable);
                L->h_ftable = nullptr;
                L->h_ftable_bytes = 0;
                if (hipHostMalloc(&L->h_ftable, tb + tb / 2 + 1024) != hipSuccess) return fail(L, IMLS_ERR_DEVICE, "hipHostMalloc (filter table)");
                L->h_ftable_bytes = tb + tb / 2 + 1024;
            }
            (void)hipSetDevice(L->device);
            if (int rc = filter_batch(L->stream, fj, L->fscratch, L->ftable, L->h_ftable, L->h_ftable_bytes, L->err)) return rc;
            if (hs) hs->mark("filter-launch");
            if (hipStreamSynchronize(L->stream) != hipSuccess) return fail(L, IMLS_ERR_DEVICE, "batched filter failed");
            if (hs) hs->mark("filter-wait");
        }
    }
    std::vector<BuildJob> jobs;
    std::vector<std::pair<imls_ctx*, int>> who;   // (context, 0 target / 1 source)
    for (size_t k = 0; k < n; ++k) {
        imls_ctx* c = ctxs[k];
        if (c->tgt_pending) {
            c->tgt_pending = false;
            if (hipEventSynchronize(c->ev_tgt) != hipSuccess) return fail(L, IMLS_ERR_DEVICE, "target filter failed");
            c->stage_pending[0] = false;
            c->M = c->h_cnt[0];
            c->Pl = c->levels = 0;
            c->has_target = c->M > 0;
            timed_end(c, 1, c->tgt_slot);
            c->tgt_slot = -1;
            if (c->M > 0) {
                const int Lv = (c->M + c->B - 1) / c->B;
                int P = 1;
                while (P < Lv) P <<= 1;
                if (!grow(c->lkeys, (size_t)Lv * 8 + 16) || !grow(c->mpt, (size_t)c->M * 36 + 64) ||
                    !grow(c->nodes, (size_t)(P + 1) * 48))
                    return fail(L, IMLS_ERR_DEVICE, "hipMalloc (index)");
                jobs.push_back(BuildJob{(const float4*)c->tpt.p, (const float4*)c->tnr.p, c->M, c->B,
                                        (unsigned long long*)c->lkeys.p, (float4*)c->mpt.p, (float4*)c->nodes.p, nullptr, 0, 0});
                who.push_back({c, 0});
            }
        }
        if (c->src_pending) {
            c->src_pending = false;
            if (hipEventSynchronize(c->ev_src) != hipSuccess) return fail(L, IMLS_ERR_DEVICE, "source filter failed");
            c->stage_pending[1] = false;
            c->N = c->h_cnt[1];
            c->has_source = c->N > 0;
            c->src_kept_out = nullptr;
            if (c->N > 0) {
                if (!grow(c->qperm, (size_t)c->N * 4 + 16)) return fail(L, IMLS_ERR_DEVICE, "hipMalloc (source order)");
                if (n == 1 && c == L && c->N <= kSmallOrderN) {
                    // a lone small frame: its source order in one launch (index.hip), not the
                    // batched build's 6-8 — the same permutation
                    if (int rc = small_source_order(L->stream, (const float4*)c->spt.p, c->N, (unsigned*)c->qperm.p, L->err))
                        return fail(L, rc, L->err);
                } else {
                    jobs.push_back(BuildJob{(const float4*)c->spt.p, nullptr, c->N, 0, nullptr, nullptr, nullptr,
                                            (unsigned*)c->qperm.p, 0, 0});
                    who.push_back({c, 1});
                }
            }
            if (int rc = ensure_solve(c, c->N)) return fail(L, rc, c->err);
        }
    }
    if (jobs.empty()) return IMLS_OK;
    const size_t tb = jobs.size() * build_job_bytes();
    if (L->h_btable_bytes < tb) {
        if (L->h_btable) (void)hipHostFree(L->h_btable);
        L->h_btable = nullptr;
        L->h_btable_bytes = 0;
        if (hipHostMalloc(&L->h_btable, tb + tb / 2 + 1024) != hipSuccess) return fail(L, IMLS_ERR_DEVICE, "hipHostMalloc (build table)");
        L->h_btable_bytes = tb + tb / 2 + 1024;
    }
    (void)hipSetDevice(L->device);
    if (int rc = build_batch(L->stream, jobs, L->bscratch, L->btable, L->h_btable, L->h_btable_bytes, L->err)) return rc;
    for (size_t q = 0; q < jobs.size(); ++q)
        if (who[q].second == 0) {
            who[q].first->Pl = jobs[q].P;
            who[q].first->levels = jobs[q].levels;
        }
    for (size_t k = 0; k < n; ++k) {          // tensors set while the build was pending (config E)
        imls_ctx* c = ctxs[k];
        if (!c->ten_pending) continue;
        c->ten_pending = false;
        if (!c->has_target) { c->has_tensors = false; continue; }
        if (int rc = gather_tensors(c, L->stream, c->ten_src, c->ten_n)) return fail(L, rc, c->err);
    }
    // every member's later work on its own stream (its frame's launches when the batch is not fused)
    // is ordered after the build (a fused batch orders them after the whole batch instead)
    if (fused) return IMLS_OK;
    if (!L->ev_build && hipEventCreateWithFlags(&L->ev_build, hipEventDisableTiming) != hipSuccess)
        return fail(L, IMLS_ERR_DEVICE, "hipEventCreate (build)");
    if (hipEventRecord(L->ev_build, L->stream) != hipSuccess) return fail(L, IMLS_ERR_DEVICE, "build event");
    for (size_t k = 0; k < n; ++k)
        if (ctxs[k] != L && hipStreamWaitEvent(ctxs[k]->stream, L->ev_build, 0) != hipSuccess)
            return fail(L, IMLS_ERR_DEVICE, "build stream join");
    return IMLS_OK;
}

// A count-less load defers its NaN filter to the first use only when the caller asked for deferred
// reads (imls_set_defer: a batch then filters all its members in three launches); otherwise the
// filter is enqueued at once, behind the context's running work, so it overlaps it.  Either way
// the rule the caller sees depends on that switch alone, never on the context's history.
bool defer_filter(const imls_ctx* c) { return c->defer; }

int do_set_target(imls_ctx* c, const float* d_soa6, size_t n, size_t* n_kept) {
    if (n == 0 || n > (size_t)0x7fffffff) return fail(c, IMLS_ERR_ARG, "target size out of range");
    c->fifo_inc = false;
    if (!grow(c->tkept, n * 4 + 16)) return fail(c, IMLS_ERR_DEVICE, "hipMalloc (kept)");
    if (!c->ev_tgt && hipEventCreateWithFlags(&c->ev_tgt, hipEventDisableTiming) != hipSuccess)
        return fail(c, IMLS_ERR_DEVICE, "hipEventCreate");
    c->has_tensors = false;
    c->ten_pending = false;
    c->tgt_pending = false;
    c->tgt_filter_deferred = false;
    timed_begin(c, 1, c->tgt_slot);
    if (n_kept || !defer_filter(c)) {
        int rc = filter_async(c->stream, d_soa6, n, c->tpt, c->tnr, c->tscratch, (unsigned*)c->tkept.p, &c->h_cnt[0], c->err);
        if (rc) return rc;
    } else {
        c->tf_soa = d_soa6;                // filtered at first use (alone, or with a whole batch)
        c->tf_n = n;
        c->tgt_filter_deferred = true;
    }
    if (hipEventRecord(c->ev_tgt, c->stream) != hipSuccess) return fail(c, IMLS_ERR_DEVICE, "event record");
    c->n_target_in = n;
    c->tgt_pending = true;
    c->has_target = true;                 // provisional: the build decides (an all-NaN map has none)
    c->rnr_valid = false;
    c->has_corr = false;
    if (n_kept) {
        if (int rc2 = finish_target(c)) return rc2;
        *n_kept = (size_t)c->M;
    }
    return IMLS_OK;
}

int do_set_source(imls_ctx* c, const float* d_soa6, size_t n, size_t* n_kept, uint32_t* kept_index) {
    c->cap_iters = 0;                     // a new source drops the captured frame
    if (n == 0 || n > (size_t)0x7fffffff) return fail(c, IMLS_ERR_ARG, "source size out of range");
    if (kept_index && !grow(c->skept, n * 4)) return fail(c, IMLS_ERR_DEVICE, "hipMalloc (kept)");
    if (!c->ev_src && hipEventCreateWithFlags(&c->ev_src, hipEventDisableTiming) != hipSuccess)
        return fail(c, IMLS_ERR_DEVICE, "hipEventCreate");
    c->src_pending = false;
    c->src_filter_deferred = false;
    if (n_kept || kept_index || !defer_filter(c)) {
        int rc = filter_async(c->stream, d_soa6, n, c->spt, c->snr, c->sscratch, kept_index ? (unsigned*)c->skept.p : nullptr,
                              &c->h_cnt[1], c->err);
        if (rc) return rc;
    } else {
        c->sf_soa = d_soa6;
        c->sf_n = n;
        c->src_filter_deferred = true;
    }
    if (hipEventRecord(c->ev_src, c->stream) != hipSuccess) return fail(c, IMLS_ERR_DEVICE, "event record");
    c->src_pending = true;
    c->src_kept_out = kept_index;
    c->has_source = true;                 // provisional, as for the target
    c->has_corr = false;
    if (n_kept || kept_index) {
        if (int rc2 = finish_source(c)) return rc2;
        if (n_kept) *n_kept = (size_t)c->N;
    }
    return IMLS_OK;
}

// The target's tensors gathered to Morton order (needs the built target: its kept index and order).
int gather_tensors(imls_ctx* c, hipStream_t s, const float* d_ten6, size_t n) {
    if (!grow(c->mten, (size_t)std::max(c->M, 1) * 32)) return fail(c, IMLS_ERR_DEVICE, "hipMalloc (tensors)");
    launch_tensor_gather(s, d_ten6, n, (const unsigned*)c->tkept.p, (const float4*)c->mpt.p, c->M, (float4*)c->mten.p);
    if (hipGetLastError() != hipSuccess) return fail(c, IMLS_ERR_DEVICE, "tensor gather launch failed");
    return IMLS_OK;
}

// With the target build still pending (a count-less load) the gather waits for it too: it runs
// right after the build (alone, or with a batch's builds), reading d_ten6 then.
int do_set_tensors(imls_ctx* c, const float* d_ten6, size_t n) {
    if (!c->has_target) return fail(c, IMLS_ERR_STATE, "set_target first");
    // (the incremental FIFO index keeps no filtered → input index of the concatenation)
    if (c->fifo_inc) return fail(c, IMLS_ERR_UNSUPPORTED, "tensor inputs need a set_target map, not the FIFO index");
    if (n != c->n_target_in) return fail(c, IMLS_ERR_ARG, "tensor count must equal the last set_target's point count");
    if (c->tgt_pending) {
        c->ten_src = d_ten6;
        c->ten_n = n;
        c->ten_pending = true;
        c->has_tensors = true;
        return IMLS_OK;
    }
    if (!c->has_target) return fail(c, IMLS_ERR_STATE, "set_target first");
    if (int rc = gather_tensors(c, c->stream, d_ten6, n)) return rc;
    c->ten_pending = false;
    c->has_tensors = true;
    return IMLS_OK;
}

// tensor voting needs the target's tensors
int check_tv_ready(imls_ctx* c) {
    if (c->kp.tv && !c->has_tensors) return fail(c, IMLS_ERR_STATE, "use_tensor_voting: imls_set_target_tensors first");
    return IMLS_OK;
}

int check_device(imls_ctx* c) {
    hipError_t e = hipSetDevice(c->device);
    if (e != hipSuccess) return fail(c, IMLS_ERR_DEVICE, std::string("hipSetDevice: ") + hipGetErrorString(e));
    return IMLS_OK;
}

// One frame's prologue / epilogue as one launch each (round 4: the lone-frame latency paid ~11 µs
// for an H2D pose copy, five fills and four D2H copies around the 20 iterations).
__global__ void k_frame_init(double* __restrict__ pose, int* __restrict__ done, int* __restrict__ status,
                             int* __restrict__ iters, unsigned long long* __restrict__ trace, int trace_words,
                             unsigned long long* __restrict__ stats) {
    const int t = threadIdx.x;
    if (t < 16) pose[t] = (t % 5 == 0) ? 1.0 : 0.0;
    if (t < 4) { done[t] = 0; status[t] = 0; iters[t] = 0; }
    if (t < 16) stats[t] = 0ull;
    for (int k = t; k < trace_words; k += blockDim.x) trace[k] = 0ull;
}
// pose, iterations, status and the trace records written straight into the pinned host buffers
// (device-visible host memory; read by the host after the stream synchronisation)
__global__ void k_frame_results(const double* __restrict__ pose, const int* __restrict__ iters,
                                const int* __restrict__ status, const unsigned long long* __restrict__ trace,
                                int trace_words, double* __restrict__ h_misc, unsigned long long* __restrict__ h_trace) {
    const int t = threadIdx.x;
    if (t < 16) h_misc[t] = pose[t];
    if (t == 16) reinterpret_cast<int*>(h_misc + 16)[0] = *iters;
    if (t == 17) reinterpret_cast<int*>(h_misc + 18)[0] = *status;
    for (int k = t; k < trace_words; k += blockDim.x) h_trace[k] = trace[k];
}

}  // namespace

extern "C" {

int imls_abi_version(void) { return IMLS_GPU_ABI_VERSION; }

void imls_default_params(imls_params* p) {
    if (!p) return;
    std::memset(p, 0, sizeof(*p));
    // config.json shipped values (laser_odometry section)
    p->matching_method = IMLS_MATCH_IMLS;
    p->correspond_number = 6;
    p->h = 1.0;
    p->r = 3.0;
    p->get_normals = 1;
    p->search_number_normal = 10;
    p->r_normal = 1.0;
    p->use_projected_distance = 0;
    p->r_proj = 0.8;
    p->normal_angle_constraint = 1;
    p->angle_diff_threshold = 30.0;
    p->search_number = 20;
    p->use_tensor_voting = 0;
    p->tensor_k = 50;
    p->tensor_sigma = 0.2;
    p->tensor_distance_threshold = 0.6;
    p->picp_r = 1.5;
    p->picp_r_proj = 0.8;
    p->picp_angle_diff_threshold = 30.0;
    p->picp_use_projected_distance = 0;
    p->picp_normal_angle_constraint = 1;
    p->solve_method = IMLS_SOLVE_RANSAC;
    p->iterations = 30;
    p->delta_dist_threshold = 0.001;
    p->delta_angle_threshold = 0.0001745353;
    p->ls_threshold = 0.02;
    p->ransac_max_iterations = 5000;
    p->ransac_final_method = IMLS_FINAL_DRPM;
    p->ransac_distance_threshold = 0.8;
    p->ransac_min_inliers_percentage = 0.95;
    p->ransac_huber_threshold = 0.648;
    p->ransac_ls_threshold = 0.02;
    p->drpm_threshold = 0.05;
    p->drpm_stdev_points = 0.02;
    p->drpm_stdev_normals = 0.05;
    p->ransac_seed = 1;
    p->transform_normal = 0;
    p->max_queue_size = 1;
}

imls_ctx* imls_create(int device, const imls_params* p) {
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return nullptr;
    imls_ctx* c = new imls_ctx();
    c->device = device;
    if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&c->own, hipStreamNonBlocking) != hipSuccess) {
        delete c;
        return nullptr;
    }
    c->stream = c->own;
    register_stream(c->own, device);
    if (hipHostMalloc((void**)&c->h_misc, 32 * sizeof(double)) != hipSuccess ||
        // coherent: the NaN filter's compaction kernel writes the kept counts here directly
        hipHostMalloc((void**)&c->h_cnt, 4 * sizeof(int), hipHostMallocCoherent) != hipSuccess) {
        delete c;
        return nullptr;
    }
    imls_params d;
    imls_default_params(&d);
    d.solve_method = IMLS_SOLVE_LS;
    if (imls_set_params(c, p ? p : &d) != IMLS_OK) {
        imls_destroy(c);
        return nullptr;
    }
    return c;
}

void imls_destroy(imls_ctx* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->ustream) (void)hipStreamSynchronize(c->ustream);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    DevBuf* bufs[] = {&c->cap_mem, &c->front_mem, &c->sample_mem, &c->pca_mem, &c->tkept, &c->mten, &c->upload_ten, &c->tvn, &c->rnr, &c->ransac_mem, &c->rng, &c->lkeys, &c->tpt, &c->tnr, &c->mpt, &c->nodes, &c->tscratch, &c->treescratch, &c->permbuf, &c->qperm, &c->fb, &c->prevnn,
                      &c->upload_t, &c->spt, &c->snr, &c->sscratch,
                      &c->upload_s, &c->cs, &c->cd, &c->cn, &c->solve_mem, &c->trace_mem, &c->stats, &c->rows_d, &c->pose_tmp};
    for (DevBuf* b : bufs)
        if (b->p) (void)hipFree(b->p);
    for (auto* v : {&c->fifo}) for (auto& sl : *v) for (DevBuf* b : {&sl.buf, &sl.fpt, &sl.fnr, &sl.run}) if (b->p) (void)hipFree(b->p);
    for (auto& sl : c->slot_pool) for (DevBuf* b : {&sl.buf, &sl.fpt, &sl.fnr, &sl.run}) if (b->p) (void)hipFree(b->p);
    for (DevBuf* b : {&c->fifo_dev, &c->mkey[0], &c->mkey[1], &c->mval[0], &c->mval[1], &c->fscr}) if (b->p) (void)hipFree(b->p);
    if (c->h_fifo_cnt) (void)hipHostFree(c->h_fifo_cnt);
    if (c->h_fifo_clamp) (void)hipHostFree(c->h_fifo_clamp);
    if (c->ev_fifo) (void)hipEventDestroy(c->ev_fifo);
    if (c->macc.p) (void)hipFree(c->macc.p);
    if (c->skept.p) (void)hipFree(c->skept.p);
    for (hipEvent_t e : c->ev) (void)hipEventDestroy(e);
    if (c->h_trace) (void)hipHostFree(c->h_trace);
    if (c->h_misc) (void)hipHostFree(c->h_misc);
    if (c->h_rng) (void)hipHostFree(c->h_rng);
    if (c->ev_rng) (void)hipEventDestroy(c->ev_rng);
    if (c->tab_h) (void)hipHostFree(c->tab_h);
    if (c->h_cnt) (void)hipHostFree(c->h_cnt);
    for (int k = 0; k < 2; ++k) {
        if (c->h_stage[k]) (void)hipHostFree(c->h_stage[k]);
        if (c->ev_stage[k]) (void)hipEventDestroy(c->ev_stage[k]);
    }
    if (c->ev_tgt) (void)hipEventDestroy(c->ev_tgt);
    if (c->ev_src) (void)hipEventDestroy(c->ev_src);
    if (c->res_h) (void)hipHostFree(c->res_h);
    if (c->tab_d.p) (void)hipFree(c->tab_d.p);
    if (c->res_d.p) (void)hipFree(c->res_d.p);
    if (c->ev_batch) (void)hipEventDestroy(c->ev_batch);
    if (c->bscratch.p) (void)hipFree(c->bscratch.p);
    if (c->btable.p) (void)hipFree(c->btable.p);
    if (c->h_btable) (void)hipHostFree(c->h_btable);
    if (c->fscratch.p) (void)hipFree(c->fscratch.p);
    if (c->ftable.p) (void)hipFree(c->ftable.p);
    if (c->h_ftable) (void)hipHostFree(c->h_ftable);
    if (c->ev_build) (void)hipEventDestroy(c->ev_build);
    if (c->stream && c->stream != c->own) unregister_stream(c->stream);
    if (c->ustream) {
        unregister_stream(c->ustream);
        (void)hipStreamDestroy(c->ustream);
    }
    if (c->own) {
        unregister_stream(c->own);
        (void)hipStreamDestroy(c->own);
    }
    release_retired(c->device);
    delete c;
}

int imls_set_params(imls_ctx* c, const imls_params* p) {
    if (!c) return IMLS_ERR_ARG;
    int rc = check_params(c, p);
    if (rc) return rc;
    // the map FIFO's entries are held in the form of the mode they were pushed under (incremental
    // index: filtered points + sorted runs, device scans not copied; concatenation: raw SoA6 copies):
    // the mode may change only while the FIFO is empty
    auto inc_mode = [](int q) { return q >= 2 && q < kMaxFifoRuns; };
    if (c->rng_init && !c->fifo.empty() && inc_mode(c->P.max_queue_size) != inc_mode(p->max_queue_size))
        return fail(c, IMLS_ERR_STATE, "max_queue_size " + std::to_string(c->P.max_queue_size) + " -> " +
                                           std::to_string(p->max_queue_size) +
                                           " changes the map FIFO's index mode while it holds scans: imls_map_clear first");
    if (!c->rng_init || p->ransac_seed != c->P.ransac_seed) {   // creation, or a new seed: restart the stream
        c->rng_init = true;
        ransac_seed_host(p->ransac_seed, c->rng_seed_state);
        c->rng_dirty = true;
    }
    c->P = *p;
    c->kp = make_kparams(*p, c->opt);
    return IMLS_OK;
}

int imls_set_option(imls_ctx* c, int32_t option, double value) {
    if (!c) return IMLS_ERR_ARG;
    if (!std::isfinite(value)) return fail(c, IMLS_ERR_ARG, "option value must be finite");
    const int v = (int)value;
    const bool integral = (double)v == value;
    Options& o = c->opt;
    switch (option) {
    case IMLS_OPT_TRAVERSAL:
        if (!integral || v < IMLS_TRAVERSAL_AUTO || v > IMLS_TRAVERSAL_LANE) return fail(c, IMLS_ERR_ARG, "traversal: 0..3");
        o.traversal = v;
        break;
    case IMLS_OPT_LIST_REUSE:
        if (!integral || (v != 0 && v != 1)) return fail(c, IMLS_ERR_ARG, "list_reuse: 0 or 1");
        o.list_reuse = v;
        break;
    case IMLS_OPT_TEMPORAL_SEED:
        if (!integral || (v != 0 && v != 1)) return fail(c, IMLS_ERR_ARG, "temporal_seed: 0 or 1");
        o.temporal_seed = v;
        break;
    case IMLS_OPT_LEAF_SIZE:   // a leaf is one wave-wide load
        if (!integral || v < 4 || v > 64 || (v & (v - 1))) return fail(c, IMLS_ERR_ARG, "leaf_size: a power of two in [4, 64]");
        o.leaf_size = v;
        break;
    case IMLS_OPT_FIRST_PACKET:
        if (!integral || (v != 16 && v != 32 && v != 64)) return fail(c, IMLS_ERR_ARG, "first_packet: 16, 32 or 64");
        o.first_packet = v;
        break;
    case IMLS_OPT_FIRST_PACKET_ITERS:
        if (!integral || v < 0) return fail(c, IMLS_ERR_ARG, "first_packet_iters: >= 0");
        o.first_packet_iters = v;
        break;
    case IMLS_OPT_FIRST_PACKET_BATCHED:
        if (!integral || (v != 0 && v != 1)) return fail(c, IMLS_ERR_ARG, "first_packet_batched: 0 or 1");
        o.first_packet_batched = v;
        break;
    case IMLS_OPT_TV_SKIN:
        if (value < 0.0 || value > 1.0) return fail(c, IMLS_ERR_ARG, "tv_skin: [0, 1] m");
        o.tv_skin = value;
        break;
    case IMLS_OPT_FORCE_FALLBACK:
        if (!integral || v < 0) return fail(c, IMLS_ERR_ARG, "force_fallback: >= 0");
        o.force_fallback = v;
        break;
    default:
        return fail(c, IMLS_ERR_ARG, "unknown option");
    }
    c->B = o.leaf_size;                          // the next index build
    c->lane_mode = o.traversal == IMLS_TRAVERSAL_LANE;
    c->temporal_seed = o.temporal_seed;
    c->kp = make_kparams(c->P, o);
    return IMLS_OK;
}

int imls_get_option(imls_ctx* c, int32_t option, double* value) {
    if (!c || !value) return IMLS_ERR_ARG;
    const Options& o = c->opt;
    switch (option) {
    case IMLS_OPT_TRAVERSAL: *value = o.traversal; break;
    case IMLS_OPT_LIST_REUSE: *value = o.list_reuse; break;
    case IMLS_OPT_TEMPORAL_SEED: *value = o.temporal_seed; break;
    case IMLS_OPT_LEAF_SIZE: *value = o.leaf_size; break;
    case IMLS_OPT_FIRST_PACKET: *value = o.first_packet; break;
    case IMLS_OPT_FIRST_PACKET_ITERS: *value = o.first_packet_iters; break;
    case IMLS_OPT_FIRST_PACKET_BATCHED: *value = o.first_packet_batched; break;
    case IMLS_OPT_TV_SKIN: *value = o.tv_skin; break;
    case IMLS_OPT_FORCE_FALLBACK: *value = o.force_fallback; break;
    default: return fail(c, IMLS_ERR_ARG, "unknown option");
    }
    return IMLS_OK;
}

const char* imls_last_error(const imls_ctx* c) { return c ? c->err.c_str() : "null context"; }

int imls_seed_rng(imls_ctx* c, uint32_t seed) {
    if (!c) return IMLS_ERR_ARG;
    // the stream restarts; params.ransac_seed is left as set (contexts seeded differently still
    // batch together: frames_async compares the params without it)
    ransac_seed_host(seed, c->rng_seed_state);
    c->rng_dirty = true;
    return IMLS_OK;
}

int imls_get_rng_state(imls_ctx* c, int32_t state[34]) {
    if (!c || !state) return IMLS_ERR_ARG;
    if (c->rng_dirty || !c->rng.p) {                  // not on the device yet: the pending seed is the state
        std::memcpy(state, c->rng_seed_state, 34 * 4);
        return IMLS_OK;
    }
    if (int rc = check_device(c)) return rc;
    if (hipMemcpyAsync(state, c->rng.p, 34 * 4, hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
        hipStreamSynchronize(c->stream) != hipSuccess)
        return fail(c, IMLS_ERR_DEVICE, "rand state download");
    return IMLS_OK;
}

int imls_set_rng_state(imls_ctx* c, const int32_t state[34]) {
    if (!c || !state) return IMLS_ERR_ARG;
    const int f = state[31], r = state[32];
    if (f < 0 || f > 30 || r < 0 || r > 30 || (f - r + 31) % 31 != 3) return fail(c, IMLS_ERR_ARG, "not a glibc TYPE_3 rand() state");
    std::memcpy(c->rng_seed_state, state, 34 * 4);
    c->rng_dirty = true;
    return IMLS_OK;
}

int imls_set_stream(imls_ctx* c, void* s) {
    if (!c) return IMLS_ERR_ARG;
    hipStream_t ns = s ? (hipStream_t)s : c->own;
    if (ns != c->stream) {
        // a caller's stream joins the registry (its pending work may read this context's buffers)
        if (ns != c->own) register_stream(ns, c->device);
        if (c->stream != c->own) unregister_stream(c->stream);
    }
    c->stream = ns;
    return IMLS_OK;
}

int imls_synchronize(imls_ctx* c) {
    if (!c) return IMLS_ERR_ARG;
    return hipStreamSynchronize(c->stream) == hipSuccess ? IMLS_OK : fail(c, IMLS_ERR_DEVICE, "stream sync failed");
}

int imls_set_target(imls_ctx* c, const float* xyz, const float* nrm, size_t n, size_t stride, size_t* n_kept) {
    if (!c) return IMLS_ERR_ARG;
    if (int rc = check_device(c)) return rc;
    if (int rc = upload_soa6(c, c->upload_t, xyz, nrm, n, stride, 0)) return rc;
    return do_set_target(c, (const float*)c->upload_t.p, n, n_kept);
}

int imls_set_target_device(imls_ctx* c, const float* d_soa6, size_t n, size_t* n_kept) {
    if (!c || !d_soa6) return IMLS_ERR_ARG;
    if (int rc = check_device(c)) return rc;
    return do_set_target(c, d_soa6, n, n_kept);
}

// accumulateTargetCloud (laser_odometry.cpp:116-136) + setTargetPointCloud(accumulatedTargetCloud)
// (imls_icp.cpp:80-103): the new scan goes to a FIFO slot (`from_host`: packed + uploaded, the only
// PCIe traffic; else copied device-to-device), the oldest entry is dropped once when the FIFO holds
// more than max_queue_size (the reference's `if`, not a loop), the entries are concatenated oldest
// first into one SoA6 map in HBM (one 2-D device copy per entry) and the index is rebuilt over it.
namespace {
// ---- incremental FIFO index -----------------------------------------------------------------
// Used for max_queue_size 2 … kMaxFifoRuns − 1 (queue 1 indexes its one scan in place; a run id
// must be unique among the FIFO's entries).
bool fifo_incremental(const imls_ctx* c) { return c->P.max_queue_size >= 2 && c->P.max_queue_size < kMaxFifoRuns; }

int ensure_fifo(imls_ctx* c) {
    if (c->h_fifo_cnt) return IMLS_OK;
    if (hipHostMalloc((void**)&c->h_fifo_cnt, kMaxFifoRuns * sizeof(int), hipHostMallocCoherent) != hipSuccess ||
        // coherent: the FIFO gather kernel writes the clamp count here directly
        hipHostMalloc((void**)&c->h_fifo_clamp, 64, hipHostMallocCoherent) != hipSuccess)
        return fail(c, IMLS_ERR_DEVICE, "hipHostMalloc (FIFO)");
    *c->h_fifo_clamp = 0;
    if (!grow(c->fifo_dev, 256 + kMaxFifoRuns * sizeof(FifoRun))) return fail(c, IMLS_ERR_DEVICE, "hipMalloc (FIFO)");
    if (hipMemsetAsync(c->fifo_dev.p, 0, 256, c->stream) != hipSuccess) return fail(c, IMLS_ERR_DEVICE, "hipMemset (FIFO)");
    if (hipEventCreateWithFlags(&c->ev_fifo, hipEventDisableTiming) != hipSuccess) return fail(c, IMLS_ERR_DEVICE, "hipEventCreate");
    return IMLS_OK;
}
float* fifo_fq(imls_ctx* c) { return (float*)c->fifo_dev.p; }
unsigned* fifo_clamp(imls_ctx* c) { return (unsigned*)((char*)c->fifo_dev.p + 64); }

// the target is the FIFO's incremental index: pending until its first use (or at once with n_map)
int fifo_set_target(imls_ctx* c, size_t* n_map) {
    c->has_tensors = false;
    c->ten_pending = false;
    c->tgt_filter_deferred = false;
    c->has_corr = false;
    c->rnr_valid = false;
    if (c->map_points == 0) {             // empty map (max_queue_size 0 or empty scans): no target
        c->tgt_pending = false;
        c->has_target = false;
        c->fifo_inc = false;
        c->M = 0;
        if (n_map) *n_map = 0;
        return IMLS_OK;
    }
    if (!c->ev_tgt && hipEventCreateWithFlags(&c->ev_tgt, hipEventDisableTiming) != hipSuccess)
        return fail(c, IMLS_ERR_DEVICE, "hipEventCreate");
    if (c->tgt_slot < 0) timed_begin(c, 1, c->tgt_slot);
    if (hipEventRecord(c->ev_tgt, c->stream) != hipSuccess) return fail(c, IMLS_ERR_DEVICE, "event record");
    c->n_target_in = c->map_points;
    c->fifo_inc = true;
    c->tgt_pending = true;
    c->has_target = true;                 // provisional: the build decides (an all-NaN map has none)
    if (n_map) {
        if (int rc = finish_target(c)) return rc;
        *n_map = (size_t)c->M;
    }
    return IMLS_OK;
}

// The build: the kept counts (one wait for every pending filter), the frame (first build, or after
// a scan fell outside it), the runs not sorted yet, the merged order (drop evicted runs, merge the
// new ones after the kept ones: the FIFO is oldest first), the index from it.
int fifo_build(imls_ctx* c) {
    if (hipEventSynchronize(c->ev_tgt) != hipSuccess) return fail(c, IMLS_ERR_DEVICE, "map filter failed");
    c->stage_pending[0] = false;
    hipStream_t s = c->stream;
    size_t M = 0;
    for (auto& e : c->fifo) {
        if (e.nk < 0) e.nk = e.n ? c->h_fifo_cnt[e.id] : 0;
        M += (size_t)e.nk;
    }
    c->M = (int)M;
    c->has_target = M > 0;
    if (M == 0) {
        timed_end(c, 1, c->tgt_slot);
        c->tgt_slot = -1;
        return IMLS_OK;
    }
    if (M > (size_t)0x7fffffff) return fail(c, IMLS_ERR_CAPACITY, "map too large");
    {   // the build's scratch, before anything is enqueued (its steps never reallocate it)
        int max_run = 0, nruns = 0;
        for (auto& e : c->fifo) { max_run = std::max(max_run, e.nk); nruns += e.nk > 0; }
        if (!grow(c->fscr, fifo_scratch_bytes(max_run, nruns, (int)M))) return fail(c, IMLS_ERR_DEVICE, "hipMalloc (FIFO scratch)");
    }
    // re-frame when the last build's new scans fell outside the frame (their keys were clamped)
    if (c->fq_valid && *c->h_fifo_clamp != 0) c->fq_valid = false;
    if (!c->fq_valid) {
        // every entry's filtered points stay in its fpt / fnr while it is in the FIFO: re-key them all
        std::vector<std::pair<const float4*, int>> pts;
        for (auto& e : c->fifo)
            if (e.nk > 0) {
                pts.push_back({(const float4*)e.fpt.p, e.nk});
                e.sorted = false;
            }
        if (int rc = fifo_frame(s, pts, fifo_fq(c), c->fscr, c->err)) return rc;
        if (hipMemsetAsync(fifo_clamp(c), 0, 4, s) != hipSuccess) return fail(c, IMLS_ERR_DEVICE, "hipMemset (clamp)");
        c->merged_ids.clear();
        c->m_n = 0;
        c->fq_valid = true;
    }
    for (auto& e : c->fifo)
        if (e.nk > 0 && !e.sorted) {
            if (int rc = fifo_run_build(s, (const float4*)e.fpt.p, (const float4*)e.fnr.p, e.nk, fifo_fq(c), fifo_clamp(c), e.run,
                                        c->fscr, c->err))
                return rc;
            e.sorted = true;
        }
    // the merged order: its runs must be a prefix of the FIFO's (new runs are the newest) — else restart
    auto merged = [&](int id) { return std::find(c->merged_ids.begin(), c->merged_ids.end(), id) != c->merged_ids.end(); };
    bool seen_new = false, prefix = true;
    unsigned live = 0;
    int kept_n = 0;
    for (auto& e : c->fifo) {
        if (e.nk <= 0) continue;
        if (!merged(e.id)) { seen_new = true; continue; }
        if (seen_new) prefix = false;
        live |= 1u << e.id;
        kept_n += e.nk;
    }
    if (!prefix) { c->merged_ids.clear(); c->m_n = 0; live = 0; kept_n = 0; }
    // the current order's buffers keep their m_n entries when they grow (a plain grow drops them:
    // the merge would read stale run ids); the other pair is output only
    if (!grow_keep(c->mkey[c->mcur], M * 8 + 64, (size_t)c->m_n * 8, s) ||
        !grow_keep(c->mval[c->mcur], M * 4 + 64, (size_t)c->m_n * 4, s) || !grow(c->mkey[c->mcur ^ 1], M * 8 + 64) ||
        !grow(c->mval[c->mcur ^ 1], M * 4 + 64))
        return fail(c, IMLS_ERR_DEVICE, "hipMalloc (FIFO order)");
    auto K = [&](int k) { return (unsigned long long*)c->mkey[k].p; };
    auto V = [&](int k) { return (unsigned*)c->mval[k].p; };
    if (c->m_n > 0 && kept_n != c->m_n) {            // evicted runs: stable compaction
        if (int rc = fifo_keep(s, K(c->mcur), V(c->mcur), c->m_n, live, K(c->mcur ^ 1), V(c->mcur ^ 1), c->fscr, c->err)) return rc;
        c->mcur ^= 1;
    }
    c->m_n = c->m_n > 0 ? kept_n : 0;
    std::vector<int> ids;
    for (auto& e : c->fifo)
        if (e.nk > 0 && (live >> e.id & 1u)) ids.push_back(e.id);
    for (auto& e : c->fifo) {
        if (e.nk <= 0 || (live >> e.id & 1u)) continue;
        if (int rc = fifo_merge(s, K(c->mcur), V(c->mcur), c->m_n, fifo_run_keys(e.run.p, e.nk), (unsigned)e.id, e.nk,
                                K(c->mcur ^ 1), V(c->mcur ^ 1), c->fscr, c->err))
            return rc;
        c->mcur ^= 1;
        c->m_n += e.nk;
        ids.push_back(e.id);
    }
    c->merged_ids = ids;
    // run table (by value in the gather launch): each run's records and its offset in the
    // concatenation (the libnabo tie order)
    FifoRunTable rt{};
    unsigned off = 0;
    for (auto& e : c->fifo) {
        if (e.nk <= 0) continue;
        rt.r[e.id] = FifoRun{fifo_run_pts(e.run.p, e.nk), fifo_run_nrm(e.run.p, e.nk), off, 0u};
        off += (unsigned)e.nk;
    }
    // the gather also copies this build's clamp count into the host's coherent word, read at the next
    // build (after its wait for the map filter, which this stream runs after the gather)
    int rc = fifo_index(s, K(c->mcur), V(c->mcur), c->M, rt, fifo_fq(c), fifo_clamp(c), c->h_fifo_clamp, c->B, c->lkeys,
                        c->mpt, c->nodes, c->treescratch, &c->Pl, &c->levels, c->err);
    if (rc) return rc;
    (void)hipEventRecord(c->ev_fifo, s);
    timed_end(c, 1, c->tgt_slot);
    c->tgt_slot = -1;
    return IMLS_OK;
}

}  // namespace

static int map_push(imls_ctx* c, const float* xyz, const float* nrm, size_t n, size_t stride, const float* d_soa6,
                    size_t* n_map) {
    if (n > (size_t)0x7fffffff) return fail(c, IMLS_ERR_ARG, "scan too large");
    // max_queue_size 1 with a device scan (the shipped config, device frames): the map IS this
    // scan, dropped at the next push — index it where it lies (its NaN filter reads it on this
    // stream, as the slot copy would), no FIFO copy
    if (d_soa6 && c->P.max_queue_size == 1) {
        for (auto& e : c->fifo)
            if (!e.ghost) c->slot_pool.push_back(e);
        c->fifo.clear();
        c->merged_ids.clear();
        c->m_n = 0;
        imls_ctx::MapSlot ghost;          // bookkeeping only: its data stays with the caller
        ghost.n = n;
        ghost.ghost = true;
        c->fifo.push_back(ghost);
        c->map_points = n;
        if (n == 0) {
            c->tgt_pending = false;
            c->has_target = false;
            c->has_corr = false;
            c->M = 0;
            if (n_map) *n_map = 0;
            return IMLS_OK;
        }
        return do_set_target(c, d_soa6, n, n_map);
    }
    imls_ctx::MapSlot sl;
    if (!c->slot_pool.empty()) { sl = c->slot_pool.back(); c->slot_pool.pop_back(); }
    sl.n = n;
    sl.ghost = false;
    sl.nk = -1;
    sl.sorted = false;
    const bool inc = fifo_incremental(c);
    sl.id = -1;                           // a pooled slot's run id / run belong to its last use
    if (inc) {
        for (const auto& e : c->fifo)     // a scan indexed in place (max_queue_size was 1) is not held
            if (e.ghost && e.n > 0) return fail(c, IMLS_ERR_STATE, "map FIFO holds a scan pushed with max_queue_size 1 (not kept): push again");
        sl.id = (int)(c->fifo_seq++ % kMaxFifoRuns);
        // an id is reused after kMaxFifoRuns pushes: if the merged order still holds its old run
        // (that many pushes without a build), the merged order restarts from the runs
        if (std::find(c->merged_ids.begin(), c->merged_ids.end(), sl.id) != c->merged_ids.end()) {
            c->merged_ids.clear();
            c->m_n = 0;
        }
    }
    if (n > 0) {
        int rc = IMLS_OK;
        const float* raw = d_soa6;
        if (!d_soa6 || !inc) {            // the incremental index filters a device scan where it lies
            if (!grow(sl.buf, n * 24)) { c->slot_pool.push_back(sl); return fail(c, IMLS_ERR_DEVICE, "hipMalloc (map slot)"); }
            if (d_soa6) {
                if (hipMemcpyAsync(sl.buf.p, d_soa6, n * 24, hipMemcpyDeviceToDevice, c->stream) != hipSuccess)
                    rc = fail(c, IMLS_ERR_DEVICE, "map slot copy");
            } else {
                rc = upload_soa6(c, sl.buf, xyz, nrm, n, stride, 0);
            }
            raw = (const float*)sl.buf.p;
        }
        // incremental: this scan's NaN filter now, on the stream (its kept count into the pinned word
        // of its run id); its run is sorted at the next build
        if (!rc && inc && (rc = ensure_fifo(c)) == IMLS_OK)
            rc = filter_async(c->stream, raw, n, sl.fpt, sl.fnr, c->tscratch, nullptr, &c->h_fifo_cnt[sl.id], c->err);
        if (rc) { c->slot_pool.push_back(sl); return rc; }
    }
    c->fifo.push_back(sl);
    c->map_points += n;
    if (c->fifo.size() > (size_t)std::max(c->P.max_queue_size, 0)) {
        c->map_points -= c->fifo.front().n;
        if (!c->fifo.front().ghost) c->slot_pool.push_back(c->fifo.front());
        c->fifo.pop_front();
    }
    if (inc) return fifo_set_target(c, n_map);
    for (const auto& e : c->fifo)     // a scan indexed in place (max_queue_size was 1) is not held
        if (e.ghost && e.n > 0) return fail(c, IMLS_ERR_STATE, "map FIFO holds a scan pushed with max_queue_size 1 (not kept): push again");
    const size_t M = c->map_points;
    if (M == 0) {                     // empty map (max_queue_size 0 or empty scans): no target
        c->tgt_pending = false;
        c->has_target = false;
        c->has_corr = false;
        c->M = 0;
        if (n_map) *n_map = 0;
        return IMLS_OK;
    }
    for (const auto& e : c->fifo)     // one non-empty entry (max_queue_size 1): index it in place
        if (e.n == M) return do_set_target(c, (const float*)e.buf.p, M, n_map);
    if (!grow(c->macc, M * 24)) return fail(c, IMLS_ERR_DEVICE, "hipMalloc (map)");
    size_t off = 0;
    for (const auto& e : c->fifo) {
        if (e.n == 0) continue;
        if (hipMemcpy2DAsync((float*)c->macc.p + off, M * 4, e.buf.p, e.n * 4, e.n * 4, 6, hipMemcpyDeviceToDevice,
                             c->stream) != hipSuccess)
            return fail(c, IMLS_ERR_DEVICE, "map assembly copy");
        off += e.n;
    }
    return do_set_target(c, (const float*)c->macc.p, M, n_map);
}

int imls_map_push(imls_ctx* c, const float* xyz, const float* nrm, size_t n, size_t stride, size_t* n_map) {
    if (!c) return IMLS_ERR_ARG;
    if (n > 0 && (!xyz || !nrm || stride < 3)) return fail(c, IMLS_ERR_ARG, "bad cloud pointer/stride");
    if (int rc = check_device(c)) return rc;
    return map_push(c, xyz, nrm, n, stride, nullptr, n_map);
}

int imls_map_push_device(imls_ctx* c, const float* d_soa6, size_t n, size_t* n_map) {
    if (!c || (n > 0 && !d_soa6)) return IMLS_ERR_ARG;
    if (int rc = check_device(c)) return rc;
    return map_push(c, nullptr, nullptr, n, 0, d_soa6, n_map);
}

int imls_map_clear(imls_ctx* c) {
    if (!c) return IMLS_ERR_ARG;
    for (auto& e : c->fifo)
        if (!e.ghost) c->slot_pool.push_back(e);
    c->fifo.clear();
    c->map_points = 0;
    c->merged_ids.clear();
    c->m_n = 0;
    c->fq_valid = false;
    return IMLS_OK;
}

int imls_map_size(imls_ctx* c, size_t* entries, size_t* points) {
    if (!c) return IMLS_ERR_ARG;
    if (entries) *entries = c->fifo.size();
    if (points) *points = c->map_points;
    return IMLS_OK;
}

int imls_set_target_tensors(imls_ctx* c, const float* tens, size_t n, size_t stride) {
    if (!c || !tens || n == 0 || stride < 6) return fail(c, IMLS_ERR_ARG, "bad tensor pointer/size/stride");
    if (int rc = check_device(c)) return rc;
    std::vector<float> h(6 * n);
    for (size_t i = 0; i < n; ++i)
        for (int k = 0; k < 6; ++k) h[(size_t)k * n + i] = tens[i * stride + k];
    if (!grow(c->upload_ten, h.size() * 4)) return fail(c, IMLS_ERR_DEVICE, "hipMalloc (upload)");
    if (hipMemcpyAsync(c->upload_ten.p, h.data(), h.size() * 4, hipMemcpyHostToDevice, c->stream) != hipSuccess)
        return fail(c, IMLS_ERR_DEVICE, "tensor upload failed");
    int rc = do_set_tensors(c, (const float*)c->upload_ten.p, n);
    if (rc) return rc;
    return hipStreamSynchronize(c->stream) == hipSuccess ? IMLS_OK : fail(c, IMLS_ERR_DEVICE, "tensor upload failed");
}

int imls_set_target_tensors_device(imls_ctx* c, const float* d_ten6, size_t n) {
    if (!c || !d_ten6) return IMLS_ERR_ARG;
    if (int rc = check_device(c)) return rc;
    return do_set_tensors(c, d_ten6, n);
}

void imls_tv_encode_pca(const float* evals, const float* evecs, size_t n, int32_t k, float* out) {
    // CustomTensorVoting::myCustomFunctionWithEigen (scan_registration.cpp:358-381), float arithmetic
    const float kf = (float)k;
    for (size_t i = 0; i < n; ++i) {
        const float a0 = std::fabs(evals[3 * i]), a1 = std::fabs(evals[3 * i + 1]), a2 = std::fabs(evals[3 * i + 2]);
        const float l1 = std::max(a0, std::max(a1, a2));
        const float l3 = std::min(a0, std::min(a1, a2));
        const float l2 = ((a0 + a1) + a2) - (l1 + l3);
        const float* e = evecs + 9 * i;           // columns: e1 = e[0..2] (stick tail), e2 = e[3..5] (plate tail)
        float T[6];
        if (l1 >= l2 && l2 >= l3) {
            const float s1 = (l1 - l2) / kf, s3 = l3 / kf;
            const int rr[6] = {0, 0, 0, 1, 1, 2}, cc[6] = {0, 1, 2, 1, 2, 2};
            for (int m = 0; m < 6; ++m) {
                const float S = e[rr[m]] * e[cc[m]];
                const float Pm = S + e[3 + rr[m]] * e[3 + cc[m]];
                T[m] = s1 * S + s3 * Pm;
            }
        } else {
            T[0] = 1.f; T[1] = 0.f; T[2] = 0.f; T[3] = 1.f; T[4] = 0.f; T[5] = 1.f;   // unit ball (377-380)
        }
        for (int m = 0; m < 6; ++m) out[6 * i + m] = T[m];
    }
}

int imls_set_source(imls_ctx* c, const float* xyz, const float* nrm, size_t n, size_t stride, size_t* n_kept,
                    uint32_t* kept_index) {
    if (!c) return IMLS_ERR_ARG;
    if (int rc = check_device(c)) return rc;
    if (int rc = upload_soa6(c, c->upload_s, xyz, nrm, n, stride, 1)) return rc;
    return do_set_source(c, (const float*)c->upload_s.p, n, n_kept, kept_index);
}

int imls_set_source_device(imls_ctx* c, const float* d_soa6, size_t n, size_t* n_kept) {
    if (!c || !d_soa6) return IMLS_ERR_ARG;
    if (int rc = check_device(c)) return rc;
    return do_set_source(c, d_soa6, n, n_kept, nullptr);
}

int imls_project(imls_ctx* c, const double pose[16], float* x_out, float* y_out, float* n_out, uint32_t* src_index_out,
                 size_t* n_valid, uint64_t reject[IMLS_NUM_REJ]) {
    if (!c || !pose) return IMLS_ERR_ARG;
    if (int rc = check_device(c)) return rc;
    if (int rc = ensure_built(c)) return rc;
    if (!c->has_target || !c->has_source) return fail(c, IMLS_ERR_STATE, "set_target and set_source first");
    if (int rc = ensure_solve(c, c->N)) return rc;
    if (int rc = check_tv_ready(c)) return rc;
    if (int rc = ensure_map_normals(c)) return rc;
    if (!grow(c->pose_tmp, 32 * 8) || !grow(c->stats, 128)) return fail(c, IMLS_ERR_DEVICE, "hipMalloc");
    double* dpose = (double*)c->pose_tmp.p;
    int* dzero = (int*)(dpose + 16);
    hipMemcpyAsync(dpose, pose, 16 * 8, hipMemcpyHostToDevice, c->stream);
    hipMemsetAsync(dzero, 0, 16, c->stream);
    hipMemsetAsync(c->st.trace, 0, sizeof(imls_iter_trace), c->stream);
    hipMemsetAsync(c->stats.p, 0, 128, c->stream);
    int slot;
    hipEvent_t marks[3];
    timed_begin(c, 0, slot);
    launch_project(c->stream, tree_view(c), (const float4*)c->spt.p, (const float4*)c->snr.p, (const unsigned*)c->qperm.p,
                   c->N, dpose, dzero, c->kp, (float4*)c->cs.p, (float4*)c->cd.p, (float4*)c->cn.p, c->st.partial1,
                   c->st.trace, stats_ptr(c), fb_list(c), fb_count(c), c->lane_mode,
                   nullptr, (int*)c->prevnn.p, 0, project_marks(c, marks));
    timed_end(c, 0, slot);
    std::vector<float> hs((size_t)c->N * 4), hd((size_t)c->N * 4), hn((size_t)c->N * 4);
    imls_iter_trace tr;
    hipMemcpyAsync(hs.data(), c->cs.p, hs.size() * 4, hipMemcpyDeviceToHost, c->stream);
    hipMemcpyAsync(hd.data(), c->cd.p, hd.size() * 4, hipMemcpyDeviceToHost, c->stream);
    hipMemcpyAsync(hn.data(), c->cn.p, hn.size() * 4, hipMemcpyDeviceToHost, c->stream);
    hipMemcpyAsync(&tr, c->st.trace, sizeof(tr), hipMemcpyDeviceToHost, c->stream);
    if (hipStreamSynchronize(c->stream) != hipSuccess) return fail(c, IMLS_ERR_DEVICE, std::string("project: ") + hipGetErrorString(hipGetLastError()));
    harvest_timing(c);
    size_t k = 0;
    for (int i = 0; i < c->N; ++i) {
        if (hs[4 * i + 3] == 0.f) continue;
        for (int d = 0; d < 3; ++d) {
            if (x_out) x_out[3 * k + d] = hs[4 * i + d];
            if (y_out) y_out[3 * k + d] = hd[4 * i + d];
            if (n_out) n_out[3 * k + d] = hn[4 * i + d];
        }
        if (src_index_out) src_index_out[k] = (uint32_t)i;
        ++k;
    }
    if (n_valid) *n_valid = k;
    if (reject) std::memcpy(reject, tr.reject, sizeof(tr.reject));
    c->has_corr = true;
    return IMLS_OK;
}

int imls_solve(imls_ctx* c, double delta_out[16], int* ok) {
    if (!c || !delta_out) return IMLS_ERR_ARG;
    if (!c->has_corr) return fail(c, IMLS_ERR_STATE, "imls_project first");
    if (int rc = check_device(c)) return rc;
    hipMemsetAsync(c->st.done, 0, 16, c->stream);
    hipMemsetAsync(c->st.status, 0, 16, c->stream);
    if (int rc = prepare_ransac(c, c->N)) return rc;
    int slot;
    timed_begin(c, 2, slot);
    launch_solve(c->stream, solve_launch(c, nullptr, 0));
    timed_end(c, 2, slot);
    int status = 0;
    hipMemcpyAsync(delta_out, c->st.delta, 16 * 8, hipMemcpyDeviceToHost, c->stream);
    hipMemcpyAsync(&status, c->st.status, sizeof(int), hipMemcpyDeviceToHost, c->stream);
    if (hipStreamSynchronize(c->stream) != hipSuccess) return fail(c, IMLS_ERR_DEVICE, "solve failed");
    harvest_timing(c);
    if (ok) *ok = status == IMLS_FRAME_SOLVE_FAILED ? 0 : 1;
    return IMLS_OK;
}

int imls_solve_correspondences(imls_ctx* c, int32_t method, const double* s, const double* d, const double* n,
                               const double* w, size_t N, double delta_out[16], int* ok) {
    if (!c || !s || !d || !n || !delta_out) return IMLS_ERR_ARG;
    if (method != IMLS_SOLVE_LS && method != IMLS_SOLVE_WEIGHTED_LS && method != IMLS_SOLVE_RANSAC &&
        method != IMLS_SOLVE_DRPM)
        return fail(c, IMLS_ERR_UNSUPPORTED, "method");
    if (N > (size_t)0x3fffffff) return fail(c, IMLS_ERR_ARG, "N too large");
    if (int rc = check_device(c)) return rc;
    if (int rc = ensure_solve(c, (int)std::max<size_t>(N, 1))) return rc;
    size_t bytes = (9 * N + N) * 8 + 64;
    if (!grow(c->rows_d, bytes)) return fail(c, IMLS_ERR_DEVICE, "hipMalloc (rows)");
    double* r = (double*)c->rows_d.p;
    hipMemcpyAsync(r, s, 3 * N * 8, hipMemcpyHostToDevice, c->stream);
    hipMemcpyAsync(r + 3 * N, d, 3 * N * 8, hipMemcpyHostToDevice, c->stream);
    hipMemcpyAsync(r + 6 * N, n, 3 * N * 8, hipMemcpyHostToDevice, c->stream);
    const double* dw = nullptr;
    if (w) {
        hipMemcpyAsync(r + 9 * N, w, N * 8, hipMemcpyHostToDevice, c->stream);
        dw = r + 9 * N;
    }
    hipMemsetAsync(c->st.done, 0, 16, c->stream);
    hipMemsetAsync(c->st.status, 0, 16, c->stream);
    const int saved = c->P.solve_method;
    c->P.solve_method = method;
    const int rc0 = prepare_ransac(c, (int)std::max<size_t>(N, 1));
    c->P.solve_method = saved;
    if (rc0) return rc0;
    if (method == IMLS_SOLVE_DRPM && !grow(c->ransac_mem, ransac_bytes((int)std::max<size_t>(N, 1))))
        return fail(c, IMLS_ERR_DEVICE, "hipMalloc (DRPM)");
    SolveLaunch L = solve_launch(c, nullptr, 0);
    L.N = (int)N;
    L.blocks1 = 0;
    L.kp.solve_method = method;
    L.cs = L.cd = L.cn = nullptr;
    L.rows_d = r;
    L.weights = dw;
    L.rows_are_double = 1;
    launch_solve(c->stream, L);
    int status = 0;
    hipMemcpyAsync(delta_out, c->st.delta, 16 * 8, hipMemcpyDeviceToHost, c->stream);
    hipMemcpyAsync(&status, c->st.status, sizeof(int), hipMemcpyDeviceToHost, c->stream);
    if (hipStreamSynchronize(c->stream) != hipSuccess) return fail(c, IMLS_ERR_DEVICE, "solve failed");
    if (ok) *ok = status == IMLS_FRAME_SOLVE_FAILED ? 0 : 1;
    return IMLS_OK;
}

int imls_register_frame_async(imls_ctx* c) {
    if (!c) return IMLS_ERR_ARG;
    if (c->batch_member) return fail(c, IMLS_ERR_STATE, "the context is part of a pending batch");
    if (int rc = check_device(c)) return rc;
    if (int rc = ensure_built(c)) return rc;
    if (!c->has_target || !c->has_source) return fail(c, IMLS_ERR_STATE, "set_target and set_source first");
    if (int rc = ensure_solve(c, c->N)) return rc;
    if (int rc = check_tv_ready(c)) return rc;
    const int iters = c->P.iterations;
    if (int rc = ensure_trace(c, iters)) return rc;
    if (!grow(c->stats, 128)) return fail(c, IMLS_ERR_DEVICE, "hipMalloc");
    const int trace_words = std::max(iters, 1) * (int)(sizeof(imls_iter_trace) / 8);
    k_frame_init<<<1, 256, 0, c->stream>>>(c->st.pose, c->st.done, c->st.status, c->st.iters,
                                           (unsigned long long*)c->trace_mem.p, trace_words,
                                           (unsigned long long*)c->stats.p);
    imls_iter_trace* tr = (imls_iter_trace*)c->trace_mem.p;
    if (int rc = ensure_map_normals(c)) return rc;
    const TreeView tv = tree_view(c);
    if (int rc = prepare_ransac(c, c->N)) return rc;
    c->cap_iters = 0;
    c->cap_run = -1;
    if (c->capture && iters > 0) {
        if (!grow(c->cap_mem, (size_t)iters * c->N * 48)) return fail(c, IMLS_ERR_DEVICE, "hipMalloc (capture)");
        c->cap_iters = iters;
        c->cap_N = c->N;
    }
    for (int it = 0; it < iters; ++it) {
        int slot;
        hipEvent_t marks[3];
        timed_begin(c, 0, slot);
        launch_project(c->stream, tv, (const float4*)c->spt.p, (const float4*)c->snr.p, (const unsigned*)c->qperm.p, c->N,
                       c->st.pose, c->st.done, kp_at(c->kp, it), (float4*)c->cs.p, (float4*)c->cd.p, (float4*)c->cn.p,
                       c->st.partial1, tr + it, stats_ptr(c), fb_list(c), fb_count(c), c->lane_mode,
                       c->st.delta, (int*)c->prevnn.p, it > 0 && c->temporal_seed, project_marks(c, marks));
        timed_end(c, 0, slot);
        if (c->cap_iters) {   // this iteration's correspondences (stale, and never read, once the frame stopped)
            char* dst = (char*)c->cap_mem.p + (size_t)it * c->N * 48;
            const size_t nb = (size_t)c->N * 16;
            if (hipMemcpyAsync(dst, c->cs.p, nb, hipMemcpyDeviceToDevice, c->stream) != hipSuccess ||
                hipMemcpyAsync(dst + nb, c->cd.p, nb, hipMemcpyDeviceToDevice, c->stream) != hipSuccess ||
                hipMemcpyAsync(dst + 2 * nb, c->cn.p, nb, hipMemcpyDeviceToDevice, c->stream) != hipSuccess) {
                c->cap_iters = 0;
                return fail(c, IMLS_ERR_DEVICE, "capture copy");
            }
        }
        timed_begin(c, 2, slot);
        launch_solve(c->stream, solve_launch(c, tr + it, 1));
        timed_end(c, 2, slot);
    }
    k_frame_results<<<1, 256, 0, c->stream>>>(c->st.pose, c->st.iters, c->st.status, (const unsigned long long*)tr,
                                              iters * (int)(sizeof(imls_iter_trace) / 8), c->h_misc,
                                              (unsigned long long*)c->h_trace);
    if (hipGetLastError() != hipSuccess) return fail(c, IMLS_ERR_DEVICE, "launch failed");
    c->pending = true;
    c->pending_iters = iters;
    c->has_corr = true;
    return IMLS_OK;
}

int imls_register_frame_result(imls_ctx* c, double pose_out[16], int* iters_run, int* status, imls_iter_trace* trace) {
    if (!c) return IMLS_ERR_ARG;
    if (!c->pending) return fail(c, IMLS_ERR_STATE, "no frame pending");
    c->pending = false;
    hipError_t e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) return fail(c, IMLS_ERR_DEVICE, std::string("frame failed: ") + hipGetErrorString(e));
    harvest_timing(c);
    const int* misc = (const int*)(c->h_misc + 16);     // iters (pinned, copied by register_frame_async)
    const int st = *(const int*)(c->h_misc + 18);       // status
    if (pose_out) std::memcpy(pose_out, c->h_misc, 16 * 8);
    if (iters_run) *iters_run = misc[0];
    if (status) *status = st;
    if (c->cap_iters) c->cap_run = misc[0];
    if (trace && c->pending_iters > 0) std::memcpy(trace, c->h_trace, (size_t)c->pending_iters * sizeof(imls_iter_trace));
    return IMLS_OK;
}

int imls_register_frame(imls_ctx* c, double pose_out[16], int* iters_run, int* status, imls_iter_trace* trace) {
    int rc = imls_register_frame_async(c);
    if (rc) return rc;
    return imls_register_frame_result(c, pose_out, iters_run, status, trace);
}

}  // extern "C"

// ------------------------------------------------------------------------------------------------
// Batched registration (imls_register_frames*): the frames loaded into n contexts run through ONE
// launch sequence — every per-iteration kernel once for all frames (grid y = frame) — on the lead
// context's stream, so n small frames fill the GPU together instead of n queues of tiny launches.
// ------------------------------------------------------------------------------------------------
namespace {

constexpr int kResStride = 20;   // per frame: pose[16], iters, status

// rPose = I, done / status / iters = 0, the frame's trace and counters cleared (one launch for the
// whole batch instead of six fills per frame)
__global__ void k_batch_init(const PairDev* __restrict__ tab, int iters) {
    const PairDev A = tab[blockIdx.x];
    const int t = threadIdx.x;
    if (t < 16) A.st.pose[t] = (t % 5 == 0) ? 1.0 : 0.0;
    if (t == 0) { *A.st.done = 0; *A.st.status = 0; *A.st.iters = 0; }
    if (A.stats && t < 16) A.stats[t] = 0ull;
    unsigned long long* tr = reinterpret_cast<unsigned long long*>(A.trace);
    const int words = iters * (int)(sizeof(imls_iter_trace) / 8);
    for (int k = t; k < words; k += blockDim.x) tr[k] = 0ull;
}

// per frame: pose, iterations, status ([n][kResStride]), then every frame's trace records gathered
// after them ([n][iters] records) — one device-to-host copy for the whole batch
__global__ void k_batch_results(const PairDev* __restrict__ tab, int n, double* __restrict__ out, int iters) {
    const int words = iters * (int)(sizeof(imls_iter_trace) / 8);
    unsigned long long* tout = reinterpret_cast<unsigned long long*>(out + (size_t)n * kResStride);
    for (int k = blockIdx.x; k < n; k += gridDim.x) {
        const PairDev A = tab[k];
        const int t = threadIdx.x;
        if (t < 16) out[(size_t)k * kResStride + t] = A.st.pose[t];
        if (t == 16) out[(size_t)k * kResStride + 16] = (double)*A.st.iters;
        if (t == 17) out[(size_t)k * kResStride + 17] = (double)*A.st.status;
        const unsigned long long* tr = reinterpret_cast<const unsigned long long*>(A.trace);
        for (int w = t; w < words; w += blockDim.x) tout[(size_t)k * words + w] = tr[w];
    }
}

// The batched path covers both matchers (tensor-voting normals included) with the LS-family solvers
// and RANSAC (+ its LS / weighted LS / DRPM final solve); the projected-distance rule and the exact
// per-lane mode keep one launch sequence per frame (each on its own context stream, so they still
// overlap).
bool batch_fusable(const imls_ctx* c) {
    return !c->lane_mode && !c->kp.proj &&
           (c->P.solve_method == IMLS_SOLVE_LS || c->P.solve_method == IMLS_SOLVE_WEIGHTED_LS ||
            c->P.solve_method == IMLS_SOLVE_RANSAC);
}

PairDev pair_dev(imls_ctx* c) {
    PairDev A{};
    A.t = tree_view(c);
    A.spt = (const float4*)c->spt.p;
    A.snr = (const float4*)c->snr.p;
    A.qperm = (const unsigned*)c->qperm.p;
    A.N = c->N;
    A.cs = (float4*)c->cs.p;
    A.cd = (float4*)c->cd.p;
    A.cn = (float4*)c->cn.p;
    A.lists = (int*)c->prevnn.p;
    A.st = c->st;
    A.trace = (imls_iter_trace*)c->trace_mem.p;
    A.stats = stats_ptr(c);
    A.fb_list = fb_list(c);
    A.fb_count = fb_count(c);
    if (c->P.solve_method == IMLS_SOLVE_RANSAC) A.rf = ransac_frame(c->ransac_mem.p, c->N, (int*)c->rng.p);
    return A;
}

int frames_async(imls_ctx* const* ctxs, size_t n) {
    if (!ctxs || n == 0 || !ctxs[0]) return IMLS_ERR_ARG;
    HostSplit hs;
    imls_ctx* L = ctxs[0];
    if (L->batch_pending) return fail(L, IMLS_ERR_STATE, "a batch led by this context is pending");
    if (int rc = check_device(L)) return rc;
    for (size_t k = 0; k < n; ++k) {
        imls_ctx* c = ctxs[k];
        if (!c) return fail(L, IMLS_ERR_ARG, "null context in the batch");
        c->cap_iters = 0;                 // batched frames capture nothing: drop an older capture
        if (c->device != L->device) return fail(L, IMLS_ERR_ARG, "batch contexts must share one device");
        imls_params pc = c->P, pl = L->P;
        pc.ransac_seed = pl.ransac_seed = 0;    // each context runs its own rand() stream
        if (std::memcmp(&pc, &pl, sizeof(imls_params)) != 0)
            return fail(L, IMLS_ERR_ARG, "batch contexts must share their params (context " + std::to_string(k) + ")");
        if (!same_options(c->opt, L->opt))
            return fail(L, IMLS_ERR_ARG, "batch contexts must share their options (imls_set_option)");
        if (c->pending || c->batch_member || (k > 0 && c->batch_pending))
            return fail(L, IMLS_ERR_STATE, "context " + std::to_string(k) + " has a frame pending");
    }
    {   // no context twice (sorted copy: O(n log n) for batches of thousands of frames)
        std::vector<imls_ctx*> sorted(ctxs, ctxs + n);
        std::sort(sorted.begin(), sorted.end());
        if (std::adjacent_find(sorted.begin(), sorted.end()) != sorted.end())
            return fail(L, IMLS_ERR_ARG, "a context appears twice in the batch");
    }
    // every member's deferred build: its filter count (one wait each, all filters already enqueued)
    // then all the members' index builds in one launch sequence on the lead's stream
    hs.mark("checks");
    bool fuse = batch_fusable(L) && (L->P.solve_method != IMLS_SOLVE_RANSAC || n <= (size_t)kMaxRansacBatch);
    if (int rc = batch_builds(L, ctxs, n, fuse, &hs))
        return rc;
    // a batch of ONE small frame takes the single-frame launches — the lone-frame path with the exact
    // stage fused into the wave-per-query traversal (two launches per ICP iteration, not three; the
    // same results): the 2000-query config B variant 1450 → 1835 pairs/s (profiles/r05_ab/r05n_q).
    // A large frame keeps the table-driven kernels, measured faster in flight (435-445 vs 430-433
    // pairs/s on config B, though each launch alone is slower: profiles/r05_ab/r05n)
    if (n == 1 && L->has_source && L->N <= kSmallRows && (L->kp.qwave > 0 || (L->kp.qwave < 0 && L->N <= kQwaveAutoN))) {
        fuse = false;                     // (its builds ran on its own stream: nothing to join)
    }
    hs.mark("filters+builds");
    (void)hipSetDevice(L->device);
    for (size_t k = 0; k < n; ++k) {
        imls_ctx* c = ctxs[k];
        if (!c->has_target || !c->has_source)
            return fail(L, IMLS_ERR_STATE, "context " + std::to_string(k) + ": set_target and set_source first");
    }
    L->members.assign(ctxs, ctxs + n);
    L->batch_fused = fuse;
    if (!L->batch_fused) {
        // one launch sequence per frame, each on its own context stream
        for (size_t k = 0; k < n; ++k) {
            if (int rc = imls_register_frame_async(ctxs[k])) {
                for (size_t j = 0; j < k; ++j) (void)imls_register_frame_result(ctxs[j], nullptr, nullptr, nullptr, nullptr);
                if (k > 0) L->err = imls_last_error(ctxs[k]);
                return rc;
            }
        }
        for (size_t k = 0; k < n; ++k) ctxs[k]->batch_member = true;
        L->batch_pending = true;
        return IMLS_OK;
    }
    const int iters = L->P.iterations;
    const size_t res_bytes = n * (kResStride * sizeof(double) + (size_t)std::max(iters, 0) * sizeof(imls_iter_trace));
    if ((size_t)L->tab_cap < n) {
        if (L->tab_h) (void)hipHostFree(L->tab_h);
        L->tab_h = nullptr;
        L->tab_cap = 0;
        if (hipHostMalloc((void**)&L->tab_h, n * sizeof(PairDev)) != hipSuccess)
            return fail(L, IMLS_ERR_DEVICE, "hipHostMalloc (batch)");
        L->tab_cap = (int)n;
    }
    if (L->res_h_bytes < res_bytes) {
        if (L->res_h) (void)hipHostFree(L->res_h);
        L->res_h = nullptr;
        L->res_h_bytes = 0;
        if (hipHostMalloc((void**)&L->res_h, res_bytes) != hipSuccess) return fail(L, IMLS_ERR_DEVICE, "hipHostMalloc (batch)");
        L->res_h_bytes = res_bytes;
    }
    if (!grow(L->tab_d, n * sizeof(PairDev)) || !grow(L->res_d, res_bytes))
        return fail(L, IMLS_ERR_DEVICE, "hipMalloc (batch)");
    if (!L->ev_batch && hipEventCreateWithFlags(&L->ev_batch, hipEventDisableTiming) != hipSuccess)
        return fail(L, IMLS_ERR_DEVICE, "hipEventCreate (batch)");
    hipStream_t s = L->stream;
    L->member_n.assign(n, 0);
    bool any_nrm = false;
    int max_m = 0;
    for (size_t k = 0; k < n; ++k) {
        imls_ctx* c = ctxs[k];
        if (int rc = ensure_solve(c, c->N)) return fail(L, rc, c->err);
        if (int rc = ensure_trace(c, iters)) return fail(L, rc, c->err);
        if (!grow(c->stats, 128)) return fail(L, IMLS_ERR_DEVICE, "hipMalloc");
        // count-mode map normals (get_normals false): flagged here, computed for all the frames that
        // need them by one batched launch ahead of the iterations
        const bool need_nrm = !c->P.get_normals && c->P.recompute_normal_count_mode &&
                              !(c->rnr_valid && c->rnr_k == c->P.search_number_normal && c->rnr_r == c->P.r_normal);
        if (need_nrm) {
            if (!grow(c->rnr, (size_t)std::max(c->M, 1) * 16)) return fail(L, IMLS_ERR_DEVICE, "hipMalloc (normals)");
            c->rnr_valid = true;
            c->rnr_k = c->P.search_number_normal;
            c->rnr_r = c->P.r_normal;
            any_nrm = true;
            max_m = std::max(max_m, c->M);
        }
        if (int rc = check_tv_ready(c)) return fail(L, rc, "context " + std::to_string(k) + ": " + c->err);
        if (int rc = prepare_ransac(c, c->N)) return fail(L, rc, c->err);
        L->tab_h[k] = pair_dev(c);
        L->tab_h[k].recompute_normals = need_nrm ? 1 : 0;
        L->member_n[k] = c->N;
        if (c != L && hipStreamQuery(c->stream) != hipSuccess) {
            // work of the frame still queued on its own stream (uploads, a counted filter or build):
            // the batch waits for it (an idle stream's work is complete: no join)
            if (!c->ev_batch && hipEventCreateWithFlags(&c->ev_batch, hipEventDisableTiming) != hipSuccess)
                return fail(L, IMLS_ERR_DEVICE, "hipEventCreate (batch)");
            if (hipEventRecord(c->ev_batch, c->stream) != hipSuccess || hipStreamWaitEvent(s, c->ev_batch, 0) != hipSuccess)
                return fail(L, IMLS_ERR_DEVICE, "batch stream join");
        }
    }
    (void)hipSetDevice(L->device);
    hs.mark("members");
    const PairDev* tab = (const PairDev*)L->tab_d.p;
    hipMemcpyAsync(L->tab_d.p, L->tab_h, n * sizeof(PairDev), hipMemcpyHostToDevice, s);
    k_batch_init<<<(unsigned)n, 64, 0, s>>>(tab, iters);
    if (any_nrm && launch_map_normals_batch(s, tab, (int)n, max_m, L->P.search_number_normal, L->P.r_normal))
        return fail(L, IMLS_ERR_DEVICE, "batched map normal launch failed");
    const KParams kp = L->kp;
    const RansacParams rp = ransac_params(L->P);
    const int* nh = L->member_n.data();
    for (int it = 0; it < iters; ++it) {
        int slot;
        timed_begin(L, 0, slot);
        launch_project_batch(s, tab, nh, (int)n, kp, it, it > 0 && L->temporal_seed);
        timed_end(L, 0, slot);
        timed_begin(L, 2, slot);
        if (kp.solve_method == IMLS_SOLVE_RANSAC) {
            if (launch_ransac_batch(s, tab, nh, (int)n, kp, rp, it))
                return fail(L, IMLS_ERR_CAPACITY, "RANSAC batch larger than kMaxRansacBatch frames");
        } else
            launch_solve_batch(s, tab, nh, (int)n, kp, it);
        timed_end(L, 2, slot);
    }
    hs.mark("iterations");
    k_batch_results<<<(unsigned)std::min<size_t>(n, 1024), 64, 0, s>>>(tab, (int)n, (double*)L->res_d.p, std::max(iters, 0));
    hipMemcpyAsync(L->res_h, L->res_d.p, res_bytes, hipMemcpyDeviceToHost, s);
    L->batch_traces = iters > 0;
    if (hipGetLastError() != hipSuccess) return fail(L, IMLS_ERR_DEVICE, "batch launch failed");
    // every member's later work (its next uploads / index build) is ordered after the batch
    if (hipEventRecord(L->ev_batch, s) != hipSuccess) return fail(L, IMLS_ERR_DEVICE, "batch event");
    for (size_t k = 1; k < n; ++k)
        if (hipStreamWaitEvent(ctxs[k]->stream, L->ev_batch, 0) != hipSuccess) return fail(L, IMLS_ERR_DEVICE, "batch stream join");
    for (size_t k = 0; k < n; ++k) { ctxs[k]->has_corr = true; ctxs[k]->batch_member = true; }
    L->batch_pending = true;
    return IMLS_OK;
}

int frames_result(imls_ctx* L, double* poses_out, int32_t* iters_out, int32_t* status_out, imls_iter_trace* traces) {
    if (!L) return IMLS_ERR_ARG;
    if (!L->batch_pending) return fail(L, IMLS_ERR_STATE, "no batch pending");
    L->batch_pending = false;
    const size_t n = L->members.size();
    for (imls_ctx* m : L->members) m->batch_member = false;
    const int iters = L->P.iterations;
    if (!L->batch_fused) {
        int first = IMLS_OK;
        for (size_t k = 0; k < n; ++k) {
            double pose[16];
            int it = 0, st = 0;
            const int rc = imls_register_frame_result(L->members[k], pose, &it, &st,
                                                      traces ? traces + k * (size_t)std::max(iters, 0) : nullptr);
            if (rc != IMLS_OK) {
                if (first == IMLS_OK) { first = rc; L->err = "frame " + std::to_string(k) + ": " + imls_last_error(L->members[k]); }
                continue;
            }
            if (poses_out) std::memcpy(poses_out + 16 * k, pose, sizeof(pose));
            if (iters_out) iters_out[k] = it;
            if (status_out) status_out[k] = st;
        }
        return first;
    }
    hipError_t e = hipStreamSynchronize(L->stream);
    if (e != hipSuccess) return fail(L, IMLS_ERR_DEVICE, std::string("batch failed: ") + hipGetErrorString(e));
    harvest_timing(L);
    for (size_t k = 0; k < n; ++k) {
        const double* r = L->res_h + k * kResStride;
        if (poses_out) std::memcpy(poses_out + 16 * k, r, 16 * sizeof(double));
        if (iters_out) iters_out[k] = (int32_t)r[16];
        if (status_out) status_out[k] = (int32_t)r[17];
        if (traces && iters > 0)
            std::memcpy(traces + k * (size_t)iters,
                        reinterpret_cast<const imls_iter_trace*>(L->res_h + n * kResStride) + k * (size_t)iters,
                        (size_t)iters * sizeof(imls_iter_trace));
    }
    return IMLS_OK;
}

}  // namespace

extern "C" {

int imls_register_frames_async(imls_ctx* const* ctxs, size_t n) { return frames_async(ctxs, n); }

int imls_register_frames_result(imls_ctx* lead, double* poses_out, int32_t* iters_out, int32_t* status_out,
                                imls_iter_trace* traces) {
    return frames_result(lead, poses_out, iters_out, status_out, traces);
}

int imls_register_frames(imls_ctx* const* ctxs, size_t n, double* poses_out, int32_t* iters_out, int32_t* status_out,
                         imls_iter_trace* traces) {
    if (int rc = frames_async(ctxs, n)) return rc;
    return frames_result(ctxs[0], poses_out, iters_out, status_out, traces);
}

}  // extern "C"

struct imls_batch {
    std::vector<imls_ctx*> ctx;
    std::string err;
};

extern "C" {

imls_batch* imls_batch_create(int device, const imls_params* p, int32_t streams) {
    if (streams < 1 || streams > 256) return nullptr;
    imls_batch* b = new imls_batch();
    for (int s = 0; s < streams; ++s) {
        imls_ctx* c = imls_create(device, p);
        if (!c) {
            imls_batch_destroy(b);
            return nullptr;
        }
        b->ctx.push_back(c);
    }
    return b;
}

void imls_batch_destroy(imls_batch* b) {
    if (!b) return;
    for (imls_ctx* c : b->ctx) imls_destroy(c);
    delete b;
}

const char* imls_batch_last_error(const imls_batch* b) { return b ? b->err.c_str() : "null batch"; }

int imls_register_batch(imls_batch* b, size_t n_pairs, const imls_pair_input* pairs, double* poses_out,
                        int32_t* iters_out, int32_t* status_out) {
    if (!b) return IMLS_ERR_ARG;
    if (n_pairs > 0 && !pairs) { b->err = "null pairs"; return IMLS_ERR_ARG; }
    // groups of S pairs (one per context): upload + index every pair of the group, then register the
    // group as ONE launch sequence (imls_register_frames)
    const size_t S = b->ctx.size();
    for (size_t g = 0; g < n_pairs; g += S) {
        const size_t m = std::min(S, n_pairs - g);
        for (size_t k = 0; k < m; ++k) {
            imls_ctx* c = b->ctx[k];
            const imls_pair_input& q = pairs[g + k];
            // independent pairs: each starts the RANSAC rand() stream from params.ransac_seed (as the
            // reference's process does for its first frame), so a pair's result does not depend on
            // `streams` or on the pairs its context handled before
            ransac_seed_host(c->P.ransac_seed, c->rng_seed_state);
            c->rng_dirty = true;
            int rc = imls_set_target(c, q.tgt_xyz, q.tgt_nrm, q.n_tgt, q.stride_floats, nullptr);
            if (rc == IMLS_OK) rc = imls_set_source(c, q.src_xyz, q.src_nrm, q.n_src, q.stride_floats, nullptr, nullptr);
            if (rc != IMLS_OK) {
                b->err = "pair " + std::to_string(g + k) + ": " + imls_last_error(c);
                return rc;
            }
        }
        const int rc = imls_register_frames(b->ctx.data(), m, poses_out ? poses_out + 16 * g : nullptr,
                                            iters_out ? iters_out + g : nullptr, status_out ? status_out + g : nullptr,
                                            nullptr);
        if (rc != IMLS_OK) {
            b->err = "pairs " + std::to_string(g) + "..: " + imls_last_error(b->ctx[0]);
            return rc;
        }
    }
    return IMLS_OK;
}

void imls_default_front_params(imls_front_params* p) {
    if (!p) return;
    p->n_scans = 64;            // planetary_slam_VLP_32.launch: scan_line 64, minimum_range 2, maximum_range 150
    p->minimum_range = 2.0f;
    p->maximum_range = 150.0f;
    p->scan_period = 0.1f;      // scan_registration.cpp:55
    p->is_dense = 0;
}

int imls_scan_front_end(imls_ctx* c, const imls_front_params* p, const float* xyz, size_t stride_floats, size_t n,
                        float* out_xyzi, uint32_t* out_index, int32_t* ring_sizes, size_t* n_out) {
    if (!c || !p || !out_xyzi || !ring_sizes || !n_out || (n > 0 && !xyz)) return IMLS_ERR_ARG;
    if (int rc = check_device(c)) return rc;
    int slot;
    timed_begin(c, 7, slot);
    const int rc = front_end_run(c->stream, *p, xyz, stride_floats, n, c->front_mem, out_xyzi, out_index, ring_sizes,
                                 n_out, c->err);
    timed_end(c, 7, slot);
    harvest_timing(c);
    return rc;
}

void imls_default_pca_params(imls_pca_params* p) {
    // scan_registration section of the shipped config.json (read at scan_registration.cpp:1140-1145, 1451, 1133)
    if (!p) return;
    p->window_size = 3;
    p->iter_step = 1;
    p->knn_distance_threshold = 10.f;
    p->neighbor_scan = 0;
    p->distance_threshold = 0.02f;
    p->valid_points_threshold = 0.8f;
    p->use_all_points = 1;
    p->planarity_threshold = 0.05f;
}

int imls_ring_normals_pca(imls_ctx* c, const imls_pca_params* p, const float* xyz, size_t stride,
                          const int32_t* ring_sizes, int32_t n_rings, uint32_t* index_out, float* normal_out,
                          float* evals_out, float* evecs_out, float* features_out, uint8_t* flags_out, size_t* n_out,
                          uint64_t counters[2]) {
    if (!c) return IMLS_ERR_ARG;
    if (!p || !ring_sizes || n_rings <= 0 || n_rings > 4096 || stride < 3)
        return fail(c, IMLS_ERR_ARG, "bad pca params / ring sizes / stride");
    if (p->window_size < 0 || p->iter_step <= 0 || p->neighbor_scan < 0 || p->neighbor_scan > 1)
        return fail(c, IMLS_ERR_ARG, "bad pca window_size / iter_step / neighbor_scan");
    long long total = 0;
    for (int i = 0; i < n_rings; ++i) total += ring_sizes[i];
    if (total > 0 && !xyz) return fail(c, IMLS_ERR_ARG, "null xyz");
    if (total >= (1ll << 31)) return fail(c, IMLS_ERR_CAPACITY, "cloud too large");
    if (int rc = check_device(c)) return rc;
    int slot = -1;
    hipEvent_t marks[2];
    hipEvent_t* mk = nullptr;
    if (c->timing && (slot = ev_pair(c)) >= 0) {
        marks[0] = c->ev[slot];
        marks[1] = c->ev[slot + 1];
        c->ev_pairs[5].push_back({slot, slot + 1});
        mk = marks;
    }
    int rc = ring_pca_run(c->stream, *p, xyz, stride, ring_sizes, n_rings, c->pca_mem, mk, index_out, normal_out,
                          evals_out, evecs_out, features_out, flags_out, n_out, counters, c->err);
    if (c->timing) harvest_timing(c);
    return rc;
}

void imls_default_sample_params(imls_sample_params* p, int32_t method) {
    // scan_registration.sample_method.{normal, major_axis} of the shipped config.json (784-799)
    if (!p) return;
    p->method = method;
    p->r = 0.5f;
    p->r_proj = 1.5f;
    p->max_total_points = 2000;
    p->azimuth_bins = 8;
    p->elevation_bins = 8;
    p->min_points_per_bin = 20;
    p->max_points_per_bin = method == IMLS_SAMPLE_NORMAL ? 100 : 200;
    p->sampling_strategy = method == IMLS_SAMPLE_NORMAL ? 1 : 0;   // normal: "random", major_axis: "FPS"
    p->shuffle_seed = 0;
    p->rand_seed = 1;
}

int imls_sample_point_cloud(imls_ctx* c, const imls_sample_params* p, const float* xyz, const float* nrm,
                            size_t stride, size_t n, const int32_t* candidates, size_t n_cand, const float* last_xyz,
                            size_t last_stride, size_t m, int32_t* sampled_out, size_t* n_sampled,
                            float* bin_weights_out) {
    if (!c) return IMLS_ERR_ARG;
    if (!p || stride < 3 || (n_cand > 0 && (!xyz || !nrm || !candidates || !sampled_out)))
        return fail(c, IMLS_ERR_ARG, "bad sample params / pointers / stride");
    if (p->method < 0 || p->method > 1 || p->azimuth_bins <= 0 || p->elevation_bins <= 0 || p->azimuth_bins > 1024 ||
        p->elevation_bins > 1024 || p->sampling_strategy < 0 || p->sampling_strategy > 1)
        return fail(c, IMLS_ERR_ARG, "bad sample method / bins / strategy");
    if (p->method == IMLS_SAMPLE_MAJOR_AXIS && m > 0 && (!last_xyz || last_stride < 3))
        return fail(c, IMLS_ERR_ARG, "major_axis needs last_pcl_cloud");
    if (n >= (1ull << 31) || m >= (1ull << 31)) return fail(c, IMLS_ERR_CAPACITY, "cloud too large");
    if (int rc = check_device(c)) return rc;
    int slot = -1;
    hipEvent_t marks[2];
    hipEvent_t* mk = nullptr;
    if (c->timing && (slot = ev_pair(c)) >= 0) {
        marks[0] = c->ev[slot];
        marks[1] = c->ev[slot + 1];
        c->ev_pairs[6].push_back({slot, slot + 1});
        mk = marks;
    }
    int rc = sample_run(c->stream, *p, xyz, nrm, stride, n, candidates, n_cand, last_xyz, last_stride, m,
                        c->sample_mem, mk, sampled_out, n_sampled, bin_weights_out, c->err);
    if (mk && rc == IMLS_OK && p->method != IMLS_SAMPLE_MAJOR_AXIS) c->ev_pairs[6].pop_back();   // no kernel recorded
    if (c->timing) harvest_timing(c);
    return rc;
}

int imls_enable_stats(imls_ctx* c, int enable) {
    if (!c) return IMLS_ERR_ARG;
    c->collect_stats = enable != 0;
    return IMLS_OK;
}

int imls_enable_timing(imls_ctx* c, int enable) {
    if (!c || enable < 0 || enable > 2) return IMLS_ERR_ARG;
    c->timing = enable;
    return IMLS_OK;
}

int imls_capture_correspondences(imls_ctx* c, int on) {
    if (!c) return IMLS_ERR_ARG;
    c->capture = on != 0;
    return IMLS_OK;
}

int imls_captured_correspondences(imls_ctx* c, int iter, size_t cap, float* x_out, float* y_out, float* n_out,
                                  uint32_t* src_index_out, size_t* n_valid) {
    if (!c || !n_valid) return IMLS_ERR_ARG;
    if (c->pending) return fail(c, IMLS_ERR_STATE, "collect the frame first (imls_register_frame_result)");
    // the captured frame's iterations only: a later set_source or batch drops the capture (its rows
    // index the old source), and iterations at or past the frame's iters_run hold stale rows
    if (c->cap_iters == 0 || c->cap_run < 0) return fail(c, IMLS_ERR_STATE, "no captured frame");
    if (iter < 0 || iter >= std::min(c->cap_iters, c->cap_run))
        return fail(c, IMLS_ERR_STATE, "no captured iteration " + std::to_string(iter));
    if (int rc = check_device(c)) return rc;
    const size_t N = (size_t)c->cap_N;
    std::vector<float> h(N * 12);
    if (hipMemcpy(h.data(), (const char*)c->cap_mem.p + (size_t)iter * N * 48, N * 48, hipMemcpyDeviceToHost) != hipSuccess)
        return fail(c, IMLS_ERR_DEVICE, "capture download");
    const float *hs = h.data(), *hd = hs + 4 * N, *hn = hs + 8 * N;
    size_t nv = 0;
    for (size_t i = 0; i < N; ++i) nv += hs[4 * i + 3] != 0.f ? 1 : 0;
    *n_valid = nv;
    const bool want = x_out || y_out || n_out || src_index_out;
    if (!want) return IMLS_OK;            // size query
    if (nv > cap) return fail(c, IMLS_ERR_ARG, "capacity " + std::to_string(cap) + " < " + std::to_string(nv) + " rows");
    size_t k = 0;
    for (size_t i = 0; i < N; ++i) {
        if (hs[4 * i + 3] == 0.f) continue;   // rejected (erased from in_cloud by the reference)
        for (int d = 0; d < 3; ++d) {
            if (x_out) x_out[3 * k + d] = hs[4 * i + d];
            if (y_out) y_out[3 * k + d] = hd[4 * i + d];
            if (n_out) n_out[3 * k + d] = hn[4 * i + d];
        }
        if (src_index_out) src_index_out[k] = (uint32_t)i;
        ++k;
    }
    return IMLS_OK;
}

int imls_set_defer(imls_ctx* c, int on) {
    if (!c) return IMLS_ERR_ARG;
    c->defer = on != 0;
    return IMLS_OK;
}

int imls_timing_origin(imls_ctx* c) {
    if (!c) return IMLS_ERR_ARG;
    if (int rc = check_device(c)) return rc;
    if (c->device < 0 || c->device >= kMaxDevices) return fail(c, IMLS_ERR_ARG, "device index");
    std::lock_guard<std::mutex> lk(g_origin_mu);
    hipEvent_t& o = g_origin[c->device];
    if (!o && hipEventCreate(&o) != hipSuccess) return fail(c, IMLS_ERR_DEVICE, "hipEventCreate (origin)");
    if (hipEventRecord(o, c->stream) != hipSuccess || hipEventSynchronize(o) != hipSuccess)
        return fail(c, IMLS_ERR_DEVICE, "origin event");
    g_origin_set[c->device] = true;
    for (auto& v : c->iv) v.clear();
    return IMLS_OK;
}

int imls_timing_intervals(imls_ctx* c, int kernel, double* out, size_t cap, size_t* n) {
    if (!c || kernel < 0 || kernel >= kTimingKinds || !n) return IMLS_ERR_ARG;
    const auto& v = c->iv[kernel];
    *n = v.size();
    for (size_t k = 0; k < v.size() && k < cap && out; ++k) {
        out[2 * k] = v[k].first;
        out[2 * k + 1] = v[k].second;
    }
    return IMLS_OK;
}

int imls_kernel_timing(imls_ctx* c, int kernel, double* total_ms, uint64_t* launches) {
    if (!c || kernel < 0 || kernel >= kTimingKinds) return IMLS_ERR_ARG;
    if (total_ms) *total_ms = c->t_ms[kernel];
    if (launches) *launches = c->t_n[kernel];
    return IMLS_OK;
}

int imls_reset_timing(imls_ctx* c) {
    if (!c) return IMLS_ERR_ARG;
    for (int k = 0; k < kTimingKinds; ++k) { c->t_ms[k] = 0; c->t_n[k] = 0; c->ev_pairs[k].clear(); c->iv[k].clear(); }
    c->ev_used = 0;
    return IMLS_OK;
}

int imls_traversal_stats(imls_ctx* c, uint64_t out[8]) {
    if (!c || !out) return IMLS_ERR_ARG;
#ifdef IMLS_DEBUG_WAVE_TRACE
    constexpr int kOut = 16;   // debug build: the caller passes 16 slots
#else
    constexpr int kOut = 8;
#endif
    unsigned long long st[kOut] = {};
    if (c->stats.p) hipMemcpy(st, c->stats.p, sizeof(st), hipMemcpyDeviceToHost);
    for (int k = 0; k < kOut; ++k) out[k] = st[k];
    return IMLS_OK;
}

int imls_index_stats(imls_ctx* c, uint64_t out[8]) {
    if (!c || !out) return IMLS_ERR_ARG;
    if (int rc = ensure_built(c)) return rc;
    unsigned long long st[2] = {0, 0};
    if (c->stats.p) hipMemcpy(st, c->stats.p, 16, hipMemcpyDeviceToHost);
    out[0] = (uint64_t)c->M;
    out[1] = (uint64_t)((c->M + c->B - 1) / c->B);
    out[2] = (uint64_t)c->Pl;
    out[3] = (uint64_t)c->levels;
    out[4] = st[0];   // Σ k_q (neighbours returned to queries reaching the IMLS function)
    out[5] = st[1];   // queries whose NN-1 was found
    out[6] = (uint64_t)c->N;
    out[7] = (uint64_t)c->B;
    return IMLS_OK;
}

}  // extern "C"
