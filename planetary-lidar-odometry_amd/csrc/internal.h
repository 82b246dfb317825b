// internal.h — shared declarations of the HIP IMLS-ICP path (gfx950 only).
//
// HBM layout (SoA-of-float4, 16-B aligned, one record per point):
//   target, filtered order   : tpt[M]  = (x, y, z, 0)      tnr[M] = (nx, ny, nz, 0)
//   target, Morton order     : mpt[M]  = (x, y, z, bits(filtered index))   ← leaf scans
//   tree (implicit, complete): node i ∈ [1, P) holds the AABBs of children 2i, 2i+1 as
//                              3 float4 (lo_l.xyz, hi_l.x | hi_l.yz, lo_r.xy | lo_r.z, hi_r.xyz);
//                              leaf node P + b = bucket b = mpt[b·B, min((b+1)·B, M)).
//   source, filtered order   : spt[N], snr[N] float4
//   correspondences, per source index (uncompacted): cs[N] = (x, valid), cd[N] = (y, ·),
//                              cn[N] = (n, ·) float4 — source order is implicit in the index.
#pragma once
#include <cstddef>
#include <hip/hip_runtime.h>
#include <cstdint>
#include <string>
#include <vector>

#include "../../include/imls_gpu.h"

namespace imlsgpu {

constexpr int kBlock = 256;            // threads per block for streaming kernels
constexpr int kProjBlock = 128;        // threads per block for the projection kernel
constexpr int kStackDepth = 24;        // traversal stack entries per lane (tree depth ≤ 24)
constexpr int kHistBins = 65536;       // residual histogram bins (top 16 bits of float |r|: 1/128 octave)
constexpr int kCandCap = 8192;         // exact-select candidates handled in LDS per boundary bin
constexpr int kNormEq = 28;            // 21 (JᵀJ upper) + 6 (Jᵀb) + 1 (row count)

// Device-side per-iteration record, laid out as imls_iter_trace.
static_assert(sizeof(imls_iter_trace) == 16 * 8 * 2 + 8 * 8, "trace layout");

struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
};

// Grow-only device buffers (api.hip).  A buffer being replaced may still be read by work already
// enqueued on any of the library's streams, and hipFree would wait for the whole device (every
// context's work in flight, and the host).  So the old buffer is RETIRED instead: an event is
// recorded on every registered stream of its device that still has work, and the buffer is handed
// out again (to any grow of a size it fits) only once all of those events have completed; retired
// buffers are freed at teardown (imls_destroy).  devbuf_grow(b, bytes, alloc): no-op when b holds
// `bytes`, else b becomes a buffer of ≥ alloc bytes (alloc ≥ bytes: the caller's headroom).
bool devbuf_grow(DevBuf& b, size_t bytes, size_t alloc);
void devbuf_retire(DevBuf& b);         // b → retired (empty afterwards)
// the streams the library enqueues on (context, upload and caller-set streams), reference counted
void register_stream(hipStream_t s, int device);
void unregister_stream(hipStream_t s);
// teardown: free every retired buffer of `device` (hipFree waits for the device)
void release_retired(int device);

// Parameters the kernels need, in a flat POD copied by value into launches.
struct KParams {
    double h2, r2, cos_thr;   // cos_thr = cos(angle_thr_deg · π/180): the angle gates' fast path
    double angle_thr_deg;
    int K;                    // search_number
    int angle_on;
    int get_normals;
    int transform_normal;
    int correspond_number;
    int solve_method;
    double ls_threshold;
    double delta_dist, delta_angle;
    int matcher;              // imls_match_method: 0 IMLS, 1 plane_ICP (NN-1 tangent-plane projection)
    int proj;                 // projected-distance candidate rule (brute force in the reference)
    double gate_dist, gate_proj;   // proj mode: ‖p−x‖ < gate_dist and ‖(p−x)×n_s‖ < gate_proj
    // traversal tuning: documented runtime options (imls_set_option, include/imls_gpu.h), fixed
    // constants otherwise (project.hip: kSeedHalf, kReseed, kSparseLanes, kWide)
    int qwave;                // traversal: −1 auto (one wave per query up to kQwaveAutoN queries), 0 packets, 1 wave per query
    int packet;               // packet traversal: queries per wave in this launch (64, or 32 / 16: see pk_small)
    int pk_small, pk_iters;   // the first pk_iters ICP iterations (mostly seeding lanes) use pk_small-query packets
    int pk_batch;             // … in batched launches too (imls_register_frames; off: measured slower there)
    int reuse;                // Verlet reuse of a query's list without traversal while its certificate holds
    int force_fb;             // test hook: every force_fb-th query slot's list treated as uncertified (0 off)
    int xcd;                  // batched projection: frames grouped per XCD round-robin slot (−1 auto: ≥ 16 frames)
    int tv;                   // tensor-voting normals (use_tensor_voting && !get_normals, IMLS matcher)
    int tv_k;                 // use_tensor_voting.k (≤ kTvMaxK)
    double tv_sigma, tv_thr;  // use_tensor_voting.sigma, .distance_threshold
    float tv_skin;            // TV ball lists reused while the query moved ≤ skin (m); 0 = every iteration walks the tree
    int bfs;                  // this launch's packet walks start breadth-first (the first IMLS_BFS_ITERS iterations)
};
// the parameters of ICP iteration `it`'s projection launch (packet size of the traversal)
#ifndef IMLS_BFS_ITERS
#define IMLS_BFS_ITERS 0   // breadth-first top levels: measured slower (profiles/r06_bfs_rejected/), off
#endif
inline KParams kp_at(const KParams& k, int it) {
    KParams r = k;
    r.packet = it >= 0 && it < k.pk_iters ? k.pk_small : 64;
    r.bfs = it >= 0 && it < IMLS_BFS_ITERS;
    return r;
}
constexpr int kTvMaxK = 64;    // tensor-voting kNN size handled on device
constexpr int kTvList = 64;    // TV skin list: ball(ρ + skin) members stored per query (more: not stored)
// per-query TV state behind TreeView::tvn, arrays of N: voted normal (double4), skin reference
// (float4: x, count), skin list (kTvList Morton positions), summed tensor (9 doubles)
constexpr size_t kTvBytesPerQuery = 32 + 16 + 4 * kTvList + 72;

struct TreeView {
    const float4* mpt;        // map points in Morton order, w = original index (bits)
    const float4* mnr;        // their normals, same order
    const unsigned* ipos;     // original index → Morton position
    const float4* nodes;      // 3 float4 per internal node, index 1..P-1 (entry 0 unused)
    const float4* tpt;
    const float4* tnr;
    int M, B, P, levels;
    const unsigned long long* lkeys;   // [L] Morton key of each leaf's first point (seed search)
    const float* qparams;              // [4] Morton quantisation: bbox lo xyz, scale
    int L;                             // leaves holding points
    const float4* mten;                // TV: input tensors in Morton order, 2 float4 per point
                                       //     (xx, xy, xz, yy | yz, zz, 0, 0), or null
    const double4* tvn;                // TV: per source index, the voted normal + found flag (w)
};

// 48-bit Morton code with isotropic quantisation (one scale for all axes keeps buckets compact);
// shared by the index build and the query-side seed search so both quantise identically.
__device__ __forceinline__ unsigned long long spread3_16(unsigned v) {
    unsigned long long x = v & 0xFFFFull;
    x = (x | (x << 16)) & 0x0000FF0000FFull;
    x = (x | (x << 8)) & 0x00F00F00F00Full;
    x = (x | (x << 4)) & 0x0C30C30C30C3ull;
    x = (x | (x << 2)) & 0x249249249249ull;
    return x;
}
__device__ __forceinline__ unsigned long long morton48(float x, float y, float z, const float* __restrict__ qp) {
    const float qmax = 65535.f, sc = qp[3];
    const unsigned qx = (unsigned)fminf(fmaxf((x - qp[0]) * sc, 0.f), qmax);
    const unsigned qy = (unsigned)fminf(fmaxf((y - qp[1]) * sc, 0.f), qmax);
    const unsigned qz = (unsigned)fminf(fmaxf((z - qp[2]) * sc, 0.f), qmax);
    return spread3_16(qx) | (spread3_16(qy) << 1) | (spread3_16(qz) << 2);
}

// Sum of v over the wave's 64 lanes, valid in lane 63 only: an inclusive scan of each 16-lane row by
// DPP row shifts (1, 2, 4, 8), then row_bcast:15 and row_bcast:31 carry the row totals into lane 63 —
// VALU moves only (a __shfl_xor butterfly is 12 ds_bpermute LDS round trips per fp64 sum).  A fixed
// association: the same bits on every run and in every kernel that uses it.
template <int CTRL, int ROWS>
__device__ __forceinline__ double dpp_add_f64(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)(unsigned)(unsigned long long)b, CTRL, ROWS, 0xf, true);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(unsigned)((unsigned long long)b >> 32), CTRL, ROWS, 0xf, true);
    return v + __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}
__device__ __forceinline__ double wave_total(double v) {
    v = dpp_add_f64<0x111, 0xf>(v);    // row_shr:1
    v = dpp_add_f64<0x112, 0xf>(v);    // row_shr:2
    v = dpp_add_f64<0x114, 0xf>(v);    // row_shr:4
    v = dpp_add_f64<0x118, 0xf>(v);    // row_shr:8  → lane 15 of each row holds its row's sum
    v = dpp_add_f64<0x142, 0xa>(v);    // row_bcast:15 into rows 1 and 3
    v = dpp_add_f64<0x143, 0xc>(v);    // row_bcast:31 into rows 2 and 3 → lane 63 holds the total
    return v;
}

// The wave's totals of 28 values per lane (a[28..31] = 0): recursive halving — at lane bit 2h each
// lane keeps one half of its 2h values and adds the partner's copy of that half (32 fp64 exchanges,
// where 28 wave_total reductions issue 168 DPP steps); lane 2k returns value k's total.  A fixed
// association, shared by the solve kernels' normal-equation reductions (block_sum28 and block_normeq
// of solve_common.h, k_collect); the projection kernels keep wave_total (their 64 extra VGPRs spill
// the traversal's 96-register budget).
__device__ __forceinline__ double xor_f64(double v, int m) {
    const long long b = __double_as_longlong(v);
    const int lo = __shfl_xor((int)(unsigned)(b & 0xffffffffll), m, 64);
    const int hi = __shfl_xor((int)(unsigned)((unsigned long long)b >> 32), m, 64);
    return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}
template <int H>
__device__ __forceinline__ void wave_halve(double (&a)[32], int lane) {
    const bool up = (lane & (2 * H)) != 0;
#pragma unroll
    for (int i = 0; i < H; ++i) {
        const double send = up ? a[i] : a[H + i];
        const double keep = up ? a[H + i] : a[i];
        a[i] = keep + xor_f64(send, 2 * H);
    }
    if constexpr (H > 1) wave_halve<H / 2>(a, lane);   // static indices at every level (no stack array)
}
__device__ __forceinline__ double wave_sum28(double (&a)[32]) {
    const int lane = threadIdx.x & 63;
    wave_halve<16>(a, lane);
    return a[0] + xor_f64(a[0], 1);
}

// Solver scratch living in device memory (one per context).
struct SolveState {
    double* pose;             // [16] current rPose
    double* delta;            // [16] last Δ
    double* x0;               // [8]  first LS solution
    int* done;                // [1]  frame finished (converged / too few / failed)
    int* status;              // [1]  imls_frame_status
    int* iters;               // [1]  iterations run
    unsigned* hist;           // [kHistBins]
    unsigned* coarse;         // [kHistBins / 256] the same histogram, 256 bins per entry
    unsigned* cand_count;     // [2]
    unsigned long long* cand_lo;   // [kCandCap*?] (key bits) pairs with row index
    unsigned* cand_lo_row;
    unsigned long long* cand_hi;
    unsigned* cand_hi_row;
    int* sel;                 // [8] select metadata: b_lo, b_hi, c_lo, c_hi, lower, upper, nvalid
    double* partial1;         // [blocks × kNormEq] pass-1 block partials
    double* partial2;         // [blocks × kNormEq] pass-2 block partials
    double* keys;             // [N] |r|
    imls_iter_trace* trace;   // [iterations]
    int partial_cap;
};

// RANSAC state of one context (ransac.hip), carved from its RANSAC scratch by ransac_frame().
struct RansacDev {
    int* rng;          // [34] glibc state (persistent)
    int* counts;       // [kHypMax]
    double* T;         // [kHypMax × 16]
    int* best;         // [1]
    int* evaluated;    // [1]
    int* rdone;        // [1] RANSAC finished (early exit or max iterations)
    double* bestT;     // [16]
    int* active;       // [1] the frame was still running when this solve began
};
struct DrpmDev {
    double* H;         // [36] row-major
    double* g;         // [6]
    double* U;         // [36] eigenvectors as columns: U[k·6 + r] = component r of vector k
    double* ev;        // [6] ascending
    double* slabs;     // [blocks × kDrpmSlab]
};
struct RansacFrame {
    double* all;       // [10·cap] the compacted valid correspondences (fp64 Rows layout)
    double* inl;       // [10·cap] the inliers of the best Δ with their weights
    int* blkcnt;       // [nb + 1] compaction block counts → offsets
    double* blkw;      // [nb + 1] compaction block Σw
    int *cnt_all, *cnt_in;
    double* wsum;      // Σw of the inliers
    RansacDev R;
    DrpmDev Dv;
    int cap;           // max(N, 1)
};

// One registration of a batched launch (imls_register_frames): everything a per-iteration kernel
// reads or writes for that frame.  The batch's table of these lives in device memory; a batched
// kernel takes its frame from tab[blockIdx.y] (a wave-uniform, read-only load: scalar) and runs the
// same body as the single-frame kernel, so a frame gives bit-identical results either way.
struct PairDev {
    TreeView t;
    const float4* spt;
    const float4* snr;
    const unsigned* qperm;
    int N;
    float4 *cs, *cd, *cn;
    int* lists;                        // [KL][N] + worst keys + xref/nref (prevnn_bytes)
    SolveState st;
    imls_iter_trace* trace;            // [iterations]
    unsigned long long* stats;         // traversal / neighbour counters
    unsigned* fb_list;                 // uncertified queries (exact fallback) + their count
    unsigned* fb_count;
    RansacFrame rf;                    // RANSAC scratch (solve_method RANSAC), else zero
    int recompute_normals;             // map normals (count mode) to compute into t.mnr before the batch
};

// The batched kernels' view of their frame's record.  A pointer loaded from the frame table is
// generic to the compiler, so every access through it was a FLAT load — counted on vmcnt and lgkmcnt
// alike, so consuming one also waits for the kernel's LDS traffic, and a flat load after an LDS store
// it might alias waits for that store (k_knn_wave_b 181 vs k_knn_wave 166 µs per launch on config
// B's pair, profiles/r05_flat/).  The table holds HBM pointers only: device_view loads each pointer
// field as a global-address-space value, and the address-space inference turns every access through
// it into a global load.  (Host code never sees the qualifier: it is defined for the device pass only.)
#if defined(__HIP_DEVICE_COMPILE__)
#define IMLS_GAS __attribute__((address_space(1)))
#else
#define IMLS_GAS
#endif
__device__ __forceinline__ const void* gfield(const void* base, size_t off) {
    typedef const void IMLS_GAS* gvp;
    return (const void*)*reinterpret_cast<const gvp*>(reinterpret_cast<const char*>(base) + off);
}
#define IMLS_GLOBAL_FIELD(A, pa, f) (A).f = (decltype((A).f))gfield((pa), offsetof(PairDev, f))
__device__ __forceinline__ PairDev device_view(const PairDev* pa) {
    PairDev A = *pa;
    IMLS_GLOBAL_FIELD(A, pa, t.mpt); IMLS_GLOBAL_FIELD(A, pa, t.mnr); IMLS_GLOBAL_FIELD(A, pa, t.ipos);
    IMLS_GLOBAL_FIELD(A, pa, t.nodes); IMLS_GLOBAL_FIELD(A, pa, t.tpt); IMLS_GLOBAL_FIELD(A, pa, t.tnr);
    IMLS_GLOBAL_FIELD(A, pa, t.lkeys); IMLS_GLOBAL_FIELD(A, pa, t.qparams); IMLS_GLOBAL_FIELD(A, pa, t.mten);
    IMLS_GLOBAL_FIELD(A, pa, t.tvn);
    IMLS_GLOBAL_FIELD(A, pa, spt); IMLS_GLOBAL_FIELD(A, pa, snr); IMLS_GLOBAL_FIELD(A, pa, qperm);
    IMLS_GLOBAL_FIELD(A, pa, cs); IMLS_GLOBAL_FIELD(A, pa, cd); IMLS_GLOBAL_FIELD(A, pa, cn);
    IMLS_GLOBAL_FIELD(A, pa, lists); IMLS_GLOBAL_FIELD(A, pa, trace); IMLS_GLOBAL_FIELD(A, pa, stats);
    IMLS_GLOBAL_FIELD(A, pa, fb_list); IMLS_GLOBAL_FIELD(A, pa, fb_count);
    IMLS_GLOBAL_FIELD(A, pa, st.pose); IMLS_GLOBAL_FIELD(A, pa, st.delta); IMLS_GLOBAL_FIELD(A, pa, st.x0);
    IMLS_GLOBAL_FIELD(A, pa, st.done); IMLS_GLOBAL_FIELD(A, pa, st.status); IMLS_GLOBAL_FIELD(A, pa, st.iters);
    IMLS_GLOBAL_FIELD(A, pa, st.hist); IMLS_GLOBAL_FIELD(A, pa, st.coarse); IMLS_GLOBAL_FIELD(A, pa, st.cand_count);
    IMLS_GLOBAL_FIELD(A, pa, st.cand_lo); IMLS_GLOBAL_FIELD(A, pa, st.cand_lo_row); IMLS_GLOBAL_FIELD(A, pa, st.cand_hi);
    IMLS_GLOBAL_FIELD(A, pa, st.cand_hi_row); IMLS_GLOBAL_FIELD(A, pa, st.sel); IMLS_GLOBAL_FIELD(A, pa, st.partial1);
    IMLS_GLOBAL_FIELD(A, pa, st.partial2); IMLS_GLOBAL_FIELD(A, pa, st.keys); IMLS_GLOBAL_FIELD(A, pa, st.trace);
    return A;
}

// index.hip — two phases, so many frames' uploads and filters can be enqueued before one wait:
// (A) filter_async: NaN filter + order-keeping compaction (kept: filtered → input index, nullable),
//     the kept count copied to pinned *h_count behind it;
// (B) with that count known: build_target_tree (Morton sort, leaf boxes, node records) or
//     source_order (the source's Morton order = the wave kernels' query order).
int filter_async(hipStream_t s, const float* d_soa6, size_t n_in, DevBuf& pt, DevBuf& nr, DevBuf& scratch,
                 unsigned* d_kept, int* h_count, std::string& err);
// (A) for many frames at once (deferred filters of a batch's members), one launch sequence; the
// kept counts land in each job's pinned host word once the stream has passed it.
struct FilterJob {
    const float* soa;
    size_t n;
    DevBuf *pt, *nr;                   // grown to n records here
    unsigned* kept;                    // nullable
    int* h_count;
};
int filter_batch(hipStream_t s, const std::vector<FilterJob>& jobs, DevBuf& scratch, DevBuf& table, void* h_table,
                 size_t h_table_bytes, std::string& err);
size_t filter_job_bytes();
int build_target_tree(hipStream_t s, int M, int bucket, DevBuf& lkeys, DevBuf& tpt, DevBuf& tnr, DevBuf& mpt,
                      DevBuf& nodes, DevBuf& scratch, DevBuf& treescratch, DevBuf& permbuf, int* P_out, int* levels_out,
                      std::string& err);
int source_order(hipStream_t s, int N, DevBuf& spt, DevBuf& scratch, DevBuf& qperm, std::string& err);
// a small frame's source order (≤ kSmallOrderN points) in one launch — the same permutation
constexpr int kSmallOrderN = 2048;
int small_source_order(hipStream_t s, const float4* pts, int N, unsigned* perm, std::string& err);
// (B) for many frames at once, one launch sequence: each job a target tree (B > 0: lkeys [L + 2]
// words, mpt [3·n] records, nodes [(P+1)·3] float4, sized by the caller; P / levels returned in the
// job) or a source order (B = 0: perm [n]).  h_table: pinned host memory for the job table.
struct BuildJob {
    const float4* pts;
    const float4* nrm;
    int n, B;
    unsigned long long* lkeys;
    float4* mpt;
    float4* nodes;
    unsigned* perm;
    int P, levels;                     // out (targets)
};
int build_batch(hipStream_t s, std::vector<BuildJob>& jobs, DevBuf& scratch, DevBuf& table, void* h_table,
                size_t h_table_bytes, std::string& err);
size_t build_job_bytes();              // bytes per job of the device job table

// index.hip — incremental index of the map FIFO (api.hip map_push / finish_target).  A run = one
// scan's filtered points Morton-sorted under the FIFO's fixed quantisation: [n] sorted keys, [n]
// records (xyz, bits(local filtered index)), [n] normals, 256-B aligned parts of one buffer.
struct FifoRun {
    const float4* rpt;
    const float4* rnr;
    unsigned off;                      // concatenated filtered index of the run's first point
    unsigned pad;
};
constexpr int kMaxFifoRuns = 32;       // run ids (5 bits of a merged entry's value; 27 bits of position)
struct FifoRunTable { FifoRun r[kMaxFifoRuns]; };   // by value in the gather launch (768 B of arguments)
inline size_t fifo_part(size_t bytes) { return (bytes + 255) / 256 * 256; }
inline size_t fifo_run_bytes(int n) { return fifo_part((size_t)n * 8) + 2 * fifo_part((size_t)n * 16); }
inline unsigned long long* fifo_run_keys(void* run, int) { return (unsigned long long*)run; }
inline float4* fifo_run_pts(void* run, int n) { return (float4*)((char*)run + fifo_part((size_t)n * 8)); }
inline float4* fifo_run_nrm(void* run, int n) { return (float4*)((char*)run + fifo_part((size_t)n * 8) + fifo_part((size_t)n * 16)); }
// scratch every fifo_* step of one build fits in (sized before the build enqueues anything: the
// steps share it in stream order and never reallocate it under a pending kernel)
size_t fifo_scratch_bytes(int max_run, int nruns, int M);
// the FIFO's quantisation frame (fq: lo xyz, scale) from the bboxes of filtered point sets
int fifo_frame(hipStream_t s, const std::vector<std::pair<const float4*, int>>& runs, float* fq, DevBuf& scratch,
               std::string& err);
// one run from n filtered points (clamp: device counter of points outside fq's cube)
int fifo_run_build(hipStream_t s, const float4* fpt, const float4* fnr, int n, const float* fq, unsigned* clamp,
                   DevBuf& run, DevBuf& scratch, std::string& err);
// stable compaction of a merged order to the entries of live runs (bit id of `live`)
int fifo_keep(hipStream_t s, const unsigned long long* key, const unsigned* val, int n, unsigned live,
              unsigned long long* okey, unsigned* oval, DevBuf& scratch, std::string& err);
// merge(A, run B) by key, A first on equal keys; B's values become (bid << 27) | index
int fifo_merge(hipStream_t s, const unsigned long long* a, const unsigned* av, int na, const unsigned long long* b,
               unsigned bid, int nb, unsigned long long* okey, unsigned* oval, DevBuf& scratch, std::string& err);
// the target index from the merged order (records, ipos, leaf keys + fq, leaf boxes, tree)
// (clamp: the device clamp counter, copied to the host's coherent word h_clamp behind the build)
int fifo_index(hipStream_t s, const unsigned long long* mkey, const unsigned* mval, int M, const FifoRunTable& runs,
               const float* fq, const unsigned* clamp, unsigned* h_clamp, int B, DevBuf& lkeys, DevBuf& mpt, DevBuf& nodes,
               DevBuf& treescratch, int* P_out, int* levels_out, std::string& err);

// project.hip
// k_knn_wave → k_finish (+ the exact k_project_lane fallback for uncertified queries); lane_mode
// runs every query through k_project_lane.  partial1 receives project_blocks(N) slabs.
void launch_project(hipStream_t s, const TreeView& t, const float4* spt, const float4* snr,
                    const unsigned* qperm, int N, const double* pose, const int* done, const KParams& kp,
                    float4* cs, float4* cd, float4* cn, double* partial1, imls_iter_trace* tr,
                    unsigned long long* nbr_stats, unsigned* fb_list, unsigned* fb_count, int lane_mode,
                    const double* delta, int* lists, int use_prev, hipEvent_t* marks = nullptr);
// delta: last pose increment (read when use_prev); lists: [KL][N] positions + [N] worst keys,
// kept across ICP iterations (temporal seed); marks: 3 events recorded before k_knn_wave, between
// it and k_finish, and after k_finish (timing), or null
constexpr int kMaxKL = 46;       // list entries per query at most (the lone-frame path: K + 12 for K ≤ 32, capped)
// per-query reference position + list guarantee (float4 xref[N]) and the key the list's answer
// relied on (float nref[N]), after the [kMaxKL+1][N] list block
__host__ __device__ inline float4* xref_of(int* lists, int N) {
    return reinterpret_cast<float4*>(reinterpret_cast<char*>(lists) + ((size_t)(kMaxKL + 1) * N * 4 + 255) / 256 * 256);
}
// then the compacted traversal lists of the packet kernel's later ICP iterations (round 6: per
// traversal block, the slots whose list could not be reused, unsigned cmp[N]) and their counts (one
// word per block, cmp_count[N / 64 + 1])
__host__ __device__ inline unsigned* cmp_of(int* lists, int N) {
    return reinterpret_cast<unsigned*>(reinterpret_cast<char*>(xref_of(lists, N)) + ((size_t)N * 20 + 255) / 256 * 256);
}
__host__ __device__ inline unsigned* cmp_count_of(int* lists, int N) { return cmp_of(lists, N) + ((size_t)N + 63) / 64 * 64; }
inline size_t prevnn_bytes(int N) {
    return ((size_t)(kMaxKL + 1) * N * 4 + 255) / 256 * 256 + ((size_t)N * 20 + 255) / 256 * 256 + ((size_t)N + 63) / 64 * 256 +
           ((size_t)N / 64 + 2) * 4 + 512;
}
constexpr int kStatSkipped = 6;   // nbr_stats slot: lanes whose list was reused without traversal
int project_blocks(int N);
// k_finish: the exact stage one lane per query (0) or one quad per query (1: round 6, measured slower —
// DESIGN §5 round 6; kept for same-box A/B builds, tools/build_full_variant.sh quad -DIMLS_FINISH_QUAD=1)
#ifndef IMLS_FINISH_QUAD
#define IMLS_FINISH_QUAD 0
#endif
constexpr int kPass1Block = IMLS_FINISH_QUAD ? 64 : 256;   // queries per k_finish block (one pass-1 slab each)
constexpr int kPass1Fallback = 64;     // k_project_lane fallback blocks (one slab each, after the k_finish slabs)
// Batched projection: one launch per kernel for all `npairs` frames of tab (device), iteration
// `it` (trace slot), every frame at its own pose / done flag.  n_host: the frames' N (grid shapes).
void launch_project_batch(hipStream_t s, const PairDev* tab, const int* n_host, int npairs, const KParams& kp, int it,
                          int use_prev);

// solve.hip
void launch_solve_chain(hipStream_t s, int N, int blocks1, const KParams& kp, const float4* cs,
                        const float4* cd, const float4* cn, const double* rows_d, const double* weights,
                        SolveState& st, imls_iter_trace* tr, int update_pose, int rows_are_double,
                        const int* count = nullptr, const double* wsum = nullptr);
// N above which the float-row LS takes the grid chain (below: one block, k_solve_small)
constexpr int kQwaveAutoN = 16384;  // auto traversal choice: one wave per query up to this many queries
constexpr int kSmallRows = 4096;
int solve_blocks(int N);
// Batched LS / weighted-LS solve + pose update for all frames of tab (float rows from the batched
// projection): k_solve_small over the frames with N ≤ kSmallRows, the grid chain over the others.
// src 0: float rows of the batched projection; src 1: every frame's RANSAC inlier rows (fp64, the
// grid chain always; n_host = the frames' RANSAC caps), pass 1 included.
void launch_solve_batch(hipStream_t s, const PairDev* tab, const int* n_host, int npairs, const KParams& kp, int it,
                        int src = 0);
// pass 1 over every frame's RANSAC inlier rows (weighted: w / Σw)
void launch_rows_pass1_batch(hipStream_t s, const PairDev* tab, const int* cap_host, int npairs, int weighted);

// normals.hip — map normals recomputed from the map (get_normals=false, count mode), Morton order
int launch_map_normals(hipStream_t s, const TreeView& t, int K, double r_normal, float4* out);
int launch_map_normals_batch(hipStream_t s, const PairDev* tab, int npairs, int maxM, int K, double r_normal);

// tv.hip — tensor voting (VoteForAny, imls_icp.cpp:171-296): the voted normal of every source point
// at the current pose → tvn[N]; input tensors gathered to Morton order once per target
void launch_tv_vote(hipStream_t s, const TreeView& t, const float4* spt, int N, const double* pose, const int* done,
                    const KParams& kp, double4* tvn, int use_prev);
void launch_tensor_gather(hipStream_t s, const float* ten6_in, size_t n_in, const unsigned* kept, const float4* mpt, int M,
                          float4* mten);
void launch_tv_vote_batch(hipStream_t s, const PairDev* tab, const int* n_host, int npairs, const KParams& kp,
                          int use_prev);

// ransac.hip — RANSAC (+ final LS / weighted LS / DRPM) and the solve-method dispatcher
constexpr int kHypMax = 8192;          // hypotheses per chunk (chunks: 16, then up to kHypMax each)
struct RansacParams {
    int max_iterations;
    double distance_threshold, min_inliers_percentage, huber_threshold;
    int final_method;                  // imls_final_method
    double ls_threshold, drpm_threshold, drpm_stdev_points, drpm_stdev_normals;
};
struct SolveLaunch {
    int N;                             // rows (float rows: source count; fp64 rows: row count)
    int blocks1;                       // pass-1 slabs already in st.partial1 (float rows from k_finish)
    KParams kp;
    const float4 *cs, *cd, *cn;
    const double* rows_d;              // fp64 rows [s 3N | d 3N | n 3N] (host API) or null
    const double* weights;
    SolveState st;
    imls_iter_trace* tr;
    int update_pose, rows_are_double;
    const int* count;
    void* scratch;                     // ransac_bytes(N) device bytes (RANSAC only)
    int* rng;                          // [34] glibc rand() state, device (RANSAC only)
    RansacParams ransac;
};
void launch_solve(hipStream_t s, const SolveLaunch& L);
size_t ransac_bytes(int cap);
RansacFrame ransac_frame(void* scratch, int cap, int* rng);   // the carve of ransac_bytes(cap)
int ransac_init_tables(int device);    // the rand() jump table on `device` (current), once per device
constexpr int kMaxRansacBatch = 1024;  // frames per batched RANSAC launch
// Batched RANSAC (+ final LS / weighted LS / DRPM) for all frames of tab, ICP iteration `it`:
// one launch per step for the whole batch, every frame at its own count / rand() stream / done flag.
int launch_ransac_batch(hipStream_t s, const PairDev* tab, const int* n_host, int npairs, const KParams& kp,
                         const RansacParams& rp, int it);
void ransac_seed_host(uint32_t seed, int st[34]);

// scanreg.hip — ring-neighbourhood PCA normals + geometric-features presample (imls_ring_normals_pca)
int ring_pca_run(hipStream_t s, const imls_pca_params& p, const float* xyz, size_t stride, const int32_t* sizes,
                 int n_rings, DevBuf& mem, hipEvent_t* marks, uint32_t* index_out, float* normal_out,
                 float* evals_out, float* evecs_out, float* features_out, uint8_t* flags_out, size_t* n_out,
                 uint64_t counters[2], std::string& err);

// front.hip — scan front end: NaN + range filter, ring assignment, relative time (imls_scan_front_end)
int front_end_run(hipStream_t s, const imls_front_params& p, const float* xyz_host, size_t stride, size_t n_in,
                  DevBuf& mem, float* out_xyzi, uint32_t* out_index, int32_t* ring_sizes, size_t* n_out,
                  std::string& err);

// sample.hip — samplePointCloud "normal" / "major_axis" (imls_sample_point_cloud)
int sample_run(hipStream_t s, const imls_sample_params& p, const float* xyz, const float* nrm, size_t stride, size_t n,
               const int32_t* cand, size_t n_cand, const float* last_xyz, size_t last_stride, size_t m, DevBuf& mem,
               hipEvent_t* marks, int32_t* sampled_out, size_t* n_sampled, float* bin_weights_out, std::string& err);

}  // namespace imlsgpu
