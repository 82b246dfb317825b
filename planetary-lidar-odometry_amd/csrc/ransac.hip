// ransac.hip — SolveMotionEstimationProblemRANSAC (solver.cpp:222-385) with farthestPointSampling
// (common.cpp:19-82) and SolveMotionEstimationProblemDRPM (solver.cpp:486-603, degeneracy.h:14-131)
// on device, plus the solve-method dispatcher used by the ICP loop.
//
// Data flow per RANSAC solve (all on the context's stream, no host sync):
//   1. the valid correspondences (float rows, source order) are compacted, order kept, into fp64
//      rows S/D/N — the reference's std::vector<Vector3d> inputs; the TOO_FEW gate
//      (laser_odometry.cpp:570-576) runs on their count;
//   2. hypotheses in chunks (16, then up to kHypMax): k_ransac_hyp runs one hypothesis per block at
//      a time — its glibc rand() draw (the FPS start index) by the jump table below, FPS (two
//      arg-max passes, first index wins ties as the sequential `>` does), the 3×6 column-pivoted
//      Householder QR basic solution (Eigen ColPivHouseholderQR, not normal equations: a rank-3
//      system squared would misjudge the rank), Δ, and the inlier count; k_ransac_select (one
//      wave) scans the chunk in order with the reference's strict `>` and early exit
//      (best > ⌊pct·N⌋) and commits exactly the draws consumed; later chunks return at once;
//   3. inliers of the best Δ are compacted (order kept) with weights
//      w = √a < h₂ ? a : 2h₂√a − h₂², a = e^{−|r|}, h₂ = huber·distance (solver.cpp:334-356),
//      normalised by Σw (361-364; the division happens where the weight is read);
//   4. final solve: LS (trimmed, RANSAC's own threshold) / weighted LS through the LS chain on the
//      fp64 inlier rows, or DRPM: H = Σ w a aᵀ and g = Σ w a b (pass 1 of the LS chain), a cyclic
//      Jacobi eigendecomposition (SelfAdjointEigenSolver order: ascending), the per-point noise
//      mean/variance along the eigenvectors, normal-CDF probabilities with SNR factor 10, and
//      x = U·diag(p/λ)·Uᵀ g when min p < threshold, else the weighted solve.
// Batched frames (imls_register_frames, launch_ransac_batch): every step above is one launch for
// all frames (grid y = frame, the same bodies; each frame keeps its own count, rand() stream, chunk
// progress and done flag).
#include <algorithm>
#include <mutex>
#include <vector>

#include "solve_common.h"

namespace imlsgpu {
namespace {

// threads per hypothesis: one wave for small frames (its serial part — QR, Δ by one lane — then
// overlaps with other hypotheses on the same CU instead of idling three more waves), four for
// large ones (the three passes over the rows dominate).  Exact either way (arg-max and counts).
constexpr int kHypSmallRows = 4096;
__host__ __device__ constexpr int hyp_block_of(int cap) { return cap <= kHypSmallRows ? 64 : 256; }
#ifndef IMLS_QR_WAVE
#define IMLS_QR_WAVE 1                // a hypothesis' 3×6 QR by one wave, a column per lane (round 6)
#endif
constexpr int kHypUnroll = 8;        // FPS passes: rows per thread whose loads are in flight together
constexpr int kHypGrid = 8192;        // batched hypothesis grid (blocks stride over the running frames' items)
constexpr int kDrpmSlab = 42;         // 36 noise-mean terms + 6 variance terms per block
#ifdef IMLS_DEBUG_WAVE_TRACE
// phase clocks (100 MHz ticks) of block 0's hypothesis [0..5] and of k_drpm_head_small [8..13];
// [6], [14]: call counts (tools/ransac_probe.py with the debug build)
__device__ unsigned long long g_dbg_ransac[16];
#define RSTAMP(k) do { if (dbg_on) { g_dbg_ransac[k] += wall_clock64() - dbg_t; dbg_t = wall_clock64(); } } while (0)
#else
#define RSTAMP(k) do { } while (0)
#endif

// ---------------------------------------------------------------------------------------------
// glibc random() TYPE_3 (what rand() returns): state = a ring of 31 words + front / rear indices
// (st[31], st[32]; rear = front − 3 mod 31).  rand() adds ring[rear] into ring[front], returns that
// word >> 1 and advances both: the word sequence is x_i = x_{i−31} + x_{i−3} (mod 2^32), and with
// s_j = ring[(front + j) % 31] = x_{i−31+j} the k-th next word is x_{i+k} = Σ_j C[k][j]·s_j (mod 2^32)
// for fixed integer rows C[k] (C[m−31] = e_m for m < 31, C[k] = C[k−31] + C[k−3]).  So the draw of
// every hypothesis of a chunk is an independent 31-term dot product with the committed state (no
// serial replay), and committing `used` draws rebuilds the ring in one parallel step.  Integer
// arithmetic mod 2^32: exact in any summation order.
// ---------------------------------------------------------------------------------------------
__device__ unsigned g_rand_jump[kHypMax * 31];   // C[k][j], k < kHypMax (host-built, ransac_init_tables)

// x_{i+k} from the committed state; called by a whole wave (lanes < 31 hold one term each)
__device__ __forceinline__ unsigned rand_word_ahead(const int* __restrict__ st, int k) {
    const int lane = threadIdx.x & 63;
    unsigned term = 0u;
    if (lane < 31) {
        const int f = st[31];
        term = g_rand_jump[(size_t)k * 31 + lane] * (unsigned)st[(f + lane) % 31];
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) term += (unsigned)__shfl_xor((int)term, o, 64);
    return term;
}

// commit `used` draws: ring'[(front + used + j) % 31] = x_{i+used−31+j}; called by one whole wave
__device__ __forceinline__ void rand_commit(int* __restrict__ st, int used) {
    const int lane = threadIdx.x & 63;
    const int f = st[31], r = st[32];
    const unsigned sj = lane < 31 ? (unsigned)st[(f + lane) % 31] : 0u;   // s_j in lane j
    unsigned sv[31];                                                      // … and in every lane
#pragma unroll
    for (int j = 0; j < 31; ++j) sv[j] = (unsigned)__builtin_amdgcn_readlane((int)sj, j);
    const unsigned kept = (unsigned)__shfl((int)sj, used + lane, 64);     // x_{i+used−31+j} = s_{used+j}
    const int idx = used - 31 + lane;
    unsigned acc = 0u;
    if (lane < 31 && idx >= 0) {
#pragma unroll
        for (int j = 0; j < 31; ++j) acc += g_rand_jump[(size_t)idx * 31 + j] * sv[j];
    }
    __builtin_amdgcn_wave_barrier();
    if (lane < 31) st[(f + used + lane) % 31] = (int)(idx < 0 ? kept : acc);
    if (lane == 0) { st[31] = (f + used) % 31; st[32] = (r + used) % 31; }
}

// ---------------------------------------------------------------------------------------------
// Order-keeping compaction (count → scan → scatter) into fp64 row arrays of stride `cap`
// ---------------------------------------------------------------------------------------------
struct CompactOut {
    double* rows;       // [10·cap]: s[3·cap] | d[3·cap] | n[3·cap] (xyz per row) | w[cap] — the Rows layout
    int* count;         // [1]
    double* wsum;       // [1] Σw of the kept rows (inlier pass) — may be null
    int cap;
};

// Predicate + payload: valid correspondences of the projection (float rows), or inliers of Δ.
struct Source {
    const float4 *cs, *cd, *cn;       // float rows (valid flag cs.w), or null
    const double* rows;               // fp64 rows (Rows layout, stride cap) with count, or null
    const int* count;
    int cap;
    const double* T;                  // inlier pass: Δ (row-major 4×4)
    double dist_thr, h2;
    __device__ __forceinline__ bool get(int i, double s[3], double d[3], double n[3], double& w) const {
        if (cs) {
            const float4 s4 = cs[i];
            if (s4.w == 0.f) return false;
            const float4 d4 = cd[i], n4 = cn[i];
            s[0] = s4.x; s[1] = s4.y; s[2] = s4.z;
            d[0] = d4.x; d[1] = d4.y; d[2] = d4.z;
            n[0] = n4.x; n[1] = n4.y; n[2] = n4.z;
            w = 1.0;
            return true;
        }
        if (i >= *count) return false;
        const size_t c3 = 3 * (size_t)cap;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            s[k] = rows[3 * (size_t)i + k];
            d[k] = rows[c3 + 3 * (size_t)i + k];
            n[k] = rows[2 * c3 + 3 * (size_t)i + k];
        }
        if (!T) { w = 1.0; return true; }
        // solver.cpp:301-314 / 334-356: point-to-plane distance of Δ·s
        double tp[3];
#pragma unroll
        for (int r = 0; r < 3; ++r) tp[r] = ((T[r * 4] * s[0] + T[r * 4 + 1] * s[1]) + T[r * 4 + 2] * s[2]) + T[r * 4 + 3];
        const double dist = fabs(((tp[0] - d[0]) * n[0] + (tp[1] - d[1]) * n[1]) + (tp[2] - d[2]) * n[2]);
        if (!(dist < dist_thr)) return false;
        const double ar = exp(-fabs(dist));
        w = sqrt(ar) < h2 ? ar : 2 * h2 * sqrt(ar) - h2 * h2;
        return true;
    }
};

__device__ __forceinline__ void compact_count_body(const Source& src, int n, int* __restrict__ blkcnt,
                                                   double* __restrict__ blkw) {
    __shared__ int wc[kBlock / 64];
    __shared__ double ws[kBlock / 64];
    const int i = blockIdx.x * kBlock + threadIdx.x;
    double s[3], d[3], nn[3], w = 0.0;
    const bool keep = i < n && src.get(i, s, d, nn, w);
    const unsigned long long m = __ballot(keep);
    const double wv = wave_sum(keep ? w : 0.0);
    if ((threadIdx.x & 63) == 0) { wc[threadIdx.x >> 6] = __popcll(m); ws[threadIdx.x >> 6] = wv; }
    __syncthreads();
    if (threadIdx.x == 0) {
        int c = 0;
        double sw = 0.0;
        for (int k = 0; k < kBlock / 64; ++k) { c += wc[k]; sw += ws[k]; }
        blkcnt[blockIdx.x] = c;
        blkw[blockIdx.x] = sw;
    }
}

// What runs after a compaction, by thread 0 with the kept count (one launch fewer each): the RANSAC
// begin (the TOO_FEW gate, laser_odometry.cpp:570-576, and the selection reset) after the valid-row
// compaction; the empty-inlier check after the inlier one.
struct CompactPost {
    int kind;                         // 0 none, 1 RANSAC begin, 2 inlier check
    int correspond_number, update_pose;
    SolveState st;
    imls_iter_trace* tr;
    RansacDev R;
};
__device__ __forceinline__ void ransac_begin_t0(int n, int correspond_number, int update_pose, const SolveState& st,
                                                imls_iter_trace* tr, const RansacDev& R) {
    *R.active = 1;
    if (update_pose && n < correspond_number) {
        *st.status = IMLS_FRAME_TOO_FEW;
        *st.done = 1;
        if (tr) tr->n_valid = (unsigned long long)n;
        return;
    }
    *R.best = 0;
    *R.evaluated = 0;
    *R.rdone = n < 3 ? 1 : 0;   // FPS needs three distinct points
#pragma unroll
    for (int k = 0; k < 16; ++k) R.bestT[k] = (k % 5 == 0) ? 1.0 : 0.0;
}
__device__ __forceinline__ void compact_post(const CompactPost& P, int n) {
    if (P.kind == 1) {
        ransac_begin_t0(n, P.correspond_number, P.update_pose, P.st, P.tr, P.R);
    } else if (P.kind == 2 && n == 0) {   // nothing to solve on (the oracle's N == 0 → false): a failed solve
        *P.st.status = IMLS_FRAME_SOLVE_FAILED;
        *P.st.done = 1;
    }
}
// a finished frame skips the compaction; its RANSAC solve is then inactive (no trace record)
__device__ __forceinline__ bool compact_skip(const CompactPost& P) {
    if (!*P.st.done) return false;
    if (P.kind == 1 && threadIdx.x == 0) *P.R.active = 0;
    return true;
}

// One block: exclusive scan of the block counts (in place), total count and Σw in fixed order.
__device__ __forceinline__ void compact_scan_body(int* __restrict__ blkcnt, const double* __restrict__ blkw, int nb,
                                                  const CompactOut& out, const CompactPost& P) {
    __shared__ int sc[1024];
    __shared__ double sw[1024];
    int carry = 0;
    double wcarry = 0.0;
    for (int base = 0; base < nb; base += 1024) {
        const int b = base + threadIdx.x;
        const int v = b < nb ? blkcnt[b] : 0;
        sc[threadIdx.x] = v;
        sw[threadIdx.x] = b < nb ? blkw[b] : 0.0;
        __syncthreads();
        for (int off = 1; off < 1024; off <<= 1) {
            const int t = threadIdx.x >= off ? sc[threadIdx.x - off] : 0;
            __syncthreads();
            sc[threadIdx.x] += t;
            __syncthreads();
        }
        if (b < nb) blkcnt[b] = carry + sc[threadIdx.x] - v;
        if (threadIdx.x == 0) {
            double acc = 0.0;
            for (int k = 0; k < 1024 && base + k < nb; ++k) acc += sw[k];
            sw[0] = acc;   // reuse after the scan: chunk sum
        }
        __syncthreads();
        carry += sc[1023];
        wcarry += sw[0];
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        *out.count = carry;
        if (out.wsum) *out.wsum = wcarry;
        compact_post(P, carry);
    }
}

// The whole compaction in one 1024-thread block (count + scan + scatter, for caps ≤ kCompactOne):
// tiles of 1024 rows in order; Σw accumulated exactly as the three-kernel path does it (per-wave
// sums, 4 waves per 256-row block in order, then the block sums in block order) — same bits.
constexpr int kCompactOne = 16384;
__device__ __forceinline__ void compact_one_body(const Source& src, int n, const CompactOut& out, const CompactPost& P) {
    __shared__ int wc[16];
    __shared__ double ws[16];
    __shared__ int sbase;
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    if (t == 0) sbase = 0;
    double wacc = 0.0;                                     // thread 0
    for (int tile = 0; tile < n; tile += 1024) {
        const int i = tile + t;
        double s[3], d[3], nn[3], w = 0.0;
        const bool keep = i < n && src.get(i, s, d, nn, w);
        const unsigned long long m = __ballot(keep);
        const double wvs = wave_sum(keep ? w : 0.0);
        if (lane == 0) { wc[wv] = __popcll(m); ws[wv] = wvs; }
        __syncthreads();
        int off = sbase;
        for (int k = 0; k < wv; ++k) off += wc[k];
        off += __popcll(m & ((1ull << lane) - 1ull));
        if (keep) {
            const size_t c3 = 3 * (size_t)out.cap, o = (size_t)off;
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                out.rows[3 * o + k] = s[k];
                out.rows[c3 + 3 * o + k] = d[k];
                out.rows[2 * c3 + 3 * o + k] = nn[k];
            }
            out.rows[3 * c3 + o] = w;
        }
        __syncthreads();
        if (t == 0) {
            int tot = 0;
            for (int b = 0; b < 4; ++b) {
                if (tile + 256 * b >= n) break;            // blocks past n do not exist in the 3-kernel path
                double sw = 0.0;
                for (int k = 0; k < 4; ++k) { sw += ws[4 * b + k]; tot += wc[4 * b + k]; }
                wacc += sw;
            }
            sbase += tot;
        }
        __syncthreads();
    }
    if (t == 0) {
        *out.count = sbase;
        if (out.wsum) *out.wsum = wacc;
        compact_post(P, sbase);
    }
}

__device__ __forceinline__ void compact_scatter_body(const Source& src, int n, const int* __restrict__ blkoff,
                                                     const CompactOut& out) {
    __shared__ int wc[kBlock / 64];
    const int i = blockIdx.x * kBlock + threadIdx.x;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    double s[3], d[3], nn[3], w = 0.0;
    const bool keep = i < n && src.get(i, s, d, nn, w);
    const unsigned long long m = __ballot(keep);
    if (lane == 0) wc[wv] = __popcll(m);
    __syncthreads();
    int off = blkoff[blockIdx.x];
    for (int k = 0; k < wv; ++k) off += wc[k];
    off += __popcll(m & ((1ull << lane) - 1ull));
    if (keep) {
        const size_t c3 = 3 * (size_t)out.cap, o = (size_t)off;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            out.rows[3 * o + k] = s[k];
            out.rows[c3 + 3 * o + k] = d[k];
            out.rows[2 * c3 + 3 * o + k] = nn[k];
        }
        out.rows[3 * c3 + o] = w;
    }
}

__global__ __launch_bounds__(kBlock) void k_compact_count(Source src, int n, int* __restrict__ blkcnt,
                                                          double* __restrict__ blkw, const int* __restrict__ done) {
    if (done && *done) return;
    compact_count_body(src, n, blkcnt, blkw);
}
__global__ __launch_bounds__(1024) void k_compact_scan(int* __restrict__ blkcnt, const double* __restrict__ blkw, int nb,
                                                       CompactOut out, CompactPost P) {
    if (compact_skip(P)) return;
    compact_scan_body(blkcnt, blkw, nb, out, P);
}
__global__ __launch_bounds__(1024) void k_compact_one(Source src, int n, CompactOut out, CompactPost P) {
    if (compact_skip(P)) return;
    compact_one_body(src, n, out, P);
}
__global__ __launch_bounds__(kBlock) void k_compact_scatter(Source src, int n, const int* __restrict__ blkoff, CompactOut out,
                                                            const int* __restrict__ done) {
    if (done && *done) return;
    compact_scatter_body(src, n, blkoff, out);
}

// The two compactions of a batched frame: mode 0 = its valid float rows (the projection's output)
// → F.all; mode 1 = the inliers of its best Δ, weighted → F.inl (+ Σw).
__device__ __forceinline__ int frame_compact(const PairDev& A, int mode, double dist_thr, double h2, Source& src,
                                             CompactOut& out) {
    const RansacFrame& F = A.rf;
    src = Source{};
    if (mode == 0) {
        src.cs = A.cs; src.cd = A.cd; src.cn = A.cn;
        out = CompactOut{F.all, F.cnt_all, nullptr, F.cap};
        return A.N;
    }
    src.rows = F.all; src.count = F.cnt_all; src.cap = F.cap; src.T = F.R.bestT;
    src.dist_thr = dist_thr; src.h2 = h2;
    out = CompactOut{F.inl, F.cnt_in, F.wsum, F.cap};
    return F.cap;
}
__global__ __launch_bounds__(kBlock) void k_compact_count_b(const PairDev* __restrict__ tab, int mode, double dist_thr,
                                                            double h2) {
    const PairDev A = device_view(tab + blockIdx.y);
    Source src;
    CompactOut out;
    const int n = frame_compact(A, mode, dist_thr, h2, src, out);
    if ((int)blockIdx.x >= (n + kBlock - 1) / kBlock || *A.st.done) return;
    compact_count_body(src, n, A.rf.blkcnt, A.rf.blkw);
}
__device__ __forceinline__ CompactPost frame_post(const PairDev& A, int mode, int correspond_number, int it) {
    return CompactPost{mode == 0 ? 1 : 2, correspond_number, 1, A.st, A.trace + it, A.rf.R};
}
__global__ __launch_bounds__(1024) void k_compact_scan_b(const PairDev* __restrict__ tab, int mode, int correspond_number,
                                                         int it) {
    const PairDev A = device_view(tab + blockIdx.y);
    const CompactPost P = frame_post(A, mode, correspond_number, it);
    if (compact_skip(P)) return;
    Source src;
    CompactOut out;
    const int n = frame_compact(A, mode, 0.0, 0.0, src, out);
    compact_scan_body(A.rf.blkcnt, A.rf.blkw, (n + kBlock - 1) / kBlock, out, P);
}
__global__ __launch_bounds__(1024) void k_compact_one_b(const PairDev* __restrict__ tab, int mode, double dist_thr, double h2,
                                                        int correspond_number, int it) {
    const PairDev A = device_view(tab + blockIdx.y);
    const CompactPost P = frame_post(A, mode, correspond_number, it);
    if (compact_skip(P)) return;
    Source src;
    CompactOut out;
    const int n = frame_compact(A, mode, dist_thr, h2, src, out);
    compact_one_body(src, n, out, P);
}
__global__ __launch_bounds__(kBlock) void k_compact_scatter_b(const PairDev* __restrict__ tab, int mode, double dist_thr,
                                                              double h2) {
    const PairDev A = device_view(tab + blockIdx.y);
    Source src;
    CompactOut out;
    const int n = frame_compact(A, mode, dist_thr, h2, src, out);
    if ((int)blockIdx.x >= (n + kBlock - 1) / kBlock || *A.st.done) return;
    compact_scatter_body(src, n, A.rf.blkcnt, out);
}

// stand-alone DRPM with no rows fails like the oracle's solve_drpm (N == 0 → false)
__global__ void k_drpm_guard(const int* __restrict__ c, SolveState st) {
    if (threadIdx.x == 0 && *c == 0) { *st.status = IMLS_FRAME_SOLVE_FAILED; *st.done = 1; }
}

__global__ void k_set_count(int* __restrict__ c, int v) {
    if (threadIdx.x == 0) *c = v;
}

// gate on the count, reset the RANSAC selection state (host fp64 rows, no compaction to fold it into)
__global__ void k_ransac_begin(const int* __restrict__ count, int correspond_number, int update_pose, SolveState st,
                               imls_iter_trace* tr, RansacDev R) {
    if (threadIdx.x) return;
    if (*st.done) { *R.active = 0; return; }
    ransac_begin_t0(*count, correspond_number, update_pose, st, tr, R);
}

// block arg-max of (value, index): larger value, then smaller index
template <int NT>
__device__ __forceinline__ void argmax_pair(double& v, int& i, double* sv, int* si) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const double ov = __shfl_xor(v, o, 64);
        const int oi = __shfl_xor(i, o, 64);
        if (ov > v || (ov == v && oi < i)) { v = ov; i = oi; }
    }
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    if (lane == 0) { sv[wv] = v; si[wv] = i; }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int k = 1; k < NT / 64; ++k)
            if (sv[k] > sv[0] || (sv[k] == sv[0] && si[k] < si[0])) { sv[0] = sv[k]; si[0] = si[k]; }
    }
    __syncthreads();
    v = sv[0];
    i = si[0];
    __syncthreads();
}

// Eigen ColPivHouseholderQR(R×6).solve(b): basic solution (free unknowns zero).  R is tiny (3);
// every loop is unrolled with constant indices, the pivot swap is predicated.
template <int RR>
__device__ void colpiv_qr_small(double A[RR][6], double b[RR], double x[6]) {
    constexpr int C = 6, S = RR < C ? RR : C;
    const double eps = DBL_EPSILON;
    double nu[C], nd[C], hc[S];
    int perm[C];
#pragma unroll
    for (int k = 0; k < C; ++k) {
        double s = 0;
#pragma unroll
        for (int r = 0; r < RR; ++r) s += A[r][k] * A[r][k];
        nu[k] = nd[k] = sqrt(s);
        perm[k] = k;
    }
    double maxnorm = 0;
#pragma unroll
    for (int k = 0; k < C; ++k) maxnorm = fmax(maxnorm, nu[k]);
    const double thr_helper = (maxnorm * eps) * (maxnorm * eps) / (double)RR;
    const double ndt = sqrt(eps);
    int nonzero = S;
    double maxpivot = 0;
#pragma unroll
    for (int k = 0; k < S; ++k) {
        int big = k;
        double bv = nu[k];
#pragma unroll
        for (int j = k + 1; j < C; ++j)
            if (nu[j] > bv) { bv = nu[j]; big = j; }
        if (nonzero == S && bv * bv < thr_helper * (double)(RR - k)) nonzero = k;
#pragma unroll
        for (int j = k + 1; j < C; ++j) {
            if (j == big) {
#pragma unroll
                for (int r = 0; r < RR; ++r) { const double t = A[r][k]; A[r][k] = A[r][j]; A[r][j] = t; }
                double t = nu[k]; nu[k] = nu[j]; nu[j] = t;
                t = nd[k]; nd[k] = nd[j]; nd[j] = t;
                const int ti = perm[k]; perm[k] = perm[j]; perm[j] = ti;
            }
        }
        // makeHouseholderInPlace on column k, rows k..RR−1
        const double c0 = A[k][k];
        double tail = 0;
#pragma unroll
        for (int r = k + 1; r < RR; ++r) tail += A[r][k] * A[r][k];
        double tau, beta;
        if (tail <= DBL_MIN) {
            tau = 0;
            beta = c0;
#pragma unroll
            for (int r = k + 1; r < RR; ++r) A[r][k] = 0;
        } else {
            beta = sqrt(c0 * c0 + tail);
            if (c0 >= 0) beta = -beta;
#pragma unroll
            for (int r = k + 1; r < RR; ++r) A[r][k] = A[r][k] / (c0 - beta);
            tau = (beta - c0) / beta;
        }
        hc[k] = tau;
        A[k][k] = beta;
        if (fabs(beta) > maxpivot) maxpivot = fabs(beta);
        if (tau != 0) {
#pragma unroll
            for (int j = k + 1; j < C; ++j) {
                double tmp = A[k][j];
#pragma unroll
                for (int r = k + 1; r < RR; ++r) tmp += A[r][k] * A[r][j];
                A[k][j] -= tau * tmp;
#pragma unroll
                for (int r = k + 1; r < RR; ++r) A[r][j] -= tau * A[r][k] * tmp;
            }
        }
#pragma unroll
        for (int j = k + 1; j < C; ++j) {
            if (nu[j] != 0) {
                double temp = fabs(A[k][j]) / nu[j];
                temp = (1 + temp) * (1 - temp);
                temp = temp < 0 ? 0 : temp;
                const double r2 = nu[j] / nd[j];
                const double temp2 = temp * r2 * r2;
                if (temp2 <= ndt) {
                    double s = 0;
#pragma unroll
                    for (int r = k + 1; r < RR; ++r) s += A[r][j] * A[r][j];
                    nd[j] = nu[j] = sqrt(s);
                } else {
                    nu[j] *= sqrt(temp);
                }
            }
        }
    }
    const double thr = eps * (double)S;
    int nz = 0;
#pragma unroll
    for (int i = 0; i < S; ++i) nz += (i < nonzero && fabs(A[i][i]) > thr * maxpivot) ? 1 : 0;
#pragma unroll
    for (int c = 0; c < C; ++c) x[c] = 0;
    if (nz == 0) return;
#pragma unroll
    for (int k = 0; k < S; ++k) {
        if (k < nz) {
            const double tau = hc[k];
            if (RR - k == 1) {
                b[k] *= 1 - tau;
            } else if (tau != 0) {
                double tmp = b[k];
#pragma unroll
                for (int r = k + 1; r < RR; ++r) tmp += A[r][k] * b[r];
                b[k] -= tau * tmp;
#pragma unroll
                for (int r = k + 1; r < RR; ++r) b[r] -= tau * A[r][k] * tmp;
            }
        }
    }
#pragma unroll
    for (int i = S - 1; i >= 0; --i) {
        if (i < nz) {
            double s = b[i];
#pragma unroll
            for (int j = i + 1; j < S; ++j)
                if (j < nz) s -= A[i][j] * b[j];
            b[i] = s / A[i][i];
        }
    }
#pragma unroll
    for (int c = 0; c < C; ++c) {
        double v = 0;
#pragma unroll
        for (int i = 0; i < S; ++i)
            if (i < nz && perm[i] == c) v = b[i];
        x[c] = v;
    }
}

// colpiv_qr_small<3> by one wave (round 6), lane c < 6 holding column c of A (a[r] = A[r][c]) with its
// norms and original index: the pivot search reads the six norms, a swap exchanges two lanes' columns,
// the Householder vector of column k is formed by every lane from lane k's column (the same scalar
// expressions, so the same bits everywhere), and the update and the norm downdate of the columns
// right of k run on their own lanes — the one-lane routine's operations, each on the lane that owns
// the column, so x is its result bit for bit.  The back-substitution (3×3) runs on every lane from the
// gathered factor.  A hypothesis block's QR 4.8 µs on one lane (tools/ransac_probe.py phase clocks).
__device__ void colpiv_qr3_wave(double a[3], double b[3], double x[6]) {
    constexpr int RR = 3, C = 6, S = 3;
    const int lane = threadIdx.x & 63;
    const double eps = DBL_EPSILON;
    double nu, nd;
    int perm = lane;
    {
        double sq = 0;
#pragma unroll
        for (int r = 0; r < RR; ++r) sq += a[r] * a[r];
        nu = nd = sqrt(sq);
    }
    double maxnorm = 0;
#pragma unroll
    for (int k = 0; k < C; ++k) maxnorm = fmax(maxnorm, readlane_f64(nu, k));
    const double thr_helper = (maxnorm * eps) * (maxnorm * eps) / (double)RR;
    const double ndt = sqrt(eps);
    int nonzero = S;
    double maxpivot = 0;
    double hc[S];
#pragma unroll
    for (int k = 0; k < S; ++k) {
        int big = k;
        double bv = readlane_f64(nu, k);
#pragma unroll
        for (int j = k + 1; j < C; ++j) {
            const double nj = readlane_f64(nu, j);
            if (nj > bv) { bv = nj; big = j; }
        }
        if (nonzero == S && bv * bv < thr_helper * (double)(RR - k)) nonzero = k;
        if (big != k) {                       // wave-uniform: exchange the columns of lanes k and big
            double ak[RR], ab[RR];
#pragma unroll
            for (int r = 0; r < RR; ++r) { ak[r] = readlane_f64(a[r], k); ab[r] = readlane_f64(a[r], big); }
            const double nuk = readlane_f64(nu, k), nub = readlane_f64(nu, big);
            const double ndk = readlane_f64(nd, k), ndb = readlane_f64(nd, big);
            const int pk = __builtin_amdgcn_readlane(perm, k), pb = __builtin_amdgcn_readlane(perm, big);
            if (lane == k) {
#pragma unroll
                for (int r = 0; r < RR; ++r) a[r] = ab[r];
                nu = nub; nd = ndb; perm = pb;
            } else if (lane == big) {
#pragma unroll
                for (int r = 0; r < RR; ++r) a[r] = ak[r];
                nu = nuk; nd = ndk; perm = pk;
            }
        }
        // makeHouseholderInPlace on column k, rows k..RR−1 (every lane, from lane k's column)
        double col[RR];
#pragma unroll
        for (int r = 0; r < RR; ++r) col[r] = readlane_f64(a[r], k);
        const double c0 = col[k];
        double tail = 0;
#pragma unroll
        for (int r = k + 1; r < RR; ++r) tail += col[r] * col[r];
        double tau, beta, v[RR];
        if (tail <= DBL_MIN) {
            tau = 0;
            beta = c0;
#pragma unroll
            for (int r = k + 1; r < RR; ++r) v[r] = 0;
        } else {
            beta = sqrt(c0 * c0 + tail);
            if (c0 >= 0) beta = -beta;
#pragma unroll
            for (int r = k + 1; r < RR; ++r) v[r] = col[r] / (c0 - beta);
            tau = (beta - c0) / beta;
        }
        hc[k] = tau;
        if (lane == k) {
            a[k] = beta;
#pragma unroll
            for (int r = k + 1; r < RR; ++r) a[r] = v[r];
        }
        if (fabs(beta) > maxpivot) maxpivot = fabs(beta);
        if (lane > k && lane < C) {
            if (tau != 0) {
                double tmp = a[k];
#pragma unroll
                for (int r = k + 1; r < RR; ++r) tmp += v[r] * a[r];
                a[k] -= tau * tmp;
#pragma unroll
                for (int r = k + 1; r < RR; ++r) a[r] -= tau * v[r] * tmp;
            }
            if (nu != 0) {
                double temp = fabs(a[k]) / nu;
                temp = (1 + temp) * (1 - temp);
                temp = temp < 0 ? 0 : temp;
                const double r2 = nu / nd;
                const double temp2 = temp * r2 * r2;
                if (temp2 <= ndt) {
                    double sq = 0;
#pragma unroll
                    for (int r = k + 1; r < RR; ++r) sq += a[r] * a[r];
                    nd = nu = sqrt(sq);
                } else {
                    nu *= sqrt(temp);
                }
            }
        }
    }
    // the factor's first S columns and the permutation, on every lane; the one-lane solve from here
    double A[RR][S];
    int pm[S];
#pragma unroll
    for (int c = 0; c < S; ++c) {
#pragma unroll
        for (int r = 0; r < RR; ++r) A[r][c] = readlane_f64(a[r], c);
        pm[c] = __builtin_amdgcn_readlane(perm, c);
    }
    const double thr = eps * (double)S;
    int nz = 0;
#pragma unroll
    for (int i = 0; i < S; ++i) nz += (i < nonzero && fabs(A[i][i]) > thr * maxpivot) ? 1 : 0;
#pragma unroll
    for (int c = 0; c < C; ++c) x[c] = 0;
    if (nz == 0) return;
#pragma unroll
    for (int k = 0; k < S; ++k) {
        if (k < nz) {
            const double tau = hc[k];
            if (RR - k == 1) {
                b[k] *= 1 - tau;
            } else if (tau != 0) {
                double tmp = b[k];
#pragma unroll
                for (int r = k + 1; r < RR; ++r) tmp += A[r][k] * b[r];
                b[k] -= tau * tmp;
#pragma unroll
                for (int r = k + 1; r < RR; ++r) b[r] -= tau * A[r][k] * tmp;
            }
        }
    }
#pragma unroll
    for (int i = S - 1; i >= 0; --i) {
        if (i < nz) {
            double sacc = b[i];
#pragma unroll
            for (int j = i + 1; j < S; ++j)
                if (j < nz) sacc -= A[i][j] * b[j];
            b[i] = sacc / A[i][i];
        }
    }
#pragma unroll
    for (int c = 0; c < C; ++c) {
        double val = 0;
#pragma unroll
        for (int i = 0; i < S; ++i)
            if (i < nz && pm[i] == c) val = b[i];
        x[c] = val;
    }
}

// Hypothesis h of the current chunk, by one block: its draw (the FPS start) from the committed
// rand() state, FPS(3), the 3×6 QR, Δ, its inlier count.
template <int NT>
__device__ __forceinline__ void ransac_hyp_one(const double* __restrict__ S, const double* __restrict__ Dp,
                                               const double* __restrict__ Np, int n, const RansacDev& R,
                                               double dist_thr, int h) {
    __shared__ double sv[NT / 64];
    __shared__ int si[NT / 64];
    __shared__ double T[16];
    __shared__ int cnt_s[NT / 64];
#ifdef IMLS_DEBUG_WAVE_TRACE
    const bool dbg_on = blockIdx.x == 0 && threadIdx.x == 0 && h == 0;
    long long dbg_t = wall_clock64();
    if (dbg_on) g_dbg_ransac[6] += 1;
#endif
    const int f0 = (int)(rand_word_ahead(R.rng, h) >> 1) % n;   // rand() % n (solver.cpp / common.cpp:49)
    // The two FPS passes: the taken points' coordinates in registers, each thread's rows in groups of
    // kHypUnroll whose loads are all issued before the first compare (round 6: the loop reloaded
    // s_f0 and waited on every row's load in turn — one L2 round trip per row, the lone frame's
    // k_ransac_hyp 31 µs per chunk).  A thread still visits its rows in ascending order and keeps the
    // first maximum (strict `>`), so the arg-max — larger value, then smaller index — is unchanged.
    const double a0 = S[3 * (size_t)f0], a1 = S[3 * (size_t)f0 + 1], a2 = S[3 * (size_t)f0 + 2];
    auto dist = [](double x0, double x1, double x2, const double (&b)[3]) {   // pdist(s, a, b): ‖s_a − s_b‖
        const double dx = x0 - b[0], dy = x1 - b[1], dz = x2 - b[2];
        return sqrt((dx * dx + dy * dy) + dz * dz);
    };
    auto load_rows = [&](int i0, double (&p)[kHypUnroll][3]) {
#pragma unroll
        for (int u = 0; u < kHypUnroll; ++u) {
            const size_t i3 = 3 * (size_t)min(i0 + u * NT, n - 1);
            p[u][0] = S[i3]; p[u][1] = S[i3 + 1]; p[u][2] = S[i3 + 2];
        }
    };
    // pass 1: farthest from f0 (common.cpp:48-66: strict `>` from −1, taken points skipped)
    double bv = -1.0;
    int bi = 0x7fffffff;
    for (int i0 = threadIdx.x; i0 < n; i0 += kHypUnroll * NT) {
        double p[kHypUnroll][3];
        load_rows(i0, p);
#pragma unroll
        for (int u = 0; u < kHypUnroll; ++u) {
            const int i = i0 + u * NT;
            if (i >= n || i == f0) continue;
            const double md = dist(a0, a1, a2, p[u]);
            if (md > bv) { bv = md; bi = i; }
        }
    }
    argmax_pair<NT>(bv, bi, sv, si);
    RSTAMP(0);
    const int f1 = bi;
    // pass 2: farthest from {f0, f1} by the running minimum distance
    const double c0 = S[3 * (size_t)f1], c1 = S[3 * (size_t)f1 + 1], c2 = S[3 * (size_t)f1 + 2];
    bv = -1.0;
    bi = 0x7fffffff;
    for (int i0 = threadIdx.x; i0 < n; i0 += kHypUnroll * NT) {
        double p[kHypUnroll][3];
        load_rows(i0, p);
#pragma unroll
        for (int u = 0; u < kHypUnroll; ++u) {
            const int i = i0 + u * NT;
            if (i >= n || i == f0 || i == f1) continue;
            const double md = fmin(dist(a0, a1, a2, p[u]), dist(c0, c1, c2, p[u]));
            if (md > bv) { bv = md; bi = i; }
        }
    }
    argmax_pair<NT>(bv, bi, sv, si);
    RSTAMP(1);
    const int f2 = bi;
#if IMLS_QR_WAVE
    if (threadIdx.x < 64) {                   // wave 0: lane c builds column c of the 3×6 system
        const int id[3] = {f0, f1, f2};
        const int lane = threadIdx.x, cc = lane < 6 ? lane : 0;
        double a[3], b[3], x[6];
#pragma unroll
        for (int r = 0; r < 3; ++r) {
            const int k = id[r];
            const double s0 = S[3 * k], s1 = S[3 * k + 1], s2 = S[3 * k + 2];
            const double d0 = Dp[3 * k], d1 = Dp[3 * k + 1], d2 = Dp[3 * k + 2];
            const double n0 = Np[3 * k], n1 = Np[3 * k + 1], n2 = Np[3 * k + 2];
            const double col[6] = {n2 * s1 - n1 * s2, n0 * s2 - n2 * s0, n1 * s0 - n0 * s1, n0, n1, n2};
            double v = col[0];
#pragma unroll
            for (int c = 1; c < 6; ++c) v = cc == c ? col[c] : v;
            a[r] = v;
            double bb = n0 * (d0 - s0);
            bb = bb + n1 * (d1 - s1);
            bb = bb + n2 * (d2 - s2);
            b[r] = bb;
        }
        colpiv_qr3_wave(a, b, x);
        RSTAMP(2);
        if (lane == 0) {
            double D[16];
            delta_from_x(x, D);
            RSTAMP(3);
#pragma unroll
            for (int k = 0; k < 16; ++k) T[k] = D[k];
        }
    }
#else
    if (threadIdx.x == 0) {
        const int id[3] = {f0, f1, f2};
        double A[3][6], b[3], x[6], D[16];
#pragma unroll
        for (int r = 0; r < 3; ++r) {
            const int k = id[r];
            const double s0 = S[3 * k], s1 = S[3 * k + 1], s2 = S[3 * k + 2];
            const double d0 = Dp[3 * k], d1 = Dp[3 * k + 1], d2 = Dp[3 * k + 2];
            const double n0 = Np[3 * k], n1 = Np[3 * k + 1], n2 = Np[3 * k + 2];
            A[r][0] = n2 * s1 - n1 * s2;
            A[r][1] = n0 * s2 - n2 * s0;
            A[r][2] = n1 * s0 - n0 * s1;
            A[r][3] = n0; A[r][4] = n1; A[r][5] = n2;
            double bb = n0 * (d0 - s0);
            bb = bb + n1 * (d1 - s1);
            bb = bb + n2 * (d2 - s2);
            b[r] = bb;
        }
        colpiv_qr_small<3>(A, b, x);
        RSTAMP(2);
        delta_from_x(x, D);
        RSTAMP(3);
#pragma unroll
        for (int k = 0; k < 16; ++k) T[k] = D[k];
    }
#endif
    __syncthreads();
    int c = 0;
    for (int i = threadIdx.x; i < n; i += NT) {
        const size_t i3 = 3 * (size_t)i;
        const double s0 = S[i3], s1 = S[i3 + 1], s2 = S[i3 + 2];
        double tp[3];
#pragma unroll
        for (int r = 0; r < 3; ++r) tp[r] = ((T[r * 4] * s0 + T[r * 4 + 1] * s1) + T[r * 4 + 2] * s2) + T[r * 4 + 3];
        const double dist = fabs(((tp[0] - Dp[i3]) * Np[i3] + (tp[1] - Dp[i3 + 1]) * Np[i3 + 1]) + (tp[2] - Dp[i3 + 2]) * Np[i3 + 2]);
        c += dist < dist_thr ? 1 : 0;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
    if ((threadIdx.x & 63) == 0) cnt_s[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
        int tot = 0;
        for (int k = 0; k < NT / 64; ++k) tot += cnt_s[k];
        R.counts[h] = tot;
    }
    if (threadIdx.x < 16) R.T[(size_t)h * 16 + threadIdx.x] = T[threadIdx.x];
    RSTAMP(4);
}
// one frame: hypotheses blockIdx.x, blockIdx.x + gridDim.x, … of the chunk.
// base > 0 (a lone frame's second chunk, its hypotheses base … base + chunk − 1 of the same draw
// sequence): nothing is selected or committed between the chunks — every block first looks for a
// hypothesis of the first chunk above the inlier minimum (the first chunk's selection would have
// stopped RANSAC there) and leaves if there is one; one selection over both chunks follows (at the head
// of k_drpm_head_small), which is the two sequential selections' result: the first exceeding
// hypothesis ends the scan, the first maximum before it wins, exactly `used` draws are committed.
template <int NT>
__global__ __launch_bounds__(NT) void k_ransac_hyp(const double* __restrict__ rows, const int* __restrict__ count,
                                                   int cap, RansacDev R, double dist_thr, int chunk,
                                                   const int* __restrict__ done, int base, double min_pct) {
    if (*done || *R.rdone) return;
    const int n = *count;
    if (base > 0) {
        __shared__ int hit;
        const int min_inliers = (int)(min_pct * (double)n);   // as ransac_select_body
        if (threadIdx.x == 0) hit = 0;
        __syncthreads();
        for (int h = threadIdx.x; h < base; h += NT)
            if (R.counts[h] > min_inliers) hit = 1;
        __syncthreads();
        if (hit) return;
    }
    const size_t c3 = 3 * (size_t)cap;
    for (int h = blockIdx.x; h < chunk; h += gridDim.x)
        ransac_hyp_one<NT>(rows, rows + c3, rows + 2 * c3, n, R, dist_thr, base + h);
}

// Sequential semantics of the hypothesis loop (solver.cpp:244-326) over one chunk, by one wave: the
// loop stops at the first hypothesis whose count exceeds ⌊pct·N⌋ (best > min_inliers first holds
// there, since best ≤ min_inliers on entry); best / bestT follow the strict `>` (first maximum
// wins); exactly the draws consumed are committed.
__device__ __forceinline__ void ransac_select_body(const int* __restrict__ count, const RansacDev& R, int chunk,
                                                   int max_iterations, double min_pct) {
    const int lane = threadIdx.x & 63;
    const int n = *count;
    const int min_inliers = (int)(min_pct * (double)n);
    int best = *R.best, bi = -1, used = chunk;
    for (int base = 0; base < chunk; base += 64) {
        const int h = base + lane;
        const int c = h < chunk ? R.counts[h] : INT_MIN;
        const unsigned long long sm = __ballot(h < chunk && c > min_inliers);
        const int lim = sm ? (int)__builtin_ctzll(sm) : 63;
        int v = lane <= lim ? c : INT_MIN, vi = h;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            const int ov = __shfl_xor(v, o, 64), oi = __shfl_xor(vi, o, 64);
            if (ov > v || (ov == v && oi < vi)) { v = ov; vi = oi; }
        }
        if (v > best) { best = v; bi = vi; }
        if (sm) { used = base + lim + 1; break; }
    }
    if (bi >= 0 && lane < 16) R.bestT[lane] = R.T[(size_t)bi * 16 + lane];
    rand_commit(R.rng, used);                 // commit exactly the draws consumed
    if (lane == 0) {
        *R.best = best;
        const int evaluated = *R.evaluated + used;
        *R.evaluated = evaluated;
        if (used < chunk || best > min_inliers || evaluated >= max_iterations) *R.rdone = 1;
    }
}
__global__ __launch_bounds__(64) void k_ransac_select(const int* __restrict__ count, RansacDev R, int chunk,
                                                     int max_iterations, double min_pct, const int* __restrict__ done) {
    if (*done || *R.rdone) return;
    ransac_select_body(count, R, chunk, max_iterations, min_pct);
}

// trace of a RANSAC iteration as the oracle records it: n_valid = correspondences, n_kept = 0
__global__ void k_ransac_trace(const int* __restrict__ count_all, RansacDev R, imls_iter_trace* tr) {
    if (threadIdx.x || !*R.active || !tr) return;
    tr->n_valid = (unsigned long long)*count_all;
    tr->n_kept = 0;
}


// ---------------------------------------------------------------------------------------------
// DRPM (solver.cpp:499-603, degeneracy.h:14-131)
// ---------------------------------------------------------------------------------------------
// The wave's totals of the 42 DRPM terms by recursive halving (internal.h wave_sum28's scheme): terms
// 0..31 in one pass (31 + 1 fp64 exchanges), 32..41 padded to 16 in another (15 + 2) — 49 exchanges
// where 42 butterfly wave_sums issued 252 (round 6).  Lane 2k returns total k in r0 (k < 32) and
// total 32 + k in r1 (k < 10).  A fixed association shared by every DRPM launch (alone and batched).
template <int H, int N>
__device__ __forceinline__ void halve_n(double (&a)[N], int lane) {
    const bool up = (lane & (2 * H)) != 0;
#pragma unroll
    for (int i = 0; i < H; ++i) {
        const double send = up ? a[i] : a[H + i];
        const double keep = up ? a[H + i] : a[i];
        a[i] = keep + xor_f64(send, 2 * H);
    }
    if constexpr (H > 1) halve_n<H / 2, N>(a, lane);
}
__device__ __forceinline__ void wave_sum42(const double (&v)[kDrpmSlab], double& r0, double& r1) {
    const int lane = threadIdx.x & 63;
    double a[32];
#pragma unroll
    for (int k = 0; k < 32; ++k) a[k] = v[k];
    halve_n<16, 32>(a, lane);
    r0 = a[0] + xor_f64(a[0], 1);
    double b[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) b[k] = k < kDrpmSlab - 32 ? v[32 + k] : 0.0;
    halve_n<8, 16>(b, lane);
    r1 = b[0] + xor_f64(b[0], 1);
    r1 = r1 + xor_f64(r1, 32);
}
// lane 2k of wave wv writes its totals to red[wv][·] (the block's per-wave rows)
__device__ __forceinline__ void wave_sum42_store(const double (&v)[kDrpmSlab], double* __restrict__ row) {
    double r0, r1;
    wave_sum42(v, r0, r1);
    const int lane = threadIdx.x & 63;
    if (!(lane & 1)) {
        row[lane >> 1] = r0;
        if ((lane >> 1) < kDrpmSlab - 32) row[32 + (lane >> 1)] = r1;
    }
}

// reduce the weighted normal equations (pass-1 slabs), eigendecompose H
__device__ __forceinline__ void drpm_eig_body(const double* __restrict__ partial, int blocks, const SolveState& st,
                                              const DrpmDev& Dv) {
    if (*st.done) return;
    __shared__ double red[(256 / 64) * kNormEq];
    __shared__ double acc[kNormEq];
    double loc[kNormEq];
#pragma unroll
    for (int k = 0; k < kNormEq; ++k) loc[k] = 0.0;
    for (int b = threadIdx.x; b < blocks; b += 256)
#pragma unroll
        for (int k = 0; k < kNormEq; ++k) loc[k] += partial[(size_t)b * kNormEq + k];
    block_sum28<256>(loc, red, acc);
    if (threadIdx.x >= 64) return;
    // H (row-major, from the upper-triangle terms) and g; the eigendecomposition by wave 0, lane k
    // holding row k (sym_eig6_wave: the oracle's Jacobi, operation for operation)
    const int lane = threadIdx.x, k = lane < 6 ? lane : 0;
    double row[6];
#pragma unroll
    for (int c = 0; c < 6; ++c) {
        const int r0 = k < c ? k : c, c0 = k < c ? c : k;
        row[c] = acc[6 * r0 - r0 * (r0 - 1) / 2 + (c0 - r0)];
    }
    if (lane < 6) {
#pragma unroll
        for (int c = 0; c < 6; ++c) Dv.H[lane * 6 + c] = row[c];
        Dv.g[lane] = acc[21 + lane];
    }
    sym_eig6_wave(row, Dv.ev, Dv.U);
}

// the 42 noise terms of row i (zero when i ≥ N or the row is absent), degeneracy.h:14-72
__device__ __forceinline__ void drpm_noise_terms(const Rows& rows, int i, int N, const DrpmDev& Dv, double sp, double sn,
                                                 double (&acc)[kDrpmSlab]) {
#pragma unroll
    for (int k = 0; k < kDrpmSlab; ++k) acc[k] = 0.0;
    double a[6], b, wt;
    if (i < N && rows.get(i, a, b, wt)) {
        const size_t i3 = 3 * (size_t)i;
        const double s[3] = {rows.ds[i3], rows.ds[i3 + 1], rows.ds[i3 + 2]};
        const double n[3] = {rows.dn[i3], rows.dn[i3 + 1], rows.dn[i3 + 2]};
        // skew(v) = [0 −z y; z 0 −x; −y x 0] (degeneracy.h:7-12)
        const double nx[9] = {0, -n[2], n[1], n[2], 0, -n[0], -n[1], n[0], 0};
        const double px[9] = {0, -s[2], s[1], s[2], 0, -s[0], -s[1], s[0], 0};
        double B[36];
#pragma unroll
        for (int q = 0; q < 36; ++q) B[q] = 0.0;
#pragma unroll
        for (int r = 0; r < 3; ++r)
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                B[r * 6 + c] = -nx[r * 3 + c];
                double pn = 0;
#pragma unroll
                for (int k = 0; k < 3; ++k) pn += px[r * 3 + k] * nx[k * 3 + c];
                B[r * 6 + 3 + c] = pn;
                B[(3 + r) * 6 + 3 + c] = nx[r * 3 + c];
            }
        const double sp2 = sp * sp, sn2 = sn * sn;
        const double Nd[6] = {sp2, sp2, sp2, sn2, sn2, sn2};
        double C[36];
#pragma unroll
        for (int r = 0; r < 6; ++r)
#pragma unroll
            for (int c = 0; c < 6; ++c) {
                double v = 0;
#pragma unroll
                for (int k = 0; k < 6; ++k) v += B[r * 6 + k] * Nd[k] * B[c * 6 + k];
                C[r * 6 + c] = v * wt;
            }
#pragma unroll
        for (int q = 0; q < 36; ++q) acc[q] = C[q];
        const double sw = sqrt(wt);
        double v6[6];
#pragma unroll
        for (int r = 0; r < 3; ++r) {
            double pn = 0;
#pragma unroll
            for (int k = 0; k < 3; ++k) pn += px[r * 3 + k] * n[k];
            v6[r] = sw * pn;
            v6[3 + r] = sw * n[r];
        }
#pragma unroll
        for (int k = 0; k < 6; ++k) {
            double aa = 0, bb = 0;
#pragma unroll
            for (int r = 0; r < 6; ++r) {
                double cu = 0;
#pragma unroll
                for (int c = 0; c < 6; ++c) cu += C[r * 6 + c] * Dv.U[k * 6 + c];
                aa += Dv.U[k * 6 + r] * cu;
                bb += Dv.U[k * 6 + r] * v6[r];
            }
            acc[36 + k] = 2 * aa * aa + 4 * aa * bb * bb;
        }
    }
}

// per-point noise mean (36) and variance along the eigenvectors (6), degeneracy.h:14-72
__device__ __forceinline__ void drpm_noise_body(const Rows& rows, int N, const SolveState& st, const DrpmDev& Dv, double sp,
                                                double sn) {
    if (*st.done) return;
    __shared__ double red[(kBlock / 64) * kDrpmSlab];
    const int i = blockIdx.x * kBlock + threadIdx.x;
    double acc[kDrpmSlab];
    drpm_noise_terms(rows, i, N, Dv, sp, sn, acc);
    const int wv = threadIdx.x >> 6;
    wave_sum42_store(acc, red + wv * kDrpmSlab);
    __syncthreads();
    if (threadIdx.x < kDrpmSlab) {
        double s = 0.0;
        for (int w = 0; w < kBlock / 64; ++w) s += red[w * kDrpmSlab + threadIdx.x];
        Dv.slabs[(size_t)blockIdx.x * kDrpmSlab + threadIdx.x] = s;
    }
}

__device__ __forceinline__ double normal_cdf(double mean, double sd, double x) {
    return 0.5 * erfc(-(x - mean) / (sd * sqrt(2.0)));   // Boost.Math cdf(normal(mean, sd), x)
}

// The DRPM decision and solve from the reduced noise terms tot[42] (solver.cpp:540-603), by wave 0
// (every other thread returns): lane k < 6 evaluates prob[k] — the thread-0 loop's expressions for
// that k, so the same bits — the minimum over k in order, then either the SNR-weighted
// eigen-solution (thread 0) or the plain normal-equation solve by the whole wave (solve6_u: solve6's
// operations with a wave-uniform pivot, bit for bit), Δ and the pose update by thread 0.  Round 6:
// one thread ran all six probabilities and solve6's predicated pivot swaps (k_drpm_final 27 µs per
// call on a lone 1600-row frame, profiles/r06_calib).
__device__ __forceinline__ void drpm_solve_wave0(const SolveState& st, const DrpmDev& Dv, imls_iter_trace* tr,
                                                 const KParams& kp, double threshold, const int* __restrict__ count_all,
                                                 const int* __restrict__ count_in, int update_pose, const double* tot) {
    if (threadIdx.x >= 64) return;
    const int lane = threadIdx.x;
    const double snr = 10.0;   // solver.cpp:547
    double pk = 0.0;
    if (lane < 6) {
        const int k = lane;
        double meas = 0, exp_noise = 0;
        for (int r = 0; r < 6; ++r) {
            double hu = 0, mu = 0;
            for (int c = 0; c < 6; ++c) { hu += Dv.H[r * 6 + c] * Dv.U[k * 6 + c]; mu += tot[r * 6 + c] * Dv.U[k * 6 + c]; }
            meas += Dv.U[k * 6 + r] * hu;
            exp_noise += Dv.U[k * 6 + r] * mu;
        }
        const double sd = sqrt(tot[36 + k]);
        const double tp = meas / (1.0 + snr);
        const bool bad = isnan(exp_noise) || isnan(sd) || isnan(tp);
        pk = bad ? 0.0 : normal_cdf(exp_noise, sd, tp);
    }
    double prob[6], pmin = INFINITY;
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        prob[k] = readlane_f64(pk, k);
        pmin = fmin(pmin, prob[k]);
    }
    double x[6];
    if (pmin < threshold) {
        if (lane) return;
        double ut[6];
        for (int k = 0; k < 6; ++k) {
            const double dps = fabs(Dv.ev[k]) > 1e-10 ? prob[k] / Dv.ev[k] : 0.0;
            double acc = 0;
            for (int r = 0; r < 6; ++r) acc += Dv.U[k * 6 + r] * Dv.g[r];
            ut[k] = dps * acc;
        }
        for (int r = 0; r < 6; ++r) {
            double acc = 0;
            for (int k = 0; k < 6; ++k) acc += Dv.U[k * 6 + r] * ut[k];
            x[r] = acc;
        }
    } else {
        double ne[kNormEq];
        int k = 0;
        for (int r = 0; r < 6; ++r)
            for (int c = r; c < 6; ++c) ne[k++] = Dv.H[r * 6 + c];
        for (int r = 0; r < 6; ++r) ne[21 + r] = Dv.g[r];
        ne[27] = 0;
        solve6_u(ne, x);
        if (lane) return;
    }
    double D[16];
    delta_from_x(x, D);
    finish_iteration(st, tr, D, (double)*count_all, (double)*count_in, update_pose, kp);
}

__device__ __forceinline__ void drpm_final_body(int blocks, const SolveState& st, const DrpmDev& Dv, imls_iter_trace* tr,
                                                const KParams& kp, double threshold, const int* __restrict__ count_all,
                                                const int* __restrict__ count_in, int update_pose) {
    if (*st.done) return;
    __shared__ double red[(256 / 64) * kDrpmSlab];
    __shared__ double tot[kDrpmSlab];
    double loc[kDrpmSlab];
#pragma unroll
    for (int k = 0; k < kDrpmSlab; ++k) loc[k] = 0.0;
    for (int b = threadIdx.x; b < blocks; b += 256)
#pragma unroll
        for (int k = 0; k < kDrpmSlab; ++k) loc[k] += Dv.slabs[(size_t)b * kDrpmSlab + k];
    const int wv = threadIdx.x >> 6;
    wave_sum42_store(loc, red + wv * kDrpmSlab);
    __syncthreads();
    if (threadIdx.x < kDrpmSlab) {
        double s = 0.0;
        for (int w = 0; w < 256 / 64; ++w) s += red[w * kDrpmSlab + threadIdx.x];
        tot[threadIdx.x] = s;
    }
    __syncthreads();
    drpm_solve_wave0(st, Dv, tr, kp, threshold, count_all, count_in, update_pose, tot);
}

__global__ __launch_bounds__(256) void k_drpm_eig(const double* __restrict__ partial, int blocks, SolveState st, DrpmDev Dv) {
    drpm_eig_body(partial, blocks, st, Dv);
}
__global__ __launch_bounds__(kBlock) void k_drpm_noise(Rows rows, int N, SolveState st, DrpmDev Dv, double sp, double sn) {
    drpm_noise_body(rows, N, st, Dv, sp, sn);
}
// rtr: RANSAC's own trace record (n_valid = correspondences, n_kept = 0) when the solve was active,
// written after the final solve's; null for the stand-alone DRPM
__device__ __forceinline__ void ransac_trace_t0(const RansacDev& R, const int* __restrict__ count_all, imls_iter_trace* rtr) {
    if (threadIdx.x == 0 && rtr && *R.active) {
        rtr->n_valid = (unsigned long long)*count_all;
        rtr->n_kept = 0;
    }
}
__global__ __launch_bounds__(256) void k_drpm_final(int blocks, SolveState st, DrpmDev Dv, imls_iter_trace* tr, KParams kp,
                                                    double threshold, const int* __restrict__ count_all,
                                                    const int* __restrict__ count_in, int update_pose, RansacDev R,
                                                    imls_iter_trace* rtr) {
    drpm_final_body(blocks, st, Dv, tr, kp, threshold, count_all, count_in, update_pose);
    ransac_trace_t0(R, count_all, rtr);
}

// ---------------------------------------------------------------------------------------------
// The lone frame's DRPM head in ONE launch (round 6; frames of ≤ kSmallRows rows registered alone,
// the config C/D deployment shape): the inlier compaction, pass 1 of the weighted normal equations
// over the inliers and the eigendecomposition — three launches before (k_compact_one, k_rows_pass1,
// k_drpm_eig) — preceded by the last hypothesis chunk's selection (k_ransac_select, round 6).  One 1024-thread block runs them between block barriers; pass 1 runs as "virtual
// blocks" — block b of k_rows_pass1's grid is done by the 256-thread group (b mod 4) in round b / 4,
// with the same thread ↔ row mapping, the same per-wave reductions and the same slab order, and the
// slab sum by the first 256 threads as k_drpm_eig does it — so every value is the chain's bit for bit
// (the batched frames keep the chain: alone and batched agree).  The noise terms and the solve stay
// grid / one-block launches: fused into this block as well (virtual noise blocks, measured) the
// frame's DRPM took 102.7 µs per ICP iteration against the chain's 70 (one CU for the noise phase,
// its registers at 2 waves per SIMD; profiles/r06_ransac/).
// ---------------------------------------------------------------------------------------------
constexpr int kHeadThreads = 1024;
struct SelectArgs {                   // the last hypothesis chunk's selection (k_ransac_select's arguments)
    const int* count;
    int chunk, max_iterations;
    double min_pct;
};
__global__ __launch_bounds__(kHeadThreads) void k_drpm_head_small(SelectArgs sel, Source isrc, int cap, CompactOut out,
                                                                  CompactPost P, Rows rows, int b1, SolveState st,
                                                                  DrpmDev Dv) {
    __shared__ double red_ne[kHeadThreads / 64][kNormEq];
    __shared__ double acc[kNormEq];
    // pass 1's slabs stay in LDS (round 6: through st.partial1 the slab sum waited on a global round trip)
    __shared__ double slab[kSmallRows / kBlock][kNormEq];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, grp = tid >> 8, t = tid & 255;
    if (compact_skip(P)) return;
#ifdef IMLS_DEBUG_WAVE_TRACE
    const bool dbg_on = tid == 0;
    long long dbg_t = wall_clock64();
    if (dbg_on) g_dbg_ransac[14] += 1;
#endif
    // 0. the last chunk's selection (k_ransac_select: skipped once RANSAC finished in an earlier chunk),
    // by wave 0; its bestT feeds the compaction below
    if (!*P.R.rdone) {
        if (tid < 64) ransac_select_body(sel.count, P.R, sel.chunk, sel.max_iterations, sel.min_pct);
        __threadfence_block();
        __syncthreads();
    }
    RSTAMP(8);
    // 1. the inliers of the best Δ with their weights (k_compact_one, kind 2: an empty set fails the solve)
    compact_one_body(isrc, cap, out, P);
    __threadfence_block();
    __syncthreads();
    RSTAMP(9);
    // 2. pass 1 over the inlier rows (k_rows_pass1<kBlock>, which runs whether or not the frame is done:
    // slab b = rows [256b, 256b + 256))
    for (int base = 0; base < b1; base += kHeadThreads / kBlock) {
        const int b = base + grp, i = b * kBlock + t;
        double a[6] = {0, 0, 0, 0, 0, 0}, bb = 0, wt = 1, cnt = 0;
        if (b < b1 && i < cap && rows.get(i, a, bb, wt)) {
            const double sw = sqrt(wt);
            for (int k = 0; k < 6; ++k) a[k] = sw * a[k];
            bb = sw * bb;
            cnt = 1;
        }
        double v[32];
        int k = 0;
#pragma unroll
        for (int r = 0; r < 6; ++r)
#pragma unroll
            for (int c = r; c < 6; ++c) v[k++] = a[r] * a[c];
#pragma unroll
        for (int r = 0; r < 6; ++r) v[21 + r] = a[r] * bb;
        v[27] = cnt;
#pragma unroll
        for (int q = kNormEq; q < 32; ++q) v[q] = 0.0;
        const double sum = wave_sum28(v);
        if (!(lane & 1) && (lane >> 1) < kNormEq) red_ne[wv][lane >> 1] = sum;
        __syncthreads();
        if (t < kNormEq && b < b1) {
            double sacc = 0.0;
            for (int w = 0; w < kBlock / 64; ++w) sacc += red_ne[grp * (kBlock / 64) + w][t];
            slab[b][t] = sacc;
        }
        __syncthreads();
    }
    RSTAMP(10);
    // 3. H, g and the eigendecomposition (k_drpm_eig: a finished frame stops here; 256 threads reduce
    // the slabs, wave 0 solves)
    if (*st.done) return;
    double loc[kNormEq];
#pragma unroll
    for (int k = 0; k < kNormEq; ++k) loc[k] = 0.0;
    if (tid < 256)
        for (int b = tid; b < b1; b += 256)
#pragma unroll
            for (int k = 0; k < kNormEq; ++k) loc[k] += slab[b][k];
    double a32[32];
#pragma unroll
    for (int k = 0; k < 32; ++k) a32[k] = k < kNormEq ? loc[k] : 0.0;
    const double sum = wave_sum28(a32);
    if (wv < 4 && !(lane & 1) && (lane >> 1) < kNormEq) red_ne[wv][lane >> 1] = sum;
    __syncthreads();
    if (tid < kNormEq) {
        double sacc = 0.0;
#pragma unroll
        for (int w = 0; w < 4; ++w) sacc += red_ne[w][tid];
        acc[tid] = sacc;
    }
    __syncthreads();
    if (tid >= 64) return;
    const int k = lane < 6 ? lane : 0;
    double row[6];
#pragma unroll
    for (int c = 0; c < 6; ++c) {
        const int r0 = k < c ? k : c, c0 = k < c ? c : k;
        row[c] = acc[6 * r0 - r0 * (r0 - 1) / 2 + (c0 - r0)];
    }
    if (lane < 6) {
#pragma unroll
        for (int c = 0; c < 6; ++c) Dv.H[lane * 6 + c] = row[c];
        Dv.g[lane] = acc[21 + lane];
    }
    RSTAMP(11);
    const int sweeps = sym_eig6_wave(row, Dv.ev, Dv.U);
    RSTAMP(12);
#ifdef IMLS_DEBUG_WAVE_TRACE
    if (dbg_on) g_dbg_ransac[13] += (unsigned long long)sweeps;
#else
    (void)sweeps;
#endif
}
#ifdef IMLS_DEBUG_WAVE_TRACE
}  // namespace
}  // namespace imlsgpu
extern "C" int imls_debug_ransac(unsigned long long* out) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(imlsgpu::g_dbg_ransac), 128) == hipSuccess ? 0 : -1;
}
namespace imlsgpu {
namespace {
#endif

// ---------------------------------------------------------------------------------------------
// Batched RANSAC / DRPM kernels (launch_ransac_batch): frame = tab[blockIdx.y], the same bodies as
// the one-frame kernels above; the frame's RANSAC scratch is A.rf, its pose update always on.
// ---------------------------------------------------------------------------------------------
// The chunk's hypotheses of the frames still running, spread evenly over the grid: each block first
// lists the running frames (done / RANSAC-finished ones drop out), then strides over
// (frame, hypothesis) items — one frame without an early exit gets the whole grid, not a slice.
template <int NT>
__global__ __launch_bounds__(NT) void k_ransac_hyp_b(const PairDev* __restrict__ tab, int npairs, int chunk,
                                                            double dist_thr) {
    __shared__ int sact[kMaxRansacBatch];
    __shared__ int swc[NT / 64];
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    int na = 0;
    for (int base = 0; base < npairs; base += NT) {
        bool act = false;
        if (base + t < npairs) act = !*tab[base + t].st.done && !*tab[base + t].rf.R.rdone;
        const unsigned long long m = __ballot(act);
        if (lane == 0) swc[wv] = __popcll(m);
        __syncthreads();
        int off = na, tot = na;
        for (int k = 0; k < NT / 64; ++k) {
            off += k < wv ? swc[k] : 0;
            tot += swc[k];
        }
        if (act) sact[off + __popcll(m & ((1ull << lane) - 1ull))] = base + t;
        na = tot;
        __syncthreads();
    }
    const long long items = (long long)na * chunk;
    for (long long q = blockIdx.x; q < items; q += gridDim.x) {
        const int fr = __builtin_amdgcn_readfirstlane(sact[q % na]);
        const int h = (int)(q / na);
        const PairDev A = device_view(tab + fr);
        const size_t c3 = 3 * (size_t)A.rf.cap;
        ransac_hyp_one<NT>(A.rf.all, A.rf.all + c3, A.rf.all + 2 * c3, *A.rf.cnt_all, A.rf.R, dist_thr, h);
    }
}
__global__ __launch_bounds__(64) void k_ransac_select_b(const PairDev* __restrict__ tab, int chunk, int max_iterations,
                                                        double min_pct) {
    const PairDev A = device_view(tab + blockIdx.y);
    if (*A.st.done || *A.rf.R.rdone) return;
    ransac_select_body(A.rf.cnt_all, A.rf.R, chunk, max_iterations, min_pct);
}
// trace of a RANSAC iteration as the oracle records it (n_valid = correspondences, n_kept = 0) —
// LS / weighted-LS finals; the DRPM final writes it itself
__global__ void k_ransac_trace_b(const PairDev* __restrict__ tab, int it) {
    const PairDev A = device_view(tab + blockIdx.y);
    if (threadIdx.x || !*A.rf.R.active) return;
    A.trace[it].n_valid = (unsigned long long)*A.rf.cnt_all;
    A.trace[it].n_kept = 0;
}
__global__ __launch_bounds__(256) void k_drpm_eig_b(const PairDev* __restrict__ tab) {
    const PairDev A = device_view(tab + blockIdx.y);
    drpm_eig_body(A.st.partial1, solve_blocks_of(A.rf.cap), A.st, A.rf.Dv);
}
__global__ __launch_bounds__(kBlock) void k_drpm_noise_b(const PairDev* __restrict__ tab, double sp, double sn) {
    const PairDev A = device_view(tab + blockIdx.y);
    if ((int)blockIdx.x >= solve_blocks_of(A.rf.cap)) return;
    drpm_noise_body(frame_rows(A, 1, 1), A.rf.cap, A.st, A.rf.Dv, sp, sn);
}
__global__ __launch_bounds__(256) void k_drpm_final_b(const PairDev* __restrict__ tab, KParams kp, double threshold, int it) {
    const PairDev A = device_view(tab + blockIdx.y);
    drpm_final_body(solve_blocks_of(A.rf.cap), A.st, A.rf.Dv, A.trace + it, kp, threshold, A.rf.cnt_all, A.rf.cnt_in, 1);
    ransac_trace_t0(A.rf.R, A.rf.cnt_all, A.trace + it);
}

// chunk sizes of the hypothesis loop: 16 (the usual early exit: the shipped 95 % inlier bar is mostly
// met by the first hypotheses), 256, then the rest in chunks of kHypMax — three chunks for
// max_iterations ≤ kHypMax + 272.  (Results do not depend on the chunking: exactly the draws
// consumed are committed.)
// Hypothesis chunks.  Each hypothesis takes its own rand() word (the h-th ahead of the chunk's state)
// and the select commits exactly the words used, so any chunking gives the same result; chunks only
// trade wasted work after an early exit against launches.  Batched frames: 16, 256, then up to
// kHypMax (throughput: a frame that exits early wastes little of the shared grid).  A frame alone
// (lone = true, the deployment shape): 272, then up to kHypMax — the first two batched chunks in one
// launch (both fit one wave of blocks, so the merged launch takes about as long as the 16; round 6:
// a lone 1600-row frame without an early exit ran 3 hypothesis + 3 select launches per ICP iteration).
std::vector<int> ransac_chunks(int max_iterations, bool lone = false) {
    std::vector<int> v;
    for (int started = 0; started < max_iterations;) {
        const int want = lone ? (started == 0 ? 272 : kHypMax) : (started == 0 ? 16 : started == 16 ? 256 : kHypMax);
        const int cn = std::min(want, max_iterations - started);
        v.push_back(cn);
        started += cn;
    }
    return v;
}

}  // namespace

size_t ransac_bytes(int cap) {
    // the carve sequence of launch_solve, each piece rounded up to 256 B (+ slack per piece)
    const size_t c = (size_t)std::max(cap, 1);
    const size_t nb = (c + kBlock - 1) / kBlock + 1;
    return 2 * (10 * c + 8) * 8 + nb * (4 + 8) + (size_t)kHypMax * (4 + 16 * 8) + nb * kDrpmSlab * 8 +
           (36 + 6 + 36 + 6 + 16) * 8 + 32 * 256;
}

void launch_solve(hipStream_t s, const SolveLaunch& L) {
    const KParams& kp = L.kp;
    SolveState st = L.st;
    if (kp.solve_method == IMLS_SOLVE_DRPM) {
        // stand-alone SolveMotionEstimationProblemDRPM (solver.cpp:499-603) on host fp64 rows + weights
        const int cap = std::max(L.N, 1);
        const int b1 = solve_blocks(cap);
        char* p = (char*)L.scratch;
        auto carve = [&](size_t bytes) { char* r = p; p += (bytes + 255) / 256 * 256; return r; };
        int* cnt = (int*)carve(64);
        DrpmDev Dv;
        Dv.H = (double*)carve(36 * 8);
        Dv.g = (double*)carve(6 * 8);
        Dv.U = (double*)carve(36 * 8);
        Dv.ev = (double*)carve(6 * 8);
        Dv.slabs = (double*)carve((size_t)(b1 + 1) * kDrpmSlab * 8);
        const size_t c = (size_t)L.N;
        k_set_count<<<1, 64, 0, s>>>(cnt, L.N);
        k_drpm_guard<<<1, 64, 0, s>>>(cnt, L.st);
        Rows rows{nullptr, nullptr, nullptr, L.rows_d, L.rows_d + 3 * c, L.rows_d + 6 * c, L.weights, 1, cnt, nullptr};
        launch_rows_pass1(s, rows, cap, L.st.partial1, b1);
        k_drpm_eig<<<1, 256, 0, s>>>(L.st.partial1, b1, L.st, Dv);
        k_drpm_noise<<<b1, kBlock, 0, s>>>(rows, cap, L.st, Dv, L.ransac.drpm_stdev_points, L.ransac.drpm_stdev_normals);
        k_drpm_final<<<1, 256, 0, s>>>(b1, L.st, Dv, L.tr, kp, L.ransac.drpm_threshold, cnt, cnt, L.update_pose,
                                       RansacDev{}, nullptr);
        return;
    }
    if (kp.solve_method != IMLS_SOLVE_RANSAC) {
        launch_solve_chain(s, L.N, L.blocks1, kp, L.cs, L.cd, L.cn, L.rows_d, L.weights, st, L.tr, L.update_pose,
                           L.rows_are_double, L.count);
        return;
    }
    const int cap = std::max(L.N, 1);
    const size_t c = (size_t)cap;
    const int nb = (cap + kBlock - 1) / kBlock;
    const RansacFrame F = ransac_frame(L.scratch, cap, L.rng);
    const RansacDev& R = F.R;
    const int* done = L.st.done;

    // one compaction (valid rows → all, or inliers → inl) with its post step folded in
    auto compact = [&](const Source& src, int n, const CompactOut& out, int kind) {
        const CompactPost P{kind, kp.correspond_number, L.update_pose, L.st, L.tr, R};
        if (cap <= kCompactOne) {
            k_compact_one<<<1, 1024, 0, s>>>(src, n, out, P);
        } else {
            k_compact_count<<<nb, kBlock, 0, s>>>(src, n, F.blkcnt, F.blkw, done);
            k_compact_scan<<<1, 1024, 0, s>>>(F.blkcnt, F.blkw, nb, out, P);
            k_compact_scatter<<<nb, kBlock, 0, s>>>(src, n, F.blkcnt, out, done);
        }
    };

    // 1. compact the valid correspondences (fp64 rows from the host API are already compact), then
    //    the count gate and the selection reset
    if (!L.rows_are_double) {
        Source src{};
        src.cs = L.cs; src.cd = L.cd; src.cn = L.cn;
        compact(src, L.N, CompactOut{F.all, F.cnt_all, nullptr, cap}, 1);
    } else {
        (void)hipMemcpyAsync(F.all, L.rows_d, 9 * c * 8, hipMemcpyDeviceToDevice, s);
        k_set_count<<<1, 64, 0, s>>>(F.cnt_all, L.N);
        k_ransac_begin<<<1, 64, 0, s>>>(F.cnt_all, kp.correspond_number, L.update_pose, L.st, L.tr, R);
    }
    // 2. hypotheses in chunks, 256 threads per hypothesis (a lone frame's chunk has ~1 block per CU, so
    // the per-thread row chains, not the CU's occupancy, set the time: 64-thread blocks took 26.8 µs
    // per 272-hypothesis chunk on a 1600-row frame).  A small DRPM frame's last selection runs at the
    // head of k_drpm_head_small (one launch fewer per ICP iteration).
    // Two chunks whose draws fit the jump table (the shipped 5000 hypotheses: 272 + 4728) run without a
    // selection between them (k_ransac_hyp, base > 0): one selection over both, at the head.
    const std::vector<int> chunks = ransac_chunks(L.ransac.max_iterations, true);
    const bool fold_select = L.ransac.final_method == IMLS_FINAL_DRPM && cap <= kSmallRows;
    const bool one_select = fold_select && chunks.size() == 2 && chunks[0] + chunks[1] <= kHypMax;
    int sel_chunk = chunks.back();
    if (one_select) {
        k_ransac_hyp<256><<<chunks[0], 256, 0, s>>>(F.all, F.cnt_all, cap, R, L.ransac.distance_threshold, chunks[0],
                                                    done, 0, 0.0);
        k_ransac_hyp<256><<<chunks[1], 256, 0, s>>>(F.all, F.cnt_all, cap, R, L.ransac.distance_threshold, chunks[1],
                                                    done, chunks[0], L.ransac.min_inliers_percentage);
        sel_chunk = chunks[0] + chunks[1];
    } else {
        for (size_t ci = 0; ci < chunks.size(); ++ci) {
            const int cn = chunks[ci];
            k_ransac_hyp<256><<<cn, 256, 0, s>>>(F.all, F.cnt_all, cap, R, L.ransac.distance_threshold, cn, done, 0, 0.0);
            if (!(fold_select && ci + 1 == chunks.size()))
                k_ransac_select<<<1, 64, 0, s>>>(F.cnt_all, R, cn, L.ransac.max_iterations, L.ransac.min_inliers_percentage,
                                                 done);
        }
    }

    // 3. inliers of the best Δ with their Huber-like weights (order kept), Σw; an empty set stops
    Source isrc{};
    isrc.rows = F.all;
    isrc.count = F.cnt_all;
    isrc.cap = cap;
    isrc.T = R.bestT;
    isrc.dist_thr = L.ransac.distance_threshold;
    isrc.h2 = L.ransac.huber_threshold * L.ransac.distance_threshold;
    KParams fk = kp;
    fk.correspond_number = 0;                       // the count gate ran before RANSAC
    double* inl = F.inl;
    Rows rows{nullptr, nullptr, nullptr, inl, inl + 3 * c, inl + 6 * c, inl + 9 * c, 1, F.cnt_in, F.wsum};
    if (L.ransac.final_method == IMLS_FINAL_DRPM && cap <= kSmallRows) {
        // a small frame: compaction + pass 1 + eigendecomposition in one launch (the chain's values),
        // then the noise terms and the solve
        const int b1 = solve_blocks(cap);
        const CompactPost P{2, kp.correspond_number, L.update_pose, L.st, L.tr, R};
        const SelectArgs sel{F.cnt_all, sel_chunk, L.ransac.max_iterations, L.ransac.min_inliers_percentage};
        k_drpm_head_small<<<1, kHeadThreads, 0, s>>>(sel, isrc, cap, CompactOut{F.inl, F.cnt_in, F.wsum, cap}, P, rows, b1,
                                                     L.st, F.Dv);
        k_drpm_noise<<<b1, kBlock, 0, s>>>(rows, cap, L.st, F.Dv, L.ransac.drpm_stdev_points, L.ransac.drpm_stdev_normals);
        k_drpm_final<<<1, 256, 0, s>>>(b1, L.st, F.Dv, L.tr, fk, L.ransac.drpm_threshold, F.cnt_all, F.cnt_in, L.update_pose,
                                       R, L.tr);
        return;
    }
    compact(isrc, cap, CompactOut{F.inl, F.cnt_in, F.wsum, cap}, 2);

    // 4. final solve on the inliers (+ RANSAC's own trace record)
    switch (L.ransac.final_method) {
        case IMLS_FINAL_LS:
            fk.solve_method = IMLS_SOLVE_LS;
            fk.ls_threshold = L.ransac.ls_threshold;
            launch_solve_chain(s, cap, 0, fk, nullptr, nullptr, nullptr, inl, nullptr, st, L.tr, L.update_pose, 1, F.cnt_in, nullptr);
            if (L.tr) k_ransac_trace<<<1, 64, 0, s>>>(F.cnt_all, R, L.tr);
            break;
        case IMLS_FINAL_WEIGHTED_LS:
            fk.solve_method = IMLS_SOLVE_WEIGHTED_LS;
            launch_solve_chain(s, cap, 0, fk, nullptr, nullptr, nullptr, inl, inl + 9 * c, st, L.tr, L.update_pose, 1, F.cnt_in, F.wsum);
            if (L.tr) k_ransac_trace<<<1, 64, 0, s>>>(F.cnt_all, R, L.tr);
            break;
        default: {   // DRPM
            const int b1 = solve_blocks(cap);
            launch_rows_pass1(s, rows, cap, L.st.partial1, b1);
            k_drpm_eig<<<1, 256, 0, s>>>(L.st.partial1, b1, L.st, F.Dv);
            k_drpm_noise<<<b1, kBlock, 0, s>>>(rows, cap, L.st, F.Dv, L.ransac.drpm_stdev_points, L.ransac.drpm_stdev_normals);
            k_drpm_final<<<1, 256, 0, s>>>(b1, L.st, F.Dv, L.tr, fk, L.ransac.drpm_threshold, F.cnt_all, F.cnt_in, L.update_pose,
                                           R, L.tr);
        }
    }
}

RansacFrame ransac_frame(void* scratch, int cap, int* rng) {
    // the carve sequence sized by ransac_bytes, each piece rounded up to 256 B
    const size_t c = (size_t)std::max(cap, 1);
    const int nb = (int)((c + kBlock - 1) / kBlock);
    char* p = (char*)scratch;
    auto carve = [&](size_t bytes) { char* r = p; p += (bytes + 255) / 256 * 256; return r; };
    RansacFrame F{};
    F.cap = (int)c;
    F.all = (double*)carve((10 * c + 8) * 8);
    F.inl = (double*)carve((10 * c + 8) * 8);
    F.blkcnt = (int*)carve((size_t)(nb + 1) * 4);
    F.blkw = (double*)carve((size_t)(nb + 1) * 8);
    F.cnt_all = (int*)carve(64);
    F.cnt_in = (int*)carve(64);
    F.wsum = (double*)carve(64);
    F.R.rng = rng;
    F.R.counts = (int*)carve((size_t)kHypMax * 4);
    F.R.T = (double*)carve((size_t)kHypMax * 16 * 8);
    F.R.best = (int*)carve(64);
    F.R.evaluated = (int*)carve(64);
    F.R.rdone = (int*)carve(64);
    F.R.bestT = (double*)carve(16 * 8);
    F.R.active = (int*)carve(64);
    F.Dv.H = (double*)carve(36 * 8);
    F.Dv.g = (double*)carve(6 * 8);
    F.Dv.U = (double*)carve(36 * 8);
    F.Dv.ev = (double*)carve(6 * 8);
    F.Dv.slabs = (double*)carve((size_t)(nb + 1) * kDrpmSlab * 8);
    return F;
}

int launch_ransac_batch(hipStream_t s, const PairDev* tab, const int* n_host, int npairs, const KParams& kp,
                        const RansacParams& rp, int it) {
    if (npairs <= 0) return 0;
    if (npairs > kMaxRansacBatch) return -1;   // the select kernels keep one slot per frame in LDS
    std::vector<int> caps((size_t)npairs);
    int maxc = 1;
    for (int k = 0; k < npairs; ++k) {
        caps[k] = std::max(n_host[k], 1);
        maxc = std::max(maxc, caps[k]);
    }
    const dim3 gc((maxc + kBlock - 1) / kBlock, npairs), g1(1, npairs);
    const double h2 = rp.huber_threshold * rp.distance_threshold;
    // one compaction per frame (mode 0: valid rows → all, then the count gate and selection reset;
    // mode 1: the inliers of the best Δ, then the empty-set check)
    auto compact = [&](int mode, double dt, double hh) {
        if (maxc <= kCompactOne) {
            k_compact_one_b<<<g1, 1024, 0, s>>>(tab, mode, dt, hh, kp.correspond_number, it);
        } else {
            k_compact_count_b<<<gc, kBlock, 0, s>>>(tab, mode, dt, hh);
            k_compact_scan_b<<<g1, 1024, 0, s>>>(tab, mode, kp.correspond_number, it);
            k_compact_scatter_b<<<gc, kBlock, 0, s>>>(tab, mode, dt, hh);
        }
    };
    // 1. every frame's valid correspondences, compacted (order kept) to fp64
    compact(0, 0.0, 0.0);
    // 2. hypotheses: each chunk's items of the still-running frames spread over one grid
    for (const int cn : ransac_chunks(rp.max_iterations)) {
        const int grid = std::min(cn * npairs, kHypGrid);
        if (hyp_block_of(maxc) == 64)
            k_ransac_hyp_b<64><<<grid, 64, 0, s>>>(tab, npairs, cn, rp.distance_threshold);
        else
            k_ransac_hyp_b<256><<<grid, 256, 0, s>>>(tab, npairs, cn, rp.distance_threshold);
        k_ransac_select_b<<<g1, 64, 0, s>>>(tab, cn, rp.max_iterations, rp.min_inliers_percentage);
    }
    // 3. inliers of each frame's best Δ with their weights
    compact(1, rp.distance_threshold, h2);
    // 4. final solve
    KParams fk = kp;
    fk.correspond_number = 0;
    switch (rp.final_method) {
        case IMLS_FINAL_LS:
            fk.solve_method = IMLS_SOLVE_LS;
            fk.ls_threshold = rp.ls_threshold;
            launch_solve_batch(s, tab, caps.data(), npairs, fk, it, 1);
            break;
        case IMLS_FINAL_WEIGHTED_LS:
            fk.solve_method = IMLS_SOLVE_WEIGHTED_LS;
            launch_solve_batch(s, tab, caps.data(), npairs, fk, it, 1);
            break;
        default:
            launch_rows_pass1_batch(s, tab, caps.data(), npairs, 1);
            k_drpm_eig_b<<<g1, 256, 0, s>>>(tab);
            k_drpm_noise_b<<<dim3(solve_blocks_of(maxc), npairs), kBlock, 0, s>>>(tab, rp.drpm_stdev_points, rp.drpm_stdev_normals);
            k_drpm_final_b<<<g1, 256, 0, s>>>(tab, fk, rp.drpm_threshold, it);   // + RANSAC's trace record
    }
    if (rp.final_method == IMLS_FINAL_LS || rp.final_method == IMLS_FINAL_WEIGHTED_LS) k_ransac_trace_b<<<g1, 64, 0, s>>>(tab, it);
    return 0;
}

int ransac_init_tables(int device) {
    // C[k][j] over k < kHypMax: C[m − 31] = e_m (m < 31), C[k] = C[k − 31] + C[k − 3] (mod 2^32)
    static std::mutex mu;
    static std::vector<int> ready;
    std::lock_guard<std::mutex> lock(mu);
    if (device < 0) return -1;
    if ((int)ready.size() <= device) ready.resize(device + 1, 0);
    if (ready[device]) return 0;
    std::vector<uint32_t> T((size_t)(kHypMax + 31) * 31, 0u);
    for (int j = 0; j < 31; ++j) T[(size_t)j * 31 + j] = 1u;
    for (int k = 0; k < kHypMax; ++k)
        for (int j = 0; j < 31; ++j)
            T[(size_t)(k + 31) * 31 + j] = T[(size_t)k * 31 + j] + T[(size_t)(k + 28) * 31 + j];
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_rand_jump), T.data() + 31 * 31, (size_t)kHypMax * 31 * 4) != hipSuccess) return -1;
    ready[device] = 1;
    return 0;
}

void ransac_seed_host(uint32_t seed, int st[34]) {
    int32_t r[34];
    r[0] = (int32_t)(seed == 0 ? 1 : seed);
    for (int i = 1; i < 31; ++i) {
        const int64_t hi = r[i - 1] / 127773, lo = r[i - 1] % 127773;
        int64_t word = 16807 * lo - 2836 * hi;
        if (word < 0) word += 2147483647;
        r[i] = (int32_t)word;
    }
    uint32_t ring[31];
    for (int i = 0; i < 31; ++i) ring[i] = (uint32_t)r[i];
    int f = 3, rr = 0;
    for (int k = 0; k < 310; ++k) {   // srandom_r discards 10·31 outputs
        ring[f] += ring[rr];
        f = (f + 1) % 31;
        rr = (rr + 1) % 31;
    }
    for (int i = 0; i < 31; ++i) st[i] = (int)ring[i];
    st[31] = f;
    st[32] = rr;
    st[33] = 0;
}

}  // namespace imlsgpu
