// solve.hip — the Solving step on device: SolveMotionEstimationProblemLS (solver.cpp:74-166) and
// SolveMotionEstimationProblemWeightedLS (solver.cpp:168-220), the pose update
// rPose = Δ·rPose (laser_odometry.cpp:619) and the convergence test (laser_odometry.cpp:628-646).
//
// The reference solves the N×6 point-to-plane system with Eigen ColPivHouseholderQR, twice
// (all rows; then the rows ranked ⌊tN⌋…⌊(1−t)N⌋ by |residual|).  Here each solve is a reduction
// of the normal equations JᵀJ (21) and Jᵀb (6) in fp64 followed by a column-pivoted Cholesky of
// the 6×6 system — the same column pivoting and the same rank test (|R_kk| > 6·ε·max|R_ii|) as
// ColPivHouseholderQR, since JᵀJ's Schur-complement diagonal equals QR's updated column norms².
//
// Trim selection is exact in the total order (|r|, row): |r| (fp64) is histogrammed on the top 16
// bits of its float image (monotone), the two boundary bins are collected and sorted by
// (|r| bits, row) in LDS, everything strictly between them is reduced directly.
//
// Launch chain per LS solve: k_solve_first (1 block) → k_resid_hist → k_collect (every block
// locates the two boundary bins itself — k_find_bins' scans, redundantly, no launch of its own —
// then reduces the interior rows and collects the boundary ones) → k_solve_final (1 block; re-zeroes
// the histogram's touched groups).  (Solving the first 6×6 redundantly in every k_resid_hist block
// too was measured slower: 30.4 µs vs 14.8 + 11.2.)  Weighted LS is k_solve_first alone.  Every
// kernel returns at once when the frame's `done` flag is set.  (A "last block finishes the reduction" fusion was
// measured slower on MI355X: each block's agent-scope release fence writes back its XCD's L2.)
#include <algorithm>
#include <cfloat>

#include "solve_common.h"

namespace imlsgpu {
namespace {

constexpr int kCollectBlocks = 128;

// ---------------------------------------------------------------------------------------------
// pass 1 for double rows (host API); float rows get it fused in k_project
template <int NT>
__device__ __forceinline__ void rows_pass1_body(const Rows& rows, int N, double* __restrict__ partial) {
    __shared__ double red[(NT / 64) * kNormEq];
    __shared__ double out[kNormEq];
    const int i = blockIdx.x * NT + threadIdx.x;
    double a[6] = {0, 0, 0, 0, 0, 0}, b = 0, wt = 1, cnt = 0;
    if (i < N && rows.get(i, a, b, wt)) {
        const double sw = sqrt(wt);
        for (int k = 0; k < 6; ++k) a[k] = sw * a[k];
        b = sw * b;
        cnt = 1;
    }
    block_normeq<NT>(a, b, cnt, red, out);
    if (threadIdx.x < kNormEq) partial[(size_t)blockIdx.x * kNormEq + threadIdx.x] = out[threadIdx.x];
}
template <int NT>
__global__ __launch_bounds__(NT) void k_rows_pass1(Rows rows, int N, double* __restrict__ partial) {
    rows_pass1_body<NT>(rows, N, partial);
}
// batched: every frame's RANSAC inlier rows (grid y = frame)
__global__ __launch_bounds__(kBlock) void k_rows_pass1_b(const PairDev* __restrict__ tab, int weighted) {
    const PairDev A = device_view(tab + blockIdx.y);
    if ((int)blockIdx.x >= solve_blocks_of(A.rf.cap)) return;
    rows_pass1_body<kBlock>(frame_rows(A, 1, weighted), A.rf.cap, A.st.partial1);
}

// Reduce pass-1 partials, first solve, set up the trim; or, for WLS, the only solve.
__device__ __forceinline__ void solve_first_body(const double* __restrict__ partial, int blocks, const SolveState& st,
                                                 imls_iter_trace* tr, const KParams& kp, int weighted, int update_pose) {
    if (*st.done) return;
    __shared__ double acc[kNormEq];
    __shared__ double red[(256 / 64) * kNormEq];
    solve_first_block<256>(partial, blocks, st, tr, kp, weighted, update_pose, red, acc);
}
__global__ __launch_bounds__(256) void k_solve_first(const double* __restrict__ partial, int blocks, SolveState st,
                                                     imls_iter_trace* tr, KParams kp, int weighted, int update_pose) {
    solve_first_body(partial, blocks, st, tr, kp, weighted, update_pose);
}

// 65536 bins on the top 16 bits of the float image of |r| (sign bit 0: 8 exponent + 7 mantissa
// bits, 1/128-octave bins): monotone in |r|, so ranks map to bins; boundary bins stay small
// (fewer, wider bins were measured slower: more contention on the histogram atomics and larger
// boundary sorts).
__device__ __forceinline__ int key_bin(double key) {
    return (int)(__float_as_uint((float)key) >> 15);
}

// Block-exclusive prefix sum of one value per thread (NT threads); *all = the block total.
template <int NT>
__device__ unsigned block_exscan(unsigned v, unsigned* wsum, unsigned* all) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    unsigned inc = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const unsigned u = __shfl_up(inc, o, 64);
        if (lane >= o) inc += u;
    }
    __syncthreads();
    if (lane == 63) wsum[wv] = inc;
    __syncthreads();
    unsigned before = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < NT / 64; ++w) {
        before += w < wv ? wsum[w] : 0u;
        tot += wsum[w];
    }
    *all = tot;
    return before + inc - v;
}

// Locate the bins holding ranks `lower` and `upper` (st.sel[4..5]) → st.sel[0..3]: a scan of the
// 256 coarse bins (256 fine bins each) finds the coarse bin of each rank, a scan of that coarse
// bin's fine bins the fine one.  One block of kCoarse threads (every k_collect block runs it).
constexpr int kCoarse = kHistBins / 256;
// sel_out (LDS, nullable): the four values also land there, for the block that found them
__device__ __forceinline__ void find_bins_core(const SolveState& st, int* sel_out) {
    __shared__ unsigned wsum[kCoarse / 64];
    __shared__ int cb[2];
    __shared__ unsigned cbase[2];
    const int t = threadIdx.x;
    const unsigned c = st.coarse[t];
    unsigned all = 0;
    const unsigned ex = block_exscan<kCoarse>(c, wsum, &all);
    const long long rank[2] = {st.sel[4], st.sel[5]};
#pragma unroll
    for (int w = 0; w < 2; ++w)
        if (rank[w] >= (long long)ex && rank[w] < (long long)ex + c) { cb[w] = t; cbase[w] = ex; }
    if (t == 0) {
        if (rank[0] >= (long long)all) { st.sel[0] = -1; st.sel[2] = 0; cb[0] = -1; if (sel_out) { sel_out[0] = -1; sel_out[2] = 0; } }   // N = 0
        if (rank[1] >= (long long)all) { st.sel[1] = -1; st.sel[3] = 0; cb[1] = -1; if (sel_out) { sel_out[1] = -1; sel_out[3] = 0; } }
    }
    __syncthreads();
#pragma unroll
    for (int w = 0; w < 2; ++w) {
        const int cw = cb[w];                                  // block-uniform
        if (cw < 0) continue;
        const unsigned f = st.hist[cw * 256 + t];
        unsigned fall = 0;
        const unsigned fex = block_exscan<kCoarse>(f, wsum, &fall) + cbase[w];
        if (rank[w] >= (long long)fex && rank[w] < (long long)fex + f) {
            st.sel[w] = cw * 256 + t;
            st.sel[2 + w] = (int)fex;
            if (sel_out) { sel_out[w] = cw * 256 + t; sel_out[2 + w] = (int)fex; }
        }
    }
    __syncthreads();
}

// |r| under the first solution (solver.cpp:110) and its histogram.  Each block privatises the
// histogram window that holds realistic residuals (kResidWin bins from kResidWinLo, 2^-64 ≤ |r|
// < 2^64) in LDS and flushes its non-zero bins once: a global bin then takes at most one atomic
// per block instead of one per row (the hot bins near the residual mode serialised ~thousands).
constexpr int kResidBlock = 1024;
constexpr int kResidBlocks = 96;
constexpr int kResidWin = 16384;                          // 128 octaves of 1/128-octave bins
constexpr int kResidWinLo = (0x1F800000 >> 15);           // key_bin(2^-64)
__device__ __forceinline__ void resid_hist_core(const Rows& rows, int N, const SolveState& st, int nb, const double* x0) {
    __shared__ unsigned h[kResidWin];
    for (int k = threadIdx.x; k < kResidWin / 4; k += kResidBlock) reinterpret_cast<uint4*>(h)[k] = make_uint4(0u, 0u, 0u, 0u);
    __syncthreads();
    for (int i = blockIdx.x * kResidBlock + threadIdx.x; i < N; i += nb * kResidBlock) {
        double a[6], b, wt;
        double key = -1.0;
        if (rows.get(i, a, b, wt)) {
            double v = a[0] * x0[0];
            for (int k = 1; k < 6; ++k) v = v + a[k] * x0[k];
            key = fabs(v - b);
            const int bin = min(key_bin(key), kHistBins - 1);
            const unsigned w = (unsigned)(bin - kResidWinLo);
            if (w < (unsigned)kResidWin) {
                atomicAdd(&h[w], 1u);
            } else {
                atomicAdd(&st.hist[bin], 1u);
                atomicAdd(&st.coarse[bin >> 8], 1u);
            }
        }
        st.keys[i] = key;
    }
    __syncthreads();
    // flush, coalesced (one atomic instruction per wave and 64 bins: device-scope atomics are
    // costly on MI355X); the window's coarse sums go through LDS and out as ONE more instruction
    static_assert(kResidWinLo % 256 == 0 && kResidWin % kResidBlock == 0 && kResidWin / 256 == 64, "window layout");
    __shared__ unsigned csh[kResidWin / 256];
    if (threadIdx.x < kResidWin / 256) csh[threadIdx.x] = 0u;
    __syncthreads();
    for (int k = threadIdx.x; k < kResidWin; k += kResidBlock) {
        const unsigned v = h[k];
        if (v) atomicAdd(&st.hist[kResidWinLo + k], v);
        unsigned csum = v;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) csum += __shfl_xor(csum, o, 64);
        if ((threadIdx.x & 63) == 0 && csum) atomicAdd(&csh[k >> 8], csum);
    }
    __syncthreads();
    if (threadIdx.x < kResidWin / 256 && csh[threadIdx.x]) atomicAdd(&st.coarse[(kResidWinLo >> 8) + threadIdx.x], csh[threadIdx.x]);
}

// bitonic sort of n (power of two ≤ kCandCap) (key, row) pairs in LDS, ascending
__device__ void bitonic(unsigned long long* k, unsigned* r, int n) {
    for (int size = 2; size <= n; size <<= 1)
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            for (int i = threadIdx.x; i < n; i += blockDim.x) {
                const int j = i ^ stride;
                if (j > i) {
                    const bool up = (i & size) == 0;
                    const bool gt = k[i] > k[j] || (k[i] == k[j] && r[i] > r[j]);
                    if (gt == up) {
                        unsigned long long tk = k[i]; k[i] = k[j]; k[j] = tk;
                        unsigned tr = r[i]; r[i] = r[j]; r[j] = tr;
                    }
                }
            }
            __syncthreads();
        }
}

// The same ascending (key, row) order for n ≤ kRankSortMax pairs by counting ranks: each thread
// ranks its pairs against all n (LDS broadcast reads) and scatters them to their rank in the upper
// half of the arrays — two barriers instead of bitonic's log²(n)/2 (a trimmed-LS boundary bin holds
// ~10-30 candidates).  Keys are distinct as (key, row) pairs.  The sorted pairs are left at k/r[0, n).
constexpr int kRankSortMax = 512;
__device__ void rank_sort(unsigned long long* k, unsigned* r, int n) {
    unsigned long long* sk = k + kRankSortMax;
    unsigned* sr = r + kRankSortMax;
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        const unsigned long long ki = k[i];
        const unsigned ri = r[i];
        int rank = 0;
        for (int j = 0; j < n; ++j) rank += (k[j] < ki || (k[j] == ki && r[j] < ri)) ? 1 : 0;
        sk[rank] = ki;
        sr[rank] = ri;
    }
    __syncthreads();
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        k[i] = sk[i];
        r[i] = sr[i];
    }
    __syncthreads();
}

// Exact fallback when a boundary bin overflows kCandCap: the (key, row) at global rank `target`
// by bisection over the key bits then over rows (slow; only for massively tied residuals).
__device__ void rank_select(const double* keys, int N, long long target, unsigned long long* kout, unsigned* rout,
                            unsigned long long* sh_count) {
    unsigned long long lo = 0, hi = 0x7FF0000000000000ull;   // key bits in [0, +inf]
    while (lo < hi) {
        const unsigned long long mid = lo + (hi - lo) / 2;
        if (threadIdx.x == 0) *sh_count = 0;
        __syncthreads();
        unsigned long long c = 0;
        for (int i = threadIdx.x; i < N; i += blockDim.x) {
            const double k = keys[i];
            if (k >= 0 && (unsigned long long)__double_as_longlong(k) <= mid) ++c;
        }
        atomicAdd(sh_count, c);
        __syncthreads();
        const unsigned long long cnt = *sh_count;
        __syncthreads();
        if ((long long)cnt > target) hi = mid; else lo = mid + 1;
    }
    const unsigned long long kb = lo;
    // rank among rows with key < kb
    if (threadIdx.x == 0) *sh_count = 0;
    __syncthreads();
    unsigned long long c = 0;
    for (int i = threadIdx.x; i < N; i += blockDim.x) {
        const double k = keys[i];
        if (k >= 0 && (unsigned long long)__double_as_longlong(k) < kb) ++c;
    }
    atomicAdd(sh_count, c);
    __syncthreads();
    long long need = target - (long long)*sh_count;   // index among equal keys, by row
    __syncthreads();
    unsigned rlo = 0, rhi = (unsigned)N;
    while (rlo < rhi) {
        const unsigned mid = rlo + (rhi - rlo) / 2;
        if (threadIdx.x == 0) *sh_count = 0;
        __syncthreads();
        unsigned long long cc = 0;
        for (int i = threadIdx.x; i <= (int)mid && i < N; i += blockDim.x) {
            const double k = keys[i];
            if (k >= 0 && (unsigned long long)__double_as_longlong(k) == kb) ++cc;
        }
        atomicAdd(sh_count, cc);
        __syncthreads();
        const long long cnt = (long long)*sh_count;
        __syncthreads();
        if (cnt > need) rhi = mid; else rlo = mid + 1;
    }
    *kout = kb;
    *rout = rlo;
}

__device__ __forceinline__ bool pair_le(unsigned long long ka, unsigned ra, unsigned long long kb, unsigned rb) {
    return ka < kb || (ka == kb && ra <= rb);
}

#ifdef IMLS_DEBUG_WAVE_TRACE
__device__ unsigned long long g_dbg_final[4];
__device__ unsigned long long g_dbg_fstamp[8];   // k_solve_final phase cycles (thread 0), debug build
#define FSTAMP(k) do { if (threadIdx.x == 0) { const long long _n = wall_clock64(); g_dbg_fstamp[k] += _n - fst; fst = _n; } } while (0)
#else
#define FSTAMP(k) do { } while (0)
#endif
// The trimmed second solve (solver.cpp:124-166) by one block of NT threads, after k_collect:
// boundary candidates sorted by (|r| bits, row), exact ranks kept, interior partials added,
// solve6, Δ, pose update.  LDS: ck/cr [kCandCap], red [(NT/64)·28], out [28], shc, selk/selr [2].
template <int NT>
__device__ void final_block(const Rows& rows, int N, SolveState st, imls_iter_trace* tr,
                            const double* __restrict__ partial2, int nparts, const KParams& kp, int update_pose,
                            unsigned long long* ck, unsigned* cr, double* red, double* out, unsigned long long& shc,
                            unsigned long long* selk, unsigned* selr) {
#ifdef IMLS_DEBUG_WAVE_TRACE
    long long fst = wall_clock64();
#endif
    const int blo = st.sel[0], bhi = st.sel[1];
    const long long clo = st.sel[2], chi = st.sel[3], lo = st.sel[4], hi = st.sel[5];
    const unsigned n_lo = st.cand_count[0], n_hi = st.cand_count[1];
    double accA[kNormEq];
    for (int k = 0; k < kNormEq; ++k) accA[k] = 0.0;
    auto add_row = [&](unsigned row) {
        double aa[6], bb, ww;
        rows.get((int)row, aa, bb, ww);
        int k = 0;
        for (int r = 0; r < 6; ++r)
            for (int c = r; c < 6; ++c) accA[k++] += aa[r] * aa[c];
        for (int r = 0; r < 6; ++r) accA[21 + r] += aa[r] * bb;
        accA[27] += 1.0;
    };
    const bool overflow = n_lo > (unsigned)kCandCap || n_hi > (unsigned)kCandCap;
#ifdef IMLS_DEBUG_WAVE_TRACE
    if (threadIdx.x == 0) {   // boundary-bin candidate counts (debug build): solves, Σ n_lo, Σ n_hi, max
        atomicAdd(&g_dbg_final[0], 1ull);
        atomicAdd(&g_dbg_final[1], (unsigned long long)n_lo);
        atomicAdd(&g_dbg_final[2], (unsigned long long)n_hi);
        atomicMax(&g_dbg_final[3], (unsigned long long)(n_lo > n_hi ? n_lo : n_hi));
    }
#endif
    if (!overflow) {
        for (int which = 0; which < 2; ++which) {
            const unsigned n = which ? n_hi : n_lo;
            if (which == 1 && bhi == blo) break;
            if (n == 0) continue;
            int np = 1;
            while (np < (int)n) np <<= 1;
            const unsigned long long* gk = which ? st.cand_hi : st.cand_lo;
            const unsigned* gr = which ? st.cand_hi_row : st.cand_lo_row;
            for (int i = threadIdx.x; i < np; i += NT) {
                ck[i] = i < (int)n ? gk[i] : ~0ull;
                cr[i] = i < (int)n ? gr[i] : ~0u;
            }
            __syncthreads();
            FSTAMP(0);
            if ((int)n <= kRankSortMax) rank_sort(ck, cr, (int)n);
            else bitonic(ck, cr, np);
            FSTAMP(1);
            const long long base = which ? chi : clo;
            for (int i = threadIdx.x; i < (int)n; i += NT) {
                const long long rank = base + i;
                if (rank >= lo && rank <= hi) add_row(cr[i]);
            }
            __syncthreads();
            FSTAMP(2);
        }
    } else {
        if (threadIdx.x == 0) shc = 0;
        rank_select(st.keys, N, lo, &selk[0], &selr[0], &shc);
        rank_select(st.keys, N, hi, &selk[1], &selr[1], &shc);
        __syncthreads();
        for (int i = threadIdx.x; i < N; i += NT) {
            const double key = st.keys[i];
            if (key < 0) continue;
            const int bin = min(key_bin(key), kHistBins - 1);
            if (bin != blo && bin != bhi) continue;   // interior rows came from k_collect
            const unsigned long long kb = (unsigned long long)__double_as_longlong(key);
            if (pair_le(selk[0], selr[0], kb, (unsigned)i) && pair_le(kb, (unsigned)i, selk[1], selr[1])) add_row((unsigned)i);
        }
    }
    // the interior partials from k_collect, then one block reduction
    for (int q = threadIdx.x; q < nparts; q += NT)
#pragma unroll
        for (int k = 0; k < kNormEq; ++k) accA[k] += partial2[(size_t)q * kNormEq + k];
    block_sum28<NT>(accA, red, out);
    FSTAMP(3);
    if (threadIdx.x >= 64) return;
    double x[6], D[16];
    solve6_u(out, x);             // wave 0 (solve_common.h)
    if (threadIdx.x != 0) return;
    FSTAMP(4);
    delta_from_x(x, D);
    FSTAMP(5);
    finish_iteration(st, tr, D, (double)st.sel[6], out[27], update_pose, kp);
    FSTAMP(6);
}

// Reduce rows strictly between the boundary bins; collect the boundary rows.
// The boundary bins, found by EVERY block (k_find_bins' scans, redundantly: no launch between the
// histogram and the collection); the histogram is re-zeroed by k_solve_final.
template <int NT>
__device__ __forceinline__ void collect_body(const Rows& rows, int N, const SolveState& st, double* __restrict__ partial2,
                                             int nb) {
    static_assert(NT == kCoarse, "one thread per coarse bin");
    if (*st.done) return;
    __shared__ double red[(NT / 64) * kNormEq];
    __shared__ int sel[4];
    find_bins_core(st, sel);
    const int blo = sel[0], bhi = sel[1];
    double acc[kNormEq];
    for (int k = 0; k < kNormEq; ++k) acc[k] = 0.0;
    for (int i = blockIdx.x * NT + threadIdx.x; i < N; i += nb * NT) {
        const double key = st.keys[i];
        if (key < 0) continue;
        const int bin = min(key_bin(key), kHistBins - 1);
        if (bin > blo && bin < bhi) {
            double a[6], b, wt;
            rows.get(i, a, b, wt);
            int k = 0;
            for (int r = 0; r < 6; ++r)
                for (int c = r; c < 6; ++c) acc[k++] += a[r] * a[c];
            for (int r = 0; r < 6; ++r) acc[21 + r] += a[r] * b;
            acc[27] += 1.0;
        } else if (bin == blo || bin == bhi) {
            const int which = (bin == blo) ? 0 : 1;
            const unsigned pos = atomicAdd(&st.cand_count[which], 1u);
            if (pos < (unsigned)kCandCap) {
                unsigned long long* ck = which ? st.cand_hi : st.cand_lo;
                unsigned* cr = which ? st.cand_hi_row : st.cand_lo_row;
                ck[pos] = (unsigned long long)__double_as_longlong(key);
                cr[pos] = (unsigned)i;
            }
        }
    }
    // block reduction of the 28 partial sums
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    {
        double v[32];
#pragma unroll
        for (int k = 0; k < 32; ++k) v[k] = k < kNormEq ? acc[k] : 0.0;
        const double s = wave_sum28(v);      // internal.h
        if (!(lane & 1) && (lane >> 1) < kNormEq) red[wv * kNormEq + (lane >> 1)] = s;
    }
    __syncthreads();
    if (threadIdx.x < kNormEq) {
        double s = 0.0;
        for (int w = 0; w < NT / 64; ++w) s += red[w * kNormEq + threadIdx.x];
        partial2[(size_t)blockIdx.x * kNormEq + threadIdx.x] = s;
    }
}

constexpr int kFinalBlock = 256;
__device__ __forceinline__ void solve_final_body(const Rows& rows, int N, const SolveState& st, imls_iter_trace* tr,
                                                 const double* __restrict__ partial2, int nparts, const KParams& kp,
                                                 int update_pose) {
    if (*st.done) return;
    // the histogram was read by k_collect: zero it for the next solve — only the 256-bin groups
    // whose coarse count is non-zero (residuals occupy a few octaves of the 65536 bins)
    static_assert(kFinalBlock == kHistBins / 256, "one thread per coarse bin");
    {
        if (st.coarse[threadIdx.x] != 0u) {
            uint4* h = reinterpret_cast<uint4*>(st.hist + (size_t)threadIdx.x * 256);
#pragma unroll 4
            for (int b = 0; b < 64; ++b) h[b] = make_uint4(0u, 0u, 0u, 0u);
            st.coarse[threadIdx.x] = 0u;
        }
    }
    __shared__ unsigned long long ck[kCandCap];
    __shared__ unsigned cr[kCandCap];
    __shared__ double red[(kFinalBlock / 64) * kNormEq];
    __shared__ double out[kNormEq];
    __shared__ unsigned long long shc;
    __shared__ unsigned long long selk[2];
    __shared__ unsigned selr[2];
    final_block<kFinalBlock>(rows, N, st, tr, partial2, nparts, kp, update_pose, ck, cr, red, out, shc, selk, selr);
}

// Small systems (≤ kSmallRows rows, e.g. the ≤2000-query frames of the config-C stream): the whole
// LS solve in ONE block — pass-1 normal equations from the rows, first solve, |r| keys of the valid rows into
// LDS, boundary bins ordered by (|r| bits, row), ranks [lo, hi] re-reduced, second solve, pose update —
// instead of five launches whose fixed latency dominates at this size.  The same row arithmetic and
// the same exact (|r|, row) trim as the chain; the SUMS are associated differently: each thread adds
// its rows t + k·512 in k order, then block_sum28 — not the chain's 256-row slabs — so every frame of
// ≤ kSmallRows rows (batched or alone, whichever projection kernels produced its rows) takes this
// kernel and the projection writes no slabs for it (project.hip).
constexpr int kSmallBlock = 512;     // 8 waves: ≤ kSmallPer rows per thread, kept in registers between passes
constexpr int kSmallPer = kSmallRows / kSmallBlock;
static_assert(kSmallRows % kSmallBlock == 0, "rows per thread");
constexpr unsigned long long kNoKey = ~0ull;   // k_solve_small: slot of an invalid row
constexpr int kSmallBins = 4096;     // LDS histogram: top 12 bits of the float image of |r| (1/16 octave)
__device__ __forceinline__ int small_bin(unsigned long long keybits) {
    return (int)(__float_as_uint((float)__longlong_as_double((long long)keybits)) >> 19);
}
#ifdef IMLS_DEBUG_WAVE_TRACE
__device__ unsigned long long g_dbg_solve[8];
#define DBG_STAMP(k) do { if (threadIdx.x == 0) g_dbg_solve[k] += wall_clock64() - dbg_t; dbg_t = wall_clock64(); } while (0)
#else
#define DBG_STAMP(k) do { } while (0)
#endif
// the row of a float correspondence as Rows::get builds it (solver.cpp:95-103), from its floats
__device__ __forceinline__ void small_a(const float4& s4, const float4& n4, double a[6]) {
    const double s[3] = {s4.x, s4.y, s4.z}, n[3] = {n4.x, n4.y, n4.z};
    a[0] = n[2] * s[1] - n[1] * s[2];
    a[1] = n[0] * s[2] - n[2] * s[0];
    a[2] = n[1] * s[0] - n[0] * s[1];
    a[3] = n[0]; a[4] = n[1]; a[5] = n[2];
}
__device__ __forceinline__ double small_b(const float4& s4, const float4& d4, const float4& n4) {
    const double s[3] = {s4.x, s4.y, s4.z}, d[3] = {d4.x, d4.y, d4.z}, n[3] = {n4.x, n4.y, n4.z};
    double b = n[0] * (d[0] - s[0]);
    b = b + n[1] * (d[1] - s[1]);
    b = b + n[2] * (d[2] - s[2]);
    return b;
}
// (round 4) 512 threads, each owning rows t + k·512: each row's s, n and b stay in registers from the
// residual pass to the kept-row sums (no second gather), valid rows are counted by wave ballots,
// the histogram scan is a wave-shuffle block scan and the boundary candidates are ranked by
// counting (rank_sort) — the phases were latency chains of 256 threads × 8 rows (31 µs per solve on
// a 1949-row frame, tools/frame_probe.py).  Float rows only (the projection's; RANSAC rows take
// the grid chain).
__device__ __forceinline__ void solve_small_body(const Rows& rows, int N, const SolveState& st, imls_iter_trace* tr,
                                                 const KParams& kp,
                                                 int weighted, int update_pose) {
    // the stop flag is read with the rows, not ahead of them (one dependent load fewer; the rows
    // are only read before the test)
    const int stopped = *st.done;
#ifdef IMLS_DEBUG_WAVE_TRACE
    long long dbg_t = wall_clock64();
#endif
    __shared__ unsigned long long ck[kSmallRows];
    __shared__ unsigned long long qk[kSmallRows];
    __shared__ unsigned qr[kSmallRows];
    __shared__ unsigned hist[kSmallBins];
    __shared__ unsigned wsum[kSmallBlock / 64];
    __shared__ int bsel[5];
    __shared__ int ncand;
    __shared__ double red[(kSmallBlock / 64) * kNormEq];
    __shared__ double acc[kNormEq];
    __shared__ double xs[6];
    __shared__ int nkey;
    __shared__ int stop;
    const int t = threadIdx.x, lane = t & 63;
    double loc[kNormEq];
#pragma unroll
    for (int k = 0; k < kNormEq; ++k) loc[k] = 0.0;
    auto add_row = [&](const double (&a)[6], double b) {
        int q = 0;
        for (int p = 0; p < 6; ++p)
            for (int c = p; c < 6; ++c) loc[q++] += a[p] * a[c];
        for (int p = 0; p < 6; ++p) loc[21 + p] += a[p] * b;
        loc[27] += 1.0;
    };
    if (t == 0) { nkey = 0; stop = 0; }
    // this thread's rows: s (w = valid flag), n, and b = n·(d − s), kept in registers for every pass.
    // Pass 1 (the normal equations of every valid row, solver.cpp:89-107) is formed here from them
    // (round 4): the lone-frame path then needs no slab launch, and every small frame — batched or
    // alone, whatever exact stage produced its rows — sums them in this one order
    float4 rs[kSmallPer], rn[kSmallPer];
    double rb[kSmallPer];
    static_assert(kSmallPer % 2 == 0, "two row groups");
    // the rows in two groups of kSmallPer/2 per thread, each group's s, y and n loaded together
    // (unconditional loads from a clamped row index, values selected after: a load behind `r < N`
    // or the valid flag became a branch with its own wait — 24 dependent round trips per thread);
    // the second group only when the frame has rows there (block-uniform), its loads ordered after
    // the first group's by an asm dependency (all rows in flight at once spilled ~60 VGPRs)
    const int rmax = N > 0 ? N - 1 : 0;
    const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
    constexpr int kGrp = kSmallPer / 2;
    int tg = t;
    auto load_group = [&](int k0) {
        float4 c[kGrp], d[kGrp], n[kGrp];
#pragma unroll
        for (int u = 0; u < kGrp; ++u) {
            const int rr = min(tg + (k0 + u) * kSmallBlock, rmax);
            c[u] = rows.cs[rr];
            d[u] = rows.cd[rr];
            n[u] = rows.cn[rr];
        }
#pragma unroll
        for (int u = 0; u < kGrp; ++u) {
            const int k = k0 + u;
            const int r = t + k * kSmallBlock;
            rs[k] = r < N ? c[u] : z4;
            const bool v = r < N && rs[k].w != 0.f;
            rn[k] = v ? n[u] : z4;
            rb[k] = small_b(rs[k], v ? d[u] : z4, rn[k]);
        }
    };
    load_group(0);
    if (N > kGrp * kSmallBlock) {
        asm volatile("" : "+v"(tg) : "v"(rb[0]), "v"(rb[kGrp - 1]));
        load_group(kGrp);
    } else {
#pragma unroll
        for (int k = kGrp; k < kSmallPer; ++k) { rs[k] = z4; rn[k] = z4; rb[k] = 0.0; }
    }
    if (stopped) return;              // block-uniform, before any LDS write or barrier
#pragma unroll
    for (int k = 0; k < kSmallPer; ++k) {
        if (t + k * kSmallBlock < N && rs[k].w != 0.f) {
            double a[6];
            small_a(rs[k], rn[k], a);
            add_row(a, rb[k]);
        }
    }
    block_sum28<kSmallBlock>(loc, red, acc);
    DBG_STAMP(0);
    const double nvalid = acc[27];
    if (t < 64) {                     // wave 0: the 6×6 solve by its 64 lanes (solve6_u)
        double x[6];
        if (update_pose && nvalid < (double)kp.correspond_number) {   // laser_odometry.cpp:570-576
            if (t == 0) {
                *st.status = IMLS_FRAME_TOO_FEW;
                *st.done = 1;
                if (tr) tr->n_valid = (unsigned long long)nvalid;
                stop = 1;
            }
        } else {
            solve6_u(acc, x);
            if (t == 0) {
                if (weighted) {
                    double D[16];
                    delta_from_x(x, D);
                    finish_iteration(st, tr, D, nvalid, nvalid, update_pose, kp);
                    stop = 1;
                }
                for (int k = 0; k < 6; ++k) xs[k] = x[k];
            }
        }
    }
    __syncthreads();
    DBG_STAMP(1);
    if (stop) return;
    // |r| under the first solution, valid rows only (solver.cpp:110-122).  Keys stay at their row's
    // slot (invalid rows hold a sentinel) so every later pass walks the rows in a fixed order
    int mine = 0;
#pragma unroll
    for (int k = 0; k < kSmallPer; ++k) {
        const int r = t + k * kSmallBlock;
        const bool v = r < N && rs[k].w != 0.f;
        unsigned long long kb = kNoKey;
        if (v) {
            double a[6];
            small_a(rs[k], rn[k], a);
            double val = a[0] * xs[0];
            for (int q = 1; q < 6; ++q) val = val + a[q] * xs[q];
            kb = (unsigned long long)__double_as_longlong(fabs(val - rb[k]));
        }
        if (r < N) ck[r] = kb;
        mine += __popcll(__ballot(v));
    }
    if (lane == 0 && mine) atomicAdd(&nkey, mine);
    for (int b = t; b < kSmallBins; b += kSmallBlock) hist[b] = 0u;
    __syncthreads();
    DBG_STAMP(2);
    const int n = nkey;
    const long long lo = (long long)(kp.ls_threshold * (double)n);
    long long hi = (long long)((1 - kp.ls_threshold) * (double)n);
    if (hi > n - 1) hi = n - 1;       // Q11
    if (n == 0 || lo > hi) {          // no valid row (stand-alone solve, or correspond_number <= 0): as the oracle
        if (t == 0) { *st.status = IMLS_FRAME_SOLVE_FAILED; *st.done = 1; }
        return;                       // n, lo, hi are block-uniform: every thread leaves here
    }
    // exact ranks at the two trim boundaries: a 4096-bin LDS histogram of the float image of |r|
    // (monotone) locates the boundary bins; only their rows are ordered by (|r| bits, row)
#pragma unroll
    for (int k = 0; k < kSmallPer; ++k) {
        const int r = t + k * kSmallBlock;
        if (r < N && ck[r] != kNoKey) atomicAdd(&hist[small_bin(ck[r])], 1u);
    }
    __syncthreads();
    {
        constexpr int per = kSmallBins / kSmallBlock;
        unsigned loc_sum = 0;
#pragma unroll
        for (int k = 0; k < per; ++k) loc_sum += hist[t * per + k];
        unsigned total;
        long long cum = block_exscan<kSmallBlock>(loc_sum, wsum, &total);
#pragma unroll
        for (int k = 0; k < per; ++k) {
            const long long c = hist[t * per + k];
            if (lo >= cum && lo < cum + c) { bsel[0] = t * per + k; bsel[2] = (int)cum; }
            if (hi >= cum && hi < cum + c) { bsel[1] = t * per + k; bsel[3] = (int)cum; }
            cum += c;
        }
        if (t == 0) ncand = 0;
    }
    __syncthreads();
    const int blo = bsel[0], bhi = bsel[1];
    if (t == 0) bsel[4] = (int)hist[blo];           // candidates of the lower boundary bin
#pragma unroll
    for (int k = 0; k < kSmallPer; ++k) {
        const int r = t + k * kSmallBlock;
        if (r >= N || ck[r] == kNoKey) continue;
        const int b = small_bin(ck[r]);
        if (b == blo || b == bhi) {
            const int at = atomicAdd(&ncand, 1);
            qk[at] = ck[r];
            qr[at] = (unsigned)r;
        }
    }
    __syncthreads();
    const int nc = ncand;
    if (nc <= kRankSortMax) {
        rank_sort(qk, qr, nc);
    } else {
        int np = 1;
        while (np < nc) np <<= 1;
        for (int i = nc + t; i < np; i += kSmallBlock) { qk[i] = ~0ull; qr[i] = ~0u; }
        __syncthreads();
        bitonic(qk, qr, np);
    }
    DBG_STAMP(3);
#pragma unroll
    for (int k = 0; k < kNormEq; ++k) loc[k] = 0.0;
#pragma unroll
    for (int k = 0; k < kSmallPer; ++k) {           // interior bins: kept without ranking (registers)
        const int r = t + k * kSmallBlock;
        if (r >= N || ck[r] == kNoKey) continue;
        const int b = small_bin(ck[r]);
        if (b > blo && b < bhi) {
            double a[6];
            small_a(rs[k], rn[k], a);
            add_row(a, rb[k]);
        }
    }
    for (int q = t; q < nc; q += kSmallBlock) {    // boundary bins: exact rank = bin base + order
        const int b = small_bin(qk[q]);
        int first = 0;                              // first candidate of this bin in sorted order
        if (b == bhi && bhi != blo) first = bsel[4];  // candidates of blo sort before those of bhi
        const long long rank = (long long)(b == blo ? bsel[2] : bsel[3]) + (q - first);
        if (rank >= lo && rank <= hi) {
            double a[6], bb, wt;
            rows.get((int)qr[q], a, bb, wt);
            add_row(a, bb);
        }
    }
    block_sum28<kSmallBlock>(loc, red, acc);
    DBG_STAMP(4);
    if (t >= 64) return;
    double x[6], D[16];
    solve6_u(acc, x);
    if (t != 0) return;
    DBG_STAMP(5);
    delta_from_x(x, D);
    DBG_STAMP(6);
    finish_iteration(st, tr, D, (double)n, acc[27], update_pose, kp);
    DBG_STAMP(7);
}


// ---------------------------------------------------------------------------------------------
// Kernels: one frame (arguments by value) and batched (frame = tab[blockIdx.y], float rows from the
// batched projection; blocks past the frame's own grid leave at once).  Both run the same bodies.
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(kResidBlock) void k_resid_hist(Rows rows, int N, SolveState st) {
    if (*st.done) return;
    resid_hist_core(rows, N, st, (int)gridDim.x, st.x0);
}
template <int NT>
__global__ __launch_bounds__(NT) void k_collect(Rows rows, int N, SolveState st, double* __restrict__ partial2) {
    collect_body<NT>(rows, N, st, partial2, (int)gridDim.x);
}
__global__ __launch_bounds__(kFinalBlock) void k_solve_final(Rows rows, int N, SolveState st, imls_iter_trace* tr,
                                                            const double* __restrict__ partial2, int nparts, KParams kp,
                                                            int update_pose) {
    solve_final_body(rows, N, st, tr, partial2, nparts, kp, update_pose);
}
__global__ __launch_bounds__(kSmallBlock) void k_solve_small(Rows rows, int N, SolveState st, imls_iter_trace* tr, KParams kp,
                                                            int weighted, int update_pose) {
    solve_small_body(rows, N, st, tr, kp, weighted, update_pose);
}

// grid shapes of the chain, per frame (shared by the one-frame and the batched launches)
__host__ __device__ __forceinline__ int resid_blocks_of(int N) {
    const int b = (N + kResidBlock - 1) / kResidBlock;
    return b < kResidBlocks ? b : kResidBlocks;
}
__host__ __device__ __forceinline__ int collect_blocks_of(int N) {
    const int b = (N + kBlock * 4 - 1) / (kBlock * 4);
    return b < 1 ? 1 : (b < kCollectBlocks ? b : kCollectBlocks);
}
__host__ __device__ __forceinline__ int pass1_blocks_of(int N) {   // project_blocks(N): wave slabs + fallback slabs
    return (N + kPass1Block - 1) / kPass1Block + kPass1Fallback;
}
// batched chain: src 0 = the projection's float rows (k_solve_small for N ≤ kSmallRows, the grid
// chain above), src 1 = the RANSAC inlier rows (the grid chain always, as launch_solve runs it)
__device__ __forceinline__ int frame_rows_n(const PairDev& A, int src) { return src ? A.rf.cap : A.N; }
__device__ __forceinline__ bool frame_big(const PairDev& A, int src) { return src || A.N > kSmallRows; }

__global__ __launch_bounds__(kSmallBlock) void k_solve_small_b(const PairDev* __restrict__ tab, KParams kp, int weighted,
                                                              int it) {
    const PairDev A = device_view(tab + blockIdx.y);
    if (A.N > kSmallRows) return;
    solve_small_body(frame_rows(A, 0, 0), A.N, A.st, A.trace + it, kp, weighted, 1);
}
__global__ __launch_bounds__(256) void k_solve_first_b(const PairDev* __restrict__ tab, KParams kp, int weighted, int it,
                                                       int src) {
    const PairDev A = device_view(tab + blockIdx.y);
    if (!frame_big(A, src)) return;
    solve_first_body(A.st.partial1, src ? solve_blocks_of(A.rf.cap) : pass1_blocks_of(A.N), A.st, A.trace + it, kp,
                     weighted, 1);
}
__global__ __launch_bounds__(kResidBlock) void k_resid_hist_b(const PairDev* __restrict__ tab, int src) {
    const PairDev A = device_view(tab + blockIdx.y);
    const int N = frame_rows_n(A, src);
    const int nb = resid_blocks_of(N);
    if (!frame_big(A, src) || (int)blockIdx.x >= nb || *A.st.done) return;
    resid_hist_core(frame_rows(A, src, 0), N, A.st, nb, A.st.x0);
}
__global__ __launch_bounds__(kBlock) void k_collect_b(const PairDev* __restrict__ tab, int src) {
    const PairDev A = device_view(tab + blockIdx.y);
    const int N = frame_rows_n(A, src);
    const int nb = collect_blocks_of(N);
    if (!frame_big(A, src) || (int)blockIdx.x >= nb) return;
    collect_body<kBlock>(frame_rows(A, src, 0), N, A.st, A.st.partial2, nb);
}
__global__ __launch_bounds__(kFinalBlock) void k_solve_final_b(const PairDev* __restrict__ tab, KParams kp, int it, int src) {
    const PairDev A = device_view(tab + blockIdx.y);
    if (!frame_big(A, src)) return;
    const int N = frame_rows_n(A, src);
    solve_final_body(frame_rows(A, src, 0), N, A.st, A.trace + it, A.st.partial2, collect_blocks_of(N), kp, 1);
}

}  // namespace

int solve_blocks(int N) { return (N + kBlock - 1) / kBlock; }

void launch_rows_pass1(hipStream_t s, const Rows& rows, int N, double* partial, int blocks) {
    k_rows_pass1<kBlock><<<blocks, kBlock, 0, s>>>(rows, N, partial);
}

void launch_solve_chain(hipStream_t s, int N, int blocks1, const KParams& kp, const float4* cs, const float4* cd,
                        const float4* cn, const double* rows_d, const double* weights, SolveState& st,
                        imls_iter_trace* tr, int update_pose, int rows_are_double, const int* count, const double* wsum) {
    Rows rows{cs, cd, cn, nullptr, nullptr, nullptr, weights, rows_are_double, count, wsum};
    if (rows_are_double) {
        rows.ds = rows_d;
        rows.dd = rows_d + 3 * (size_t)N;
        rows.dn = rows_d + 6 * (size_t)N;
        blocks1 = solve_blocks(N);
        k_rows_pass1<kBlock><<<blocks1, kBlock, 0, s>>>(rows, N, st.partial1);
    }
    const int weighted = kp.solve_method == IMLS_SOLVE_WEIGHTED_LS;
    if (!rows_are_double && N <= kSmallRows) {
        k_solve_small<<<1, kSmallBlock, 0, s>>>(rows, N, st, tr, kp, weighted, update_pose);
        return;
    }
    k_solve_first<<<1, 256, 0, s>>>(st.partial1, blocks1, st, tr, kp, weighted, update_pose);
    if (weighted) return;
    k_resid_hist<<<resid_blocks_of(N), kResidBlock, 0, s>>>(rows, N, st);
    const int cb = collect_blocks_of(N);
    k_collect<kBlock><<<cb, kBlock, 0, s>>>(rows, N, st, st.partial2);
    k_solve_final<<<1, kFinalBlock, 0, s>>>(rows, N, st, tr, st.partial2, cb, kp, update_pose);
}

}  // namespace imlsgpu

#ifdef IMLS_DEBUG_WAVE_TRACE
extern "C" int imls_debug_solve(unsigned long long* out) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(imlsgpu::g_dbg_solve), 64) == hipSuccess ? 0 : -1;
}
extern "C" int imls_debug_final(unsigned long long* out) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(imlsgpu::g_dbg_final), 32) == hipSuccess &&
                   hipMemcpyFromSymbol(out + 4, HIP_SYMBOL(imlsgpu::g_dbg_fstamp), 64) == hipSuccess
               ? 0 : -1;
}
#endif

namespace imlsgpu {
void launch_rows_pass1_batch(hipStream_t s, const PairDev* tab, const int* cap_host, int npairs, int weighted) {
    int maxc = 1;
    for (int k = 0; k < npairs; ++k) maxc = std::max(maxc, cap_host[k]);
    k_rows_pass1_b<<<dim3(solve_blocks_of(maxc), npairs), kBlock, 0, s>>>(tab, weighted);
}

void launch_solve_batch(hipStream_t s, const PairDev* tab, const int* n_host, int npairs, const KParams& kp, int it,
                        int src) {
    if (npairs <= 0) return;
    int maxN = 0;
    bool any_small = false, any_large = false;
    for (int k = 0; k < npairs; ++k) {
        maxN = std::max(maxN, n_host[k]);
        (n_host[k] <= kSmallRows && !src ? any_small : any_large) = true;
    }
    const int weighted = kp.solve_method == IMLS_SOLVE_WEIGHTED_LS;
    if (src) launch_rows_pass1_batch(s, tab, n_host, npairs, weighted);
    if (any_small) k_solve_small_b<<<dim3(1, npairs), kSmallBlock, 0, s>>>(tab, kp, weighted, it);
    if (!any_large) return;
    k_solve_first_b<<<dim3(1, npairs), 256, 0, s>>>(tab, kp, weighted, it, src);
    if (weighted) return;
    k_resid_hist_b<<<dim3(resid_blocks_of(maxN), npairs), kResidBlock, 0, s>>>(tab, src);
    k_collect_b<<<dim3(collect_blocks_of(maxN), npairs), kBlock, 0, s>>>(tab, src);
    k_solve_final_b<<<dim3(1, npairs), kFinalBlock, 0, s>>>(tab, kp, it, src);
}
}  // namespace imlsgpu
