// ransac.hip — SolveMotionEstimationProblemRANSAC (solver.cpp:222-385) with farthestPointSampling
// (common.cpp:19-82) and SolveMotionEstimationProblemDRPM (solver.cpp:486-603, degeneracy.h:14-131)
// on device, plus the solve-method dispatcher used by the ICP loop.
//
// Data flow per RANSAC solve (all on the context's stream, no host sync):
//   1. the valid correspondences (float rows, source order) are compacted, order kept, into fp64
//      rows S/D/N — the reference's std::vector<Vector3d> inputs; the TOO_FEW gate
//      (laser_odometry.cpp:570-576) runs on their count;
//   2. hypotheses in growing chunks (16, 64, 256, 1024, 4096): k_ransac_draws replays glibc rand()
//      (one draw per hypothesis: the FPS start index), k_ransac_hyp runs one hypothesis per block —
//      FPS (two arg-max passes, first index wins ties as the sequential `>` does), the 3×6
//      column-pivoted Householder QR basic solution (Eigen ColPivHouseholderQR, not normal
//      equations: a rank-3 system squared would misjudge the rank), Δ, and the inlier count;
//      k_ransac_select scans the chunk in order with the reference's strict `>` and early exit
//      (best > ⌊pct·N⌋) and commits exactly the draws consumed; later chunks return at once;
//   3. inliers of the best Δ are compacted (order kept) with weights
//      w = √a < h₂ ? a : 2h₂√a − h₂², a = e^{−|r|}, h₂ = huber·distance (solver.cpp:334-356),
//      normalised by Σw (361-364; the division happens where the weight is read);
//   4. final solve: LS (trimmed, RANSAC's own threshold) / weighted LS through the LS chain on the
//      fp64 inlier rows, or DRPM: H = Σ w a aᵀ and g = Σ w a b (pass 1 of the LS chain), a cyclic
//      Jacobi eigendecomposition (SelfAdjointEigenSolver order: ascending), the per-point noise
//      mean/variance along the eigenvectors, normal-CDF probabilities with SNR factor 10, and
//      x = U·diag(p/λ)·Uᵀ g when min p < threshold, else the weighted solve.
#include "solve_common.h"

namespace imlsgpu {
namespace {

constexpr int kHypBlock = 256;
constexpr int kDrpmSlab = 42;         // 36 noise-mean terms + 6 variance terms per block

// ---------------------------------------------------------------------------------------------
// glibc random() TYPE_3 (what rand() returns), state = 31 words + front/rear indices
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ int rand_next(int* st) {
    unsigned* ring = reinterpret_cast<unsigned*>(st);
    const int f = st[31], r = st[32];
    ring[f] += ring[r];
    const int out = (int)(ring[f] >> 1);
    st[31] = (f + 1) % 31;
    st[32] = (r + 1) % 31;
    return out;
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

__global__ __launch_bounds__(kBlock) void k_compact_count(Source src, int n, int* __restrict__ blkcnt,
                                                          double* __restrict__ blkw, const int* __restrict__ done) {
    if (done && *done) return;
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

// One block: exclusive scan of the block counts (in place), total count and Σw in fixed order.
__global__ __launch_bounds__(1024) void k_compact_scan(int* __restrict__ blkcnt, const double* __restrict__ blkw, int nb,
                                                       CompactOut out, const int* __restrict__ done) {
    if (done && *done) return;
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
    }
}

__global__ __launch_bounds__(kBlock) void k_compact_scatter(Source src, int n, const int* __restrict__ blkoff, CompactOut out,
                                                            const int* __restrict__ done) {
    if (done && *done) return;
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

// ---------------------------------------------------------------------------------------------
// RANSAC state (device, one per context)
// ---------------------------------------------------------------------------------------------
struct RansacDev {
    int* rng;          // [34] glibc state (persistent)
    int* first;        // [kHypMax] FPS start index per hypothesis of the current chunk
    int* counts;       // [kHypMax]
    double* T;         // [kHypMax × 16]
    int* best;         // [1]
    int* evaluated;    // [1]
    int* rdone;        // [1] RANSAC finished (early exit or max iterations)
    double* bestT;     // [16]
    int* active;       // [1] the frame was still running when this solve began
};

// stand-alone DRPM with no rows fails like the oracle's solve_drpm (N == 0 → false)
__global__ void k_drpm_guard(const int* __restrict__ c, SolveState st) {
    if (threadIdx.x == 0 && *c == 0) { *st.status = IMLS_FRAME_SOLVE_FAILED; *st.done = 1; }
}

__global__ void k_set_count(int* __restrict__ c, int v) {
    if (threadIdx.x == 0) *c = v;
}

// gate on the compacted count, reset the RANSAC selection state
__global__ void k_ransac_begin(const int* __restrict__ count, int correspond_number, int update_pose, SolveState st,
                               imls_iter_trace* tr, RansacDev R) {
    if (threadIdx.x) return;
    *R.active = *st.done ? 0 : 1;
    if (*st.done) return;
    const int n = *count;
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

__global__ void k_ransac_draws(const int* __restrict__ count, RansacDev R, int chunk, const int* __restrict__ done) {
    if (threadIdx.x || *done || *R.rdone) return;
    __shared__ int st[34];   // LDS: the ring is indexed dynamically
    for (int k = 0; k < 34; ++k) st[k] = R.rng[k];
    const int n = *count;
    for (int h = 0; h < chunk; ++h) R.first[h] = rand_next(st) % n;
}

// block arg-max of (value, index): larger value, then smaller index
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
        for (int k = 1; k < kHypBlock / 64; ++k)
            if (sv[k] > sv[0] || (sv[k] == sv[0] && si[k] < si[0])) { sv[0] = sv[k]; si[0] = si[k]; }
    }
    __syncthreads();
    v = sv[0];
    i = si[0];
    __syncthreads();
}

// ‖s_a − s_b‖ as Eigen's (a − b).norm() evaluates it
__device__ __forceinline__ double pdist(const double* s, int a, int b) {
    const double dx = s[3 * (size_t)a] - s[3 * (size_t)b], dy = s[3 * (size_t)a + 1] - s[3 * (size_t)b + 1],
                 dz = s[3 * (size_t)a + 2] - s[3 * (size_t)b + 2];
    return sqrt((dx * dx + dy * dy) + dz * dz);
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

// One hypothesis per block: FPS(3) from the drawn start, 3×6 QR, Δ, inlier count.
__global__ __launch_bounds__(kHypBlock) void k_ransac_hyp(const double* __restrict__ rows, const int* __restrict__ count,
                                                          int cap, RansacDev R, double dist_thr, const int* __restrict__ done) {
    if (*done || *R.rdone) return;
    __shared__ double sv[kHypBlock / 64];
    __shared__ int si[kHypBlock / 64];
    __shared__ double T[16];
    __shared__ int cnt_s[kHypBlock / 64];
    const int h = blockIdx.x, n = *count;
    const size_t c3 = 3 * (size_t)cap;
    const double* S = rows;
    const double* Dp = rows + c3;
    const double* Np = rows + 2 * c3;
    const int f0 = R.first[h];
    // pass 1: farthest from f0 (common.cpp:48-66: strict `>` from −1, taken points skipped)
    double bv = -1.0;
    int bi = 0x7fffffff;
    for (int i = threadIdx.x; i < n; i += kHypBlock) {
        if (i == f0) continue;
        const double md = pdist(S, f0, i);
        if (md > bv) { bv = md; bi = i; }
    }
    argmax_pair(bv, bi, sv, si);
    const int f1 = bi;
    // pass 2: farthest from {f0, f1} by the running minimum distance
    bv = -1.0;
    bi = 0x7fffffff;
    for (int i = threadIdx.x; i < n; i += kHypBlock) {
        if (i == f0 || i == f1) continue;
        const double md = fmin(pdist(S, f0, i), pdist(S, f1, i));
        if (md > bv) { bv = md; bi = i; }
    }
    argmax_pair(bv, bi, sv, si);
    const int f2 = bi;
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
        delta_from_x(x, D);
#pragma unroll
        for (int k = 0; k < 16; ++k) T[k] = D[k];
    }
    __syncthreads();
    int c = 0;
    for (int i = threadIdx.x; i < n; i += kHypBlock) {
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
        for (int k = 0; k < kHypBlock / 64; ++k) tot += cnt_s[k];
        R.counts[h] = tot;
    }
    if (threadIdx.x < 16) R.T[(size_t)h * 16 + threadIdx.x] = T[threadIdx.x];
}

// Sequential semantics of the hypothesis loop (solver.cpp:244-326) over one chunk.
__global__ void k_ransac_select(const int* __restrict__ count, RansacDev R, int chunk, int max_iterations, double min_pct,
                                const int* __restrict__ done) {
    if (threadIdx.x || *done || *R.rdone) return;
    const int n = *count;
    const int min_inliers = (int)(min_pct * (double)n);
    int best = *R.best, used = 0;
    bool stop = false;
    for (int h = 0; h < chunk && !stop; ++h) {
        ++used;
        if (R.counts[h] > best) {
            best = R.counts[h];
            for (int k = 0; k < 16; ++k) R.bestT[k] = R.T[(size_t)h * 16 + k];
        }
        if (best > min_inliers) stop = true;
    }
    __shared__ int st[34];
    for (int k = 0; k < 34; ++k) st[k] = R.rng[k];
    for (int k = 0; k < used; ++k) (void)rand_next(st);       // commit exactly the draws consumed
    for (int k = 0; k < 34; ++k) R.rng[k] = st[k];
    *R.best = best;
    *R.evaluated += used;
    if (stop || *R.evaluated >= max_iterations) *R.rdone = 1;
}

// trace of a RANSAC iteration as the oracle records it: n_valid = correspondences, n_kept = 0
__global__ void k_ransac_trace(const int* __restrict__ count_all, RansacDev R, imls_iter_trace* tr) {
    if (threadIdx.x || !*R.active || !tr) return;
    tr->n_valid = (unsigned long long)*count_all;
    tr->n_kept = 0;
}

__global__ void k_ransac_check_inliers(const int* __restrict__ count_in, SolveState st, imls_iter_trace* tr) {
    if (threadIdx.x || *st.done) return;
    if (*count_in == 0) {   // nothing to solve on (the oracle's N == 0 → false): stop like a failed solve
        *st.status = IMLS_FRAME_SOLVE_FAILED;
        *st.done = 1;
    }
}

// ---------------------------------------------------------------------------------------------
// DRPM (solver.cpp:499-603, degeneracy.h:14-131)
// ---------------------------------------------------------------------------------------------
struct DrpmDev {
    double* H;        // [36] row-major
    double* g;        // [6]
    double* U;        // [36] eigenvectors as columns: U[k·6 + r] = component r of vector k
    double* ev;       // [6] ascending
    double* slabs;    // [blocks × kDrpmSlab]
};

// reduce the weighted normal equations (pass-1 slabs), eigendecompose H
__global__ __launch_bounds__(256) void k_drpm_eig(const double* __restrict__ partial, int blocks, SolveState st, DrpmDev Dv) {
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
    if (threadIdx.x) return;
    double H[36];
    int k = 0;
    for (int r = 0; r < 6; ++r)
        for (int c = r; c < 6; ++c) { H[r * 6 + c] = acc[k]; H[c * 6 + r] = acc[k]; ++k; }
    for (int q = 0; q < 36; ++q) Dv.H[q] = H[q];
    for (int r = 0; r < 6; ++r) Dv.g[r] = acc[21 + r];
    double ev[6], U[36];
    sym_eig<6>(H, ev, U);
    for (int q = 0; q < 36; ++q) Dv.U[q] = U[q];
    for (int r = 0; r < 6; ++r) Dv.ev[r] = ev[r];
}

// per-point noise mean (36) and variance along the eigenvectors (6), degeneracy.h:14-72
__global__ __launch_bounds__(kBlock) void k_drpm_noise(Rows rows, int N, SolveState st, DrpmDev Dv, double sp, double sn) {
    if (*st.done) return;
    __shared__ double red[(kBlock / 64) * kDrpmSlab];
    const int i = blockIdx.x * kBlock + threadIdx.x;
    double acc[kDrpmSlab];
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
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
    for (int k = 0; k < kDrpmSlab; ++k) {
        const double v = wave_sum(acc[k]);
        if (lane == 0) red[wv * kDrpmSlab + k] = v;
    }
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

__global__ __launch_bounds__(256) void k_drpm_final(int blocks, SolveState st, DrpmDev Dv, imls_iter_trace* tr, KParams kp,
                                                    double threshold, const int* __restrict__ count_all,
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
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
    for (int k = 0; k < kDrpmSlab; ++k) {
        const double v = wave_sum(loc[k]);
        if (lane == 0) red[wv * kDrpmSlab + k] = v;
    }
    __syncthreads();
    if (threadIdx.x < kDrpmSlab) {
        double s = 0.0;
        for (int w = 0; w < 256 / 64; ++w) s += red[w * kDrpmSlab + threadIdx.x];
        tot[threadIdx.x] = s;
    }
    __syncthreads();
    if (threadIdx.x) return;
    double prob[6], pmin = INFINITY;
    const double snr = 10.0;   // solver.cpp:547
    for (int k = 0; k < 6; ++k) {
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
        prob[k] = bad ? 0.0 : normal_cdf(exp_noise, sd, tp);
        pmin = fmin(pmin, prob[k]);
    }
    double x[6];
    if (pmin < threshold) {
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
        solve6(ne, x);
    }
    double D[16];
    delta_from_x(x, D);
    finish_iteration(st, tr, D, (double)*count_all, (double)*count_in, update_pose, kp);
}

}  // namespace

size_t ransac_bytes(int cap) {
    // the carve sequence of launch_solve, each piece rounded up to 256 B (+ slack per piece)
    const size_t c = (size_t)std::max(cap, 1);
    const size_t nb = (c + kBlock - 1) / kBlock + 1;
    return 2 * (10 * c + 8) * 8 + nb * (4 + 8) + (size_t)kHypMax * (4 + 4 + 16 * 8) + nb * kDrpmSlab * 8 +
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
        k_drpm_final<<<1, 256, 0, s>>>(b1, L.st, Dv, L.tr, kp, L.ransac.drpm_threshold, cnt, cnt, L.update_pose);
        return;
    }
    if (kp.solve_method != IMLS_SOLVE_RANSAC) {
        launch_solve_chain(s, L.N, L.blocks1, kp, L.cs, L.cd, L.cn, L.rows_d, L.weights, st, L.tr, L.update_pose,
                           L.rows_are_double, L.count);
        return;
    }
    // carve the RANSAC scratch
    const int cap = std::max(L.N, 1);
    const size_t c = (size_t)cap;
    const int nb = (cap + kBlock - 1) / kBlock;
    char* p = (char*)L.scratch;
    auto carve = [&](size_t bytes) { char* r = p; p += (bytes + 255) / 256 * 256; return r; };
    double* all = (double*)carve((10 * c + 8) * 8);
    double* inl = (double*)carve((10 * c + 8) * 8);
    int* blkcnt = (int*)carve((size_t)(nb + 1) * 4);
    double* blkw = (double*)carve((size_t)(nb + 1) * 8);
    int* cnt_all = (int*)carve(64);
    int* cnt_in = (int*)carve(64);
    double* wsum = (double*)carve(64);
    RansacDev R;
    R.rng = L.rng;
    R.first = (int*)carve((size_t)kHypMax * 4);
    R.counts = (int*)carve((size_t)kHypMax * 4);
    R.T = (double*)carve((size_t)kHypMax * 16 * 8);
    R.best = (int*)carve(64);
    R.evaluated = (int*)carve(64);
    R.rdone = (int*)carve(64);
    R.bestT = (double*)carve(16 * 8);
    R.active = (int*)carve(64);
    DrpmDev Dv;
    Dv.H = (double*)carve(36 * 8);
    Dv.g = (double*)carve(6 * 8);
    Dv.U = (double*)carve(36 * 8);
    Dv.ev = (double*)carve(6 * 8);
    Dv.slabs = (double*)carve((size_t)(nb + 1) * kDrpmSlab * 8);
    const int* done = L.st.done;

    // 1. compact the valid correspondences (fp64 rows from the host API are already compact)
    Source src{};
    CompactOut out{all, cnt_all, nullptr, cap};
    if (!L.rows_are_double) {
        src.cs = L.cs; src.cd = L.cd; src.cn = L.cn;
        k_compact_count<<<nb, kBlock, 0, s>>>(src, L.N, blkcnt, blkw, done);
        k_compact_scan<<<1, 1024, 0, s>>>(blkcnt, blkw, nb, out, done);
        k_compact_scatter<<<nb, kBlock, 0, s>>>(src, L.N, blkcnt, out, done);
    } else {
        (void)hipMemcpyAsync(all, L.rows_d, 9 * c * 8, hipMemcpyDeviceToDevice, s);
        k_set_count<<<1, 64, 0, s>>>(cnt_all, L.N);
    }
    k_ransac_begin<<<1, 64, 0, s>>>(cnt_all, kp.correspond_number, L.update_pose, L.st, L.tr, R);

    // 2. hypotheses in growing chunks
    int started = 0;
    for (int chunk = 16; started < L.ransac.max_iterations; chunk *= 4) {
        const int cn = std::min(std::min(chunk, kHypMax), L.ransac.max_iterations - started);
        k_ransac_draws<<<1, 64, 0, s>>>(cnt_all, R, cn, done);
        k_ransac_hyp<<<cn, kHypBlock, 0, s>>>(all, cnt_all, cap, R, L.ransac.distance_threshold, done);
        k_ransac_select<<<1, 64, 0, s>>>(cnt_all, R, cn, L.ransac.max_iterations, L.ransac.min_inliers_percentage, done);
        started += cn;
    }

    // 3. inliers of the best Δ with their Huber-like weights (order kept), Σw
    Source isrc{};
    isrc.rows = all;
    isrc.count = cnt_all;
    isrc.cap = cap;
    isrc.T = R.bestT;
    isrc.dist_thr = L.ransac.distance_threshold;
    isrc.h2 = L.ransac.huber_threshold * L.ransac.distance_threshold;
    CompactOut iout{inl, cnt_in, wsum, cap};
    k_compact_count<<<nb, kBlock, 0, s>>>(isrc, cap, blkcnt, blkw, done);
    k_compact_scan<<<1, 1024, 0, s>>>(blkcnt, blkw, nb, iout, done);
    k_compact_scatter<<<nb, kBlock, 0, s>>>(isrc, cap, blkcnt, iout, done);
    k_ransac_check_inliers<<<1, 64, 0, s>>>(cnt_in, L.st, L.tr);

    // 4. final solve on the inliers
    KParams fk = kp;
    fk.correspond_number = 0;                       // the count gate ran before RANSAC
    Rows rows{nullptr, nullptr, nullptr, inl, inl + 3 * c, inl + 6 * c, inl + 9 * c, 1, cnt_in, wsum};
    switch (L.ransac.final_method) {
        case IMLS_FINAL_LS:
            fk.solve_method = IMLS_SOLVE_LS;
            fk.ls_threshold = L.ransac.ls_threshold;
            launch_solve_chain(s, cap, 0, fk, nullptr, nullptr, nullptr, inl, nullptr, st, L.tr, L.update_pose, 1, cnt_in, nullptr);
            break;
        case IMLS_FINAL_WEIGHTED_LS:
            fk.solve_method = IMLS_SOLVE_WEIGHTED_LS;
            launch_solve_chain(s, cap, 0, fk, nullptr, nullptr, nullptr, inl, inl + 9 * c, st, L.tr, L.update_pose, 1, cnt_in, wsum);
            break;
        default: {   // DRPM
            const int b1 = solve_blocks(cap);
            launch_rows_pass1(s, rows, cap, L.st.partial1, b1);
            k_drpm_eig<<<1, 256, 0, s>>>(L.st.partial1, b1, L.st, Dv);
            k_drpm_noise<<<b1, kBlock, 0, s>>>(rows, cap, L.st, Dv, L.ransac.drpm_stdev_points, L.ransac.drpm_stdev_normals);
            k_drpm_final<<<1, 256, 0, s>>>(b1, L.st, Dv, L.tr, fk, L.ransac.drpm_threshold, cnt_all, cnt_in, L.update_pose);
        }
    }
    if (L.tr) k_ransac_trace<<<1, 64, 0, s>>>(cnt_all, R, L.tr);
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
