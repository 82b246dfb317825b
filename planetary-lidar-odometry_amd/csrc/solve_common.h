// solve_common.h — device helpers shared by the LS chain (solve.hip) and the RANSAC / DRPM
// solvers (ransac.hip): the correspondence-row accessor, block reductions, the 6×6 column-pivoted
// solve, Δ from x (Rodrigues + polar factor) and the pose update / convergence test.
#pragma once
#include <cfloat>

#include "internal.h"

namespace imlsgpu {

// One correspondence row of the point-to-plane system (solver.cpp:89-107).
struct Rows {
    const float4 *cs, *cd, *cn;           // float rows from the projection (valid flag in cs.w)
    const double *ds, *dd, *dn, *w;       // or double rows (host API / RANSAC inliers), all valid
    int is_double;
    const int* count;                     // double rows: device-side row count (rows ≥ count absent)
    const double* wsum;                   // weights are w[i] / *wsum when set (RANSAC normalisation)
    __device__ __forceinline__ bool get(int i, double a[6], double& b, double& wt) const {
        double s[3], d[3], n[3];
        if (is_double) {
#pragma unroll
            for (int k = 0; k < 3; ++k) { s[k] = ds[3 * i + k]; d[k] = dd[3 * i + k]; n[k] = dn[3 * i + k]; }
            if (count && i >= *count) return false;
            wt = w ? (wsum ? w[i] / *wsum : w[i]) : 1.0;
        } else {
            const float4 s4 = cs[i];
            if (s4.w == 0.f) return false;
            const float4 d4 = cd[i], n4 = cn[i];
            s[0] = s4.x; s[1] = s4.y; s[2] = s4.z;
            d[0] = d4.x; d[1] = d4.y; d[2] = d4.z;
            n[0] = n4.x; n[1] = n4.y; n[2] = n4.z;
            wt = 1.0;
        }
        // solver.cpp:95-103
        a[0] = n[2] * s[1] - n[1] * s[2];
        a[1] = n[0] * s[2] - n[2] * s[0];
        a[2] = n[1] * s[0] - n[0] * s[1];
        a[3] = n[0]; a[4] = n[1]; a[5] = n[2];
        b = n[0] * (d[0] - s[0]);
        b = b + n[1] * (d[1] - s[1]);
        b = b + n[2] * (d[2] - s[2]);
        return true;
    }
};

// Rows of a batched frame: the projection's float rows (src 0) or the frame's RANSAC inlier rows
// (src 1: fp64, device-side count; weights w / Σw when weighted) — what launch_solve builds for the
// same solve of a one-frame launch.
__device__ __forceinline__ Rows frame_rows(const PairDev& A, int src, int weighted) {
    if (!src) return Rows{A.cs, A.cd, A.cn, nullptr, nullptr, nullptr, nullptr, 0, nullptr, nullptr};
    const size_t c = (size_t)A.rf.cap;
    const double* r = A.rf.inl;
    return Rows{nullptr, nullptr, nullptr, r, r + 3 * c, r + 6 * c, weighted ? r + 9 * c : nullptr, 1, A.rf.cnt_in,
                weighted ? A.rf.wsum : nullptr};
}
__host__ __device__ __forceinline__ int solve_blocks_of(int N) { return (N + kBlock - 1) / kBlock; }

// pass 1 of the LS chain (weighted normal equations) on any rows; solve.hip
void launch_rows_pass1(hipStream_t s, const Rows& rows, int N, double* partial, int blocks);

namespace {

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// Block-reduce the 28 normal-equation terms of (a, b, weight, count); result valid in thread 0's
// `out` (all threads must call).  red: [nwaves][28] LDS.
template <int NT>
__device__ void block_normeq(const double a[6], double b, double cnt, double* red, double out[kNormEq]) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    double v[32];
    int k = 0;
#pragma unroll
    for (int r = 0; r < 6; ++r)
#pragma unroll
        for (int c = r; c < 6; ++c) v[k++] = a[r] * a[c];
#pragma unroll
    for (int r = 0; r < 6; ++r) v[21 + r] = a[r] * b;
    v[27] = cnt;
#pragma unroll
    for (int q = kNormEq; q < 32; ++q) v[q] = 0.0;
    const double s = wave_sum28(v);
    if (!(lane & 1) && (lane >> 1) < kNormEq) red[wv * kNormEq + (lane >> 1)] = s;
    __syncthreads();
    if (threadIdx.x < kNormEq) {
        double s = 0.0;
        for (int w = 0; w < NT / 64; ++w) s += red[w * kNormEq + threadIdx.x];
        out[threadIdx.x] = s;
    }
    __syncthreads();
}

// Block-sum 28 per-thread values (all threads call); result in out[0..27] (LDS) after the call.
// Within a wave by wave_sum28 (internal.h): k_solve_small's two block sums 4.8 / 3.9 → 4.0 / 2.7 µs
// on a 1949-row frame (28 wave_total reductions before).
template <int NT>
__device__ void block_sum28(const double (&v)[kNormEq], double* red, double* out) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    double a[32];
#pragma unroll
    for (int k = 0; k < 32; ++k) a[k] = k < kNormEq ? v[k] : 0.0;
    const double s = wave_sum28(a);
    if (!(lane & 1) && (lane >> 1) < kNormEq) red[wv * kNormEq + (lane >> 1)] = s;
    __syncthreads();
    if (threadIdx.x < kNormEq) {
        double s = 0.0;
#pragma unroll
        for (int w = 0; w < NT / 64; ++w) s += red[w * kNormEq + threadIdx.x];
        out[threadIdx.x] = s;
    }
    __syncthreads();
}

// Column-pivoted Cholesky solve of the 6×6 normal equations (see file header).  Unknowns past the
// numerical rank are set to zero (Eigen's basic solution).  Returns the rank.
__device__ inline int solve6(const double* ne, double x[6]) {
    // every index below is a compile-time constant (full unroll; the pivot swap is a predicated
    // swap over the candidate rows), so the system stays in registers — no scratch traffic
    double A[6][6], g[6];
    int perm[6];
    {
        int k = 0;
#pragma unroll
        for (int r = 0; r < 6; ++r)
#pragma unroll
            for (int c = r; c < 6; ++c) { A[r][c] = ne[k]; A[c][r] = ne[k]; ++k; }
    }
#pragma unroll
    for (int r = 0; r < 6; ++r) { g[r] = ne[21 + r]; perm[r] = r; }
    const double eps = DBL_EPSILON;
    double maxpiv = 0.0;
    int rank = 6;
    bool stop = false;
#pragma unroll
    for (int j = 0; j < 6; ++j) {
        if (!stop) {
            int p = j;
            double best = A[j][j];
#pragma unroll
            for (int q = j + 1; q < 6; ++q)
                if (A[q][q] > best) { best = A[q][q]; p = q; }
#pragma unroll
            for (int q = j + 1; q < 6; ++q) {
                if (q == p) {
#pragma unroll
                    for (int c = 0; c < 6; ++c) { const double t = A[j][c]; A[j][c] = A[q][c]; A[q][c] = t; }
#pragma unroll
                    for (int r = 0; r < 6; ++r) { const double t = A[r][j]; A[r][j] = A[r][q]; A[r][q] = t; }
                    const double t = g[j]; g[j] = g[q]; g[q] = t;
                    const int ti = perm[j]; perm[j] = perm[q]; perm[q] = ti;
                }
            }
            const double d = A[j][j];
            const double rkk = d > 0 ? sqrt(d) : 0.0;
            if (rkk > maxpiv) maxpiv = rkk;
            if (!(rkk > eps * 6.0 * maxpiv) || !(d > 0)) {
                rank = j;
                stop = true;
            } else {
                A[j][j] = rkk;
                const double inv = 1.0 / rkk;   // one division per pivot (round 4: the column scaled by it)
#pragma unroll
                for (int r = j + 1; r < 6; ++r) A[r][j] = A[r][j] * inv;
#pragma unroll
                for (int r = j + 1; r < 6; ++r)
#pragma unroll
                    for (int c = j + 1; c <= r; ++c) {
                        A[r][c] = A[r][c] - A[r][j] * A[c][j];
                        A[c][r] = A[r][c];
                    }
            }
        }
    }
    double y[6] = {0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int r = 0; r < 6; ++r) {
        if (r < rank) {
            double s = g[r];
#pragma unroll
            for (int c = 0; c < r; ++c) s -= A[r][c] * y[c];
            y[r] = s / A[r][r];
        }
    }
#pragma unroll
    for (int r = 5; r >= 0; --r) {
        if (r < rank) {
            double s = y[r];
#pragma unroll
            for (int c = r + 1; c < 6; ++c)
                if (c < rank) s -= A[c][r] * y[c];
            y[r] = s / A[r][r];
        }
    }
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        double v = 0.0;
#pragma unroll
        for (int r = 0; r < 6; ++r)
            if (r < rank && perm[r] == k) v = y[r];
        x[k] = v;
    }
    return rank;
}

// solve6 with the pivot made wave-uniform (readfirstlane): the row / column swap of pivot p is a
// scalar branch to one static swap (a few dozen moves), not solve6's ~700 predicated selects over
// every candidate row, and not the one-wave form's chain of LDS permutes per pivot (element (r, c) in
// lane 6r + c: 3.6 µs per solve vs 2.8 here, tools/frame_probe.py phases).  Every lane (or the one
// calling lane) holds the whole system and performs exactly solve6's operations: x is solve6's bit for bit.
__device__ __forceinline__ int solve6_u(const double* ne, double x[6]) {
    double A[6][6], g[6];
    int perm[6];
    {
        int k = 0;
#pragma unroll
        for (int r = 0; r < 6; ++r)
#pragma unroll
            for (int c = r; c < 6; ++c) { A[r][c] = ne[k]; A[c][r] = ne[k]; ++k; }
    }
#pragma unroll
    for (int r = 0; r < 6; ++r) { g[r] = ne[21 + r]; perm[r] = r; }
    const double eps = DBL_EPSILON;
    double maxpiv = 0.0;
    int rank = 6;
#pragma unroll
    for (int j = 0; j < 6; ++j) {
        int p = j;
        double best = A[j][j];
#pragma unroll
        for (int q = j + 1; q < 6; ++q)
            if (A[q][q] > best) { best = A[q][q]; p = q; }
        p = __builtin_amdgcn_readfirstlane(p);
#pragma unroll
        for (int q = j + 1; q < 6; ++q) {
            if (q == p) {                 // uniform: one taken branch per pivot
#pragma unroll
                for (int c = 0; c < 6; ++c) { const double t = A[j][c]; A[j][c] = A[q][c]; A[q][c] = t; }
#pragma unroll
                for (int r = 0; r < 6; ++r) { const double t = A[r][j]; A[r][j] = A[r][q]; A[r][q] = t; }
                const double t = g[j]; g[j] = g[q]; g[q] = t;
                const int ti = perm[j]; perm[j] = perm[q]; perm[q] = ti;
            }
        }
        const double d = A[j][j];
        const double rkk = d > 0 ? sqrt(d) : 0.0;
        if (rkk > maxpiv) maxpiv = rkk;
        if (__builtin_amdgcn_readfirstlane((!(rkk > eps * 6.0 * maxpiv) || !(d > 0)) ? 1 : 0)) {
            rank = j;
            break;
        }
        A[j][j] = rkk;
        const double inv = 1.0 / rkk;
#pragma unroll
        for (int r = j + 1; r < 6; ++r) A[r][j] = A[r][j] * inv;
#pragma unroll
        for (int r = j + 1; r < 6; ++r)
#pragma unroll
            for (int c = j + 1; c <= r; ++c) {
                A[r][c] = A[r][c] - A[r][j] * A[c][j];
                A[c][r] = A[r][c];
            }
    }
    double y[6] = {0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int r = 0; r < 6; ++r) {
        if (r < rank) {
            double s = g[r];
#pragma unroll
            for (int c = 0; c < r; ++c) s -= A[r][c] * y[c];
            y[r] = s / A[r][r];
        }
    }
#pragma unroll
    for (int r = 5; r >= 0; --r) {
        if (r < rank) {
            double s = y[r];
#pragma unroll
            for (int c = r + 1; c < 6; ++c)
                if (c < rank) s -= A[c][r] * y[c];
            y[r] = s / A[r][r];
        }
    }
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        double v = 0.0;
#pragma unroll
        for (int r = 0; r < 6; ++r)
            if (r < rank && perm[r] == k) v = y[r];
        x[k] = v;
    }
    return rank;
}

// Δ from x (solver.cpp:140-163): R = AngleAxis(‖ω‖, ω̂) (Eigen AngleAxis::toRotationMatrix), then
// the JacobiSVD U·Vᵀ re-orthonormalisation as the polar factor (Newton iteration).
__device__ inline void delta_from_x(const double x[6], double D[16]) {
    const double wx = x[0], wy = x[1], wz = x[2];
    double sq = wx * wx;
    sq = sq + wy * wy;
    sq = sq + wz * wz;
    const double ang = sqrt(sq);
    double ax = 0, ay = 0, az = 0;
    if (sq > 0) { ax = wx / ang; ay = wy / ang; az = wz / ang; }   // (ang = ‖ω‖: the same root)
    double s, c;
    sincos(ang, &s, &c);              // one shared argument reduction (round 5: sin + cos)
    const double sx = s * ax, sy = s * ay, sz = s * az;
    const double c1x = (1 - c) * ax, c1y = (1 - c) * ay, c1z = (1 - c) * az;
    double R[9];
    double tmp = c1x * ay; R[1] = tmp - sz; R[3] = tmp + sz;
    tmp = c1x * az; R[2] = tmp + sy; R[6] = tmp - sy;
    tmp = c1y * az; R[5] = tmp - sx; R[7] = tmp + sx;
    R[0] = c1x * ax + c; R[4] = c1y * ay + c; R[8] = c1z * az + c;
    // A step that reproduces the iterate before last has entered a 2-cycle (an element alternating by
    // an ulp: |Δ| ≥ 1e-16 forever — 35 % of small rotations run all 20 steps): the 20th iterate is
    // then known from the parity of the steps left, bit for bit what the remaining steps would give
    // (the cycle repeats its maxd and det, so neither exit fires in it).
    double P[9];
    bool have_prev = false;
    for (int it = 0; it < 20; ++it) {
        const double* a = R;
        const double det = a[0] * (a[4] * a[8] - a[5] * a[7]) - a[1] * (a[3] * a[8] - a[5] * a[6]) + a[2] * (a[3] * a[7] - a[4] * a[6]);
        if (det == 0) break;
        const double cof[9] = {a[4] * a[8] - a[5] * a[7], a[5] * a[6] - a[3] * a[8], a[3] * a[7] - a[4] * a[6],
                               a[2] * a[7] - a[1] * a[8], a[0] * a[8] - a[2] * a[6], a[1] * a[6] - a[0] * a[7],
                               a[1] * a[5] - a[2] * a[4], a[2] * a[3] - a[0] * a[5], a[0] * a[4] - a[1] * a[3]};
        // one division per step (its reciprocal scales the cofactors; round 5: was nine)
        const double rdet = 1.0 / det;
        double maxd = 0, n[9];
        bool cyc = have_prev;
        for (int k = 0; k < 9; ++k) {
            n[k] = 0.5 * (a[k] + cof[k] * rdet);
            maxd = fmax(maxd, fabs(n[k] - a[k]));
            cyc = cyc && __double_as_longlong(n[k]) == __double_as_longlong(P[k]);
        }
        if (maxd < 1e-16) {
            for (int k = 0; k < 9; ++k) R[k] = n[k];
            break;
        }
        if (cyc) {                    // n = the iterate before last: 19 − it steps remain
            if ((19 - it) % 2 == 0)
                for (int k = 0; k < 9; ++k) R[k] = n[k];
            break;
        }
        for (int k = 0; k < 9; ++k) { P[k] = R[k]; R[k] = n[k]; }
        have_prev = true;
    }
    for (int k = 0; k < 16; ++k) D[k] = 0.0;
    for (int r = 0; r < 3; ++r) for (int cc = 0; cc < 3; ++cc) D[r * 4 + cc] = R[r * 3 + cc];
    D[3] = x[3]; D[7] = x[4]; D[11] = x[5]; D[15] = 1.0;
}

// rPose = Δ·rPose, trace, convergence (laser_odometry.cpp:619-646); single thread.
__device__ inline void finish_iteration(SolveState st, imls_iter_trace* tr, const double D[16], double nvalid, double nkept,
                                 int update_pose, const KParams& kp) {
    for (int k = 0; k < 16; ++k) st.delta[k] = D[k];
    if (tr) {
        for (int k = 0; k < 16; ++k) tr->delta[k] = D[k];
        tr->n_valid = (unsigned long long)nvalid;
        tr->n_kept = (unsigned long long)nkept;
    }
    if (!update_pose) return;
    double Pn[16];
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) {
            double s = D[i * 4 + 0] * st.pose[0 * 4 + j];
            s = s + D[i * 4 + 1] * st.pose[1 * 4 + j];
            s = s + D[i * 4 + 2] * st.pose[2 * 4 + j];
            s = s + D[i * 4 + 3] * st.pose[3 * 4 + j];
            Pn[i * 4 + j] = s;
        }
    for (int k = 0; k < 16; ++k) st.pose[k] = Pn[k];
    if (tr) for (int k = 0; k < 16; ++k) tr->pose[k] = Pn[k];
    *st.iters += 1;
    const double dd = sqrt(D[3] * D[3] + D[7] * D[7] + D[11] * D[11]);
    double ct = ((D[0] + D[5] + D[10]) - 1.0) / 2.0;
    ct = fmin(1.0, fmax(ct, -1.0));
    const double da = acos(ct);
    if (dd < kp.delta_dist && da < kp.delta_angle) {
        *st.status = IMLS_FRAME_CONVERGED;
        *st.done = 1;
    }
}


// The first LS solve (or the only one, weighted LS) over `blocks` pass-1 slabs, by one block of
// NT threads: reduce, too-few gate (laser_odometry.cpp:570-576), solve6, and for LS the trim
// ranks (solver.cpp:118-134, Q11) for the selection that follows.  red: LDS [(NT/64)·28],
// acc: LDS [28].  Run by k_solve_first.
template <int NT>
__device__ void solve_first_block(const double* __restrict__ partial, int blocks, SolveState st, imls_iter_trace* tr,
                                  const KParams& kp, int weighted, int update_pose, double* red, double* acc) {
    const int t = threadIdx.x;
    double loc[kNormEq];
#pragma unroll
    for (int k = 0; k < kNormEq; ++k) loc[k] = 0.0;
    for (int b = t; b < blocks; b += NT)
#pragma unroll
        for (int k = 0; k < kNormEq; ++k) loc[k] += partial[(size_t)b * kNormEq + k];
    if (t < 2) st.cand_count[t] = 0u;
    block_sum28<NT>(loc, red, acc);
    if (t >= 64) return;
    const double nvalid = acc[27];
    if (update_pose && nvalid < (double)kp.correspond_number) {
        if (t == 0) {
            *st.status = IMLS_FRAME_TOO_FEW;
            *st.done = 1;
            if (tr) tr->n_valid = (unsigned long long)nvalid;
        }
        return;
    }
    double x[6];
    solve6_u(acc, x);              // wave 0
    if (t != 0) return;
    if (weighted) {
        double D[16];
        delta_from_x(x, D);
        finish_iteration(st, tr, D, nvalid, nvalid, update_pose, kp);
        return;
    }
    for (int k = 0; k < 6; ++k) st.x0[k] = x[k];
    const long long N = (long long)nvalid;
    long long lo = (long long)(kp.ls_threshold * (double)N);
    long long hi = (long long)((1 - kp.ls_threshold) * (double)N);
    if (hi > N - 1) hi = N - 1;       // Q11
    if (N == 0 || lo > hi) {          // no valid row: solve fails (the oracle's solve_ls returns false)
        *st.status = IMLS_FRAME_SOLVE_FAILED;
        *st.done = 1;
        return;
    }
    st.sel[4] = (int)lo;
    st.sel[5] = (int)hi;
    st.sel[6] = (int)N;
}

// Cyclic Jacobi on a symmetric N×N (ascending eigenvalues, eigenvectors as columns:
// U[c·N + r]); identical sweep order to the oracle's sym_eig (Eigen SelfAdjointEigenSolver order).
template <int N>
__device__ void sym_eig(const double* Hin, double* ev, double* U) {
    double a[N][N], v[N][N];
#pragma unroll
    for (int r = 0; r < N; ++r)
#pragma unroll
        for (int c = 0; c < N; ++c) { a[r][c] = Hin[r * N + c]; v[r][c] = r == c ? 1.0 : 0.0; }
    for (int sweep = 0; sweep < 100; ++sweep) {
        double off = 0;
#pragma unroll
        for (int p = 0; p < N; ++p)
#pragma unroll
            for (int q = p + 1; q < N; ++q) off += a[p][q] * a[p][q];
        if (off < 1e-300) break;
#pragma unroll
        for (int p = 0; p < N; ++p)
#pragma unroll
            for (int q = p + 1; q < N; ++q) {
                const double apq = a[p][q];
                if (apq != 0) {
                    const double app = a[p][p], aqq = a[q][q];
                    const double theta = (aqq - app) / (2 * apq);
                    const double t = (theta >= 0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1));
                    const double c = 1 / sqrt(t * t + 1), s = t * c;
#pragma unroll
                    for (int k = 0; k < N; ++k) {
                        const double akp = a[k][p], akq = a[k][q];
                        a[k][p] = c * akp - s * akq;
                        a[k][q] = s * akp + c * akq;
                    }
#pragma unroll
                    for (int k = 0; k < N; ++k) {
                        const double apk = a[p][k], aqk = a[q][k];
                        a[p][k] = c * apk - s * aqk;
                        a[q][k] = s * apk + c * aqk;
                    }
#pragma unroll
                    for (int k = 0; k < N; ++k) {
                        const double vkp = v[k][p], vkq = v[k][q];
                        v[k][p] = c * vkp - s * vkq;
                        v[k][q] = s * vkp + c * vkq;
                    }
                }
            }
    }
    // ascending order, ties keep index order (std::sort on distinct diagonal values)
    int ord[N];
    double dg[N];
#pragma unroll
    for (int k = 0; k < N; ++k) { ord[k] = k; dg[k] = a[k][k]; }
#pragma unroll
    for (int i = 1; i < N; ++i)
#pragma unroll
        for (int j = i; j > 0; --j) {
            const bool sw = dg[j] < dg[j - 1];
            const double td = dg[j];
            const int to = ord[j];
            dg[j] = sw ? dg[j - 1] : dg[j];
            ord[j] = sw ? ord[j - 1] : ord[j];
            dg[j - 1] = sw ? td : dg[j - 1];
            ord[j - 1] = sw ? to : ord[j - 1];
        }
#pragma unroll
    for (int c = 0; c < N; ++c) {
        ev[c] = dg[c];
#pragma unroll
        for (int r = 0; r < N; ++r) {
            double val = 0;
#pragma unroll
            for (int k = 0; k < N; ++k) val = ord[c] == k ? v[r][k] : val;
            U[c * N + r] = val;
        }
    }
}

__device__ __forceinline__ double readlane_f64(double x, int l) {
    const long long b = __double_as_longlong(x);
    const int lo = __builtin_amdgcn_readlane((int)(unsigned)(b & 0xffffffffll), l);
    const int hi = __builtin_amdgcn_readlane((int)(unsigned)((unsigned long long)b >> 32), l);
    return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}

constexpr double kDrpmEigRelTol = 1e-30;   // the oracle's DRPM Jacobi stop (imls_oracle.cpp sym_eig)

// sym_eig<6> by one wave, lane k < 6 holding row k of the matrix and of the eigenvector accumulator:
// the same sweeps, rotations and per-element expressions in the same order (a rotation's column
// update is lane-local, its row update reads rows p and q after it, as the sequential loops do), so
// the result is the one-thread routine's (with the relative stop below); ~6× shorter dependency chains.  a_row: row k of the
// symmetric input (lanes < 6).  Every lane of the wave calls; ev / U (as sym_eig) written by lanes < 6.
__device__ inline int sym_eig6_wave(const double (&a_row)[6], double* __restrict__ ev, double* __restrict__ U) {
    constexpr int N = 6;
    const int lane = threadIdx.x & 63;
    double a[N], v[N];
#pragma unroll
    for (int c = 0; c < N; ++c) { a[c] = a_row[c]; v[c] = lane == c ? 1.0 : 0.0; }
    // stop at off-diagonal mass < max(1e-300, 1e-30·‖H‖_F²) (the oracle's sym_eig with DRPM's rel_tol)
    double fro = 0;
#pragma unroll
    for (int r = 0; r < N; ++r)
#pragma unroll
        for (int c = 0; c < N; ++c) {
            const double x = readlane_f64(a[c], r);
            fro += x * x;
        }
    const double stop = fmax(1e-300, kDrpmEigRelTol * fro);
    int sweeps = 0;
    for (int sweep = 0; sweep < 100; ++sweep) {
        double off = 0;
#pragma unroll
        for (int p = 0; p < N; ++p)
#pragma unroll
            for (int q = p + 1; q < N; ++q) {
                const double apq = readlane_f64(a[q], p);
                off += apq * apq;
            }
        if (off < stop) break;
        ++sweeps;
#pragma unroll
        for (int p = 0; p < N; ++p)
#pragma unroll
            for (int q = p + 1; q < N; ++q) {
                const double apq = readlane_f64(a[q], p);
                if (apq != 0) {
                    const double app = readlane_f64(a[p], p), aqq = readlane_f64(a[q], q);
                    const double theta = (aqq - app) / (2 * apq);
                    const double t = (theta >= 0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1));
                    const double c = 1 / sqrt(t * t + 1), s = t * c;
                    {
                        const double akp = a[p], akq = a[q];
                        a[p] = c * akp - s * akq;
                        a[q] = s * akp + c * akq;
                    }
                    double rp[N], rq[N];
#pragma unroll
                    for (int k = 0; k < N; ++k) { rp[k] = readlane_f64(a[k], p); rq[k] = readlane_f64(a[k], q); }
#pragma unroll
                    for (int k = 0; k < N; ++k) {
                        const double apk = rp[k], aqk = rq[k];
                        if (lane == p) a[k] = c * apk - s * aqk;
                        if (lane == q) a[k] = s * apk + c * aqk;
                    }
                    {
                        const double vkp = v[p], vkq = v[q];
                        v[p] = c * vkp - s * vkq;
                        v[q] = s * vkp + c * vkq;
                    }
                }
            }
    }
    int ord[N];
    double dg[N];
#pragma unroll
    for (int k = 0; k < N; ++k) { ord[k] = k; dg[k] = readlane_f64(a[k], k); }
#pragma unroll
    for (int i = 1; i < N; ++i)
#pragma unroll
        for (int j = i; j > 0; --j) {
            const bool sw = dg[j] < dg[j - 1];
            const double td = dg[j];
            const int to = ord[j];
            dg[j] = sw ? dg[j - 1] : dg[j];
            ord[j] = sw ? ord[j - 1] : ord[j];
            dg[j - 1] = sw ? td : dg[j - 1];
            ord[j - 1] = sw ? to : ord[j - 1];
        }
    if (lane < N) {
#pragma unroll
        for (int c = 0; c < N; ++c) {
            if (lane == c) ev[c] = dg[c];
            double val = 0;
#pragma unroll
            for (int k = 0; k < N; ++k) val = ord[c] == k ? v[k] : val;
            U[c * N + lane] = val;
        }
    }
    return sweeps;   // sweeps run (the debug build records them)
}

}  // namespace
}  // namespace imlsgpu
