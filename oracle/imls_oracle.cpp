// imls_oracle.cpp — CPU restatement of the reference IMLS-ICP path.  TEST INFRASTRUCTURE ONLY
// (see imls_oracle.h for who may load it and for the "parity unpinned" statement).
//
// Every function cites the reference file:line it restates (paths relative to the reference
// repo root).  Arithmetic is double on float storage, in the reference's evaluation order and
// without FMA contraction (the reference is built for baseline x86-64, no -mfma; this file is
// compiled with -ffp-contract=off), so the GPU path can be compared bit-for-bit where the
// reference's own arithmetic is deterministic.
#include "imls_oracle.h"

#include <algorithm>
#include <array>
#include <cfloat>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <limits>
#include <numeric>
#include <sstream>
#include <vector>

namespace {

constexpr double kInf = std::numeric_limits<double>::infinity();

inline bool finite3(double a, double b, double c) { return std::isfinite(a) && std::isfinite(b) && std::isfinite(c); }

// ------------------------------------------------------------------------------------------
// Cloud storage (float storage, double arithmetic — SURVEY Q9)
// ------------------------------------------------------------------------------------------
struct Cloud {
    std::vector<float> x, y, z, nx, ny, nz;
    size_t size() const { return x.size(); }
};

// RemoveNANandINFData (imls_icp.cpp:58-72): pcl::isFinite checks xyz only (Q8); order kept.
Cloud load_filtered(const float* soa6, size_t n, std::vector<uint32_t>* kept = nullptr) {
    Cloud c;
    for (size_t i = 0; i < n; ++i) {
        float px = soa6[i], py = soa6[n + i], pz = soa6[2 * n + i];
        if (!(std::isfinite(px) && std::isfinite(py) && std::isfinite(pz))) continue;
        c.x.push_back(px); c.y.push_back(py); c.z.push_back(pz);
        c.nx.push_back(soa6[3 * n + i]); c.ny.push_back(soa6[4 * n + i]); c.nz.push_back(soa6[5 * n + i]);
        if (kept) kept->push_back((uint32_t)i);
    }
    return c;
}

// ------------------------------------------------------------------------------------------
// Exact kNN with libnabo NNSearchD semantics (call sites imls_icp.cpp:372-375, 605-607).
//   accept  : d² ≤ maxRadius² (inclusive), strictly better than the current K-th,
//             and (ALLOW_SELF_MATCH or d² > DBL_EPSILON);
//   d²      : ((q−p)x² + (q−p)y²) + (q−p)z², double, no FMA;
//   output  : sorted ascending (SORT_RESULTS); unfound slots d² = +inf.
// libnabo breaks exact distance ties by tree-visit order (unspecified); this restatement uses
// the total order (d², index) and the GPU path uses the same.
// ------------------------------------------------------------------------------------------
struct KdTree {
    struct Node { int dim; double split; int left, right, begin, end; };
    std::vector<double> px, py, pz;   // bucket-permuted coordinates
    std::vector<int32_t> pid;         // original (filtered) index
    std::vector<Node> nodes;
    static constexpr int kBucket = 8;

    void build(const Cloud& c) {
        size_t n = c.size();
        std::vector<int32_t> order(n);
        std::iota(order.begin(), order.end(), 0);
        nodes.clear();
        nodes.reserve(2 * (n / kBucket + 1) + 1);
        if (n) build_rec(c, order, 0, (int)n);
        px.resize(n); py.resize(n); pz.resize(n); pid.resize(n);
        for (size_t i = 0; i < n; ++i) {
            px[i] = c.x[order[i]]; py[i] = c.y[order[i]]; pz[i] = c.z[order[i]]; pid[i] = order[i];
        }
    }
    int build_rec(const Cloud& c, std::vector<int32_t>& ord, int b, int e) {
        int id = (int)nodes.size();
        nodes.push_back({-1, 0.0, -1, -1, b, e});
        if (e - b <= kBucket) return id;
        double lo[3] = {kInf, kInf, kInf}, hi[3] = {-kInf, -kInf, -kInf};
        for (int i = b; i < e; ++i) {
            double v[3] = {c.x[ord[i]], c.y[ord[i]], c.z[ord[i]]};
            for (int d = 0; d < 3; ++d) { lo[d] = std::min(lo[d], v[d]); hi[d] = std::max(hi[d], v[d]); }
        }
        int dim = 0;
        for (int d = 1; d < 3; ++d) if (hi[d] - lo[d] > hi[dim] - lo[dim]) dim = d;
        if (!(hi[dim] > lo[dim])) return id;  // all points identical: keep one leaf
        const float* coord = dim == 0 ? c.x.data() : dim == 1 ? c.y.data() : c.z.data();
        int mid = (b + e) / 2;
        std::nth_element(ord.begin() + b, ord.begin() + mid, ord.begin() + e,
                         [&](int32_t a, int32_t q) { return coord[a] < coord[q]; });
        double split = coord[ord[mid]];
        nodes[id].dim = dim;
        nodes[id].split = split;
        int l = build_rec(c, ord, b, mid);
        int r = build_rec(c, ord, mid, e);
        nodes[id].left = l;
        nodes[id].right = r;
        return id;
    }

    struct Heap {
        int K;
        double d[64];
        int32_t i[64];
        int n;
        void reset(int k) { K = k; n = 0; }
        double worst() const { return n < K ? kInf : d[K - 1]; }
        static bool less(double da, int32_t ia, double db, int32_t ib) { return da < db || (da == db && ia < ib); }
        void push(double dd, int32_t ii) {
            if (n == K && !less(dd, ii, d[K - 1], i[K - 1])) return;
            int pos = n < K ? n++ : K - 1;
            while (pos > 0 && less(dd, ii, d[pos - 1], i[pos - 1])) { d[pos] = d[pos - 1]; i[pos] = i[pos - 1]; --pos; }
            d[pos] = dd; i[pos] = ii;
        }
    };

    void knn(const double q[3], int K, double max_r2, bool allow_self, Heap& h) const {
        h.reset(K);
        if (nodes.empty()) return;
        double off[3] = {0, 0, 0};
        rec(0, q, 0.0, off, max_r2, allow_self, h);
    }
    void rec(int id, const double q[3], double rd, double off[3], double max_r2, bool self, Heap& h) const {
        const Node& nd = nodes[id];
        if (nd.dim < 0) {
            for (int k = nd.begin; k < nd.end; ++k) {
                double dx = q[0] - px[k], dy = q[1] - py[k], dz = q[2] - pz[k];
                double d2 = dx * dx;
                d2 = d2 + dy * dy;
                d2 = d2 + dz * dz;
                if (d2 <= max_r2 && (self || d2 > DBL_EPSILON)) h.push(d2, pid[k]);
            }
            return;
        }
        double diff = q[nd.dim] - nd.split;
        int nearc = diff < 0 ? nd.left : nd.right, farc = diff < 0 ? nd.right : nd.left;
        rec(nearc, q, rd, off, max_r2, self, h);
        double old = off[nd.dim];
        double nrd = rd - old * old + diff * diff;
        double bound = std::min(max_r2, h.worst());
        if (nrd <= bound * (1.0 + 1e-9) + 1e-300) {   // relaxed: pruning must never drop a tie
            off[nd.dim] = diff;
            rec(farc, q, nrd, off, max_r2, self, h);
            off[nd.dim] = old;
        }
    }
};

// ------------------------------------------------------------------------------------------
// Small linear algebra restating the Eigen calls the reference makes.
// ------------------------------------------------------------------------------------------
struct Mat4 { double m[16]; };
inline Mat4 mat4_identity() { Mat4 r{}; r.m[0] = r.m[5] = r.m[10] = r.m[15] = 1.0; return r; }
// Eigen 4×4 lazy product: res(i,j) = ((a(i,0)b(0,j) + a(i,1)b(1,j)) + a(i,2)b(2,j)) + a(i,3)b(3,j)
inline Mat4 mat4_mul(const Mat4& a, const Mat4& b) {
    Mat4 r;
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) {
            double s = a.m[i * 4 + 0] * b.m[0 * 4 + j];
            s = s + a.m[i * 4 + 1] * b.m[1 * 4 + j];
            s = s + a.m[i * 4 + 2] * b.m[2 * 4 + j];
            s = s + a.m[i * 4 + 3] * b.m[3 * 4 + j];
            r.m[i * 4 + j] = s;
        }
    return r;
}

// Eigen::ColPivHouseholderQR<MatrixXd>(A).solve(b) — Householder QR with column pivoting
// (Eigen/src/QR/ColPivHouseholderQR.h: computeInPlace + _solve_impl; makeHouseholderInPlace,
// applyHouseholderOnTheLeft).  Rank-deficient systems get Eigen's "basic solution": the
// non-pivot unknowns are zero (SURVEY Q15 for the 3×6 RANSAC solves).
int colpiv_qr_solve(std::vector<double>& A /* rows×cols row-major, destroyed */, int rows, int cols,
                    std::vector<double> b, double* x) {
    const int size = std::min(rows, cols);
    auto at = [&](int r, int c) -> double& { return A[(size_t)r * cols + c]; };
    std::vector<double> hcoeffs(size), colNormsU(cols), colNormsD(cols);
    std::vector<int> transp(size);
    for (int k = 0; k < cols; ++k) {
        double s = 0;
        for (int r = 0; r < rows; ++r) s += at(r, k) * at(r, k);
        colNormsD[k] = colNormsU[k] = std::sqrt(s);
    }
    double maxnorm = 0;
    for (int k = 0; k < cols; ++k) maxnorm = std::max(maxnorm, colNormsU[k]);
    const double eps = std::numeric_limits<double>::epsilon();
    const double threshold_helper = (maxnorm * eps) * (maxnorm * eps) / (double)rows;
    const double norm_downdate_threshold = std::sqrt(eps);
    int nonzero_pivots = size;
    double maxpivot = 0;
    for (int k = 0; k < size; ++k) {
        int big = k;
        for (int j = k + 1; j < cols; ++j) if (colNormsU[j] > colNormsU[big]) big = j;
        double big_sq = colNormsU[big] * colNormsU[big];
        if (nonzero_pivots == size && big_sq < threshold_helper * (double)(rows - k)) nonzero_pivots = k;
        transp[k] = big;
        if (k != big) {
            for (int r = 0; r < rows; ++r) std::swap(at(r, k), at(r, big));
            std::swap(colNormsU[k], colNormsU[big]);
            std::swap(colNormsD[k], colNormsD[big]);
        }
        // makeHouseholderInPlace on column k, rows k..rows-1
        double c0 = at(k, k), tail = 0;
        for (int r = k + 1; r < rows; ++r) tail += at(r, k) * at(r, k);
        double tau, beta;
        const double tol = std::numeric_limits<double>::min();
        if (tail <= tol) {
            tau = 0; beta = c0;
            for (int r = k + 1; r < rows; ++r) at(r, k) = 0;
        } else {
            beta = std::sqrt(c0 * c0 + tail);
            if (c0 >= 0) beta = -beta;
            for (int r = k + 1; r < rows; ++r) at(r, k) = at(r, k) / (c0 - beta);
            tau = (beta - c0) / beta;
        }
        hcoeffs[k] = tau;
        at(k, k) = beta;
        if (std::abs(beta) > maxpivot) maxpivot = std::abs(beta);
        // applyHouseholderOnTheLeft to the bottom-right corner (rows k.., cols k+1..)
        if (tau != 0) {
            for (int j = k + 1; j < cols; ++j) {
                double tmp = at(k, j);
                for (int r = k + 1; r < rows; ++r) tmp += at(r, k) * at(r, j);
                at(k, j) -= tau * tmp;
                for (int r = k + 1; r < rows; ++r) at(r, j) -= tau * at(r, k) * tmp;
            }
        }
        // column-norm downdate
        for (int j = k + 1; j < cols; ++j) {
            if (colNormsU[j] != 0) {
                double temp = std::abs(at(k, j)) / colNormsU[j];
                temp = (1 + temp) * (1 - temp);
                temp = temp < 0 ? 0 : temp;
                double r2 = colNormsU[j] / colNormsD[j];
                double temp2 = temp * r2 * r2;
                if (temp2 <= norm_downdate_threshold) {
                    double s = 0;
                    for (int r = k + 1; r < rows; ++r) s += at(r, j) * at(r, j);
                    colNormsD[j] = colNormsU[j] = std::sqrt(s);
                } else {
                    colNormsU[j] *= std::sqrt(temp);
                }
            }
        }
    }
    // nonzeroPivots(): |R(i,i)| > threshold()·maxpivot, threshold() = eps·diagonalSize
    const double thr = eps * (double)size;
    int nz = 0;
    for (int i = 0; i < nonzero_pivots; ++i) nz += (std::abs(at(i, i)) > thr * maxpivot);
    std::vector<int> perm(cols);
    std::iota(perm.begin(), perm.end(), 0);
    for (int k = 0; k < size; ++k) std::swap(perm[k], perm[transp[k]]);
    for (int c = 0; c < cols; ++c) x[c] = 0;
    if (nz == 0) return 0;
    // c = Qᵀ b using the first nz reflectors
    for (int k = 0; k < nz; ++k) {
        double tau = hcoeffs[k];
        if (rows - k == 1) { b[k] *= 1 - tau; continue; }
        if (tau == 0) continue;
        double tmp = b[k];
        for (int r = k + 1; r < rows; ++r) tmp += at(r, k) * b[r];
        b[k] -= tau * tmp;
        for (int r = k + 1; r < rows; ++r) b[r] -= tau * at(r, k) * tmp;
    }
    // back substitution on the nz×nz upper triangle
    for (int i = nz - 1; i >= 0; --i) {
        double s = b[i];
        for (int j = i + 1; j < nz; ++j) s -= at(i, j) * b[j];
        b[i] = s / at(i, i);
    }
    for (int i = 0; i < nz; ++i) x[perm[i]] = b[i];
    return nz;
}

// Polar factor of a 3×3 matrix (what JacobiSVD U·Vᵀ returns for a full-rank input,
// solver.cpp:149-158): Newton iteration X ← (X + X⁻ᵀ)/2.  For the near-orthogonal rotations
// AngleAxis produces it agrees with U·Vᵀ to rounding; det < 0 never occurs for AngleAxis output.
void polar3(double R[9]) {
    for (int it = 0; it < 20; ++it) {
        const double* a = R;
        double det = a[0] * (a[4] * a[8] - a[5] * a[7]) - a[1] * (a[3] * a[8] - a[5] * a[6]) + a[2] * (a[3] * a[7] - a[4] * a[6]);
        if (det == 0) return;
        // inverse transpose = cofactor / det
        double cof[9] = {a[4] * a[8] - a[5] * a[7], a[5] * a[6] - a[3] * a[8], a[3] * a[7] - a[4] * a[6],
                         a[2] * a[7] - a[1] * a[8], a[0] * a[8] - a[2] * a[6], a[1] * a[6] - a[0] * a[7],
                         a[1] * a[5] - a[2] * a[4], a[2] * a[3] - a[0] * a[5], a[0] * a[4] - a[1] * a[3]};
        double maxd = 0, n[9];
        for (int k = 0; k < 9; ++k) { n[k] = 0.5 * (a[k] + cof[k] / det); maxd = std::max(maxd, std::abs(n[k] - a[k])); }
        std::memcpy(R, n, sizeof(n));
        if (maxd < 1e-16) break;
    }
}

// x[0:3] = rotation vector, x[3:6] = translation → Δ (solver.cpp:140-163):
// R = AngleAxisd(‖ω‖, ω.normalized()).toRotationMatrix() (Eigen/src/Geometry/AngleAxis.h), then
// the SVD re-orthonormalisation.  ω = 0 → normalized() returns 0 → R = I.
void delta_from_x(const double x[6], double D[16]) {
    double wx = x[0], wy = x[1], wz = x[2];
    double sq = (wx * wx + wy * wy) + wz * wz;
    double ang = std::sqrt(sq);
    double ax = 0, ay = 0, az = 0;
    if (sq > 0) { double nrm = std::sqrt(sq); ax = wx / nrm; ay = wy / nrm; az = wz / nrm; }
    double s = std::sin(ang), c = std::cos(ang);
    double sx = s * ax, sy = s * ay, sz = s * az;
    double c1x = (1 - c) * ax, c1y = (1 - c) * ay, c1z = (1 - c) * az;
    double R[9];
    double tmp = c1x * ay; R[1] = tmp - sz; R[3] = tmp + sz;
    tmp = c1x * az; R[2] = tmp + sy; R[6] = tmp - sy;
    tmp = c1y * az; R[5] = tmp - sx; R[7] = tmp + sx;
    R[0] = c1x * ax + c; R[4] = c1y * ay + c; R[8] = c1z * az + c;
    polar3(R);
    for (int i = 0; i < 16; ++i) D[i] = 0;
    for (int r = 0; r < 3; ++r) for (int cc = 0; cc < 3; ++cc) D[r * 4 + cc] = R[r * 3 + cc];
    D[3] = x[3]; D[7] = x[4]; D[11] = x[5]; D[15] = 1;
}

// Row of the point-to-plane system (solver.cpp:89-104).
inline void plane_row(const double* s, const double* d, const double* n, double a[6], double& b) {
    a[0] = n[2] * s[1] - n[1] * s[2];
    a[1] = n[0] * s[2] - n[2] * s[0];
    a[2] = n[1] * s[0] - n[0] * s[1];
    a[3] = n[0]; a[4] = n[1]; a[5] = n[2];
    double e0 = d[0] - s[0], e1 = d[1] - s[1], e2 = d[2] - s[2];
    b = (n[0] * e0 + n[1] * e1) + n[2] * e2;
}

// SolveMotionEstimationProblemLS (solver.cpp:74-166).  Ties in the |r| ordering (unstable
// std::sort, Q10) are broken by row index.  The upper rank is clamped to N−1 (Q11: the
// reference reads out of bounds when threshold·N rounds to N).
bool solve_ls(const double* s, const double* d, const double* n, size_t N, double threshold, double D[16], size_t* kept) {
    if (N == 0) return false;
    std::vector<double> A(N * 6), b(N);
    for (size_t i = 0; i < N; ++i) plane_row(s + 3 * i, d + 3 * i, n + 3 * i, &A[6 * i], b[i]);
    std::vector<double> Aw = A;
    double x[6];
    colpiv_qr_solve(Aw, (int)N, 6, b, x);
    std::vector<double> res(N);
    for (size_t i = 0; i < N; ++i) {
        const double* a = &A[6 * i];
        double v = a[0] * x[0];
        for (int k = 1; k < 6; ++k) v = v + a[k] * x[k];
        res[i] = v - b[i];
    }
    std::vector<size_t> idx(N);
    std::iota(idx.begin(), idx.end(), 0);
    std::sort(idx.begin(), idx.end(), [&](size_t i1, size_t i2) {
        double a1 = std::abs(res[i1]), a2 = std::abs(res[i2]);
        return a1 < a2 || (a1 == a2 && i1 < i2);
    });
    size_t lo = (size_t)(threshold * (double)N);
    size_t hi = (size_t)((1 - threshold) * (double)N);
    if (hi > N - 1) hi = N - 1;
    if (lo > hi) return false;
    size_t m = hi - lo + 1;
    std::vector<double> Af(m * 6), bf(m);
    for (size_t i = lo; i <= hi; ++i) {
        std::memcpy(&Af[(i - lo) * 6], &A[idx[i] * 6], 6 * sizeof(double));
        bf[i - lo] = b[idx[i]];
    }
    colpiv_qr_solve(Af, (int)m, 6, bf, x);
    if (kept) *kept = m;
    delta_from_x(x, D);
    return true;
}

// SolveMotionEstimationProblemWeightedLS (solver.cpp:168-220): rows scaled by √w, one QR.
bool solve_wls(const double* s, const double* d, const double* n, const double* w, size_t N, double D[16]) {
    if (N == 0) return false;
    std::vector<double> A(N * 6), b(N);
    for (size_t i = 0; i < N; ++i) {
        plane_row(s + 3 * i, d + 3 * i, n + 3 * i, &A[6 * i], b[i]);
        double sw = std::sqrt(w ? w[i] : 1.0);
        for (int k = 0; k < 6; ++k) A[6 * i + k] = sw * A[6 * i + k];
        b[i] = sw * b[i];
    }
    double x[6];
    colpiv_qr_solve(A, (int)N, 6, b, x);
    delta_from_x(x, D);
    return true;
}

constexpr double kDrpmEigRelTol = 1e-30;

// Symmetric 6×6 eigendecomposition (Eigen::SelfAdjointEigenSolver semantics: ascending
// eigenvalues, unit eigenvectors as columns).  Cyclic Jacobi; every DRPM quantity that uses the
// eigenvectors is invariant to their sign (degeneracy.h:14-131), so the sign is unpinned-safe.
// Stops when the off-diagonal mass is below max(1e-300, rel_tol·‖H‖_F²): rel_tol = 1e-30 (DRPM) is
// the usual Jacobi criterion off(A) ≤ 1e-15·‖A‖ (4 sweeps where the absolute one needs ~12);
// rel_tol = 0 sweeps on until the off-diagonal terms underflow.
void sym_eig(int n, const double* Hin, double* ev, double* U /* col-major: U[c*n+r] */, double rel_tol = 0.0) {
    std::vector<double> a(Hin, Hin + n * n), v(n * n, 0.0);
    for (int i = 0; i < n; ++i) v[i * n + i] = 1;
    double fro = 0;
    for (int i = 0; i < n * n; ++i) fro += a[i] * a[i];
    const double stop = std::max(1e-300, rel_tol * fro);
    for (int sweep = 0; sweep < 100; ++sweep) {
        double off = 0;
        for (int p = 0; p < n; ++p) for (int q = p + 1; q < n; ++q) off += a[p * n + q] * a[p * n + q];
        if (off < stop) break;
        for (int p = 0; p < n; ++p)
            for (int q = p + 1; q < n; ++q) {
                double apq = a[p * n + q];
                if (apq == 0) continue;
                double app = a[p * n + p], aqq = a[q * n + q];
                double theta = (aqq - app) / (2 * apq);
                double t = (theta >= 0 ? 1.0 : -1.0) / (std::abs(theta) + std::sqrt(theta * theta + 1));
                double c = 1 / std::sqrt(t * t + 1), s = t * c;
                for (int k = 0; k < n; ++k) {
                    double akp = a[k * n + p], akq = a[k * n + q];
                    a[k * n + p] = c * akp - s * akq;
                    a[k * n + q] = s * akp + c * akq;
                }
                for (int k = 0; k < n; ++k) {
                    double apk = a[p * n + k], aqk = a[q * n + k];
                    a[p * n + k] = c * apk - s * aqk;
                    a[q * n + k] = s * apk + c * aqk;
                }
                for (int k = 0; k < n; ++k) {
                    double vkp = v[k * n + p], vkq = v[k * n + q];
                    v[k * n + p] = c * vkp - s * vkq;
                    v[k * n + q] = s * vkp + c * vkq;
                }
            }
    }
    std::vector<int> ord(n);
    std::iota(ord.begin(), ord.end(), 0);
    std::sort(ord.begin(), ord.end(), [&](int i, int j) { return a[i * n + i] < a[j * n + j]; });
    for (int c = 0; c < n; ++c) {
        ev[c] = a[ord[c] * n + ord[c]];
        for (int r = 0; r < n; ++r) U[c * n + r] = v[r * n + ord[c]];
    }
}

// Boost.Math cdf(normal_distribution(mean, sd), x) = erfc(−(x−mean)/(sd·√2))/2.
inline double normal_cdf(double mean, double sd, double x) { return 0.5 * std::erfc(-(x - mean) / (sd * std::sqrt(2.0))); }

inline void skew(const double v[3], double S[9]) {
    // degeneracy.h:7-12: [0 −z y; z 0 −x; −y x 0]
    S[0] = 0; S[1] = -v[2]; S[2] = v[1];
    S[3] = v[2]; S[4] = 0; S[5] = -v[0];
    S[6] = -v[1]; S[7] = v[0]; S[8] = 0;
}

// SolveMotionEstimationProblemDRPM (solver.cpp:499-603) with degeneracy::ComputeNoiseEstimate
// (degeneracy.h:14-72), ComputeSignalToNoiseProbabilities (74-105) and SolveWithSnrProbabilities
// (107-131).  snr_factor = 10 (solver.cpp:547).
bool solve_drpm(const double* s, const double* d, const double* n, const double* w, size_t N,
                double threshold, double sp, double sn, double D[16]) {
    if (N == 0) return false;
    std::vector<double> A(N * 6), b(N), Aw(N * 6), bw(N);
    for (size_t i = 0; i < N; ++i) {
        plane_row(s + 3 * i, d + 3 * i, n + 3 * i, &A[6 * i], b[i]);
        double sw = std::sqrt(w[i]);
        for (int k = 0; k < 6; ++k) Aw[6 * i + k] = sw * A[6 * i + k];
        bw[i] = sw * b[i];
    }
    double H[36] = {0}, g[6] = {0};
    for (size_t i = 0; i < N; ++i)
        for (int r = 0; r < 6; ++r) {
            for (int c = 0; c < 6; ++c) H[r * 6 + c] += Aw[6 * i + r] * Aw[6 * i + c];
            g[r] += Aw[6 * i + r] * bw[i];
        }
    double ev[6], U[36];
    sym_eig(6, H, ev, U, kDrpmEigRelTol);
    // noise estimate
    double mean[36] = {0}, var[6] = {0};
    const double sp2 = sp * sp, sn2 = sn * sn;
    for (size_t i = 0; i < N; ++i) {
        double nx[9], px[9];
        skew(n + 3 * i, nx);
        skew(s + 3 * i, px);
        double B[36] = {0};
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c) {
                B[r * 6 + c] = -nx[r * 3 + c];
                double pn = 0;
                for (int k = 0; k < 3; ++k) pn += px[r * 3 + k] * nx[k * 3 + c];
                B[r * 6 + 3 + c] = pn;
                B[(3 + r) * 6 + 3 + c] = nx[r * 3 + c];
            }
        double Ndiag[6] = {sp2, sp2, sp2, sn2, sn2, sn2};
        double C[36];
        for (int r = 0; r < 6; ++r)
            for (int c = 0; c < 6; ++c) {
                double acc = 0;
                for (int k = 0; k < 6; ++k) acc += B[r * 6 + k] * Ndiag[k] * B[c * 6 + k];
                C[r * 6 + c] = acc * w[i];
            }
        for (int k = 0; k < 36; ++k) mean[k] += C[k];
        double sw = std::sqrt(w[i]), v[6];
        for (int r = 0; r < 3; ++r) {
            double pn = 0;
            for (int k = 0; k < 3; ++k) pn += px[r * 3 + k] * n[3 * i + k];
            v[r] = sw * pn;
            v[3 + r] = sw * n[3 * i + r];
        }
        for (int k = 0; k < 6; ++k) {
            const double* u = &U[k * 6];
            double a = 0, bb = 0;
            for (int r = 0; r < 6; ++r) {
                double cu = 0;
                for (int c = 0; c < 6; ++c) cu += C[r * 6 + c] * u[c];
                a += u[r] * cu;
                bb += u[r] * v[r];
            }
            var[k] += 2 * a * a + 4 * a * bb * bb;
        }
    }
    double prob[6];
    const double snr = 10.0;
    double pmin = kInf;
    for (int k = 0; k < 6; ++k) {
        const double* u = &U[k * 6];
        double meas = 0, exp_noise = 0;
        for (int r = 0; r < 6; ++r) {
            double hu = 0, mu = 0;
            for (int c = 0; c < 6; ++c) { hu += H[r * 6 + c] * u[c]; mu += mean[r * 6 + c] * u[c]; }
            meas += u[r] * hu;
            exp_noise += u[r] * mu;
        }
        double sd = std::sqrt(var[k]);
        double tp = meas / (1.0 + snr);
        bool nan = std::isnan(exp_noise) || std::isnan(sd) || std::isnan(tp);
        prob[k] = nan ? 0.0 : normal_cdf(exp_noise, sd, tp);
        pmin = std::min(pmin, prob[k]);
    }
    double x[6];
    if (pmin < threshold) {
        double dps[6];
        for (int k = 0; k < 6; ++k) dps[k] = std::abs(ev[k]) > 1e-10 ? prob[k] / ev[k] : 0.0;
        double ut[6];
        for (int k = 0; k < 6; ++k) { double acc = 0; for (int r = 0; r < 6; ++r) acc += U[k * 6 + r] * g[r]; ut[k] = dps[k] * acc; }
        for (int r = 0; r < 6; ++r) { double acc = 0; for (int k = 0; k < 6; ++k) acc += U[k * 6 + r] * ut[k]; x[r] = acc; }
    } else {
        colpiv_qr_solve(Aw, (int)N, 6, bw, x);
    }
    delta_from_x(x, D);
    return true;
}

// glibc random() TYPE_3 (degree 31, separation 3) as rand() uses it; srand(seed) init.
void rand_seed(int32_t* st, uint32_t seed) {
    int32_t r[34];
    r[0] = (int32_t)(seed == 0 ? 1 : seed);
    for (int i = 1; i < 31; ++i) {
        int64_t hi = r[i - 1] / 127773, lo = r[i - 1] % 127773;
        int64_t word = 16807 * lo - 2836 * hi;
        if (word < 0) word += 2147483647;
        r[i] = (int32_t)word;
    }
    for (int i = 31; i < 34; ++i) r[i] = r[i - 31];
    // state layout: st[0..30] = ring, st[31] = front idx, st[32] = rear idx
    uint32_t ring[31];
    for (int i = 0; i < 31; ++i) ring[i] = (uint32_t)r[i];
    // discard 310 outputs (glibc srandom_r runs random_r 10*31 times)
    int f = 3, rr = 0;
    for (int k = 0; k < 310; ++k) {
        ring[f] += ring[rr];
        f = (f + 1) % 31; rr = (rr + 1) % 31;
    }
    for (int i = 0; i < 31; ++i) st[i] = (int32_t)ring[i];
    st[31] = f; st[32] = rr; st[33] = 0;
}
int32_t rand_next(int32_t* st) {
    uint32_t* ring = reinterpret_cast<uint32_t*>(st);
    int f = st[31], r = st[32];
    ring[f] += ring[r];
    int32_t out = (int32_t)(ring[f] >> 1);
    st[31] = (f + 1) % 31; st[32] = (r + 1) % 31;
    return out;
}

// farthestPointSampling (common.cpp:19-82) for std::vector<Eigen::Vector3d>.
void fps3(const double* s, size_t N, int32_t* rs, int out[3]) {
    std::vector<double> md(N);
    int first = rand_next(rs) % (int)N;
    out[0] = first;
    auto dist = [&](size_t a, size_t b) {
        double dx = s[3 * a] - s[3 * b], dy = s[3 * a + 1] - s[3 * b + 1], dz = s[3 * a + 2] - s[3 * b + 2];
        return std::sqrt((dx * dx + dy * dy) + dz * dz);
    };
    for (size_t i = 0; i < N; ++i) md[i] = dist(first, i);
    for (int sc = 1; sc < 3; ++sc) {
        double maxd = -1.0;
        int far = -1;
        for (size_t i = 0; i < N; ++i) {
            bool taken = false;
            for (int k = 0; k < sc; ++k) taken |= (out[k] == (int)i);
            if (!taken && md[i] > maxd) { maxd = md[i]; far = (int)i; }
        }
        out[sc] = far;
        for (size_t i = 0; i < N; ++i) md[i] = std::min(md[i], dist(far, i));
    }
}

// SolveMotionEstimationProblemRANSAC (solver.cpp:222-385).
bool solve_ransac(const double* s, const double* d, const double* n, size_t N, const imls_params* p, int32_t* rs, double D[16]) {
    if (N == 0) return false;
    const int min_inliers = (int)(p->ransac_min_inliers_percentage * (double)N);
    int best = 0;
    double bestT[16];
    Mat4 I = mat4_identity();
    std::memcpy(bestT, I.m, sizeof(bestT));
    for (int it = 0; it < p->ransac_max_iterations; ++it) {
        int id[3];
        fps3(s, N, rs, id);
        std::vector<double> A(18), b(3);
        for (int i = 0; i < 3; ++i) plane_row(s + 3 * id[i], d + 3 * id[i], n + 3 * id[i], &A[6 * i], b[i]);
        double x[6], T[16];
        colpiv_qr_solve(A, 3, 6, b, x);
        delta_from_x(x, T);
        int cnt = 0;
        for (size_t i = 0; i < N; ++i) {
            double tp[3];
            for (int r = 0; r < 3; ++r) tp[r] = ((T[r * 4] * s[3 * i] + T[r * 4 + 1] * s[3 * i + 1]) + T[r * 4 + 2] * s[3 * i + 2]) + T[r * 4 + 3];
            double dist = std::abs(((tp[0] - d[3 * i]) * n[3 * i] + (tp[1] - d[3 * i + 1]) * n[3 * i + 1]) + (tp[2] - d[3 * i + 2]) * n[3 * i + 2]);
            if (dist < p->ransac_distance_threshold) ++cnt;
        }
        if (cnt > best) { best = cnt; std::memcpy(bestT, T, sizeof(T)); }
        if (best > min_inliers) break;
    }
    std::vector<double> is, id_, in, w;
    const double h2 = p->ransac_huber_threshold * p->ransac_distance_threshold;
    for (size_t i = 0; i < N; ++i) {
        double tp[3];
        for (int r = 0; r < 3; ++r) tp[r] = ((bestT[r * 4] * s[3 * i] + bestT[r * 4 + 1] * s[3 * i + 1]) + bestT[r * 4 + 2] * s[3 * i + 2]) + bestT[r * 4 + 3];
        double dist = std::abs(((tp[0] - d[3 * i]) * n[3 * i] + (tp[1] - d[3 * i + 1]) * n[3 * i + 1]) + (tp[2] - d[3 * i + 2]) * n[3 * i + 2]);
        if (dist < p->ransac_distance_threshold) {
            for (int k = 0; k < 3; ++k) { is.push_back(s[3 * i + k]); id_.push_back(d[3 * i + k]); in.push_back(n[3 * i + k]); }
            double ar = std::exp(-std::abs(dist));
            w.push_back(std::sqrt(ar) < h2 ? ar : 2 * h2 * std::sqrt(ar) - h2 * h2);
        }
    }
    double ws = 0;
    for (double v : w) ws += v;
    if (ws > 0) for (double& v : w) v /= ws;
    size_t M = w.size();
    switch (p->ransac_final_method) {
        case IMLS_FINAL_LS: return solve_ls(is.data(), id_.data(), in.data(), M, p->ransac_ls_threshold, D, nullptr);
        case IMLS_FINAL_WEIGHTED_LS: return solve_wls(is.data(), id_.data(), in.data(), w.data(), M, D);
        case IMLS_FINAL_DRPM: return solve_drpm(is.data(), id_.data(), in.data(), w.data(), M, p->drpm_threshold, p->drpm_stdev_points, p->drpm_stdev_normals, D);
        default: return false;
    }
}

// ------------------------------------------------------------------------------------------
// Matching (imls_icp.cpp:301-483, 496-745).
// ------------------------------------------------------------------------------------------
struct Matcher {
    const imls_params* P;
    Cloud tgt;
    KdTree tree;
    std::vector<double> ten;   // tensor-voting input tensors [M][6] (xx xy xz yy yz zz), filtered order

    // angle test shared by imls_icp.cpp:442-451, 681-692 and laser_odometry.cpp:373-384; NaN
    // angles pass (Q8).
    static bool angle_reject_thr(const double ns[3], const double nn[3], double thr) {
        double dot = (ns[0] * nn[0] + ns[1] * nn[1]) + ns[2] * nn[2];
        double n1 = std::sqrt((ns[0] * ns[0] + ns[1] * ns[1]) + ns[2] * ns[2]);
        double n2 = std::sqrt((nn[0] * nn[0] + nn[1] * nn[1]) + nn[2] * nn[2]);
        double ca = dot / (n1 * n2);
        double angle = std::acos(ca) * 180.0 / M_PI;
        return angle > thr;
    }
    bool angle_reject(const double ns[3], const double nn[3]) const { return angle_reject_thr(ns, nn, P->angle_diff_threshold); }

    // ComputeNormal (imls_icp.cpp:753-794) is reached only through the recompute branch; under
    // libnabo's knn() return-value semantics (Q1) the branch rejects before calling it.
    // Count mode (documented intent) uses the PCA normal flipped to +z.
    bool recompute_normal(const double pt[3], double nrm[3]) const {
        if (!P->recompute_normal_count_mode) { nrm[0] = nrm[1] = nrm[2] = kInf; return false; }
        KdTree::Heap h;
        tree.knn(pt, P->search_number_normal, P->r_normal * P->r_normal, false, h);
        if (h.n < P->search_number_normal) { nrm[0] = nrm[1] = nrm[2] = kInf; return false; }
        double mu[3] = {0, 0, 0};
        for (int k = 0; k < h.n; ++k) { mu[0] += tgt.x[h.i[k]]; mu[1] += tgt.y[h.i[k]]; mu[2] += tgt.z[h.i[k]]; }
        for (double& m : mu) m /= h.n;
        double C[9] = {0};
        for (int k = 0; k < h.n; ++k) {
            double v[3] = {tgt.x[h.i[k]] - mu[0], tgt.y[h.i[k]] - mu[1], tgt.z[h.i[k]] - mu[2]};
            for (int r = 0; r < 3; ++r) for (int c = 0; c < 3; ++c) C[r * 3 + c] += v[r] * v[c];
        }
        for (double& c : C) c /= h.n;
        double ev[3], U[9];
        sym_eig(3, C, ev, U);
        double nn = std::sqrt(U[0] * U[0] + U[1] * U[1] + U[2] * U[2]);
        for (int k = 0; k < 3; ++k) nrm[k] = U[k] / nn;
        if (nrm[2] < 0) { nrm[0] = -nrm[0]; nrm[1] = -nrm[1]; nrm[2] = -nrm[2]; }
        return true;
    }

    // Tensor voting (IMLSICPMatcher::VoteForAny, imls_icp.cpp:171-296, used at 514-546 and
    // 634-643) for ONE output point x (a transformed source point, in_cloudDP column).
    //   * candidates: libnabo knn(x, k) over the target — K = tensor_k, no radius, no
    //     ALLOW_SELF_MATCH (197), sorted (d², index); unfound slots skipped (205-208);
    //   * vote of input j: r = x − p_j, dist = ‖r‖/σ; skipped unless 0 < dist < threshold
    //     (212-217); w = exp(−‖r‖²/σ) (220: σ, not σ²); R = I − 2 r̂r̂ᵀ, R' = (I − ½ r̂r̂ᵀ)R,
    //     S = w·R·T_j·R' (222-224), summed into the output tensor (226);
    //   * non-zero test (233): Eigen isZero(1e-12) — every |coeff| ≤ 1e-12 counts as zero;
    //   * decompose (245; libpointmatcher TensorVoting::decompose, UNPINNED — not in the
    //     container): SelfAdjointEigenSolver on the (non-symmetric) sum reads its LOWER triangle;
    //     eigenvalues ordered by |λ| descending, "tangents" = the eigenvector of the smallest |λ|
    //     (the vector the reference uses as the normal, 272-278 / 541-545), flipped to +z (274).
    // T_j = the target's input tensor as given (encode(AWARE_TENSOR), 179: see
    // oracle_tv_encode_pca for the reference's own encoding of PCA features).  Returns false when
    // the tensor is zero (the lookup at 637 then fails → "no normal").
    bool tv_normal(const double x[3], double nrm[3], double acc_out[9] = nullptr) const {
        KdTree::Heap h;
        tree.knn(x, P->tensor_k, kInf, false, h);
        double acc[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
        const double sigma = P->tensor_sigma;
        for (int k = 0; k < h.n; ++k) {
            const int32_t j = h.i[k];
            const double r[3] = {x[0] - (double)tgt.x[j], x[1] - (double)tgt.y[j], x[2] - (double)tgt.z[j]};
            const double nr = std::sqrt((r[0] * r[0] + r[1] * r[1]) + r[2] * r[2]);
            const double dist = nr / sigma;
            if (dist <= 0. || dist >= P->tensor_distance_threshold) continue;
            const double u[3] = {r[0] / nr, r[1] / nr, r[2] / nr};
            const double w = std::exp(-(nr * nr) / sigma);
            const double* t6 = &ten[(size_t)j * 6];
            const double T[9] = {t6[0], t6[1], t6[2], t6[1], t6[3], t6[4], t6[2], t6[4], t6[5]};
            double R[9], Rp[9], RT[9];
            for (int a = 0; a < 3; ++a)
                for (int b = 0; b < 3; ++b) R[a * 3 + b] = (a == b ? 1.0 : 0.0) - 2 * u[a] * u[b];
            for (int a = 0; a < 3; ++a)
                for (int b = 0; b < 3; ++b) {
                    double s = 0.0;
                    for (int c = 0; c < 3; ++c) s += ((a == c ? 1.0 : 0.0) - 0.5 * u[a] * u[c]) * R[c * 3 + b];
                    Rp[a * 3 + b] = s;
                }
            for (int a = 0; a < 3; ++a)
                for (int b = 0; b < 3; ++b) {
                    double s = 0.0;
                    for (int c = 0; c < 3; ++c) s += R[a * 3 + c] * T[c * 3 + b];
                    RT[a * 3 + b] = s;
                }
            for (int a = 0; a < 3; ++a)
                for (int b = 0; b < 3; ++b) {
                    double s = 0.0;
                    for (int c = 0; c < 3; ++c) s += RT[a * 3 + c] * Rp[c * 3 + b];
                    acc[a * 3 + b] += w * s;
                }
        }
        if (acc_out) std::memcpy(acc_out, acc, sizeof(acc));
        bool zero = true;
        for (double v : acc) zero = zero && std::abs(v) <= 1e-12;
        if (zero) return false;
        double A[9];
        for (int a = 0; a < 3; ++a)
            for (int b = 0; b < 3; ++b) A[a * 3 + b] = a >= b ? acc[a * 3 + b] : acc[b * 3 + a];
        double ev[3], U[9];
        sym_eig(3, A, ev, U);
        int m = 0;
        for (int c = 1; c < 3; ++c) if (std::abs(ev[c]) < std::abs(ev[m])) m = c;
        for (int k = 0; k < 3; ++k) nrm[k] = U[m * 3 + k];
        if (nrm[2] < 0) { nrm[0] = -nrm[0]; nrm[1] = -nrm[1]; nrm[2] = -nrm[2]; }
        return true;
    }

    void map_normal(int32_t j, double nrm[3]) const {
        if (P->get_normals) { nrm[0] = tgt.nx[j]; nrm[1] = tgt.ny[j]; nrm[2] = tgt.nz[j]; return; }
        double pt[3] = {tgt.x[j], tgt.y[j], tgt.z[j]};
        recompute_normal(pt, nrm);
    }

    // ImplicitMLSFunction (imls_icp.cpp:301-483), default (kd-tree) branch, and the projected-
    // distance branch (338-369, brute force over the whole map).
    bool imls(const double x[3], const double ns[3], double& height) const {
        const int K = P->search_number;
        double nd2[64];
        int32_t nid[64];
        int valid_number = K;
        if (P->use_projected_distance) {
            std::vector<std::pair<double, int>> pd;
            for (size_t j = 0; j < tgt.size(); ++j) {
                double dx = (double)tgt.x[j] - x[0], dy = (double)tgt.y[j] - x[1], dz = (double)tgt.z[j] - x[2];
                double cx = dy * ns[2] - dz * ns[1], cy = dz * ns[0] - dx * ns[2], cz = dx * ns[1] - dy * ns[0];
                double proj = std::sqrt((cx * cx + cy * cy) + cz * cz);
                double dn = std::sqrt((dx * dx + dy * dy) + dz * dz);
                if (dn < P->r_proj && proj < P->r) pd.emplace_back(proj, (int)j);
            }
            if (pd.empty()) return false;
            std::sort(pd.begin(), pd.end());
            valid_number = std::min(K, (int)pd.size());
            for (int i = 0; i < valid_number; ++i) { nid[i] = pd[i].second; nd2[i] = pd[i].first * pd[i].first; }
        } else {
            KdTree::Heap h;
            tree.knn(x, K, P->r * P->r, true, h);
            for (int i = 0; i < K; ++i) {
                if (i < h.n) { nd2[i] = h.d[i]; nid[i] = h.i[i]; }
                else { nd2[i] = kInf; nid[i] = -1; }
            }
        }
        double sp[64][3], sn[64][3];
        int ns_cnt = 0;
        for (int i = 0; i < valid_number; ++i) {
            if (!(nd2[i] < kInf && !std::isinf(nd2[i]) && !std::isnan(nd2[i]))) continue;
            int32_t j = nid[i];
            double pt[3] = {tgt.x[j], tgt.y[j], tgt.z[j]};
            if (!finite3(pt[0], pt[1], pt[2])) continue;
            double nrm[3];
            map_normal(j, nrm);
            if (!finite3(nrm[0], nrm[1], nrm[2])) continue;
            if (P->normal_angle_constraint && angle_reject(ns, nrm)) continue;
            std::memcpy(sp[ns_cnt], pt, sizeof(pt));
            std::memcpy(sn[ns_cnt], nrm, sizeof(nrm));
            ++ns_cnt;
        }
        if (ns_cnt < 3) return false;
        double hmax = std::sqrt(nd2[ns_cnt - 1]) / 3;   // Q3: indexes the sorted list
        double wsum = 0.0, psum = 0.0;
        for (int i = 0; i < ns_cnt; ++i) {
            double dx = x[0] - sp[i][0], dy = x[1] - sp[i][1], dz = x[2] - sp[i][2];
            double dn = (dx * dx + dy * dy) + dz * dz;
            double w = std::exp(-dn / hmax / hmax);
            double proj = ((w * dx) * sn[i][0] + (w * dy) * sn[i][1]) + (w * dz) * sn[i][2];
            wsum += w;
            psum += proj;
        }
        height = psum / (wsum + 1e-5);   // Q4
        return true;
    }

    // One query of ProjSourcePtToSurface's loop body (imls_icp.cpp:553-734).  Returns the reject
    // category (or -1 when the point survives, with y and nn filled).
    int project_one(const float xf[3], const float nsf[3], float y[3], float nn_out[3]) const {
        double x[3] = {xf[0], xf[1], xf[2]}, ns[3] = {nsf[0], nsf[1], nsf[2]};
        int32_t best = -1;
        double min_dist = kInf;
        if (P->use_projected_distance) {
            std::vector<std::pair<double, int>> pd;   // imls_icp.cpp:563-596
            for (size_t j = 0; j < tgt.size(); ++j) {
                double dx = (double)tgt.x[j] - x[0], dy = (double)tgt.y[j] - x[1], dz = (double)tgt.z[j] - x[2];
                double cx = dy * ns[2] - dz * ns[1], cy = dz * ns[0] - dx * ns[2], cz = dx * ns[1] - dy * ns[0];
                double proj = std::sqrt((cx * cx + cy * cy) + cz * cz);
                double dn = std::sqrt((dx * dx + dy * dy) + dz * dz);
                if (dn < P->r_proj && proj < P->r) pd.emplace_back(proj, (int)j);
            }
            if (pd.empty()) return IMLS_REJ_TOO_FAR;
            auto it = std::min_element(pd.begin(), pd.end());
            min_dist = it->first * it->first;
            best = it->second;
        } else {
            KdTree::Heap h;
            tree.knn(x, 1, P->r * P->r, false, h);   // imls_icp.cpp:605-609 (no self match)
            if (h.n == 0) return IMLS_REJ_TOO_FAR;   // InvalidIndex: counted as too far (Q18)
            best = h.i[0];
            min_dist = h.d[0];
        }
        if (best < 0 || best >= (int32_t)tgt.size()) return IMLS_REJ_NO_NORMAL;
        if (min_dist > P->h * P->h) return IMLS_REJ_TOO_FAR;
        double nn[3];
        if (P->get_normals) { nn[0] = tgt.nx[best]; nn[1] = tgt.ny[best]; nn[2] = tgt.nz[best]; }
        else if (P->use_tensor_voting) {   // imls_icp.cpp:634-643: the query's own voted normal
            if (ten.empty() || !tv_normal(x, nn)) return IMLS_REJ_NO_NORMAL;
        }
        else { double pt[3] = {tgt.x[best], tgt.y[best], tgt.z[best]}; recompute_normal(pt, nn); }
        if (!finite3(nn[0], nn[1], nn[2])) return IMLS_REJ_INVALID_NORMAL;
        if (P->normal_angle_constraint && angle_reject(ns, nn)) return IMLS_REJ_NORMAL_CONSTRAINT;
        double height;
        if (!imls(x, ns, height)) return IMLS_REJ_MLS_FAIL;
        if (std::isnan(height) || std::isinf(height)) return IMLS_REJ_NAN_INF_HEIGHT;
        y[0] = (float)(x[0] - height * nn[0]);
        y[1] = (float)(x[1] - height * nn[1]);
        y[2] = (float)(x[2] - height * nn[2]);
        nn_out[0] = (float)nn[0]; nn_out[1] = (float)nn[1]; nn_out[2] = (float)nn[2];
        return -1;
    }

    // plane_ICP_proj's loop body (laser_odometry.cpp:312-404): NN-1 within picp.r (no self match)
    // or, with use_projected_distance, the brute-force minimum of ‖(p−x)×n_s‖ under the
    // reference's swapped gate ‖p−x‖ < r·r && proj < r_proj (322); no h gate (min_dist unused);
    // unfound → "no normal" (352-357); map normal from the cloud; y = x − ((x−p)·n)·n.
    int project_one_plane(const float xf[3], const float nsf[3], float y[3], float nn_out[3]) const {
        double x[3] = {xf[0], xf[1], xf[2]}, ns[3] = {nsf[0], nsf[1], nsf[2]};
        int32_t best = -1;
        if (P->picp_use_projected_distance) {
            std::vector<std::pair<double, int>> pd;
            const double rr = P->picp_r * P->picp_r;
            for (size_t j = 0; j < tgt.size(); ++j) {
                double dx = (double)tgt.x[j] - x[0], dy = (double)tgt.y[j] - x[1], dz = (double)tgt.z[j] - x[2];
                double cx = dy * ns[2] - dz * ns[1], cy = dz * ns[0] - dx * ns[2], cz = dx * ns[1] - dy * ns[0];
                double proj = std::sqrt((cx * cx + cy * cy) + cz * cz);
                double dn = std::sqrt((dx * dx + dy * dy) + dz * dz);
                if (dn < rr && proj < P->picp_r_proj) pd.emplace_back(proj, (int)j);
            }
            if (pd.empty()) return IMLS_REJ_TOO_FAR;
            best = std::min_element(pd.begin(), pd.end())->second;
        } else {
            KdTree::Heap h;
            tree.knn(x, 1, P->picp_r * P->picp_r, false, h);
            best = h.n ? h.i[0] : -1;
        }
        if (best < 0 || best >= (int32_t)tgt.size()) return IMLS_REJ_NO_NORMAL;
        double p[3] = {tgt.x[best], tgt.y[best], tgt.z[best]};
        double nn[3] = {tgt.nx[best], tgt.ny[best], tgt.nz[best]};
        if (!finite3(nn[0], nn[1], nn[2])) return IMLS_REJ_INVALID_NORMAL;
        if (P->picp_normal_angle_constraint && angle_reject_thr(ns, nn, P->picp_angle_diff_threshold))
            return IMLS_REJ_NORMAL_CONSTRAINT;
        double v[3] = {x[0] - p[0], x[1] - p[1], x[2] - p[2]};
        double pdist = (v[0] * nn[0] + v[1] * nn[1]) + v[2] * nn[2];
        y[0] = (float)(x[0] - pdist * nn[0]);
        y[1] = (float)(x[1] - pdist * nn[1]);
        y[2] = (float)(x[2] - pdist * nn[2]);
        nn_out[0] = (float)nn[0]; nn_out[1] = (float)nn[1]; nn_out[2] = (float)nn[2];
        return -1;
    }
};

// x = float(pose·[p;1]) (laser_odometry.cpp:527-549): row-wise ((m0p0 + m1p1) + m2p2) + m3.
inline void transform_point(const double T[16], float px, float py, float pz, float out[3]) {
    double p[3] = {px, py, pz};
    for (int r = 0; r < 3; ++r) {
        double v = T[r * 4 + 0] * p[0];
        v = v + T[r * 4 + 1] * p[1];
        v = v + T[r * 4 + 2] * p[2];
        v = v + T[r * 4 + 3] * 1.0;
        out[r] = (float)v;
    }
}
inline void rotate_normal(const double T[16], float nx, float ny, float nz, float out[3]) {
    double n[3] = {nx, ny, nz};
    for (int r = 0; r < 3; ++r) {
        double v = T[r * 4 + 0] * n[0];
        v = v + T[r * 4 + 1] * n[1];
        v = v + T[r * 4 + 2] * n[2];
        out[r] = (float)v;
    }
}

struct Corr { std::vector<float> x, y, n; std::vector<uint32_t> idx; };

int g_threads = 1;   // oracle_set_threads: the secondary (all-cores) CPU baseline, SURVEY §8(d)
int g_faithful = 0;  // oracle_set_faithful: the reference's own data-structure costs (CPU baseline only)

// The "faithful" CPU baseline: the same arithmetic with the reference's container
// costs — a full 48-byte AoS copy of the source per iteration (laser_odometry.cpp:527), the
// erase-based loop over it (imls_icp.cpp:553-734: `in_cloud->erase(it)` moves the tail for every
// rejected point, O(N) each), heap-allocated kNN index/distance vectors and neighbour lists per
// query (328-329, 378-379, 602-604), out_cloud push_back, and the getXYZ/getNormals copies
// (laser_odometry.cpp:595-599).  Results are identical to project_all's.
struct Pt48 { float x, y, z, p0, nx, ny, nz, p1, in, cu, p2, p3; };
void project_all_faithful(const Matcher& m, const Cloud& src, const double T[16], bool rot_normals, Corr& c,
                          uint64_t rej[6]) {
    for (int k = 0; k < 6; ++k) rej[k] = 0;
    c.x.clear(); c.y.clear(); c.n.clear(); c.idx.clear();
    std::vector<Pt48> in_cloud(src.size());
    std::vector<uint32_t> orig(src.size());
    for (size_t i = 0; i < src.size(); ++i) {
        Pt48& q = in_cloud[i];
        q = Pt48{src.x[i], src.y[i], src.z[i], 0.f, src.nx[i], src.ny[i], src.nz[i], 0.f, 0.f, 0.f, 0.f, 0.f};
        float x[3];
        transform_point(T, src.x[i], src.y[i], src.z[i], x);
        q.x = x[0]; q.y = x[1]; q.z = x[2];
        if (rot_normals) { float nn[3]; rotate_normal(T, src.nx[i], src.ny[i], src.nz[i], nn); q.nx = nn[0]; q.ny = nn[1]; q.nz = nn[2]; }
        orig[i] = (uint32_t)i;
    }
    std::vector<Pt48> out_cloud;
    const int K = m.P->search_number;
    volatile double sink = 0.0;
    for (size_t i = 0; i < in_cloud.size();) {
        std::vector<int> nn_idx(1);                                // Eigen::VectorXi indices(1)
        std::vector<double> nn_d2(1);                              // Eigen::VectorXd dist2(1)
        std::vector<int> k_idx(K);                                 // VectorXi nearIndices(K)
        std::vector<double> k_d2(K);                               // VectorXd nearDist2(K)
        std::vector<std::array<double, 3>> nearPoints, nearNormals;
        nearPoints.reserve(K);
        nearNormals.reserve(K);
        const Pt48& q = in_cloud[i];
        float x[3] = {q.x, q.y, q.z}, ns[3] = {q.nx, q.ny, q.nz}, y[3], nn[3];
        int r = m.P->matching_method == IMLS_MATCH_PLANE_ICP ? m.project_one_plane(x, ns, y, nn) : m.project_one(x, ns, y, nn);
        sink = sink + (double)nn_idx.size() + (double)k_d2.size();
        if (r >= 0) {
            rej[r]++;
            in_cloud.erase(in_cloud.begin() + (long)i);            // it = in_cloud->erase(it)
            orig.erase(orig.begin() + (long)i);
            continue;
        }
        out_cloud.push_back(Pt48{y[0], y[1], y[2], 0.f, nn[0], nn[1], nn[2], 0.f, 0.f, 0.f, 0.f, 0.f});
        ++i;
    }
    // getXYZ(in_cloud), getXYZ(out_cloud), getNormals(out_cloud) (laser_odometry.cpp:595-599)
    std::vector<std::array<double, 3>> vin, vref, vnrm;
    for (const Pt48& p : in_cloud) vin.push_back({(double)p.x, (double)p.y, (double)p.z});
    for (const Pt48& p : out_cloud) { vref.push_back({(double)p.x, (double)p.y, (double)p.z}); vnrm.push_back({(double)p.nx, (double)p.ny, (double)p.nz}); }
    for (size_t k = 0; k < in_cloud.size(); ++k) {
        const float xs[3] = {in_cloud[k].x, in_cloud[k].y, in_cloud[k].z};
        const float ys[3] = {out_cloud[k].x, out_cloud[k].y, out_cloud[k].z};
        const float ns[3] = {out_cloud[k].nx, out_cloud[k].ny, out_cloud[k].nz};
        c.x.insert(c.x.end(), xs, xs + 3);
        c.y.insert(c.y.end(), ys, ys + 3);
        c.n.insert(c.n.end(), ns, ns + 3);
        c.idx.push_back(orig[k]);
    }
    sink = sink + (double)vin.size() + (double)vref.size() + (double)vnrm.size();
}

void project_all(const Matcher& m, const Cloud& src, const double T[16], bool rot_normals, Corr& c, uint64_t rej[6]) {
    if (g_faithful && g_threads <= 1) { project_all_faithful(m, src, T, rot_normals, c, rej); return; }
    for (int k = 0; k < 6; ++k) rej[k] = 0;
    c.x.clear(); c.y.clear(); c.n.clear(); c.idx.clear();
    if (g_threads > 1) {
        // queries are independent: evaluate them in parallel, then compact in source order (the
        // same result as the sequential loop below)
        const size_t N = src.size();
        std::vector<float> X(3 * N), Y(3 * N), NN(3 * N);
        std::vector<int> R(N);
#pragma omp parallel for schedule(dynamic, 256) num_threads(g_threads)
        for (long i = 0; i < (long)N; ++i) {
            float ns[3] = {src.nx[i], src.ny[i], src.nz[i]};
            transform_point(T, src.x[i], src.y[i], src.z[i], &X[3 * i]);
            if (rot_normals) rotate_normal(T, src.nx[i], src.ny[i], src.nz[i], ns);
            R[i] = m.P->matching_method == IMLS_MATCH_PLANE_ICP ? m.project_one_plane(&X[3 * i], ns, &Y[3 * i], &NN[3 * i])
                                                                 : m.project_one(&X[3 * i], ns, &Y[3 * i], &NN[3 * i]);
        }
        for (size_t i = 0; i < N; ++i) {
            if (R[i] >= 0) { rej[R[i]]++; continue; }
            c.x.insert(c.x.end(), &X[3 * i], &X[3 * i] + 3);
            c.y.insert(c.y.end(), &Y[3 * i], &Y[3 * i] + 3);
            c.n.insert(c.n.end(), &NN[3 * i], &NN[3 * i] + 3);
            c.idx.push_back((uint32_t)i);
        }
        return;
    }
    for (size_t i = 0; i < src.size(); ++i) {
        float x[3], ns[3] = {src.nx[i], src.ny[i], src.nz[i]}, y[3], nn[3];
        transform_point(T, src.x[i], src.y[i], src.z[i], x);
        if (rot_normals) rotate_normal(T, src.nx[i], src.ny[i], src.nz[i], ns);
        int r = m.P->matching_method == IMLS_MATCH_PLANE_ICP ? m.project_one_plane(x, ns, y, nn) : m.project_one(x, ns, y, nn);
        if (r >= 0) { rej[r]++; continue; }
        c.x.insert(c.x.end(), x, x + 3);
        c.y.insert(c.y.end(), y, y + 3);
        c.n.insert(c.n.end(), nn, nn + 3);
        c.idx.push_back((uint32_t)i);
    }
}

bool solve_dispatch(int method, const double* s, const double* d, const double* n, const double* w, size_t N,
                    const imls_params* p, int32_t* rs, double D[16], size_t* kept) {
    switch (method) {
        case IMLS_SOLVE_LS: return solve_ls(s, d, n, N, p->ls_threshold, D, kept);
        case IMLS_SOLVE_WEIGHTED_LS: return solve_wls(s, d, n, w, N, D);
        case IMLS_SOLVE_RANSAC: return solve_ransac(s, d, n, N, p, rs, D);
        case IMLS_SOLVE_DRPM: {   // stand-alone SolveMotionEstimationProblemDRPM; null weights = unit
            std::vector<double> ones;
            if (!w) { ones.assign(N, 1.0); w = ones.data(); }
            return solve_drpm(s, d, n, w, N, p->drpm_threshold, p->drpm_stdev_points, p->drpm_stdev_normals, D);
        }
        default: return false;
    }
}

}  // namespace

// Tensor-voting input tensors [6][n] (SoA, input order) → [M][6] in the filtered order.
std::vector<double> load_tensors(const float* tgt6, size_t n, const float* ten6) {
    std::vector<double> t;
    if (!ten6) return t;
    for (size_t i = 0; i < n; ++i) {
        if (!(std::isfinite(tgt6[i]) && std::isfinite(tgt6[n + i]) && std::isfinite(tgt6[2 * n + i]))) continue;
        for (int k = 0; k < 6; ++k) t.push_back(ten6[k * n + i]);
    }
    return t;
}

// ==========================================================================================
// C ABI
// ==========================================================================================
extern "C" {

int oracle_knn(const float* tgt6, size_t M, const float* q3, size_t Q, int K, double max_radius,
               int allow_self, double* d2, int32_t* idx) {
    if (K <= 0 || K > 64) return IMLS_ERR_ARG;
    Cloud t = load_filtered(tgt6, M);
    KdTree tree;
    tree.build(t);
    KdTree::Heap h;
    for (size_t q = 0; q < Q; ++q) {
        double x[3] = {q3[q], q3[Q + q], q3[2 * Q + q]};
        tree.knn(x, K, max_radius * max_radius, allow_self != 0, h);
        for (int k = 0; k < K; ++k) {
            d2[q * K + k] = k < h.n ? h.d[k] : kInf;
            idx[q * K + k] = k < h.n ? h.i[k] : -1;
        }
    }
    return IMLS_OK;
}

int oracle_project(const float* src6, size_t N, const float* tgt6, size_t M, const double pose[16],
                   const imls_params* p, float* x_out, float* y_out, float* n_out, uint32_t* src_index_out,
                   size_t* n_valid, uint64_t reject[IMLS_NUM_REJ]) {
    return oracle_project_tv(src6, N, tgt6, M, nullptr, pose, p, x_out, y_out, n_out, src_index_out, n_valid, reject);
}

int oracle_project_tv(const float* src6, size_t N, const float* tgt6, size_t M, const float* ten6, const double pose[16],
                      const imls_params* p, float* x_out, float* y_out, float* n_out, uint32_t* src_index_out,
                      size_t* n_valid, uint64_t reject[IMLS_NUM_REJ]) {
    if (!p || p->search_number <= 0 || p->search_number > 64) return IMLS_ERR_ARG;
    if (p->use_tensor_voting && (p->tensor_k <= 0 || p->tensor_k > 64)) return IMLS_ERR_ARG;
    Cloud src = load_filtered(src6, N);
    Matcher m{p, load_filtered(tgt6, M), {}, load_tensors(tgt6, M, ten6)};
    m.tree.build(m.tgt);
    Corr c;
    uint64_t rej[6];
    project_all(m, src, pose, p->transform_normal != 0, c, rej);
    size_t nv = c.idx.size();
    if (x_out) std::memcpy(x_out, c.x.data(), nv * 3 * sizeof(float));
    if (y_out) std::memcpy(y_out, c.y.data(), nv * 3 * sizeof(float));
    if (n_out) std::memcpy(n_out, c.n.data(), nv * 3 * sizeof(float));
    if (src_index_out) std::memcpy(src_index_out, c.idx.data(), nv * sizeof(uint32_t));
    if (n_valid) *n_valid = nv;
    if (reject) std::memcpy(reject, rej, sizeof(rej));
    return IMLS_OK;
}

int oracle_solve(int32_t method, const double* s, const double* d, const double* n, const double* w, size_t N,
                 const imls_params* p, int32_t* rand_state, double delta_out[16], int* ok) {
    int32_t local[34];
    if (!rand_state) { rand_seed(local, p->ransac_seed); rand_state = local; }
    bool r = solve_dispatch(method, s, d, n, w, N, p, rand_state, delta_out, nullptr);
    if (ok) *ok = r ? 1 : 0;
    return IMLS_OK;
}

int oracle_register_frame(const float* src6, size_t N, const float* tgt6, size_t M, const imls_params* p,
                          double pose_out[16], int* iters_run, int* status, imls_iter_trace* trace,
                          int corr_iter, float* corr, size_t* corr_n, double* seconds_index, double* seconds_total) {
    return oracle_register_frame_tv(src6, N, tgt6, M, nullptr, p, pose_out, iters_run, status, trace, corr_iter, corr,
                                    corr_n, seconds_index, seconds_total);
}

int oracle_register_frame_tv(const float* src6, size_t N, const float* tgt6, size_t M, const float* ten6,
                             const imls_params* p, double pose_out[16], int* iters_run, int* status,
                             imls_iter_trace* trace, int corr_iter, float* corr, size_t* corr_n,
                             double* seconds_index, double* seconds_total) {
    return oracle_register_frame_rs(src6, N, tgt6, M, ten6, p, nullptr, pose_out, iters_run, status, trace, corr_iter,
                                    corr, corr_n, seconds_index, seconds_total);
}

// rand_state (nullable, int32[34]): the process-wide glibc rand() stream RANSAC draws from, carried
// across frames like the reference's (it never calls srand); null = a fresh stream from ransac_seed.
int oracle_register_frame_rs(const float* src6, size_t N, const float* tgt6, size_t M, const float* ten6,
                             const imls_params* p, int32_t* rand_state, double pose_out[16], int* iters_run,
                             int* status, imls_iter_trace* trace, int corr_iter, float* corr, size_t* corr_n,
                             double* seconds_index, double* seconds_total) {
    if (!p || p->search_number <= 0 || p->search_number > 64) return IMLS_ERR_ARG;
    if (p->use_tensor_voting && (p->tensor_k <= 0 || p->tensor_k > 64)) return IMLS_ERR_ARG;
    auto t0 = std::chrono::steady_clock::now();
    Cloud src = load_filtered(src6, N);
    Matcher m{p, load_filtered(tgt6, M), {}, load_tensors(tgt6, M, ten6)};
    m.tree.build(m.tgt);
    auto t1 = std::chrono::steady_clock::now();
    int32_t local[34];
    int32_t* rs = rand_state;
    if (!rs) { rand_seed(local, p->ransac_seed); rs = local; }
    Mat4 pose = mat4_identity();
    int st = IMLS_FRAME_MAX_ITERS, it = 0;
    Corr c;
    std::vector<double> s, d, n;
    for (it = 0; it < p->iterations; ++it) {
        uint64_t rej[6];
        project_all(m, src, pose.m, p->transform_normal != 0, c, rej);
        size_t nv = c.idx.size();
        if (trace) {
            std::memcpy(trace[it].reject, rej, sizeof(rej));
            trace[it].n_valid = nv;
            trace[it].n_kept = 0;
        }
        if (corr && it == corr_iter) {
            for (size_t k = 0; k < nv; ++k) {
                std::memcpy(corr + 9 * k, &c.x[3 * k], 3 * sizeof(float));
                std::memcpy(corr + 9 * k + 3, &c.y[3 * k], 3 * sizeof(float));
                std::memcpy(corr + 9 * k + 6, &c.n[3 * k], 3 * sizeof(float));
            }
            if (corr_n) *corr_n = nv;
        }
        if ((long)nv < (long)p->correspond_number) { st = IMLS_FRAME_TOO_FEW; break; }
        s.assign(c.x.begin(), c.x.end());
        d.assign(c.y.begin(), c.y.end());
        n.assign(c.n.begin(), c.n.end());
        Mat4 D;
        size_t kept = 0;
        if (!solve_dispatch(p->solve_method, s.data(), d.data(), n.data(), nullptr, nv, p, rs, D.m, &kept)) {
            st = IMLS_FRAME_SOLVE_FAILED;
            break;
        }
        pose = mat4_mul(D, pose);
        if (trace) {
            std::memcpy(trace[it].delta, D.m, sizeof(D.m));
            std::memcpy(trace[it].pose, pose.m, sizeof(pose.m));
            trace[it].n_kept = kept;
        }
        double dd = std::sqrt(std::pow(D.m[3], 2) + std::pow(D.m[7], 2) + std::pow(D.m[11], 2));
        double ct = ((D.m[0] + D.m[5] + D.m[10]) - 1.0) / 2.0;
        ct = std::min(1.0, std::max(ct, -1.0));
        double da = std::acos(ct);
        if (dd < p->delta_dist_threshold && da < p->delta_angle_threshold) { ++it; st = IMLS_FRAME_CONVERGED; break; }
    }
    auto t2 = std::chrono::steady_clock::now();
    if (iters_run) *iters_run = it;
    if (status) *status = st;
    std::memcpy(pose_out, pose.m, sizeof(pose.m));
    if (seconds_index) *seconds_index = std::chrono::duration<double>(t1 - t0).count();
    if (seconds_total) *seconds_total = std::chrono::duration<double>(t2 - t0).count();
    return IMLS_OK;
}

int oracle_tv_normals(const float* tgt6, size_t M, const float* ten6, const float* q3, size_t Q, const imls_params* p,
                      double* nrm, int32_t* found, double* tensors) {
    if (!p || !ten6 || p->tensor_k <= 0 || p->tensor_k > 64) return IMLS_ERR_ARG;
    Matcher m{p, load_filtered(tgt6, M), {}, load_tensors(tgt6, M, ten6)};
    m.tree.build(m.tgt);
    for (size_t q = 0; q < Q; ++q) {
        const double x[3] = {q3[q], q3[Q + q], q3[2 * Q + q]};
        double n[3] = {0, 0, 0};
        found[q] = m.tv_normal(x, n, tensors ? tensors + 9 * q : nullptr) ? 1 : 0;
        for (int k = 0; k < 3; ++k) nrm[3 * q + k] = n[k];
    }
    return IMLS_OK;
}

void oracle_rand_seed(int32_t* state, uint32_t seed) { rand_seed(state, seed); }

// nowPose = prevLaserPose * rPose (laser_odometry.cpp:652): Eigen's 4x4 product, k = 0..3 in order.
void oracle_chain_pose(const double prev[16], const double rel[16], double out[16]) {
    Mat4 a, b;
    std::memcpy(a.m, prev, sizeof(a.m));
    std::memcpy(b.m, rel, sizeof(b.m));
    Mat4 c = mat4_mul(a, b);
    std::memcpy(out, c.m, sizeof(c.m));
}

// savePoseToFile (saver.cpp:46-54): Eigen::Quaterniond(Matrix3d) (Eigen's quaternionbase_assign_impl
// for a 3x3: trace branch, else the largest-diagonal branch with strict '>'), then
// `std::fixed << std::setprecision(6)`: ts tx ty tz qx qy qz qw.  Returns the line length.
// saveMatchedPointsToFile (saver.cpp:113-133): `sx sy sz yx yy yz` per correspondence, the doubles
// of Eigen::Vector3d built from the float clouds, default std::ostream formatting.  x3 / y3: [n][3].
// Returns the byte count written (or needed, when it exceeds cap).
size_t oracle_format_matched(const float* x3, const float* y3, size_t n, char* buf, size_t cap) {
    std::ostringstream file;
    for (size_t i = 0; i < n; ++i) {
        const double s0 = x3[3 * i], s1 = x3[3 * i + 1], s2 = x3[3 * i + 2];
        const double m0 = y3[3 * i], m1 = y3[3 * i + 1], m2 = y3[3 * i + 2];
        file << s0 << " " << s1 << " " << s2 << " " << m0 << " " << m1 << " " << m2 << "\n";
    }
    const std::string t = file.str();
    if (buf && t.size() < cap) std::memcpy(buf, t.c_str(), t.size() + 1);
    return t.size();
}

int oracle_format_pose(const double P[16], const char* timestamp, char* buf, size_t cap) {
    auto m = [&](int r, int c) { return P[r * 4 + c]; };
    double q[4];   // x y z w
    double t = (m(0, 0) + m(1, 1)) + m(2, 2);
    if (t > 0.0) {
        t = std::sqrt(t + 1.0);
        q[3] = 0.5 * t;
        t = 0.5 / t;
        q[0] = (m(2, 1) - m(1, 2)) * t;
        q[1] = (m(0, 2) - m(2, 0)) * t;
        q[2] = (m(1, 0) - m(0, 1)) * t;
    } else {
        int i = 0;
        if (m(1, 1) > m(0, 0)) i = 1;
        if (m(2, 2) > m(i, i)) i = 2;
        const int j = (i + 1) % 3, k = (j + 1) % 3;
        t = std::sqrt(((m(i, i) - m(j, j)) - m(k, k)) + 1.0);
        q[i] = 0.5 * t;
        t = 0.5 / t;
        q[3] = (m(k, j) - m(j, k)) * t;
        q[j] = (m(j, i) + m(i, j)) * t;
        q[k] = (m(k, i) + m(i, k)) * t;
    }
    return std::snprintf(buf, cap, "%s %.6f %.6f %.6f %.6f %.6f %.6f %.6f\n", timestamp, m(0, 3), m(1, 3), m(2, 3), q[0],
                         q[1], q[2], q[3]);
}
void oracle_set_threads(int n) { g_threads = n < 1 ? 1 : n; }
void oracle_set_faithful(int on) { g_faithful = on ? 1 : 0; }
int32_t oracle_rand_next(int32_t* state) { return rand_next(state); }

int oracle_colpiv_qr_solve(const double* A, int rows, int cols, const double* b, double* x) {
    std::vector<double> a(A, A + (size_t)rows * cols), bb(b, b + rows);
    return colpiv_qr_solve(a, rows, cols, bb, x);
}
void oracle_delta_from_x(const double x[6], double delta[16]) { delta_from_x(x, delta); }
int oracle_sym_eig6(const double* H, double* evals, double* evecs) { sym_eig(6, H, evals, evecs, kDrpmEigRelTol); return 0; }

}  // extern "C"
