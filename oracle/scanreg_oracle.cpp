// scanreg_oracle.cpp — CPU restatement of the reference's upstream producer: ring-neighbourhood PCA
// normals + the geometric-features presample (scan_registration.cpp).  TEST INFRASTRUCTURE ONLY
// (see imls_oracle.h): only tests/ and bench.py's cpu_baseline leg load it, as the checker.
//
// PARITY STATUS: unpinned at two third-party boundaries (neither library is in the container):
//   - pcl::KdTreeFLANN::nearestKSearch(k=1) (FLANN KDTreeSingleIndex, eps = 0: exact), distance =
//     flann::L2_Simple<float> = ((0 + d0²) + d1²) + d2² in float, returned SQUARED; restated here as
//     an exhaustive scan of the adjacent ring (ties: lowest index — FLANN's is tree-visit order);
//   - Eigen::SelfAdjointEigenSolver<Matrix3f> (ascending eigenvalues, unit eigenvectors): restated
//     by a cyclic Jacobi in double on the float covariance, rounded to float (Eigen iterates in
//     float: the two agree to float rounding of well-separated eigenpairs).  Eigen's vectorised
//     colwise().mean() / adjoint()*matrix reductions are restated as sequential float sums.
// Build: oracle/Makefile (one .so with imls_oracle.cpp).
#include <cmath>
#include <cstddef>
#include <cstdint>
#include <vector>

#include "../include/imls_gpu.h"

namespace {

struct P3 {
    float x, y, z;
};

// flann::L2_Simple<float> over the 3 xyz dims (PCL's DefaultPointRepresentation keeps the first 3
// floats of PointXYZINormal).
inline float l2_simple(const P3& a, const P3& b) {
    float r = 0.f;
    float d = a.x - b.x;
    r += d * d;
    d = a.y - b.y;
    r += d * d;
    d = a.z - b.z;
    r += d * d;
    return r;
}

// findNearestPoint (scan_registration.cpp:117-136).
bool find_nearest(const P3& q, const P3* ring, int size, int mode, float thr, int& idx) {
    if (mode == 1) return true;   // "index": neighbour index = own index (128-130)
    int best = -1;                // an empty tree returns no result (123)
    float bd = INFINITY;
    for (int k = 0; k < size; ++k) {
        float d = l2_simple(q, ring[k]);
        if (d < bd) { bd = d; best = k; }
    }
    if (best >= 0 && bd < thr) { idx = best; return true; }   // distances[0] < knn_distance_threshold (123)
    return false;
}

// Cyclic Jacobi on a symmetric 3×3 (row-major a), ascending eigenvalues, eigenvectors as columns of
// v (column-major v[c*3+r]) — SelfAdjointEigenSolver's contract.
void eig3(const double ain[9], double ev[3], double v[9]) {
    double a[9], u[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};   // u row-major: u[r*3+c]
    for (int i = 0; i < 9; ++i) a[i] = ain[i];
    for (int sweep = 0; sweep < 50; ++sweep) {
        double off = a[1] * a[1] + a[2] * a[2] + a[5] * a[5];
        if (off < 1e-300) break;
        for (int p = 0; p < 2; ++p)
            for (int q = p + 1; q < 3; ++q) {
                double apq = a[p * 3 + q];
                if (apq == 0) continue;
                double app = a[p * 3 + p], aqq = a[q * 3 + q];
                double theta = (aqq - app) / (2 * apq);
                double t = (theta >= 0 ? 1.0 : -1.0) / (std::fabs(theta) + std::sqrt(theta * theta + 1));
                double c = 1 / std::sqrt(t * t + 1), s = t * c;
                for (int k = 0; k < 3; ++k) {
                    double akp = a[k * 3 + p], akq = a[k * 3 + q];
                    a[k * 3 + p] = c * akp - s * akq;
                    a[k * 3 + q] = s * akp + c * akq;
                }
                for (int k = 0; k < 3; ++k) {
                    double apk = a[p * 3 + k], aqk = a[q * 3 + k];
                    a[p * 3 + k] = c * apk - s * aqk;
                    a[q * 3 + k] = s * apk + c * aqk;
                }
                for (int k = 0; k < 3; ++k) {
                    double ukp = u[k * 3 + p], ukq = u[k * 3 + q];
                    u[k * 3 + p] = c * ukp - s * ukq;
                    u[k * 3 + q] = s * ukp + c * ukq;
                }
            }
    }
    int o[3] = {0, 1, 2};   // stable ascending order of the diagonal
    for (int i = 1; i < 3; ++i)
        for (int j = i; j > 0 && a[o[j] * 4] < a[o[j - 1] * 4]; --j) { int t = o[j]; o[j] = o[j - 1]; o[j - 1] = t; }
    for (int c = 0; c < 3; ++c) {
        ev[c] = a[o[c] * 4];
        for (int r = 0; r < 3; ++r) v[c * 3 + r] = u[r * 3 + o[c]];
    }
}

struct PcaOut {
    int status;             // 0 = failure (count < num), 1 = ok, 2 = plane check failed
    float l[3];             // λ1 ≥ λ2 ≥ λ3, or -1s
    float evec[9];          // column-major, as stored at 1205-1207
    float margin;           // min over the window of |dist − distance_threshold| (test tolerance aid)
};

// computeNormalPCA (scan_registration.cpp:158-229) for point j of ring i.
PcaOut compute_normal_pca(const std::vector<const P3*>& rings, const std::vector<int>& sizes, int i, int j,
                          const imls_pca_params& p) {
    PcaOut o{};
    const int w = p.window_size, st = p.iter_step;
    const int num = 3 * (int(2 * w / st) + 1);                     // 161
    std::vector<P3> pts;
    pts.reserve(num);
    for (int k = -w; k <= w; k += st)                              // 166-170
        if (j + k >= 0 && j + k < sizes[i]) pts.push_back(rings[i][j + k]);
    const int nr = (int)rings.size();
    for (int a : {i - 1, i + 1}) {                                 // 173-196: previous, then next line
        if (a < 0 || a > nr - 1) continue;
        int nb = j;
        if (find_nearest(rings[i][j], rings[a], sizes[a], p.neighbor_scan, p.knn_distance_threshold, nb))
            for (int k = -w; k <= w; k += st)
                if (nb + k >= 0 && nb + k < sizes[a]) pts.push_back(rings[a][nb + k]);
    }
    const int count = (int)pts.size();
    if (count < num) return o;                                     // 198-201 (λ = 0: failure)
    // 203-205: centroid, centred covariance / (count − 1), float
    float cx = 0.f, cy = 0.f, cz = 0.f;
    for (const P3& q : pts) { cx += q.x; cy += q.y; cz += q.z; }
    cx /= (float)count; cy /= (float)count; cz /= (float)count;
    float C[6] = {0, 0, 0, 0, 0, 0};   // xx xy xz yy yz zz
    for (const P3& q : pts) {
        float dx = q.x - cx, dy = q.y - cy, dz = q.z - cz;
        C[0] += dx * dx; C[1] += dx * dy; C[2] += dx * dz;
        C[3] += dy * dy; C[4] += dy * dz; C[5] += dz * dz;
    }
    const float den = float(count - 1);
    for (float& c : C) c /= den;
    const double A[9] = {C[0], C[1], C[2], C[1], C[3], C[4], C[2], C[4], C[5]};
    double ev[3], V[9];
    eig3(A, ev, V);                                                // 207-209
    float evf[3], Vf[9];
    for (int k = 0; k < 3; ++k) evf[k] = (float)ev[k];
    for (int k = 0; k < 9; ++k) Vf[k] = (float)V[k];
    // checkPlaneValidity (138-156) with normal = col(0), centroid recomputed over the same rows
    int valid = 0;
    float margin = INFINITY;
    for (const P3& q : pts) {
        float dx = q.x - cx, dy = q.y - cy, dz = q.z - cz;
        float dist = std::fabs(Vf[0] * dx + Vf[1] * dy + Vf[2] * dz);
        if (dist < p.distance_threshold) valid++;
        margin = std::fmin(margin, std::fabs(dist - p.distance_threshold));
    }
    o.margin = margin;
    for (int k = 0; k < 9; ++k) o.evec[k] = Vf[k];
    if (!((float)valid >= p.valid_points_threshold * (float)count)) {   // 215-219: λ = -1, no swap
        o.status = 2;
        o.l[0] = o.l[1] = o.l[2] = -1.f;
        return o;
    }
    o.status = 1;
    o.l[0] = evf[2]; o.l[1] = evf[1]; o.l[2] = evf[0];             // 223-225
    for (int r = 0; r < 3; ++r) { o.evec[r] = Vf[6 + r]; o.evec[6 + r] = Vf[r]; }   // 228: swap cols 0, 2
    return o;
}

}  // namespace

extern "C" {

// The "pca" branch of scan_registration.cpp:1136-1229 + computeGeometricFeatures (279-327) + the
// invalid-index erase (1481-1489).  Same outputs as imls_ring_normals_pca (include/imls_gpu.h), plus
// margin_out[r] = the plane check's distance margin (tests tolerate flips only where it is tiny).
int oracle_ring_pca(const float* xyz, size_t stride, const int32_t* ring_sizes, int32_t n_rings,
                    const imls_pca_params* p, uint32_t* index_out, float* normal_out, float* evals_out,
                    float* evecs_out, float* features_out, uint8_t* flags_out, float* margin_out, size_t* n_out,
                    uint64_t counters[2]) {
    std::vector<int> sizes(ring_sizes, ring_sizes + n_rings), start(n_rings + 1, 0);
    for (int i = 0; i < n_rings; ++i) start[i + 1] = start[i] + sizes[i];
    std::vector<P3> cloud(start[n_rings]);
    for (int k = 0; k < start[n_rings]; ++k) cloud[k] = {xyz[k * stride], xyz[k * stride + 1], xyz[k * stride + 2]};
    std::vector<const P3*> rings(n_rings);
    for (int i = 0; i < n_rings; ++i) rings[i] = cloud.data() + start[i];
    uint64_t fail = 0, invalid = 0;
    size_t r = 0;
    for (int i = 1; i < n_rings - 1; ++i) {                                        // 1162
        if (sizes[i] == 0) continue;                                               // 1164-1165
        // scanEndInd − scanStartInd = size − 11 (1066-1068) must be ≥ 6 for lines i−1, i, i+1 (1166)
        if (sizes[i] - 11 < 6 || sizes[i - 1] - 11 < 6 || sizes[i + 1] - 11 < 6) continue;
        for (int j = 5; j < sizes[i] - 5; ++j) {                                   // 1170
            PcaOut o = compute_normal_pca(rings, sizes, i, j, *p);
            if (o.status == 0) { fail++; continue; }                               // 1177-1181
            if (o.status == 2) {
                invalid++;
                if (!p->use_all_points) continue;                                  // 1184-1191
            }
            // 1196-1200: normal = eigen_vectors.col(2).normalized(), flipped towards +z
            float nx = o.evec[6], ny = o.evec[7], nz = o.evec[8];
            float z2 = nx * nx + ny * ny + nz * nz;
            if (z2 > 0.f) { float s = std::sqrt(z2); nx /= s; ny /= s; nz /= s; }
            if (nz < 0.f) { nx = -nx; ny = -ny; nz = -nz; }
            const float l1 = o.l[0], l2 = o.l[1], l3 = o.l[2];
            // computeGeometricFeatures (295-319), float array arithmetic
            const float f[8] = {l1 + l2 + l3,
                                std::pow(l1 * l2 * l3, 1.0f / 3.0f),
                                -(l1 * std::log(l1) + l2 * std::log(l2) + l3 * std::log(l3)),
                                (l1 - l3) / l1,
                                (l1 - l2) / l1,
                                (l2 - l3) / l1,
                                l3 / (l1 + l2 + l3),
                                l3 / l1};
            uint8_t fl = (o.status == 2) ? IMLS_PCA_PLANE_INVALID : 0;
            if (f[5] > p->planarity_threshold && !(o.status == 2 && p->use_all_points)) fl |= IMLS_PCA_CANDIDATE;
            if (index_out) index_out[r] = (uint32_t)(start[i] + 5 + j);           // 1194 (Q-SR1)
            if (normal_out) { normal_out[3 * r] = nx; normal_out[3 * r + 1] = ny; normal_out[3 * r + 2] = nz; }
            if (evals_out) for (int k = 0; k < 3; ++k) evals_out[3 * r + k] = o.l[k];
            if (evecs_out) for (int k = 0; k < 9; ++k) evecs_out[9 * r + k] = o.evec[k];
            if (features_out) for (int k = 0; k < 8; ++k) features_out[8 * r + k] = f[k];
            if (flags_out) flags_out[r] = fl;
            if (margin_out) margin_out[r] = o.margin;
            r++;
        }
    }
    if (n_out) *n_out = r;
    if (counters) { counters[0] = fail; counters[1] = invalid; }
    return 0;
}

}  // extern "C"
