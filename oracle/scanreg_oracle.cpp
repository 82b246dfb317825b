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
#include <algorithm>
#include <cmath>
#include <cstddef>
#include <cstdint>
#include <limits>
#include <random>
#include <vector>

#include "../include/imls_gpu.h"

extern "C" int32_t oracle_rand_next(int32_t* state);   // glibc rand() restatement (imls_oracle.cpp)
extern "C" void oracle_rand_seed(int32_t* state, uint32_t seed);

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

// ---- samplePointCloud: "normal" / "major_axis" (scan_registration.cpp:536-806, common.cpp:19-82) ----
//
// Further unpinned semantics, beyond the two above: randomSampling seeds a fresh std::mt19937 from
// std::random_device per call (571-572) — restated with the seed shuffle_seed + k for the k-th call
// (same libstdc++ std::shuffle); farthestPointSampling's first index is rand() % n from the
// process-wide glibc stream — restated from srand(rand_seed) per call.  Eigen float/double 3-vector
// norms: Vector3f.norm() = sqrt(c0 + (c1 + c2)) (Redux.h non-vectorised unroller, size 3 < 4 floats),
// Vector3d.norm() = sqrt((c0 + c1) + c2) (SSE2: one 2-double packet + the tail).

struct SampleCloud {
    const float* xyz;
    const float* nrm;
    size_t stride;
    P3 p(size_t i) const { return {xyz[i * stride], xyz[i * stride + 1], xyz[i * stride + 2]}; }
    P3 n(size_t i) const { return {nrm[i * stride], nrm[i * stride + 1], nrm[i * stride + 2]}; }
};

inline float norm3f(float a, float b, float c) { return std::sqrt(a * a + (b * b + c * c)); }
inline double norm3d(double a, double b, double c) { return std::sqrt((a * a + b * b) + c * c); }

// computeSphericalHistogram (536-564): bins[az * elevation_bins + el] = candidate indices, in order.
std::vector<std::vector<int>> spherical_histogram(const SampleCloud& c, const int32_t* cand, size_t n_cand, int az_bins,
                                                  int el_bins) {
    std::vector<std::vector<int>> h((size_t)az_bins * el_bins);
    for (size_t k = 0; k < n_cand; ++k) {
        const int idx = cand[k];
        const P3 nn = c.n(idx);
        float azimuth = std::atan2(nn.y, nn.x);        // `using std::atan2` (51): the float overload
        float elevation = (float)::asin((double)nn.z); // ::asin(double) (no float overload in scope)
        if (azimuth < 0) azimuth += 2 * M_PI;
        elevation += M_PI / 2;
        const int ai = std::min(static_cast<int>(azimuth / (2 * M_PI / az_bins)), az_bins - 1);
        const int ei = std::min(static_cast<int>(elevation / (M_PI / el_bins)), el_bins - 1);
        h[(size_t)ai * el_bins + ei].push_back(idx);
    }
    return h;
}

struct Rng {
    uint32_t shuffle_seed;
    uint32_t calls = 0;
    int32_t glibc[34];
};

// randomSampling (566-582)
void random_sampling(const std::vector<int>& cand, int max_points, std::vector<int>& out, Rng& rng) {
    std::mt19937 gen(rng.shuffle_seed + rng.calls++);
    std::vector<int> sh = cand;
    std::shuffle(sh.begin(), sh.end(), gen);
    const int cnt = std::min(max_points, (int)sh.size());
    for (int i = 0; i < cnt; ++i) out.push_back(sh[i]);
}

// farthestPointSampling (common.cpp:19-82) over the sub-cloud `pts` (indices into c)
void farthest_point_sampling(const SampleCloud& c, const std::vector<int>& pts, int num_samples, std::vector<int>& out,
                             Rng& rng) {
    const int n = (int)pts.size();
    std::vector<double> md(n, INFINITY);
    std::vector<char> taken(n, 0);
    const int first = oracle_rand_next(rng.glibc) % n;            // 49
    out.push_back(first);
    taken[first] = 1;
    const P3 f = c.p(pts[first]);
    for (int i = 0; i < n; ++i) {
        const P3 q = c.p(pts[i]);
        md[i] = norm3d((double)f.x - q.x, (double)f.y - q.y, (double)f.z - q.z);
    }
    for (int s = 1; s < num_samples; ++s) {                        // 59-81
        double best = -1.0;
        int bi = -1;
        for (int i = 0; i < n; ++i)
            if (!taken[i] && md[i] > best) { best = md[i]; bi = i; }
        out.push_back(bi);
        taken[bi] = 1;
        const P3 b = c.p(pts[bi]);
        for (int i = 0; i < n; ++i) {
            const P3 q = c.p(pts[i]);
            md[i] = std::min(md[i], norm3d((double)b.x - q.x, (double)b.y - q.y, (double)b.z - q.z));
        }
    }
}

// the shared "sample a bin down to k points" step of normalSampling (603-622) / majorAxisSampling (735-752)
void sample_bin(const SampleCloud& c, const std::vector<int>& bin, int k, int strategy, std::vector<int>& out, Rng& rng) {
    if (strategy == 0) {
        std::vector<int> loc;
        farthest_point_sampling(c, bin, k, loc, rng);
        for (int b : loc) out.push_back(bin[b]);
    } else {
        random_sampling(bin, k, out, rng);
    }
}

// static_cast<int>(double) as the reference's x86-64 build evaluates it (cvttsd2si): truncation,
// INT_MIN for NaN / out of range (spelled out: the C++ cast is undefined there)
inline int x86_d2i(double v) {
    if (!(v > -2147483649.0 && v < 2147483648.0)) return INT32_MIN;
    return (int)v;
}

}  // namespace

extern "C" {

// scan_registration.cpp:laserCloudHandler front end, line by line: pcl::removeNaNFromPointCloud
// (862; a dense cloud is copied unchanged), removeClosedPointCloud (87-115, 863), startOri / endOri
// (899-912), the per-point ring + azimuth loop with the sequential halfPassed switch (940-1058; the
// std:: float overloads of sqrt / atan / atan2 = glibc sqrtf / atanf / atan2f), and laserCloud = the
// rings concatenated (1064-1069).  Outputs as imls_scan_front_end.
int oracle_scan_front_end(const imls_front_params* p, const float* xyz, size_t stride, size_t n, float* out_xyzi,
                          uint32_t* out_index, int32_t* ring_sizes, size_t* n_out) {
    const int NS = p->n_scans;
    *n_out = 0;
    if (NS != 16 && NS != 32 && NS != 64) return -1;
    for (int r = 0; r < NS; ++r) ring_sizes[r] = 0;
    struct Pt { float x, y, z; uint32_t i; };
    std::vector<Pt> in;
    for (size_t i = 0; i < n; ++i) {
        const float* q = xyz + i * stride;
        if (!p->is_dense && (!std::isfinite(q[0]) || !std::isfinite(q[1]) || !std::isfinite(q[2]))) continue;
        in.push_back({q[0], q[1], q[2], (uint32_t)i});
    }
    std::vector<Pt> kept;
    const float mn = p->minimum_range, mx = p->maximum_range;
    for (const Pt& q : in) {
        if (q.x * q.x + q.y * q.y + q.z * q.z < mn * mn || q.x * q.x + q.y * q.y + q.z * q.z > mx * mx) continue;
        kept.push_back(q);
    }
    const int cloudSize = (int)kept.size();
    if (cloudSize == 0) return 0;
    float startOri = -std::atan2(kept[0].y, kept[0].x);
    float endOri = -std::atan2(kept[cloudSize - 1].y, kept[cloudSize - 1].x) + 2 * M_PI;
    if (endOri - startOri > 3 * M_PI) endOri -= 2 * M_PI;
    else if (endOri - startOri < M_PI) endOri += 2 * M_PI;
    bool halfPassed = false;
    float upperBound = 0.f, lowerBound = 0.f;
    if (NS == 32) { upperBound = 15.0f; lowerBound = -25.0f; }
    else if (NS == 64) { upperBound = 2.0f; lowerBound = -24.33f; }
    static const std::vector<float> scanAngles = {-25.000, -15.639, -11.310, -8.843, -7.254, -6.148, -5.333,
                                                  -4.667,  -4.000,  -3.667,  -3.333, -3.000, -2.667, -2.333,
                                                  -2.000,  -1.667,  -1.333,  -1.000, -0.667, -0.333, 0.000,
                                                  0.333,   0.667,   1.000,   1.333,  1.667,  2.333};
    const float scanPeriod = p->scan_period;
    std::vector<std::vector<std::pair<Pt, float>>> scans(NS);
    for (int i = 0; i < cloudSize; i++) {
        Pt point = kept[i];
        float range = std::sqrt(point.x * point.x + point.y * point.y);
        float vertical_angle = std::atan(point.z / range);
        float angle = vertical_angle * 180 / M_PI;
        int scanID = 0;
        if (NS == 16) {
            scanID = x86_d2i((angle + 15) / 2 + 0.5);
            if (scanID > (NS - 1) || scanID < 0) continue;
        } else if (NS == 32) {
            float min_diff = std::numeric_limits<float>::max();
            for (size_t j = 0; j < scanAngles.size(); j++) {
                float diff = std::abs(angle - scanAngles[j]);
                if (diff < min_diff) { min_diff = diff; scanID = (int)j; }
            }
            if (scanID > (NS - 1) || scanID < 0) continue;
        } else {
            if (angle >= -8.83) scanID = x86_d2i((upperBound - angle) * 3.0 + 0.5);
            else scanID = (int)((unsigned)(NS / 2) + (unsigned)x86_d2i((-8.83 - angle) * 2.0 + 0.5));
            if (angle > upperBound || angle < lowerBound || scanID > 50 || scanID < 0) continue;
        }
        float ori = -std::atan2(point.y, point.x);
        if (!halfPassed) {
            if (ori < startOri - M_PI / 2) ori += 2 * M_PI;
            else if (ori > startOri + M_PI * 3 / 2) ori -= 2 * M_PI;
            if (ori - startOri > M_PI) halfPassed = true;
        } else {
            ori += 2 * M_PI;
            if (ori < endOri - M_PI * 3 / 2) ori += 2 * M_PI;
            else if (ori > endOri + M_PI / 2) ori -= 2 * M_PI;
        }
        float relTime = (ori - startOri) / (endOri - startOri);
        float intensity = scanID + scanPeriod * relTime;
        scans[scanID].push_back({point, intensity});
    }
    size_t k = 0;
    for (int r = 0; r < NS; ++r) {
        ring_sizes[r] = (int32_t)scans[r].size();
        for (const auto& e : scans[r]) {
            out_xyzi[4 * k] = e.first.x; out_xyzi[4 * k + 1] = e.first.y; out_xyzi[4 * k + 2] = e.first.z;
            out_xyzi[4 * k + 3] = e.second;
            if (out_index) out_index[k] = e.first.i;
            ++k;
        }
    }
    *n_out = k;
    return 0;
}


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

// samplePointCloud for "normal" / "major_axis" (scan_registration.cpp:761-806).  Same contract as
// imls_sample_point_cloud (include/imls_gpu.h).
int oracle_sample_point_cloud(const imls_sample_params* p, const float* xyz, const float* nrm, size_t stride, size_t n,
                              const int32_t* cand, size_t n_cand, const float* last_xyz, size_t last_stride, size_t m,
                              int32_t* sampled_out, size_t* n_sampled, float* bin_weights_out) {
    const SampleCloud c{xyz, nrm, stride};
    const int nb = p->azimuth_bins * p->elevation_bins;
    auto hist = spherical_histogram(c, cand, n_cand, p->azimuth_bins, p->elevation_bins);
    Rng rng{};
    rng.shuffle_seed = p->shuffle_seed;
    oracle_rand_seed(rng.glibc, p->rand_seed);
    std::vector<int> out;
    std::vector<float> w(nb, 0.0f);
    if (p->method == IMLS_SAMPLE_NORMAL) {                         // normalSampling (584-629)
        for (int b = 0; b < nb; ++b) {
            const auto& bin = hist[b];
            const int sz = (int)bin.size();
            if (sz < p->min_points_per_bin) continue;
            if (sz > p->max_points_per_bin) sample_bin(c, bin, p->max_points_per_bin, p->sampling_strategy, out, rng);
            else out.insert(out.end(), bin.begin(), bin.end());
        }
    } else {                                                       // majorAxisSampling (631-759)
        for (int b = 0; b < nb; ++b) {
            const auto& bin = hist[b];
            const int sz = (int)bin.size();
            if (sz < p->min_points_per_bin) continue;
            std::vector<int> sub;
            if (sz > p->max_points_per_bin) random_sampling(bin, p->max_points_per_bin, sub, rng);
            else sub = bin;
            std::vector<float> distances(sub.size(), 0.0f);
            int valid = 0;
            for (int idx : sub) {                                  // 670-702
                const P3 pt = c.p(idx), nn = c.n(idx);
                int cnt = 0;
                for (size_t j = 0; j < m; ++j) {                   // 679-686
                    const float dx = pt.x - last_xyz[j * last_stride], dy = pt.y - last_xyz[j * last_stride + 1],
                                dz = pt.z - last_xyz[j * last_stride + 2];
                    const float cx = dy * nn.z - dz * nn.y, cy = dz * nn.x - dx * nn.z, cz = dx * nn.y - dy * nn.x;
                    if (norm3f(dx, dy, dz) < p->r_proj && norm3f(cx, cy, cz) < p->r) cnt++;
                }
                if (cnt >= 3) {                                    // 689-701
                    float avg = 0.0f;
                    for (size_t j = 0; j < m; ++j) {
                        const float dx = pt.x - last_xyz[j * last_stride], dy = pt.y - last_xyz[j * last_stride + 1],
                                    dz = pt.z - last_xyz[j * last_stride + 2];
                        const float cx = dy * nn.z - dz * nn.y, cy = dz * nn.x - dx * nn.z, cz = dx * nn.y - dy * nn.x;
                        if (norm3f(dx, dy, dz) < p->r_proj && norm3f(cx, cy, cz) < p->r) avg += norm3f(dx, dy, dz);
                    }
                    avg /= (float)cnt;
                    distances[valid++] = avg;
                }
            }
            if (valid >= 3) {                                      // 704-711
                float total = 0.0f;
                for (float d : distances) total += d;
                w[b] = total / valid;
            }
        }
        float tw = 0.0f;                                           // 715-723
        for (float x : w) tw += x;
        for (float& x : w) x /= tw;
        for (int b = 0; b < nb; ++b) {                             // 726-758
            const auto& bin = hist[b];
            const int sz = (int)bin.size();
            if (sz < p->min_points_per_bin) continue;
            const float wk = w[b] * p->max_total_points;        // x86 cvttss2si: NaN / out of range → INT_MIN
            const int k = std::min((wk > -2147483904.0f && wk < 2147483648.0f) ? static_cast<int>(wk) : INT32_MIN, sz);
            if (sz > k) sample_bin(c, bin, k, p->sampling_strategy, out, rng);
            else out.insert(out.end(), bin.begin(), bin.end());
        }
    }
    for (size_t k = 0; k < out.size(); ++k) sampled_out[k] = out[k];
    if (n_sampled) *n_sampled = out.size();
    if (bin_weights_out) for (int b = 0; b < nb; ++b) bin_weights_out[b] = w[b];
    return 0;
}

}  // extern "C"
