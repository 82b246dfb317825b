// scanreg.hip — the upstream producer's per-point normal estimation on gfx950: ring-neighbourhood
// PCA normals (scan_registration.cpp:1136-1229, computeNormalPCA 158-229, findNearestPoint 117-136,
// checkPlaneValidity 138-156) fused with the geometric-features presample (computeGeometricFeatures
// 279-327; invalid-index erase 1481-1489).
//
// Layout: the ring-concatenated cloud `laserCloud` (1064-1069) as float4 (x, y, z, 0) in HBM, ring
// offsets ring_off[n_rings + 1].  One block = 256 consecutive centre points j of one scan line i
// (a host-built block table covers exactly the (i, j) the reference visits: lines 1 … N−2 whose
// own and adjacent line sizes pass the scanEndInd − scanStartInd ≥ 6 test, j ∈ [5, size−6]).
//
// Per block: the NN-1 of every centre in line i−1 and line i+1 ("kdtree" mode) is an exact
// exhaustive scan of that line staged through LDS in 2048-point tiles (every lane reads the same LDS
// word: broadcast, no bank conflicts); float L2 evaluated exactly as flann::L2_Simple<float>
// ((0 + d0²) + d1²) + d2² with no contraction (-ffp-contract=off), strict < in ascending index order
// (ties → lowest index).  Then the ≤ 3·(2w/s + 1) window points are re-read from HBM/L2 three times
// (centroid, covariance, plane check — float sums in the reference's row order), the 3×3 covariance
// is diagonalised by cyclic Jacobi in fp64 and rounded to float, and the outputs (normal, λ, the
// eigenvector matrix, 8 features, flags) are written per slot; an order-keeping compaction (hipcub
// exclusive scan + scatter) yields filteredLaserCloud's row order.
//
// Roofline: VALU-bound (the exhaustive NN is ~10 flop per (centre, adjacent-line point) pair:
// 2·|line| pairs per centre); HBM traffic is ~100 B per point (read 16, write ~96).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <string>
#include <vector>

#include "internal.h"

namespace imlsgpu {
namespace {

constexpr int kPcaBlock = 256;
constexpr int kPcaTile = 2048;         // adjacent-line points per LDS tile (32 KB)
constexpr int kPcaOutF = 23;           // per-slot floats: normal 3, λ 3, eigenvectors 9, features 8

__device__ __forceinline__ float l2_simple(float qx, float qy, float qz, float4 p) {
    float r = 0.f;
    float d = qx - p.x;
    r = __fadd_rn(r, __fmul_rn(d, d));
    d = qy - p.y;
    r = __fadd_rn(r, __fmul_rn(d, d));
    d = qz - p.z;
    r = __fadd_rn(r, __fmul_rn(d, d));
    return r;
}

// Cyclic Jacobi on a symmetric 3×3 (row-major), ascending eigenvalues, unit eigenvectors as
// columns (v column-major) — Eigen::SelfAdjointEigenSolver's contract, restated in fp64.
__device__ void eig3(double a[9], double ev[3], double v[9]) {
    double u[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
    for (int sweep = 0; sweep < 50; ++sweep) {
        const double off = a[1] * a[1] + a[2] * a[2] + a[5] * a[5];
        if (off < 1e-300) break;
#pragma unroll
        for (int p = 0; p < 2; ++p)
#pragma unroll
            for (int q = p + 1; q < 3; ++q) {
                const double apq = a[p * 3 + q];
                if (apq == 0) continue;
                const double app = a[p * 3 + p], aqq = a[q * 3 + q];
                const double theta = (aqq - app) / (2 * apq);
                const double t = (theta >= 0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1));
                const double c = 1 / sqrt(t * t + 1), s = t * c;
#pragma unroll
                for (int k = 0; k < 3; ++k) {
                    const double akp = a[k * 3 + p], akq = a[k * 3 + q];
                    a[k * 3 + p] = c * akp - s * akq;
                    a[k * 3 + q] = s * akp + c * akq;
                }
#pragma unroll
                for (int k = 0; k < 3; ++k) {
                    const double apk = a[p * 3 + k], aqk = a[q * 3 + k];
                    a[p * 3 + k] = c * apk - s * aqk;
                    a[q * 3 + k] = s * apk + c * aqk;
                }
#pragma unroll
                for (int k = 0; k < 3; ++k) {
                    const double ukp = u[k * 3 + p], ukq = u[k * 3 + q];
                    u[k * 3 + p] = c * ukp - s * ukq;
                    u[k * 3 + q] = s * ukp + c * ukq;
                }
            }
    }
    int o0 = 0, o1 = 1, o2 = 2;   // stable ascending order of the diagonal (insertion sort)
    if (a[o1 * 4] < a[o0 * 4]) { int t = o0; o0 = o1; o1 = t; }
    if (a[o2 * 4] < a[o1 * 4]) {
        int t = o1; o1 = o2; o2 = t;
        if (a[o1 * 4] < a[o0 * 4]) { t = o0; o0 = o1; o1 = t; }
    }
    const int o[3] = {o0, o1, o2};
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        ev[c] = a[o[c] * 4];
#pragma unroll
        for (int r = 0; r < 3; ++r) v[c * 3 + r] = u[r * 3 + o[c]];
    }
}

// NN-1 of (qx,qy,qz) among line [b, b + n) — all lanes of the block cooperate on the LDS staging.
__device__ void nn_scan(const float4* __restrict__ pts, int b, int n, float qx, float qy, float qz, bool active,
                        float4* tile, float& bd, int& best) {
    bd = INFINITY;
    best = -1;
    for (int base = 0; base < n; base += kPcaTile) {
        const int m = min(kPcaTile, n - base);
        __syncthreads();
        for (int k = threadIdx.x; k < m; k += kPcaBlock) tile[k] = pts[b + base + k];
        __syncthreads();
        if (active)
            for (int k = 0; k < m; ++k) {
                const float d = l2_simple(qx, qy, qz, tile[k]);
                if (d < bd) { bd = d; best = base + k; }
            }
    }
}

struct Seg {
    int b, n, c;   // line start, line size, window centre (-1: absent)
};

__global__ __launch_bounds__(kPcaBlock) void k_ring_pca(const float4* __restrict__ pts, const int* __restrict__ ring_off,
                                                        int n_rings, const int2* __restrict__ blocks,
                                                        imls_pca_params p, float* __restrict__ outf,
                                                        unsigned* __restrict__ keep, unsigned char* __restrict__ flags,
                                                        int n_total, unsigned long long* __restrict__ counters) {
    __shared__ float4 tile[kPcaTile];
    const int2 blk = blocks[blockIdx.x];
    const int i = blk.x;
    const int bi = ring_off[i], si = ring_off[i + 1] - bi;
    const int j = blk.y + (int)threadIdx.x;
    const bool active = j < si - 5;
    const float4 q = pts[bi + min(j, si - 1)];
    Seg seg[3];
    seg[0] = {bi, si, j};
    for (int s = 1; s < 3; ++s) {
        const int a = s == 1 ? i - 1 : i + 1;   // previous line, then next (173-196)
        seg[s] = {0, 0, -1};
        if (a < 0 || a > n_rings - 1) continue;
        const int ba = ring_off[a], sa = ring_off[a + 1] - ba;
        if (p.neighbor_scan == 1) {              // "index": own index (128-130)
            seg[s] = {ba, sa, j};
        } else {                                 // "kdtree": exact NN-1, squared float distance (117-127)
            float bd;
            int best;
            nn_scan(pts, ba, sa, q.x, q.y, q.z, active, tile, bd, best);
            if (best >= 0 && bd < p.knn_distance_threshold) seg[s] = {ba, sa, best};
        }
    }
    if (!active) return;
    const int slot = bi + j;
    const int w = p.window_size, st = p.iter_step;
    const int num = 3 * (int(2 * w / st) + 1);   // 161
    // pass 1: count + centroid (203), float, rows in the reference's push order
    int count = 0;
    float cx = 0.f, cy = 0.f, cz = 0.f;
    for (int s = 0; s < 3; ++s) {
        if (seg[s].c < 0) continue;
        for (int k = -w; k <= w; k += st) {
            const int t = seg[s].c + k;
            if (t < 0 || t >= seg[s].n) continue;
            const float4 v = pts[seg[s].b + t];
            cx = __fadd_rn(cx, v.x); cy = __fadd_rn(cy, v.y); cz = __fadd_rn(cz, v.z);
            count++;
        }
    }
    if (count < num) {                               // 198-201: pca failure, the point is skipped
        atomicAdd(&counters[0], 1ull);
        keep[slot] = 0u;
        return;
    }
    cx = __fdiv_rn(cx, (float)count); cy = __fdiv_rn(cy, (float)count); cz = __fdiv_rn(cz, (float)count);
    // pass 2: covariance / (count − 1) (204-205)
    float C0 = 0.f, C1 = 0.f, C2 = 0.f, C3 = 0.f, C4 = 0.f, C5 = 0.f;
    for (int s = 0; s < 3; ++s) {
        if (seg[s].c < 0) continue;
        for (int k = -w; k <= w; k += st) {
            const int t = seg[s].c + k;
            if (t < 0 || t >= seg[s].n) continue;
            const float4 v = pts[seg[s].b + t];
            const float dx = v.x - cx, dy = v.y - cy, dz = v.z - cz;
            C0 = __fadd_rn(C0, __fmul_rn(dx, dx)); C1 = __fadd_rn(C1, __fmul_rn(dx, dy));
            C2 = __fadd_rn(C2, __fmul_rn(dx, dz)); C3 = __fadd_rn(C3, __fmul_rn(dy, dy));
            C4 = __fadd_rn(C4, __fmul_rn(dy, dz)); C5 = __fadd_rn(C5, __fmul_rn(dz, dz));
        }
    }
    const float den = (float)(count - 1);
    C0 = __fdiv_rn(C0, den); C1 = __fdiv_rn(C1, den); C2 = __fdiv_rn(C2, den);
    C3 = __fdiv_rn(C3, den); C4 = __fdiv_rn(C4, den); C5 = __fdiv_rn(C5, den);
    double A[9] = {C0, C1, C2, C1, C3, C4, C2, C4, C5};
    double ev[3], V[9];
    eig3(A, ev, V);                                  // 207-209
    float Vf[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) Vf[k] = (float)V[k];
    // pass 3: checkPlaneValidity with normal = col(0) (138-156, 212-219)
    int valid = 0;
    for (int s = 0; s < 3; ++s) {
        if (seg[s].c < 0) continue;
        for (int k = -w; k <= w; k += st) {
            const int t = seg[s].c + k;
            if (t < 0 || t >= seg[s].n) continue;
            const float4 v = pts[seg[s].b + t];
            const float dx = v.x - cx, dy = v.y - cy, dz = v.z - cz;
            const float dist = fabsf(__fadd_rn(__fadd_rn(__fmul_rn(Vf[0], dx), __fmul_rn(Vf[1], dy)), __fmul_rn(Vf[2], dz)));
            if (dist < p.distance_threshold) valid++;
        }
    }
    const bool invalid = !((float)valid >= __fmul_rn(p.valid_points_threshold, (float)count));
    float l1, l2, l3, E[9];
    if (invalid) {                                   // 215-218: λ = -1, eigenvectors unswapped
        atomicAdd(&counters[1], 1ull);
        l1 = l2 = l3 = -1.f;
#pragma unroll
        for (int k = 0; k < 9; ++k) E[k] = Vf[k];
        if (!p.use_all_points) { keep[slot] = 0u; return; }   // 1189-1190
    } else {                                         // 223-228: descending, columns 0 ↔ 2 swapped
        l1 = (float)ev[2]; l2 = (float)ev[1]; l3 = (float)ev[0];
#pragma unroll
        for (int r = 0; r < 3; ++r) { E[r] = Vf[6 + r]; E[3 + r] = Vf[3 + r]; E[6 + r] = Vf[r]; }
    }
    // 1196-1200: normal = col(2).normalized(), flipped towards +z
    float nx = E[6], ny = E[7], nz = E[8];
    const float z2 = __fadd_rn(__fadd_rn(__fmul_rn(nx, nx), __fmul_rn(ny, ny)), __fmul_rn(nz, nz));
    if (z2 > 0.f) {
        const float sq = (float)__dsqrt_rn((double)z2);   // correctly rounded (v_sqrt_f32 is 1 ulp)
        nx = __fdiv_rn(nx, sq); ny = __fdiv_rn(ny, sq); nz = __fdiv_rn(nz, sq);
    }
    if (nz < 0.f) { nx = -nx; ny = -ny; nz = -nz; }
    // computeGeometricFeatures (295-319)
    const float sum = __fadd_rn(__fadd_rn(l1, l2), l3);
    const float f[8] = {sum,
                        powf(__fmul_rn(__fmul_rn(l1, l2), l3), 1.0f / 3.0f),
                        -(__fadd_rn(__fadd_rn(__fmul_rn(l1, logf(l1)), __fmul_rn(l2, logf(l2))), __fmul_rn(l3, logf(l3)))),
                        __fdiv_rn(l1 - l3, l1),
                        __fdiv_rn(l1 - l2, l1),
                        __fdiv_rn(l2 - l3, l1),
                        __fdiv_rn(l3, sum),
                        __fdiv_rn(l3, l1)};
    unsigned char fl = invalid ? (unsigned char)IMLS_PCA_PLANE_INVALID : (unsigned char)0;
    if (f[5] > p.planarity_threshold && !invalid) fl |= (unsigned char)IMLS_PCA_CANDIDATE;   // 323, 1481-1489
    // per-slot record, SoA [23][n_total] (coalesced across the block's consecutive slots)
    float* o = outf + slot;
    o[0] = nx; o[(size_t)1 * n_total] = ny; o[(size_t)2 * n_total] = nz;
    o[(size_t)3 * n_total] = l1; o[(size_t)4 * n_total] = l2; o[(size_t)5 * n_total] = l3;
#pragma unroll
    for (int k = 0; k < 9; ++k) o[(size_t)(6 + k) * n_total] = E[k];
#pragma unroll
    for (int k = 0; k < 8; ++k) o[(size_t)(15 + k) * n_total] = f[k];
    flags[slot] = fl;
    keep[slot] = 1u;
}

// Order-keeping compaction into the reference's row order (filteredLaserCloud push order).
__global__ void k_pca_scatter(const float* __restrict__ outf, const unsigned* __restrict__ keep,
                              const unsigned* __restrict__ pos, const unsigned char* __restrict__ flags,
                              const int* __restrict__ slot_ring, const int* __restrict__ ring_off, int n_total,
                              unsigned* __restrict__ idx_c, float* __restrict__ nrm_c, float* __restrict__ ev_c,
                              float* __restrict__ evec_c, float* __restrict__ feat_c, unsigned char* __restrict__ fl_c) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= n_total || !keep[s]) return;
    const unsigned r = pos[s];
    idx_c[r] = (unsigned)(s + 5);   // filteredIndices = scanStartInd[i] + j = slot + 5 (1066, 1194: Q-SR1)
    for (int k = 0; k < 3; ++k) nrm_c[3 * (size_t)r + k] = outf[(size_t)k * n_total + s];
    for (int k = 0; k < 3; ++k) ev_c[3 * (size_t)r + k] = outf[(size_t)(3 + k) * n_total + s];
    for (int k = 0; k < 9; ++k) evec_c[9 * (size_t)r + k] = outf[(size_t)(6 + k) * n_total + s];
    for (int k = 0; k < 8; ++k) feat_c[8 * (size_t)r + k] = outf[(size_t)(15 + k) * n_total + s];
    fl_c[r] = flags[s];
    (void)slot_ring;
    (void)ring_off;
}

size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

}  // namespace

// Host side of imls_ring_normals_pca: upload, the block table, the PCA kernel (bracketed by
// marks[0..1] when non-null), the compaction, and the D2H of the requested outputs.
int ring_pca_run(hipStream_t s, const imls_pca_params& p, const float* xyz, size_t stride, const int32_t* sizes,
                 int n_rings, DevBuf& mem, hipEvent_t* marks, uint32_t* index_out, float* normal_out,
                 float* evals_out, float* evecs_out, float* features_out, uint8_t* flags_out, size_t* n_out,
                 uint64_t counters[2], std::string& err) {
    std::vector<int> off(n_rings + 1, 0);
    for (int i = 0; i < n_rings; ++i) {
        if (sizes[i] < 0 || sizes[i] > (1 << 20)) { err = "ring size out of range"; return IMLS_ERR_ARG; }
        off[i + 1] = off[i] + sizes[i];
    }
    const int n = off[n_rings];
    // the (line, first centre) of every block: lines 1 … N−2 (1162), size tests (1164-1167), j ∈ [5, size−6] (1170)
    std::vector<int2> blocks;
    for (int i = 1; i < n_rings - 1; ++i) {
        if (sizes[i] == 0) continue;
        if (sizes[i] - 11 < 6 || sizes[i - 1] - 11 < 6 || sizes[i + 1] - 11 < 6) continue;
        for (int j0 = 5; j0 < sizes[i] - 5; j0 += kPcaBlock) blocks.push_back(make_int2(i, j0));
    }
    // device scratch: pts float4[n] | ring_off | blocks | outf[23][n] | keep | pos | flags | compact outputs | counters | cub
    size_t cub_bytes = 0;
    if (hipcub::DeviceScan::ExclusiveSum(nullptr, cub_bytes, (unsigned*)nullptr, (unsigned*)nullptr, std::max(n, 1), s) !=
        hipSuccess) { err = "hipcub scan size query failed"; return IMLS_ERR_DEVICE; }
    const size_t nn = (size_t)std::max(n, 1);
    size_t o_pts = 0, o_off = align256(o_pts + nn * 16), o_blk = align256(o_off + (n_rings + 1) * 4ull),
           o_outf = align256(o_blk + std::max<size_t>(blocks.size(), 1) * 8), o_keep = align256(o_outf + nn * 4 * kPcaOutF),
           o_pos = align256(o_keep + nn * 4), o_fl = align256(o_pos + nn * 4), o_idx = align256(o_fl + nn),
           o_nrm = align256(o_idx + nn * 4), o_ev = align256(o_nrm + nn * 12), o_evec = align256(o_ev + nn * 12),
           o_feat = align256(o_evec + nn * 36), o_flc = align256(o_feat + nn * 32), o_cnt = align256(o_flc + nn),
           o_cub = align256(o_cnt + 16), total = align256(o_cub + cub_bytes);
    if (!devbuf_grow(mem, total, total)) { err = "hipMalloc (pca scratch)"; return IMLS_ERR_DEVICE; }
    char* m = (char*)mem.p;
    std::vector<float4> h(nn);
    for (int k = 0; k < n; ++k) h[k] = make_float4(xyz[k * stride], xyz[k * stride + 1], xyz[k * stride + 2], 0.f);
    bool ok = hipMemcpyAsync(m + o_pts, h.data(), (size_t)n * 16, hipMemcpyHostToDevice, s) == hipSuccess;
    ok = ok && hipMemcpyAsync(m + o_off, off.data(), (n_rings + 1) * 4ull, hipMemcpyHostToDevice, s) == hipSuccess;
    if (!blocks.empty())
        ok = ok && hipMemcpyAsync(m + o_blk, blocks.data(), blocks.size() * 8, hipMemcpyHostToDevice, s) == hipSuccess;
    ok = ok && hipMemsetAsync(m + o_keep, 0, nn * 4, s) == hipSuccess;
    ok = ok && hipMemsetAsync(m + o_cnt, 0, 16, s) == hipSuccess;
    if (!ok) { err = "pca upload failed"; return IMLS_ERR_DEVICE; }
    if (marks) (void)hipEventRecord(marks[0], s);
    if (!blocks.empty())
        k_ring_pca<<<(unsigned)blocks.size(), kPcaBlock, 0, s>>>((const float4*)(m + o_pts), (const int*)(m + o_off),
                                                                n_rings, (const int2*)(m + o_blk), p, (float*)(m + o_outf),
                                                                (unsigned*)(m + o_keep), (unsigned char*)(m + o_fl), n,
                                                                (unsigned long long*)(m + o_cnt));
    if (marks) (void)hipEventRecord(marks[1], s);
    hipcub::DeviceScan::ExclusiveSum(m + o_cub, cub_bytes, (unsigned*)(m + o_keep), (unsigned*)(m + o_pos), (int)nn, s);
    if (n > 0)
        k_pca_scatter<<<(n + kBlock - 1) / kBlock, kBlock, 0, s>>>(
            (const float*)(m + o_outf), (const unsigned*)(m + o_keep), (const unsigned*)(m + o_pos),
            (const unsigned char*)(m + o_fl), nullptr, (const int*)(m + o_off), n, (unsigned*)(m + o_idx),
            (float*)(m + o_nrm), (float*)(m + o_ev), (float*)(m + o_evec), (float*)(m + o_feat),
            (unsigned char*)(m + o_flc));
    if (hipGetLastError() != hipSuccess) { err = "pca launch failed"; return IMLS_ERR_DEVICE; }
    unsigned last_pos = 0, last_keep = 0;
    unsigned long long cnt[2] = {0, 0};
    ok = hipMemcpyAsync(&last_pos, m + o_pos + (nn - 1) * 4, 4, hipMemcpyDeviceToHost, s) == hipSuccess;
    ok = ok && hipMemcpyAsync(&last_keep, m + o_keep + (nn - 1) * 4, 4, hipMemcpyDeviceToHost, s) == hipSuccess;
    ok = ok && hipMemcpyAsync(cnt, m + o_cnt, 16, hipMemcpyDeviceToHost, s) == hipSuccess;
    ok = ok && hipStreamSynchronize(s) == hipSuccess;
    if (!ok) { err = "pca kernel failed"; return IMLS_ERR_DEVICE; }
    const size_t r = n > 0 ? (size_t)last_pos + last_keep : 0;
    if (r > 0) {
        if (index_out) ok = ok && hipMemcpyAsync(index_out, m + o_idx, r * 4, hipMemcpyDeviceToHost, s) == hipSuccess;
        if (normal_out) ok = ok && hipMemcpyAsync(normal_out, m + o_nrm, r * 12, hipMemcpyDeviceToHost, s) == hipSuccess;
        if (evals_out) ok = ok && hipMemcpyAsync(evals_out, m + o_ev, r * 12, hipMemcpyDeviceToHost, s) == hipSuccess;
        if (evecs_out) ok = ok && hipMemcpyAsync(evecs_out, m + o_evec, r * 36, hipMemcpyDeviceToHost, s) == hipSuccess;
        if (features_out) ok = ok && hipMemcpyAsync(features_out, m + o_feat, r * 32, hipMemcpyDeviceToHost, s) == hipSuccess;
        if (flags_out) ok = ok && hipMemcpyAsync(flags_out, m + o_flc, r, hipMemcpyDeviceToHost, s) == hipSuccess;
        ok = ok && hipStreamSynchronize(s) == hipSuccess;
        if (!ok) { err = "pca download failed"; return IMLS_ERR_DEVICE; }
    }
    if (n_out) *n_out = r;
    if (counters) { counters[0] = cnt[0]; counters[1] = cnt[1]; }
    return IMLS_OK;
}

}  // namespace imlsgpu
