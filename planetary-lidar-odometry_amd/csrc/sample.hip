// sample.hip — the upstream producer's point sampling on gfx950: samplePointCloud "normal" /
// "major_axis" (scan_registration.cpp:536-806) with farthestPointSampling (common.cpp:19-82).
//
// Host: the spherical histogram of the candidates' normals (536-564, glibc atan2f / asin exactly as
// the reference evaluates them), randomSampling's shuffles (std::mt19937 + libstdc++ std::shuffle,
// 566-582), the bin weights (704-723) and the output assembly in bin order.  Device:
//   k_major_avg — the O(N_s·M) brute-force neighbour average of majorAxisSampling (670-702): one
//     wave per sample; the previous frame's cloud (scan-ring order) is cut into 64-point chunks whose
//     boxes the lanes test 64 at a time, and only chunks that can hold a point within r_proj are
//     scanned (exact: the skipped chunks provably contribute nothing); per pair the two
//     Eigen::Vector3f norm gates as square-root-free thresholds, a ballot of the lanes that pass and
//     an in-order sum (v_readlane per set bit) so the float accumulation order is the reference's;
//   k_fps — farthestPointSampling of one histogram bin per block: fp64 distances from float
//     coordinates, min-distance cache in HBM (L2-resident), block arg-max per step (largest distance,
//     lowest index on ties = the reference's strict > scan), first index from the replayed glibc
//     rand() stream.
// Roofline: k_major_avg reads 32 B of chunk box per 64 points per sample plus the surviving chunks
// (L2-resident: the previous cloud is ~2 MB); k_fps is latency-bound (one block-wide arg-max per step).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <limits>
#include <random>
#include <string>
#include <vector>

#include "internal.h"

namespace imlsgpu {
namespace {

constexpr int kAvgBlock = 1024;        // 16 waves = 16 samples per block
constexpr int kFpsBlock = 512;          // 8 waves: up to 256 VGPRs for the register-resident bin

// Correctly rounded float sqrt: v_sqrt_f32 is a 1-ulp approximation, so go through the correctly
// rounded fp64 sqrt (rounding sqrt twice, 53 → 24 bits, is innocuous: 53 ≥ 2·24 + 2).
__device__ __forceinline__ float sqrt_rn(float x) { return (float)__dsqrt_rn((double)x); }
// (Eigen::Vector3f::norm() = sqrt(c0 + (c1 + c2)): the non-vectorised unroller for 3 floats — the
// squared norms in k_major_avg keep that order)
// Eigen::Vector3d::norm() under SSE2: sqrt((c0 + c1) + c2)
__device__ __forceinline__ double norm3d(double a, double b, double c) {
    return __dsqrt_rn(__dadd_rn(__dadd_rn(__dmul_rn(a, a), __dmul_rn(b, b)), __dmul_rn(c, c)));
}

// The gates `sqrt_rn(s) < r` are evaluated as `s < T(r)` with T(r) = the smallest float whose
// correctly rounded sqrt is ≥ r (host, sqrt_threshold) — the same decisions without a square root
// per pair; the root is taken only for the pairs that pass (their in-order sum needs it).
// The previous cloud is in scan-ring order, so 64 consecutive points (a chunk) are spatially tight:
// lanes first test 64 chunk boxes at once and only chunks whose box comes within r_proj (with a
// 1e-4 relative margin over the float rounding of both sides) are scanned — point by point, in
// ascending chunk order, so the surviving pairs and their float sum are exactly the exhaustive
// loop's (679-696).
__global__ __launch_bounds__(kAvgBlock) void k_major_avg(const float4* __restrict__ spt, const float4* __restrict__ snr,
                                                         int ns, const float4* __restrict__ last, int m,
                                                         const float4* __restrict__ cbox, float t_r, float t_rproj,
                                                         int* __restrict__ cnt_out, float* __restrict__ avg_out) {
    const int lane = threadIdx.x & 63;
    const int si = blockIdx.x * (kAvgBlock / 64) + (threadIdx.x >> 6);
    if (si >= ns) return;                          // wave-uniform
    const float4 p = spt[si], n = snr[si];
    const int nchunks = (m + 63) >> 6;
    const float cull = t_rproj * (1.0f + 1e-4f);
    int cnt = 0;
    float acc = 0.f;
    for (int c0 = 0; c0 < nchunks; c0 += 64) {
        bool near = false;
        if (c0 + lane < nchunks) {
            const float4 lo = cbox[2 * (c0 + lane)], hi = cbox[2 * (c0 + lane) + 1];
            const float ex = fmaxf(fmaxf(lo.x - p.x, p.x - hi.x), 0.f);
            const float ey = fmaxf(fmaxf(lo.y - p.y, p.y - hi.y), 0.f);
            const float ez = fmaxf(fmaxf(lo.z - p.z, p.z - hi.z), 0.f);
            near = ex * ex + ey * ey + ez * ez <= cull;
        }
        unsigned long long cm = __ballot(near);
        while (cm) {
            const int c = c0 + (__ffsll((long long)cm) - 1);
            cm &= cm - 1;
            const int k = c * 64 + lane;
            bool hit = false;
            float nd = 0.f;
            if (k < m) {
                const float4 q = last[k];
                const float dx = p.x - q.x, dy = p.y - q.y, dz = p.z - q.z;   // pt − last_pt (683)
                const float sd = __fadd_rn(__fmul_rn(dx, dx), __fadd_rn(__fmul_rn(dy, dy), __fmul_rn(dz, dz)));
                if (sd < t_rproj) {
                    const float cx = __fsub_rn(__fmul_rn(dy, n.z), __fmul_rn(dz, n.y));
                    const float cy = __fsub_rn(__fmul_rn(dz, n.x), __fmul_rn(dx, n.z));
                    const float cz = __fsub_rn(__fmul_rn(dx, n.y), __fmul_rn(dy, n.x));
                    const float sc = __fadd_rn(__fmul_rn(cx, cx), __fadd_rn(__fmul_rn(cy, cy), __fmul_rn(cz, cz)));
                    hit = sc < t_r;
                    if (hit) nd = sqrt_rn(sd);
                }
            }
            unsigned long long mask = __ballot(hit);
            cnt += __popcll(mask);
            while (mask) {                         // in-order float sum of the nearby distances (691-696)
                const int b = __ffsll((long long)mask) - 1;
                acc = __fadd_rn(acc, __int_as_float(__builtin_amdgcn_readlane(__float_as_int(nd), b)));
                mask &= mask - 1;
            }
        }
    }
    if (lane == 0) {
        cnt_out[si] = cnt;
        avg_out[si] = cnt >= 3 ? __fdiv_rn(acc, (float)cnt) : 0.f;   // 697
    }
}

struct FpsJob {
    int off, n, k, first, out;   // points [off, off+n) of the packed bin clouds; k samples → out[out, out+k)
};

constexpr int kFpsPPT = 16;            // bin points per thread held in registers (bins ≤ 8192 points)

// block arg-max of (value desc, index asc) — the first maximum of the reference's strict `>` scan
__device__ __forceinline__ void fps_better(double& b, int& x, double ov, int oi) {
    if (ov > b || (ov == b && oi < x)) { b = ov; x = oi; }
}

__global__ __launch_bounds__(kFpsBlock) void k_fps(const float4* __restrict__ pts, const FpsJob* __restrict__ jobs,
                                                   double* __restrict__ md, unsigned char* __restrict__ taken,
                                                   int* __restrict__ out) {
    // one LDS slot pair per wave and iteration parity: a single barrier per sample (a wave cannot
    // overwrite parity p before every wave has passed the next barrier, i.e. finished reading p)
    __shared__ double sv[2][kFpsBlock / 64];
    __shared__ int si[2][kFpsBlock / 64];
    const FpsJob J = jobs[blockIdx.x];
    const float4* P = pts + J.off;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    int last = J.first;
    if (tid == 0) out[J.out] = last;
    const bool regs = J.n <= kFpsBlock * kFpsPPT;
    double D[kFpsPPT];
    float X[kFpsPPT], Y[kFpsPPT], Z[kFpsPPT];
    unsigned tk = 0u;                                   // bit k: point tid + k·kFpsBlock already sampled
    double* Dg = md + J.off;
    unsigned char* Tg = taken + J.off;
    if (regs) {
#pragma unroll
        for (int k = 0; k < kFpsPPT; ++k) {
            const int i = tid + k * kFpsBlock;
            const float4 q = P[i < J.n ? i : 0];
            X[k] = q.x; Y[k] = q.y; Z[k] = q.z;
            D[k] = INFINITY;
            if (i == last) tk |= 1u << k;
        }
    } else {
        for (int i = tid; i < J.n; i += kFpsBlock) { Dg[i] = INFINITY; Tg[i] = i == last; }
        __syncthreads();
    }
    for (int s = 1; s < J.k; ++s) {
        const float4 f = P[last];                       // one broadcast load
        const double fx = f.x, fy = f.y, fz = f.z;
        double best = -1.0;
        int bi = 0x7fffffff;
        if (regs) {
#pragma unroll
            for (int k = 0; k < kFpsPPT; ++k) {
                const int i = tid + k * kFpsBlock;
                if (i < J.n) {
                    const double v = fmin(D[k], norm3d(fx - (double)X[k], fy - (double)Y[k], fz - (double)Z[k]));
                    D[k] = v;
                    if (!((tk >> k) & 1u) && v > best) { best = v; bi = i; }   // ascending i: the first maximum
                }
            }
        } else {
            for (int i = tid; i < J.n; i += kFpsBlock) {
                const float4 q = P[i];
                const double v = fmin(Dg[i], norm3d(fx - (double)q.x, fy - (double)q.y, fz - (double)q.z));
                Dg[i] = v;
                if (!Tg[i] && v > best) { best = v; bi = i; }
            }
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) fps_better(best, bi, __shfl_xor(best, o), __shfl_xor(bi, o));
        const int par = s & 1;
        if (lane == 0) { sv[par][wv] = best; si[par][wv] = bi; }
        __syncthreads();
        double b = sv[par][0];
        int x = si[par][0];
#pragma unroll
        for (int w = 1; w < kFpsBlock / 64; ++w) fps_better(b, x, sv[par][w], si[par][w]);
        last = x;
        if (tid == 0) out[J.out + s] = x;
        if (regs) {
            if ((x & (kFpsBlock - 1)) == tid) tk |= 1u << (x / kFpsBlock);
        } else {
            if (tid == 0) Tg[x] = 1;
            __syncthreads();
        }
    }
}

// glibc random() TYPE_3 step on the host (the state ransac_seed_host produces)
int host_rand_next(int* st) {
    unsigned* ring = reinterpret_cast<unsigned*>(st);
    const int f = st[31], r = st[32];
    ring[f] += ring[r];
    const int out = (int)(ring[f] >> 1);
    st[31] = (f + 1) % 31;
    st[32] = (r + 1) % 31;
    return out;
}

size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }

// static_cast<int>(float) as the reference's x86-64 build evaluates it (cvttss2si): truncation, and
// the "integer indefinite" INT_MIN for NaN / out-of-range (all-zero weights make them NaN, 721-723)
// — spelled out here because the C++ cast is undefined there.
int x86_float_to_int(float v) {
    return (v > -2147483904.0f && v < 2147483648.0f) ? static_cast<int>(v) : std::numeric_limits<int>::min();
}

// Smallest float t ≥ 0 with sqrt(t) ≥ r in correctly rounded float arithmetic (x86 sqrtss is
// correctly rounded, as is the device's sqrt_rn), so `sqrt(s) < r` ⇔ `s < t` for every float s ≥ 0.
float sqrt_threshold(float r) {
    if (!(r > 0.f)) return 0.f;                        // sqrt(s) < r never holds
    if (std::isinf(r)) return INFINITY;
    float t = r * r;
    if (std::isinf(t)) t = std::numeric_limits<float>::max();
    while (t > 0.f && std::sqrt(std::nextafter(t, 0.f)) >= r) t = std::nextafter(t, 0.f);
    while (std::sqrt(t) < r) t = std::nextafter(t, INFINITY);
    return t;
}

struct HostRng {
    uint32_t seed;
    uint32_t calls = 0;
    int glibc[34];
    // randomSampling (566-582): a fresh generator per call
    void shuffle_take(const std::vector<int>& cand, int k, std::vector<int>& out) {
        std::mt19937 gen(seed + calls++);
        std::vector<int> sh = cand;
        std::shuffle(sh.begin(), sh.end(), gen);
        const int c = std::min(k, (int)sh.size());
        out.insert(out.end(), sh.begin(), sh.begin() + c);
    }
};

bool grow_buf(DevBuf& b, size_t bytes) { return devbuf_grow(b, bytes, bytes); }

}  // namespace

int sample_run(hipStream_t s, const imls_sample_params& p, const float* xyz, const float* nrm, size_t stride, size_t n,
               const int32_t* cand, size_t n_cand, const float* last_xyz, size_t last_stride, size_t m, DevBuf& mem,
               hipEvent_t* marks, int32_t* sampled_out, size_t* n_sampled, float* bin_weights_out, std::string& err) {
    const int AZ = p.azimuth_bins, EL = p.elevation_bins, NB = AZ * EL;
    // computeSphericalHistogram (536-564)
    std::vector<std::vector<int>> hist(NB);
    for (size_t k = 0; k < n_cand; ++k) {
        const int idx = cand[k];
        if (idx < 0 || (size_t)idx >= n) { err = "candidate index out of range"; return IMLS_ERR_ARG; }
        const float nx = nrm[idx * stride], ny = nrm[idx * stride + 1], nz = nrm[idx * stride + 2];
        float azimuth = std::atan2(ny, nx);              // std::atan2(float, float) (`using std::atan2`, 51)
        float elevation = (float)::asin((double)nz);     // ::asin(double)
        if (azimuth < 0) azimuth += 2 * M_PI;
        elevation += M_PI / 2;
        const int ai = std::min(static_cast<int>(azimuth / (2 * M_PI / AZ)), AZ - 1);
        const int ei = std::min(static_cast<int>(elevation / (M_PI / EL)), EL - 1);
        hist[(size_t)ai * EL + ei].push_back(idx);
    }
    HostRng rng{p.shuffle_seed};
    ransac_seed_host(p.rand_seed, rng.glibc);
    std::vector<float> w(NB, 0.0f);
    if (p.method == IMLS_SAMPLE_MAJOR_AXIS) {
        // per-bin subsets (656-664) → one device pass over all samples (670-702)
        std::vector<int> sub_all, sub_off(NB + 1, 0);
        for (int b = 0; b < NB; ++b) {
            const auto& bin = hist[b];
            if ((int)bin.size() >= p.min_points_per_bin) {
                if ((int)bin.size() > p.max_points_per_bin) rng.shuffle_take(bin, p.max_points_per_bin, sub_all);
                else sub_all.insert(sub_all.end(), bin.begin(), bin.end());
            }
            sub_off[b + 1] = (int)sub_all.size();
        }
        const int ns = (int)sub_all.size();
        std::vector<int> cnt(ns);
        std::vector<float> avg(ns);
        if (ns > 0 && m > 0) {
            std::vector<float4> hs(2 * (size_t)ns), hl(m);
            for (int k = 0; k < ns; ++k) {
                const size_t i = (size_t)sub_all[k];
                hs[k] = make_float4(xyz[i * stride], xyz[i * stride + 1], xyz[i * stride + 2], 0.f);
                hs[ns + k] = make_float4(nrm[i * stride], nrm[i * stride + 1], nrm[i * stride + 2], 0.f);
            }
            for (size_t j = 0; j < m; ++j)
                hl[j] = make_float4(last_xyz[j * last_stride], last_xyz[j * last_stride + 1], last_xyz[j * last_stride + 2], 0.f);
            const size_t nch = (m + 63) / 64;
            std::vector<float4> hb(2 * nch);                               // AABB of every 64-point chunk
            for (size_t c = 0; c < nch; ++c) {
                float4 lo = make_float4(INFINITY, INFINITY, INFINITY, 0.f), hi = make_float4(-INFINITY, -INFINITY, -INFINITY, 0.f);
                for (size_t j = c * 64; j < std::min(m, c * 64 + 64); ++j) {
                    lo.x = std::min(lo.x, hl[j].x); lo.y = std::min(lo.y, hl[j].y); lo.z = std::min(lo.z, hl[j].z);
                    hi.x = std::max(hi.x, hl[j].x); hi.y = std::max(hi.y, hl[j].y); hi.z = std::max(hi.z, hl[j].z);
                }
                // a non-finite coordinate makes the box unbounded: the chunk is always scanned
                if (!(std::isfinite(lo.x) && std::isfinite(lo.y) && std::isfinite(lo.z) && std::isfinite(hi.x) &&
                      std::isfinite(hi.y) && std::isfinite(hi.z)))
                    lo = make_float4(-INFINITY, -INFINITY, -INFINITY, 0.f), hi = make_float4(INFINITY, INFINITY, INFINITY, 0.f);
                hb[2 * c] = lo;
                hb[2 * c + 1] = hi;
            }
            const size_t o_s = 0, o_l = al256(o_s + hs.size() * 16), o_b = al256(o_l + m * 16),
                         o_c = al256(o_b + nch * 32), o_a = al256(o_c + (size_t)ns * 4), total = al256(o_a + (size_t)ns * 4);
            if (!grow_buf(mem, total)) { err = "hipMalloc (sample scratch)"; return IMLS_ERR_DEVICE; }
            char* d = (char*)mem.p;
            bool ok = hipMemcpyAsync(d + o_s, hs.data(), hs.size() * 16, hipMemcpyHostToDevice, s) == hipSuccess;
            ok = ok && hipMemcpyAsync(d + o_l, hl.data(), m * 16, hipMemcpyHostToDevice, s) == hipSuccess;
            ok = ok && hipMemcpyAsync(d + o_b, hb.data(), nch * 32, hipMemcpyHostToDevice, s) == hipSuccess;
            if (!ok) { err = "sample upload failed"; return IMLS_ERR_DEVICE; }
            if (marks) (void)hipEventRecord(marks[0], s);
            k_major_avg<<<(ns + kAvgBlock / 64 - 1) / (kAvgBlock / 64), kAvgBlock, 0, s>>>(
                (const float4*)(d + o_s), (const float4*)(d + o_s) + ns, ns, (const float4*)(d + o_l), (int)m,
                (const float4*)(d + o_b), sqrt_threshold(p.r), sqrt_threshold(p.r_proj), (int*)(d + o_c), (float*)(d + o_a));
            if (marks) (void)hipEventRecord(marks[1], s);
            ok = hipGetLastError() == hipSuccess;
            ok = ok && hipMemcpyAsync(cnt.data(), d + o_c, (size_t)ns * 4, hipMemcpyDeviceToHost, s) == hipSuccess;
            ok = ok && hipMemcpyAsync(avg.data(), d + o_a, (size_t)ns * 4, hipMemcpyDeviceToHost, s) == hipSuccess;
            ok = ok && hipStreamSynchronize(s) == hipSuccess;
            if (!ok) { err = "major-axis kernel failed"; return IMLS_ERR_DEVICE; }
        }
        for (int b = 0; b < NB; ++b) {                                     // 666-711
            if ((int)hist[b].size() < p.min_points_per_bin) continue;
            const int len = sub_off[b + 1] - sub_off[b];
            std::vector<float> distances(len, 0.0f);
            int valid = 0;
            for (int k = sub_off[b]; k < sub_off[b + 1]; ++k)
                if (cnt[k] >= 3) distances[valid++] = avg[k];
            if (valid >= 3) {
                float total = 0.0f;
                for (float x : distances) total += x;
                w[b] = total / valid;
            }
        }
        float tw = 0.0f;                                                   // 715-723
        for (float x : w) tw += x;
        for (float& x : w) x /= tw;
    }
    // per-bin decisions in bin order (the RNG streams are consumed in the reference's order)
    struct BinPlan { int kind, k, job; std::vector<int> pts; };   // kind 0 all, 1 FPS, 2 random (pts)
    std::vector<BinPlan> plan(NB);
    std::vector<FpsJob> jobs;
    std::vector<float4> fpts;
    int fout = 0;
    for (int b = 0; b < NB; ++b) {
        const auto& bin = hist[b];
        const int sz = (int)bin.size();
        plan[b].kind = -1;
        if (sz < p.min_points_per_bin) continue;
        const int k = p.method == IMLS_SAMPLE_MAJOR_AXIS
                          ? std::min(x86_float_to_int(w[b] * p.max_total_points), sz)   // 732
                          : p.max_points_per_bin;                                        // 603
        if (sz <= k) { plan[b].kind = 0; continue; }
        if (p.sampling_strategy == 0) {
            const int kk = std::max(k, 1);   // farthestPointSampling pushes its first index even for k ≤ 0 (49-50)
            FpsJob J{(int)fpts.size(), sz, kk, host_rand_next(rng.glibc) % sz, fout};
            for (int i : bin)
                fpts.push_back(make_float4(xyz[(size_t)i * stride], xyz[(size_t)i * stride + 1], xyz[(size_t)i * stride + 2], 0.f));
            plan[b].kind = 1;
            plan[b].k = kk;
            plan[b].job = fout;
            fout += kk;
            jobs.push_back(J);
        } else {
            plan[b].kind = 2;
            rng.shuffle_take(bin, k, plan[b].pts);
        }
    }
    std::vector<int> fres(fout);
    if (!jobs.empty()) {
        const size_t np = fpts.size();
        const size_t o_p = 0, o_j = al256(np * 16), o_md = al256(o_j + jobs.size() * sizeof(FpsJob)),
                     o_t = al256(o_md + np * 8), o_o = al256(o_t + np), total = al256(o_o + (size_t)fout * 4);
        if (!grow_buf(mem, total)) { err = "hipMalloc (fps scratch)"; return IMLS_ERR_DEVICE; }
        char* d = (char*)mem.p;
        bool ok = hipMemcpyAsync(d + o_p, fpts.data(), np * 16, hipMemcpyHostToDevice, s) == hipSuccess;
        ok = ok && hipMemcpyAsync(d + o_j, jobs.data(), jobs.size() * sizeof(FpsJob), hipMemcpyHostToDevice, s) == hipSuccess;
        if (!ok) { err = "fps upload failed"; return IMLS_ERR_DEVICE; }
        k_fps<<<(unsigned)jobs.size(), kFpsBlock, 0, s>>>((const float4*)(d + o_p), (const FpsJob*)(d + o_j),
                                                           (double*)(d + o_md), (unsigned char*)(d + o_t), (int*)(d + o_o));
        ok = hipGetLastError() == hipSuccess;
        ok = ok && hipMemcpyAsync(fres.data(), d + o_o, (size_t)fout * 4, hipMemcpyDeviceToHost, s) == hipSuccess;
        ok = ok && hipStreamSynchronize(s) == hipSuccess;
        if (!ok) { err = "fps kernel failed"; return IMLS_ERR_DEVICE; }
    }
    size_t r = 0;
    for (int b = 0; b < NB; ++b) {
        const auto& bin = hist[b];
        switch (plan[b].kind) {
            case 0: for (int i : bin) sampled_out[r++] = i; break;
            case 1: for (int t = 0; t < plan[b].k; ++t) sampled_out[r++] = bin[fres[plan[b].job + t]]; break;
            case 2: for (int i : plan[b].pts) sampled_out[r++] = i; break;
            default: break;
        }
    }
    if (n_sampled) *n_sampled = r;
    if (bin_weights_out) for (int b = 0; b < NB; ++b) bin_weights_out[b] = w[b];
    return IMLS_OK;
}

}  // namespace imlsgpu
