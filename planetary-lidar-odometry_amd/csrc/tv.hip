// tv.hip — tensor-voting normals on device: IMLSICPMatcher::VoteForAny (imls_icp.cpp:171-296) as
// ProjSourcePtToSurface uses it (get_normals=false, use_tensor_voting=true: 514-546, 634-643).
//
// Every ICP iteration the reference votes from the target's input tensors into every transformed
// source point x (in_cloudDP): the voters are x's libnabo knn(k) over the target (no radius, no
// self match, 197), a voter p counts when 0 < ‖x−p‖/σ < distance_threshold (212-217) and adds
// S = w·R·T_p·R' with w = exp(−‖r‖²/σ), R = I − 2r̂r̂ᵀ, R' = (I − ½r̂r̂ᵀ)R (220-226).  The query's
// normal is the "tangent" of the summed tensor (the eigenvector of its smallest |λ|, lower
// triangle, flipped to +z; 245, 272-278, 543); a zero tensor (Eigen isZero, |coeff| ≤ 1e-12) has
// none and the query is rejected as "no normal" (637-643).
//
// Voters are the k nearest, but only those within ρ = threshold·σ of x vote, and every point
// nearer than a voting one is itself within ρ: so the exact voter set is "the ≤ k best (d², index)
// of the ball of radius ρ" — a small fixed-radius search, not a k-nearest search.  One wave per
// query: the tree walk is wave-uniform (scalar node loads), a leaf is one coalesced load with one
// point per lane, ball members (fp32 screen with slack, exact fp64 libnabo metric, self match
// excluded by d² > DBL_EPSILON) are appended to an LDS buffer by ballot; a full buffer is sorted
// and cut to the best k (the k-th entry then bounds the search).  Finally the buffer is sorted by
// (d², index), lane j < k computes voter j's S in fp64, lanes 0..8 sum one component each in list
// order (the reference's order) through LDS, and k_tv_tangent runs the shared 3×3 Jacobi
// eigensolver with one thread per query.  Skin lists (below) let later ICP iterations skip the walk.
#include <algorithm>
#include <cfloat>

#include "geom.h"
#include "solve_common.h"

namespace imlsgpu {
namespace {

constexpr int kTvBlock = 256;              // 4 waves per block, one query per wave
constexpr int kTvWaves = kTvBlock / 64;
constexpr int kTvCap = 256;                // ball members buffered per query before a cut to the best k
constexpr int kTvStack = 32;               // tree depth ≤ 23 (kStackDepth − 1), one push per level
constexpr float kTvSlack = 1.0f + 2e-6f;   // fp32 screen vs exact distance: ≤ 3.1e-7 relative
static_assert(kTvCap >= kTvMaxK + 64, "a cut must leave room for one more leaf");

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// One wave sorts n (a power of two) LDS entries ascending by (key, index).
__device__ void wave_bitonic(unsigned long long* k, unsigned* ix, unsigned* ps, int n, int lane) {
    for (int size = 2; size <= n; size <<= 1)
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            for (int a = lane; a < n; a += 64) {
                const int b = a ^ stride;
                if (b > a) {
                    const bool up = (a & size) == 0;
                    const bool gt = k[a] > k[b] || (k[a] == k[b] && ix[a] > ix[b]);
                    if (gt == up) {
                        const unsigned long long tk = k[a]; k[a] = k[b]; k[b] = tk;
                        const unsigned ti = ix[a]; ix[a] = ix[b]; ix[b] = ti;
                        const unsigned tp = ps[a]; ps[a] = ps[b]; ps[b] = tp;
                    }
                }
            }
            wave_sync();
        }
}

// the summed tensors (9 doubles per query) behind the voted normals, skin references and lists
__device__ __forceinline__ double* tv_acc(double4* tvn, int N) {
    return reinterpret_cast<double*>(reinterpret_cast<unsigned*>(reinterpret_cast<float4*>(tvn + N) + N) +
                                     (size_t)N * kTvList);
}

// fp32 screen distance (the one definition every ball test uses)
__device__ __forceinline__ float screen_d2(const float4& p4, const float* xf) {
    const float ex = p4.x - xf[0], ey = p4.y - xf[1], ez = p4.z - xf[2];
    return __builtin_fmaf(ex, ex, __builtin_fmaf(ey, ey, ez * ez));
}

__device__ __forceinline__ void tv_vote_body(const TreeView& t, const float4* __restrict__ spt, int N,
                                             const double* __restrict__ pose, const int* __restrict__ done,
                                             const KParams& kp, double4* __restrict__ tvn, int use_prev, int bx) {
    if (done && *done) return;
    __shared__ unsigned long long ck[kTvWaves][kTvCap];   // exact d² bits (positive doubles order as integers)
    __shared__ unsigned ci[kTvWaves][kTvCap];             // filtered target index (the tie order)
    __shared__ unsigned cp[kTvWaves][kTvCap];             // Morton position
    __shared__ int snode[kTvWaves][kTvStack];
    __shared__ float sdist[kTvWaves][kTvStack];
    __shared__ double sx[kTvWaves][64];                   // the vote sum's ninth component
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int q = __builtin_amdgcn_readfirstlane(bx * kTvWaves + wv);
    if (q >= N) return;
    float xf[3];
    {
        double ns_unused[3];
        transform_query(pose, spt[q], make_float4(0.f, 0.f, 0.f, 0.f), 0, xf, ns_unused);
    }
    const double xd[3] = {xf[0], xf[1], xf[2]};
    const double sigma = kp.tv_sigma, thr = kp.tv_thr;
    const double rho = thr * sigma;
    const float r2s = (float)(rho * rho) * kTvSlack + 1e-30f;
    const int K = kp.tv_k;
    unsigned long long* wk = ck[wv];
    unsigned* wi = ci[wv];
    unsigned* wp = cp[wv];
    int cnt = 0;
    unsigned long long bk = ~0ull;     // after a cut: the k-th (d², index) — later members must beat it
    unsigned bi = ~0u;
    float bnd = r2s;
    auto sort_buffer = [&]() {
        int n = 1;
        while (n < cnt) n <<= 1;
        for (int a = cnt + lane; a < n; a += 64) { wk[a] = ~0ull; wi[a] = ~0u; wp[a] = 0u; }
        wave_sync();
        wave_bitonic(wk, wi, wp, n, lane);
    };
    // skin lists (Verlet): a walk stores every point of the ball of radius ρ' + skin around x (ρ' the
    // screen radius) when they fit kTvList; while the query stays within skin of that x the ball of
    // x is a subset of the stored set, so the stored set screened at x gives the same members as a
    // walk — bit-identical lists, no tree descent.  Margins (1e-5) cover the fp32 screens.
    const float skin = kp.tv_skin;
    float4* tref = reinterpret_cast<float4*>(tvn + N);
    unsigned* tlist = reinterpret_cast<unsigned*>(tref + N) + (size_t)q * kTvList;
    double* tacc = tv_acc(tvn, N);
    bool reuse = false;
    int nst = 0;
    if (use_prev && skin > 0.f) {
        const float4 xr = tref[q];
        const float dx = xf[0] - xr.x, dy = xf[1] - xr.y, dz = xf[2] - xr.z;
        reuse = xr.w >= 0.f && dx * dx + dy * dy + dz * dz <= skin * skin * (1.0f - 1e-4f);
        nst = (int)xr.w;
    }
    bool wide = !reuse && skin > 0.f;   // this walk collects the skin ball (self matches included)
    if (wide) {
        const float rs = sqrtf(r2s) * (1.0f + 1e-5f) + skin;
        bnd = rs * rs * (1.0f + 1e-5f);
    }
    // keep only the screened ball members proper (d32 ≤ r2s, no self match), in buffer order
    auto compact_ball = [&]() {
        int nc = 0;
        for (int a0 = 0; a0 < cnt; a0 += 64) {
            const int a = a0 + lane;
            bool keep = false;
            unsigned long long k0 = 0ull;
            unsigned i0 = 0u, p0 = 0u;
            if (a < cnt) {
                k0 = wk[a];
                i0 = wi[a];
                p0 = wp[a];
                keep = screen_d2(t.mpt[p0], xf) <= r2s && __longlong_as_double((long long)k0) > DBL_EPSILON;
            }
            const unsigned long long mk = __ballot(keep);
            wave_sync();
            if (keep) {
                const int at = nc + __popcll(mk & ((1ull << lane) - 1ull));
                wk[at] = k0;
                wi[at] = i0;
                wp[at] = p0;
            }
            nc += __popcll(mk);
            wave_sync();
        }
        cnt = nc;
    };
    const int P = t.P, B = t.B, M = t.M;
    int node = reuse ? 0 : 1, sp = 0;
    if (reuse) {
        bool pass = false;
        unsigned long long key = 0ull;
        unsigned oi = 0u, pos = 0u;
        if (lane < nst) {
            pos = tlist[lane];
            const float4 p4 = t.mpt[pos];
            if (screen_d2(p4, xf) <= r2s) {
                const double d2 = exact_d2(xd, p4.x, p4.y, p4.z);
                key = (unsigned long long)__double_as_longlong(d2);
                oi = __float_as_uint(p4.w);
                pass = d2 > DBL_EPSILON;
            }
        }
        const unsigned long long m = __ballot(pass);
        if (pass) {
            const int at = __popcll(m & ((1ull << lane) - 1ull));
            wk[at] = key;
            wi[at] = oi;
            wp[at] = pos;
        }
        cnt = __popcll(m);
    }
    while (node) {
        if (node < P) {
            const float4* rec = t.nodes + 3 * (size_t)node;
            const float4 a = rec[0], b = rec[1], c = rec[2];
            const float dl = box_d2(xf, a.x, a.y, a.z, a.w, b.x, b.y);
            const float dr = box_d2(xf, b.z, b.w, c.x, c.y, c.z, c.w);
            const float bs = bnd * kTvSlack;
            const bool nl = dl <= bs, nr = dr <= bs;
            if (nl && nr) {
                const bool lf = dl <= dr;
                snode[wv][sp] = lf ? 2 * node + 1 : 2 * node;
                sdist[wv][sp] = lf ? dr : dl;
                ++sp;
                node = __builtin_amdgcn_readfirstlane(lf ? 2 * node : 2 * node + 1);
                continue;
            }
            if (nl) { node = 2 * node; continue; }
            if (nr) { node = 2 * node + 1; continue; }
        } else {
            const int base = (node - P) * B, cl = min(B, M - base);
            bool pass = false;
            unsigned long long key = 0ull;
            unsigned oi = 0u;
            float d32 = __builtin_inff();
            if (lane < cl) {
                const float4 p4 = t.mpt[base + lane];
                d32 = screen_d2(p4, xf);
                if (d32 <= bnd) {
                    const double d2 = exact_d2(xd, p4.x, p4.y, p4.z);
                    key = (unsigned long long)__double_as_longlong(d2);
                    oi = __float_as_uint(p4.w);
                    pass = (wide || d2 > DBL_EPSILON) && (key < bk || (key == bk && oi < bi));   // no self match (197)
                }
            }
            unsigned long long m = __ballot(pass);
            if (wide && cnt + __popcll(m) > kTvCap) {
                // the skin ball overflows: no list for this query; back to the ball proper
                wide = false;
                bnd = r2s;
                compact_ball();
                pass = pass && d32 <= r2s && __longlong_as_double((long long)key) > DBL_EPSILON;
                m = __ballot(pass);
            }
            if (cnt + __popcll(m) > kTvCap) {
                // cut to the best k; its k-th entry bounds everything after
                sort_buffer();
                cnt = min(cnt, K);
                if (cnt == K) {
                    bk = wk[K - 1];
                    bi = wi[K - 1];
                    bnd = fminf(r2s, (float)__longlong_as_double((long long)bk) * kTvSlack + 1e-30f);
                }
                pass = pass && (key < bk || (key == bk && oi < bi));
                m = __ballot(pass);
            }
            if (pass) {
                const int at = cnt + __popcll(m & ((1ull << lane) - 1ull));
                wk[at] = key;
                wi[at] = oi;
                wp[at] = (unsigned)(base + lane);
            }
            cnt += __popcll(m);
        }
        node = 0;
        while (sp > 0) {
            --sp;
            if (sdist[wv][sp] <= bnd * kTvSlack) { node = snode[wv][sp]; break; }
        }
        node = __builtin_amdgcn_readfirstlane(node);
    }
    if (wide) {
        // the walk's skin ball: stored when it fits, then cut to the ball proper
        const bool fits = cnt <= kTvList;
        if (fits && lane < cnt) tlist[lane] = wp[lane];
        if (lane == 0) tref[q] = make_float4(xf[0], xf[1], xf[2], fits ? (float)cnt : -1.f);
        compact_ball();
    } else if (!reuse && skin > 0.f && lane == 0) {
        tref[q] = make_float4(0.f, 0.f, 0.f, -1.f);
    }
    if (cnt > 0) sort_buffer();
    const int kk = min(cnt, K);
    // voter j = list entry j (lane j): S = w·(R·T)·R' in fp64, the oracle's evaluation order
    double S[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    if (lane < kk) {
        const int pos = (int)wp[lane];
        const float4 p4 = t.mpt[pos];
        const double r[3] = {xd[0] - (double)p4.x, xd[1] - (double)p4.y, xd[2] - (double)p4.z};
        double nn2 = r[0] * r[0];
        nn2 = nn2 + r[1] * r[1];
        nn2 = nn2 + r[2] * r[2];
        const double nr = sqrt(nn2);
        const double dist = nr / sigma;
        if (!(dist <= 0. || dist >= thr)) {
            const double u[3] = {r[0] / nr, r[1] / nr, r[2] / nr};
            const double w = exp(-(nr * nr) / sigma);
            const float4 t0 = t.mten[2 * (size_t)pos], t1 = t.mten[2 * (size_t)pos + 1];
            const double T[9] = {t0.x, t0.y, t0.z, t0.y, t0.w, t1.x, t0.z, t1.x, t1.y};
            double R[9], Rp[9], RT[9];
#pragma unroll
            for (int a = 0; a < 3; ++a)
#pragma unroll
                for (int b = 0; b < 3; ++b) R[a * 3 + b] = (a == b ? 1.0 : 0.0) - 2 * u[a] * u[b];
#pragma unroll
            for (int a = 0; a < 3; ++a)
#pragma unroll
                for (int b = 0; b < 3; ++b) {
                    double s = 0.0;
#pragma unroll
                    for (int c = 0; c < 3; ++c) s += ((a == c ? 1.0 : 0.0) - 0.5 * u[a] * u[c]) * R[c * 3 + b];
                    Rp[a * 3 + b] = s;
                }
#pragma unroll
            for (int a = 0; a < 3; ++a)
#pragma unroll
                for (int b = 0; b < 3; ++b) {
                    double s = 0.0;
#pragma unroll
                    for (int c = 0; c < 3; ++c) s += R[a * 3 + c] * T[c * 3 + b];
                    RT[a * 3 + b] = s;
                }
#pragma unroll
            for (int a = 0; a < 3; ++a)
#pragma unroll
                for (int b = 0; b < 3; ++b) {
                    double s = 0.0;
#pragma unroll
                    for (int c = 0; c < 3; ++c) s += RT[a * 3 + c] * Rp[c * 3 + b];
                    S[a * 3 + b] = w * s;
                }
        }
    }
    // the votes summed in list order (the reference's): the wave's S staged in its (now free) LDS
    // buffers, component-major, and lane e < 9 runs component e's chain of adds — 9 chains side by
    // side instead of 9·k wave-wide adds of lane-broadcast values
    wave_sync();   // every lane has read its wp entry
    double* sk = reinterpret_cast<double*>(wk);
    if (lane < kk) {
#pragma unroll
        for (int e = 0; e < 4; ++e) sk[e * 64 + lane] = S[e];
#pragma unroll
        for (int e = 4; e < 8; ++e) {
            const unsigned long long b = (unsigned long long)__double_as_longlong(S[e]);
            wi[(e - 4) * 64 + lane] = (unsigned)b;
            wp[(e - 4) * 64 + lane] = (unsigned)(b >> 32);
        }
        sx[wv][lane] = S[8];
    }
    wave_sync();
    if (lane >= 9) return;
    const unsigned* lo;
    const unsigned* hi;
    int st;
    if (lane < 4) { lo = reinterpret_cast<const unsigned*>(sk + lane * 64); hi = lo + 1; st = 2; }
    else if (lane < 8) { lo = wi + (lane - 4) * 64; hi = wp + (lane - 4) * 64; st = 1; }
    else { lo = reinterpret_cast<const unsigned*>(sx[wv]); hi = lo + 1; st = 2; }
    double acc = 0.0;
    for (int j = 0; j < kk; ++j)
        acc += __longlong_as_double((long long)(((unsigned long long)hi[j * st] << 32) | lo[j * st]));
    tacc[(size_t)q * 9 + lane] = acc;
}

// The summed tensor's tangent, one thread per query (the serial 3×3 Jacobi of 64 queries shares the
// wave's instructions): Eigen isZero (|coeff| ≤ 1e-12) → no normal; else the eigenvector of the
// smallest |λ| of the lower triangle, flipped to +z (imls_icp.cpp:245, 272-278).
__device__ __forceinline__ void tv_tangent_body(int N, const int* __restrict__ done, double4* __restrict__ tvn, int q) {
    if (q >= N || (done && *done)) return;
    const double* acc = tv_acc(tvn, N) + (size_t)q * 9;
    double a9[9];
#pragma unroll
    for (int e = 0; e < 9; ++e) a9[e] = acc[e];
    bool zero = true;
#pragma unroll
    for (int e = 0; e < 9; ++e) zero = zero && fabs(a9[e]) <= 1e-12;
    if (zero) { tvn[q] = make_double4(0.0, 0.0, 0.0, 0.0); return; }
    double A[9], ev[3], U[9];
#pragma unroll
    for (int a = 0; a < 3; ++a)
#pragma unroll
        for (int b = 0; b < 3; ++b) A[a * 3 + b] = a >= b ? a9[a * 3 + b] : a9[b * 3 + a];
    sym_eig<3>(A, ev, U);
    int mi = 0;
    if (fabs(ev[1]) < fabs(ev[mi])) mi = 1;
    if (fabs(ev[2]) < fabs(ev[mi])) mi = 2;
    double n0 = U[mi * 3], n1 = U[mi * 3 + 1], n2 = U[mi * 3 + 2];
    if (n2 < 0) { n0 = -n0; n1 = -n1; n2 = -n2; }
    tvn[q] = make_double4(n0, n1, n2, 1.0);
}

__global__ __launch_bounds__(256) void k_tv_tangent(int N, const int* __restrict__ done, double4* __restrict__ tvn) {
    tv_tangent_body(N, done, tvn, (int)(blockIdx.x * blockDim.x + threadIdx.x));
}

__global__ __launch_bounds__(256) void k_tv_tangent_b(const PairDev* __restrict__ tab) {
    const PairDev A = device_view(tab + blockIdx.y);
    if (A.t.M <= 0) return;
    tv_tangent_body(A.N, A.st.done, const_cast<double4*>(A.t.tvn), (int)(blockIdx.x * blockDim.x + threadIdx.x));
}

// Input tensors [6][n_in] (input order) → Morton order, 2 float4 per point.
__global__ __launch_bounds__(kTvBlock) void k_tv_vote(TreeView t, const float4* __restrict__ spt, int N,
                                                      const double* __restrict__ pose, const int* __restrict__ done,
                                                      KParams kp, double4* __restrict__ tvn, int use_prev) {
    tv_vote_body(t, spt, N, pose, done, kp, tvn, use_prev, (int)blockIdx.x);
}

// batched (imls_register_frames): frame = tab[blockIdx.y], the same body
__global__ __launch_bounds__(kTvBlock) void k_tv_vote_b(const PairDev* __restrict__ tab, KParams kp, int use_prev) {
    const PairDev A = device_view(tab + blockIdx.y);
    if (A.t.M <= 0 || (int)blockIdx.x * kTvWaves >= A.N) return;
    tv_vote_body(A.t, A.spt, A.N, A.st.pose, A.st.done, kp, const_cast<double4*>(A.t.tvn), use_prev, (int)blockIdx.x);
}

__global__ void k_tensor_gather(const float* __restrict__ ten6, size_t n_in, const unsigned* __restrict__ kept,
                                const float4* __restrict__ mpt, int M, float4* __restrict__ mten) {
    const int m = blockIdx.x * blockDim.x + threadIdx.x;
    if (m >= M) return;
    const size_t in = kept[__float_as_uint(mpt[m].w)];
    mten[2 * (size_t)m] = make_float4(ten6[in], ten6[n_in + in], ten6[2 * n_in + in], ten6[3 * n_in + in]);
    mten[2 * (size_t)m + 1] = make_float4(ten6[4 * n_in + in], ten6[5 * n_in + in], 0.f, 0.f);
}

}  // namespace

void launch_tv_vote(hipStream_t s, const TreeView& t, const float4* spt, int N, const double* pose, const int* done,
                    const KParams& kp, double4* tvn, int use_prev) {
    if (N <= 0 || t.M <= 0) return;
    k_tv_vote<<<(N + kTvWaves - 1) / kTvWaves, kTvBlock, 0, s>>>(t, spt, N, pose, done, kp, tvn, use_prev);
    k_tv_tangent<<<(N + 255) / 256, 256, 0, s>>>(N, done, tvn);
}

void launch_tv_vote_batch(hipStream_t s, const PairDev* tab, const int* n_host, int npairs, const KParams& kp,
                          int use_prev) {
    int maxN = 0;
    for (int k = 0; k < npairs; ++k) maxN = std::max(maxN, n_host[k]);
    if (maxN <= 0) return;
    k_tv_vote_b<<<dim3((maxN + kTvWaves - 1) / kTvWaves, npairs), kTvBlock, 0, s>>>(tab, kp, use_prev);
    k_tv_tangent_b<<<dim3((maxN + 255) / 256, npairs), 256, 0, s>>>(tab);
}

void launch_tensor_gather(hipStream_t s, const float* ten6_in, size_t n_in, const unsigned* kept, const float4* mpt, int M,
                          float4* mten) {
    if (M <= 0) return;
    k_tensor_gather<<<(M + 255) / 256, 256, 0, s>>>(ten6_in, n_in, kept, mpt, M, mten);
}

}  // namespace imlsgpu
