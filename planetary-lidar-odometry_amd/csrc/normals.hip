// normals.hip — map normals recomputed from the map itself: ComputeNormal (imls_icp.cpp:753-794)
// reached through the get_normals=false branch (404-434 for the IMLS neighbours, 634-668 for
// NN-1) in the documented-intent "count" mode of SURVEY Q1 (the reference's own mode is the dead
// one: libnabo's knn() return value is 0, every candidate normal is ∞ — that mode needs no
// kernel, the matcher rejects at once).
//
// Every recomputed normal is a function of one map point only (its kNN-`search_number_normal`
// within r_normal, self match excluded: d² > DBL_EPSILON), so the whole map is done once per
// (map, parameters) and the matcher then reads it like stored normals — exactly what the
// reference computes per candidate, without the per-candidate repetition.
//
// One lane per map point (Morton order): exact fp64 kNN by a per-lane tree traversal (LDS stack,
// fp32 box pruning with slack, libnabo metric, (d², index) order), then mean, covariance / n
// (summed in list order), a cyclic Jacobi 3×3 eigendecomposition, the eigenvector of the smallest
// eigenvalue, normalised, flipped to +z.  Fewer than search_number_normal neighbours → ∞.
#include "solve_common.h"

namespace imlsgpu {
namespace {

constexpr int kNrmBlock = 128;
constexpr float kNrmSlack = 1.0f + 2e-6f;

template <int KC>
__device__ __forceinline__ void map_normals_body(const TreeView& t, int K, double r2, float4* __restrict__ out, int bx) {
    __shared__ uint2 stack[kStackDepth][kNrmBlock];
    const int tid = threadIdx.x;
    const int pos = bx * kNrmBlock + tid;
    if (pos >= t.M) return;
    const float4 q4 = t.mpt[pos];
    const float xf[3] = {q4.x, q4.y, q4.z};
    const double xd[3] = {q4.x, q4.y, q4.z};
    double ld[KC];
    int li[KC], lp[KC];
#pragma unroll
    for (int j = 0; j < KC; ++j) {
        const bool sentinel = j < KC - K;      // capacity K inside KC registers
        ld[j] = sentinel ? -1.0 : INFINITY;
        li[j] = sentinel ? -1 : 0x7fffffff;
        lp[j] = -1;
    }
    float bf = (float)r2 * kNrmSlack + 1e-30f;
    int node = 1, sp = 0;
    const int P = t.P, B = t.B, M = t.M;
    while (true) {
        if (node < P) {
            const float4* rec = t.nodes + 3 * (size_t)node;
            const float4 a = rec[0], b = rec[1], c = rec[2];
            float dl, dr;
            {
                const float lx = fmaxf(fmaxf(a.x - xf[0], 0.f), xf[0] - a.w), ly = fmaxf(fmaxf(a.y - xf[1], 0.f), xf[1] - b.x),
                            lz = fmaxf(fmaxf(a.z - xf[2], 0.f), xf[2] - b.y);
                dl = lx * lx + ly * ly + lz * lz;
                const float rx = fmaxf(fmaxf(b.z - xf[0], 0.f), xf[0] - c.y), ry = fmaxf(fmaxf(b.w - xf[1], 0.f), xf[1] - c.z),
                            rz = fmaxf(fmaxf(c.x - xf[2], 0.f), xf[2] - c.w);
                dr = rx * rx + ry * ry + rz * rz;
            }
            const bool vl = dl <= bf, vr = dr <= bf;
            if (vl && vr) {
                const bool lfirst = dl <= dr;
                stack[sp][tid] = make_uint2(lfirst ? 2 * node + 1 : 2 * node, __float_as_uint(lfirst ? dr : dl));
                ++sp;
                node = lfirst ? 2 * node : 2 * node + 1;
                continue;
            }
            node = vl ? 2 * node : (vr ? 2 * node + 1 : 0);
            if (node) continue;
        } else {
            const int s0 = (node - P) * B, e0 = min(s0 + B, M);
            for (int k = s0; k < e0; ++k) {
                const float4 p4 = t.mpt[k];
                const float ex = p4.x - xf[0], ey = p4.y - xf[1], ez = p4.z - xf[2];
                const float d32 = __builtin_fmaf(ex, ex, __builtin_fmaf(ey, ey, ez * ez));
                if (d32 > bf) continue;
                const double dx = xd[0] - (double)p4.x, dy = xd[1] - (double)p4.y, dz = xd[2] - (double)p4.z;
                double d2 = dx * dx;
                d2 = d2 + dy * dy;
                d2 = d2 + dz * dz;
                if (!(d2 <= r2 && d2 > DBL_EPSILON)) continue;
                const int oi = (int)__float_as_uint(p4.w);
                if (!(d2 < ld[KC - 1] || (d2 == ld[KC - 1] && oi < li[KC - 1]))) continue;
                bool prev = true;
#pragma unroll
                for (int j = KC - 1; j >= 0; --j) {
                    const int jm = j > 0 ? j - 1 : 0;
                    const bool sh = j > 0 && (d2 < ld[jm] || (d2 == ld[jm] && oi < li[jm]));
                    const double nd = sh ? ld[jm] : (prev ? d2 : ld[j]);
                    const int ni = sh ? li[jm] : (prev ? oi : li[j]);
                    const int np = sh ? lp[jm] : (prev ? k : lp[j]);
                    ld[j] = nd;
                    li[j] = ni;
                    lp[j] = np;
                    prev = sh;
                }
                bf = (float)fmin(r2, ld[KC - 1]) * kNrmSlack + 1e-30f;
            }
            node = 0;
        }
        while (sp > 0) {
            --sp;
            const uint2 e = stack[sp][tid];
            if (__uint_as_float(e.y) <= bf) { node = (int)e.x; break; }
        }
        if (!node) break;
    }
    int n = 0;
#pragma unroll
    for (int j = 0; j < KC; ++j) n += (j >= KC - K && ld[j] < INFINITY) ? 1 : 0;
    if (n < K) {   // imls_icp.cpp:418-421 / 654-657: too few neighbours → ∞ normal
        out[pos] = make_float4(INFINITY, INFINITY, INFINITY, 0.f);
        return;
    }
    // ComputeNormal (imls_icp.cpp:753-794) over the K neighbours in list order
    double mu[3] = {0, 0, 0};
#pragma unroll
    for (int j = 0; j < KC; ++j) {
        if (j >= KC - K) {
            const float4 p4 = t.mpt[lp[j]];
            mu[0] += p4.x; mu[1] += p4.y; mu[2] += p4.z;
        }
    }
#pragma unroll
    for (int d = 0; d < 3; ++d) mu[d] /= K;
    double C[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int j = 0; j < KC; ++j) {
        if (j >= KC - K) {
            const float4 p4 = t.mpt[lp[j]];
            const double v[3] = {p4.x - mu[0], p4.y - mu[1], p4.z - mu[2]};
#pragma unroll
            for (int r = 0; r < 3; ++r)
#pragma unroll
                for (int c = 0; c < 3; ++c) C[r * 3 + c] += v[r] * v[c];
        }
    }
#pragma unroll
    for (int k = 0; k < 9; ++k) C[k] /= K;
    double ev[3], U[9];
    sym_eig<3>(C, ev, U);
    const double nn = sqrt(U[0] * U[0] + U[1] * U[1] + U[2] * U[2]);
    double nr[3] = {U[0] / nn, U[1] / nn, U[2] / nn};
    if (nr[2] < 0) { nr[0] = -nr[0]; nr[1] = -nr[1]; nr[2] = -nr[2]; }
    out[pos] = make_float4((float)nr[0], (float)nr[1], (float)nr[2], 0.f);
}

template <int KC>
__global__ __launch_bounds__(kNrmBlock) void k_map_normals(TreeView t, int K, double r2, float4* __restrict__ out) {
    map_normals_body<KC>(t, K, r2, out, (int)blockIdx.x);
}

// batched (imls_register_frames): the maps of the frames flagged recompute_normals, grid y = frame
template <int KC>
__global__ __launch_bounds__(kNrmBlock) void k_map_normals_b(const PairDev* __restrict__ tab, int K, double r2) {
    const PairDev A = device_view(tab + blockIdx.y);
    if (!A.recompute_normals || (int)blockIdx.x * kNrmBlock >= A.t.M) return;
    map_normals_body<KC>(A.t, K, r2, const_cast<float4*>(A.t.mnr), (int)blockIdx.x);
}

}  // namespace

int launch_map_normals_batch(hipStream_t s, const PairDev* tab, int npairs, int maxM, int K, double r_normal) {
    if (maxM <= 0 || npairs <= 0) return 0;
    const dim3 g((maxM + kNrmBlock - 1) / kNrmBlock, npairs);
    const double r2 = r_normal * r_normal;
    if (K <= 8) k_map_normals_b<8><<<g, kNrmBlock, 0, s>>>(tab, K, r2);
    else if (K <= 16) k_map_normals_b<16><<<g, kNrmBlock, 0, s>>>(tab, K, r2);
    else if (K <= 32) k_map_normals_b<32><<<g, kNrmBlock, 0, s>>>(tab, K, r2);
    else return -1;
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_map_normals(hipStream_t s, const TreeView& t, int K, double r_normal, float4* out) {
    if (t.M <= 0) return 0;
    const int blocks = (t.M + kNrmBlock - 1) / kNrmBlock;
    const double r2 = r_normal * r_normal;
    if (K <= 8) k_map_normals<8><<<blocks, kNrmBlock, 0, s>>>(t, K, r2, out);
    else if (K <= 16) k_map_normals<16><<<blocks, kNrmBlock, 0, s>>>(t, K, r2, out);
    else if (K <= 32) k_map_normals<32><<<blocks, kNrmBlock, 0, s>>>(t, K, r2, out);
    else return -1;
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace imlsgpu
