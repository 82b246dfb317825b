// project.hip — fused transform + matching kernel: the GPU form of one ICP iteration's
// Matching step (laser_odometry.cpp:527-549 → IMLSICPMatcher::ProjSourcePtToSurface,
// imls_icp.cpp:496-745 → ImplicitMLSFunction, imls_icp.cpp:301-483).
//
// One lane per source point:
//   1. x = float(rPose·[p;1])  (double, the reference's evaluation order, no FMA)
//   2. one traversal of the target tree collecting, in registers,
//        NN-1 : nearest map point within r with d² > DBL_EPSILON   (knn K=1, no self match,
//               imls_icp.cpp:605-607)
//        L    : the K nearest within r, sorted by (d², index)      (knn K=search_number,
//               ALLOW_SELF_MATCH, imls_icp.cpp:372-375)
//      Candidates are screened with an fp32 distance against the current bound (× (1+2e-6)
//      slack, so no exact candidate is ever screened out) and ranked by the exact fp64 distance
//      ((dx²+dy²)+dz², the libnabo metric), so the neighbour sets equal the oracle's.
//   3. the gates of imls_icp.cpp:612-717 in the reference order, the IMLS height with the
//      h_max quirk (Q3) and the 1e-5 bias (Q4), y = float(x − height·n_NN).
//   4. outputs per source index (source order is the index; compaction is separate), reject
//      counters, and the pass-1 normal-equation partials of the LS solve (solver.cpp:89-107)
//      reduced per block: 21 JᵀJ + 6 Jᵀb + count, fp64.
// Compiled with -ffp-contract=off: every fp64 expression is evaluated as written.
#include <cfloat>

#include "internal.h"

namespace imlsgpu {
namespace {

constexpr double kInfD = __builtin_huge_val();

__device__ __forceinline__ bool lessp(double da, int ia, double db, int ib) {
    return da < db || (da == db && ia < ib);
}

__device__ __forceinline__ float box_d2(const float q[3], float lx, float ly, float lz, float hx, float hy, float hz) {
    float vx = fmaxf(fmaxf(lx - q[0], q[0] - hx), 0.f);
    float vy = fmaxf(fmaxf(ly - q[1], q[1] - hy), 0.f);
    float vz = fmaxf(fmaxf(lz - q[2], q[2] - hz), 0.f);
    return __builtin_fmaf(vx, vx, __builtin_fmaf(vy, vy, vz * vz));
}

// imls_icp.cpp:442-451 / 681-692: acos(ns·n/(|ns||n|))·180/π > threshold; NaN passes (Q8).
__device__ __forceinline__ bool angle_reject(const double ns[3], double n0, double n1, double n2, double thr) {
    double dot = ns[0] * n0;
    dot = dot + ns[1] * n1;
    dot = dot + ns[2] * n2;
    double a = ns[0] * ns[0];
    a = a + ns[1] * ns[1];
    a = a + ns[2] * ns[2];
    double b = n0 * n0;
    b = b + n1 * n1;
    b = b + n2 * n2;
    double ca = dot / (sqrt(a) * sqrt(b));
    double angle = acos(ca) * 180.0 / M_PI;
    return angle > thr;
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

template <int KCAP>
__global__ __launch_bounds__(kProjBlock) void k_project(TreeView t, const float4* __restrict__ spt,
                                                        const float4* __restrict__ snr, int N,
                                                        const double* __restrict__ pose, const int* __restrict__ done,
                                                        KParams kp, float4* __restrict__ cs, float4* __restrict__ cd,
                                                        float4* __restrict__ cn, double* __restrict__ partial1,
                                                        imls_iter_trace* __restrict__ tr,
                                                        unsigned long long* __restrict__ nbr_stats) {
    if (done && *done) return;
    __shared__ uint2 stack[kStackDepth][kProjBlock];
    __shared__ double red[kProjBlock / 64][kNormEq];
    __shared__ unsigned rej_s[IMLS_NUM_REJ + 3];
    const int tid = threadIdx.x;
    if (tid < IMLS_NUM_REJ + 3) rej_s[tid] = 0;
    __syncthreads();

    const int i = blockIdx.x * kProjBlock + tid;
    const bool active = i < N;
    int cat = -2;
    float xf[3] = {0, 0, 0}, yf[3] = {0, 0, 0}, nf[3] = {0, 0, 0};
    int kq = 0, nn_found = 0;
    if (active) {
        double T[12];
#pragma unroll
        for (int k = 0; k < 12; ++k) T[k] = pose[k];
        const float4 p = spt[i];
        const float4 nsv = snr[i];
        const double pd[3] = {p.x, p.y, p.z};
#pragma unroll
        for (int r = 0; r < 3; ++r) {
            double v = T[r * 4 + 0] * pd[0];
            v = v + T[r * 4 + 1] * pd[1];
            v = v + T[r * 4 + 2] * pd[2];
            v = v + T[r * 4 + 3] * 1.0;
            xf[r] = (float)v;
        }
        float nsf[3] = {nsv.x, nsv.y, nsv.z};
        if (kp.transform_normal) {
            const double nd[3] = {nsv.x, nsv.y, nsv.z};
#pragma unroll
            for (int r = 0; r < 3; ++r) {
                double v = T[r * 4 + 0] * nd[0];
                v = v + T[r * 4 + 1] * nd[1];
                v = v + T[r * 4 + 2] * nd[2];
                nsf[r] = (float)v;
            }
        }
        const double xd[3] = {xf[0], xf[1], xf[2]};
        const double ns[3] = {nsf[0], nsf[1], nsf[2]};

        // ---------------- traversal: NN-1 + sorted K list ----------------
        const int K = kp.K;
        double ld[KCAP];
        int li[KCAP];
#pragma unroll
        for (int j = 0; j < KCAP; ++j) {
            const bool sentinel = j < KCAP - K;   // capacity K inside KCAP registers
            ld[j] = sentinel ? -1.0 : kInfD;
            li[j] = sentinel ? -1 : 0x7fffffff;
        }
        double d1 = kInfD;
        int i1 = 0x7fffffff;
        const double r2 = kp.r2;
        double bnd = r2;
        float bf = (float)bnd * (1.0f + 2e-6f) + 1e-30f;

        int node = 1, sp = 0;
        const int P = t.P, B = t.B, M = t.M;
        while (true) {
            if (node < P) {
                const float4* rec = t.nodes + 3 * (size_t)node;
                const float4 a = rec[0], b = rec[1], c = rec[2];
                const float dl = box_d2(xf, a.x, a.y, a.z, a.w, b.x, b.y);
                const float dr = box_d2(xf, b.z, b.w, c.x, c.y, c.z, c.w);
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
                const int bucket = node - P;
                const int s0 = bucket * B, e0 = min(s0 + B, M);
                for (int k = s0; k < e0; ++k) {
                    const float4 q = t.mpt[k];
                    const float ex = q.x - xf[0], ey = q.y - xf[1], ez = q.z - xf[2];
                    const float d32 = __builtin_fmaf(ex, ex, __builtin_fmaf(ey, ey, ez * ez));
                    if (d32 > bf) continue;
                    const double dx = xd[0] - (double)q.x, dy = xd[1] - (double)q.y, dz = xd[2] - (double)q.z;
                    double d2 = dx * dx;
                    d2 = d2 + dy * dy;
                    d2 = d2 + dz * dz;
                    if (!(d2 <= r2)) continue;
                    const int oi = (int)__float_as_uint(q.w);
                    bool changed = false;
                    if (d2 > DBL_EPSILON && lessp(d2, oi, d1, i1)) { d1 = d2; i1 = oi; changed = true; }
                    if (lessp(d2, oi, ld[KCAP - 1], li[KCAP - 1])) {
                        bool prev = true;
#pragma unroll
                        for (int j = KCAP - 1; j >= 0; --j) {
                            const bool sh = (j > 0) ? lessp(d2, oi, ld[j - 1], li[j - 1]) : false;
                            const double nd = sh ? ld[(j > 0) ? j - 1 : 0] : (prev ? d2 : ld[j]);
                            const int ni = sh ? li[(j > 0) ? j - 1 : 0] : (prev ? oi : li[j]);
                            ld[j] = nd;
                            li[j] = ni;
                            prev = sh;
                        }
                        changed = true;
                    }
                    if (changed) {
                        bnd = fmin(r2, fmax(ld[KCAP - 1], d1));
                        bf = (float)bnd * (1.0f + 2e-6f) + 1e-30f;
                    }
                }
                node = 0;
            }
            // pop
            while (sp > 0) {
                --sp;
                const uint2 e = stack[sp][tid];
                if (__uint_as_float(e.y) <= bf) { node = (int)e.x; break; }
            }
            if (!node) break;
        }

        // ---------------- gates (imls_icp.cpp:612-717) ----------------
        nn_found = i1 != 0x7fffffff;
        double nn[3] = {0, 0, 0};
        if (!nn_found) {
            cat = IMLS_REJ_TOO_FAR;                  // InvalidIndex → counted as too far (Q18)
        } else if (d1 > kp.h2) {
            cat = IMLS_REJ_TOO_FAR;
        } else if (!kp.get_normals) {
            cat = IMLS_REJ_INVALID_NORMAL;           // recompute path under libnabo semantics (Q1)
        } else {
            const float4 n4 = t.tnr[i1];
            nn[0] = n4.x; nn[1] = n4.y; nn[2] = n4.z;
            if (!(isfinite(nn[0]) && isfinite(nn[1]) && isfinite(nn[2]))) {
                cat = IMLS_REJ_INVALID_NORMAL;
            } else if (kp.angle_on && angle_reject(ns, nn[0], nn[1], nn[2], kp.angle_thr_deg)) {
                cat = IMLS_REJ_NORMAL_CONSTRAINT;
            } else {
                // ImplicitMLSFunction: walk L in order, keep finite-d², finite-normal, angle-ok
                unsigned acc = 0u;
                int nacc = 0;
#pragma unroll
                for (int j = 0; j < KCAP; ++j) {
                    if (j >= KCAP - K && ld[j] < kInfD) {
                        ++kq;
                        const float4 qn = t.tnr[li[j]];
                        bool ok = isfinite(qn.x) && isfinite(qn.y) && isfinite(qn.z);
                        if (ok && kp.angle_on) ok = !angle_reject(ns, qn.x, qn.y, qn.z, kp.angle_thr_deg);
                        if (ok) { acc |= 1u << j; ++nacc; }
                    }
                }
                if (nacc < 3) {
                    cat = IMLS_REJ_MLS_FAIL;
                } else {
                    const int target = KCAP - K + nacc - 1;   // Q3: index into L, not into S
                    double dsel = 0.0;
#pragma unroll
                    for (int j = 0; j < KCAP; ++j) dsel = (j == target) ? ld[j] : dsel;
                    const double hmax = sqrt(dsel) / 3;
                    double wsum = 0.0, psum = 0.0;
#pragma unroll
                    for (int j = 0; j < KCAP; ++j) {
                        if (acc & (1u << j)) {
                            const float4 qp = t.tpt[li[j]];
                            const float4 qn = t.tnr[li[j]];
                            const double dx = xd[0] - (double)qp.x, dy = xd[1] - (double)qp.y, dz = xd[2] - (double)qp.z;
                            double dn = dx * dx;
                            dn = dn + dy * dy;
                            dn = dn + dz * dz;
                            const double w = exp(-dn / hmax / hmax);
                            double pr = (w * dx) * (double)qn.x;
                            pr = pr + (w * dy) * (double)qn.y;
                            pr = pr + (w * dz) * (double)qn.z;
                            wsum += w;
                            psum += pr;
                        }
                    }
                    const double height = psum / (wsum + 1e-5);
                    if (isnan(height) || isinf(height)) {
                        cat = IMLS_REJ_NAN_INF_HEIGHT;
                    } else {
                        yf[0] = (float)(xd[0] - height * nn[0]);
                        yf[1] = (float)(xd[1] - height * nn[1]);
                        yf[2] = (float)(xd[2] - height * nn[2]);
                        nf[0] = (float)nn[0]; nf[1] = (float)nn[1]; nf[2] = (float)nn[2];
                        cat = -1;
                    }
                }
            }
        }
        cs[i] = make_float4(xf[0], xf[1], xf[2], cat == -1 ? 1.f : 0.f);
        cd[i] = make_float4(yf[0], yf[1], yf[2], 0.f);
        cn[i] = make_float4(nf[0], nf[1], nf[2], 0.f);
    }

    // ---------------- counters ----------------
    if (cat >= 0) atomicAdd(&rej_s[cat], 1u);
    if (active) {
        if (kq) atomicAdd(&rej_s[IMLS_NUM_REJ], (unsigned)kq);
        if (nn_found) atomicAdd(&rej_s[IMLS_NUM_REJ + 1], 1u);
    }

    // ---------------- pass-1 normal equations (solver.cpp:89-107 as JᵀJ, Jᵀb) ----------------
    double a[6] = {0, 0, 0, 0, 0, 0}, bb = 0.0, one = 0.0;
    if (cat == -1) {
        const double s0 = xf[0], s1 = xf[1], s2 = xf[2];
        const double d0 = yf[0], d1_ = yf[1], d2_ = yf[2];
        const double n0 = nf[0], n1 = nf[1], n2 = nf[2];
        a[0] = n2 * s1 - n1 * s2;
        a[1] = n0 * s2 - n2 * s0;
        a[2] = n1 * s0 - n0 * s1;
        a[3] = n0; a[4] = n1; a[5] = n2;
        bb = n0 * (d0 - s0);
        bb = bb + n1 * (d1_ - s1);
        bb = bb + n2 * (d2_ - s2);
        one = 1.0;
    }
    const int lane = tid & 63, wv = tid >> 6;
    int k = 0;
#pragma unroll
    for (int r = 0; r < 6; ++r) {
#pragma unroll
        for (int c = r; c < 6; ++c) {
            const double v = wave_sum(a[r] * a[c]);
            if (lane == 0) red[wv][k] = v;
            ++k;
        }
    }
#pragma unroll
    for (int r = 0; r < 6; ++r) {
        const double v = wave_sum(a[r] * bb);
        if (lane == 0) red[wv][21 + r] = v;
    }
    {
        const double v = wave_sum(one);
        if (lane == 0) red[wv][27] = v;
    }
    __syncthreads();
    if (tid < kNormEq) {
        double s = 0.0;
#pragma unroll
        for (int w = 0; w < kProjBlock / 64; ++w) s += red[w][tid];
        partial1[(size_t)blockIdx.x * kNormEq + tid] = s;
    }
    if (tid < IMLS_NUM_REJ && rej_s[tid]) atomicAdd((unsigned long long*)&tr->reject[tid], (unsigned long long)rej_s[tid]);
    if (nbr_stats && tid >= IMLS_NUM_REJ && tid < IMLS_NUM_REJ + 2 && rej_s[tid])
        atomicAdd(&nbr_stats[tid - IMLS_NUM_REJ], (unsigned long long)rej_s[tid]);
}

}  // namespace

int project_blocks(int N) { return (N + kProjBlock - 1) / kProjBlock; }

void launch_project(hipStream_t s, const TreeView& t, const float4* spt, const float4* snr, int N, const double* pose,
                    const int* done, const KParams& kp, float4* cs, float4* cd, float4* cn, double* partial1,
                    imls_iter_trace* tr, unsigned long long* nbr_stats) {
    const int blocks = project_blocks(N);
    if (kp.K <= 8)
        k_project<8><<<blocks, kProjBlock, 0, s>>>(t, spt, snr, N, pose, done, kp, cs, cd, cn, partial1, tr, nbr_stats);
    else if (kp.K <= 16)
        k_project<16><<<blocks, kProjBlock, 0, s>>>(t, spt, snr, N, pose, done, kp, cs, cd, cn, partial1, tr, nbr_stats);
    else if (kp.K <= 20)
        k_project<20><<<blocks, kProjBlock, 0, s>>>(t, spt, snr, N, pose, done, kp, cs, cd, cn, partial1, tr, nbr_stats);
    else
        k_project<32><<<blocks, kProjBlock, 0, s>>>(t, spt, snr, N, pose, done, kp, cs, cd, cn, partial1, tr, nbr_stats);
}

}  // namespace imlsgpu
