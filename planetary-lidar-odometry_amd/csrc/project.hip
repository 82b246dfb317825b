// project.hip — fused transform + matching kernels: the GPU form of one ICP iteration's Matching
// step (laser_odometry.cpp:527-549 → IMLSICPMatcher::ProjSourcePtToSurface, imls_icp.cpp:496-745
// → ImplicitMLSFunction, imls_icp.cpp:301-483).
//
// k_knn_wave (hot kernel 1) — wave-coherent ("packet") traversal of the target tree:
//   * a wave owns 64 queries taken in Morton order of the source scan, so they are neighbours;
//   * ONE traversal per wave: the node index and the LDS stack (node + its box, so a pop needs no
//     memory round trip) are wave-uniform, node records come through the scalar cache; a child is
//     entered when any lane's box distance is within that lane's bound (ballot), near-first by
//     lane majority;
//   * a leaf (B ≤ 64 Morton-consecutive map points) is ONE coalesced float4 load, each point is
//     broadcast to all lanes by v_readlane and tested against each lane's register top-(K+4)
//     list keyed by the fp32 distance;
//   * bounds: iteration 0 seeds each lane from its nearest leaf (greedy descent); later ICP
//     iterations prefill the list with the previous iteration's neighbours re-measured at the
//     new pose (temporal coherence: the pose changes little), so few leaf points insert;
//   * output: the list positions (Morton order) and the worst key W per query, to HBM.
// k_finish (hot kernel 2) — one lane per query: the exact stage — fp64 distances
//   ((dx²+dy²)+dz², the libnabo metric, no FMA) of the list, sorted by (d², index), the radius
//   filter (d² ≤ r², inclusive), NN-1 = first entry with d² > DBL_EPSILON (no self match,
//   imls_icp.cpp:605-607), L = first K (ALLOW_SELF_MATCH, imls_icp.cpp:372-375);
//   CERTIFICATION — every map point outside the list has d²₆₄ ≥ W/(1+3.1e-7)
//   (|d²₃₂ − d²₆₄| ≤ 5·2⁻²⁴·d²), so the result is exact iff the largest exact distance it relies
//   on is < W/(1+4e-7); uncertified queries (near-ties at the list edge, > K+4 duplicates) are
//   appended to a list that k_project_lane re-runs exactly.  Then the gates
//   (imls_icp.cpp:612-717 in order), IMLS height with the h_max quirk (Q3) and the 1e-5 bias (Q4),
//   y = float(x − height·n_NN), and the pass-1 normal-equation partials of the LS solve
//   (solver.cpp:89-107): 21 JᵀJ + 6 Jᵀb + count per block, fp64.
// k_project_lane — one lane per query, exact fp64 list during the traversal (the fallback, and
// the IMLS_TRAVERSAL_LANE reference mode, imls_set_option).
// Compiled with -ffp-contract=off: every fp64 expression evaluates as written.
#include <algorithm>
#include <cfloat>

#include "internal.h"
#include "geom.h"

namespace imlsgpu {
namespace {

constexpr double kInfD = __builtin_huge_val();
constexpr float kInfF = __builtin_huge_valf();
constexpr int kWaveBlock = 256;
// constant address space view of read-only device data: wave-uniform loads through it are scalar
typedef float kf4v __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(4))) const kf4v kconst_f4;
// a value an earlier launch wrote and the whole wave reads (the done flag, the last Δ): through the
// constant address space, i.e. scalar loads — not a per-lane (flat, in the batched kernels) load
__device__ __forceinline__ int ld_const(const int* p) { return *(const __attribute__((address_space(4))) int*)p; }
__device__ __forceinline__ double ld_const(const double* p) { return *(const __attribute__((address_space(4))) double*)p; }
constexpr int kFallbackBlocks = 64;
constexpr int kFallbackBlocksBatched = 4;   // physical blocks per frame of a large batch (same slabs)
// queries per k_finish block = per pass-1 slab (the quad exact stage: 64; the one-lane form: 256)
constexpr int kFinishPerBlock = IMLS_FINISH_QUAD ? kWaveBlock / 4 : kWaveBlock;
static_assert(kFinishPerBlock == kPass1Block && kFallbackBlocks == kPass1Fallback, "pass-1 slab layout (solve.hip)");
// the later ICP iterations' packet traversal in two launches (reuse decision + compacted walk, round 6):
// measured slower (a walk's cost is its node visits, which compaction only concentrates into fewer,
// longer walks — profiles/r06_compact_rejected/), off; kept for same-box A/B builds
#ifndef IMLS_COMPACT
#define IMLS_COMPACT 0
#endif
constexpr int kWideMax = 8;         // packet traversal: children tested per step (2^wide, wide ≤ 3)
constexpr int kWaveStack = 64;       // its stack: ≤ 7 entries per step × ⌈23/3⌉ steps
constexpr int kFStack = 256;        // frontier traversal's stack per wave (see knn_qwave_body)
constexpr int kFBatchMax = 128;     // above this many entries: one entry per step (DFS growth ≤ 8 × 7)
// frontier stack bound: a step at ≤ kFBatchMax entries pushes ≤ 8 groups × 8 children; above it one
// entry per step grows the stack by ≤ 7 per descent step, and a walk descends ≤ ⌈(kStackDepth−1)/kWide⌉
// steps (the index refuses deeper trees, index.hip) — so fsp never exceeds kFStack
static_assert(kFBatchMax + 64 + 7 * ((24 + 2) / 3) <= kFStack, "frontier stack bound");
#ifndef IMLS_SEED_CHUNK
#define IMLS_SEED_CHUNK 8
#endif
constexpr int kSeedChunk = IMLS_SEED_CHUNK;   // per-lane reseed: points loaded per batch
constexpr int kSeedTab = 1024;                // seed search: coarse leaf-key table entries in LDS (8 KB)
// traversal constants (measured in rounds 1-4; no runtime selectors)
constexpr int kSeedHalf = 1;        // a seed scans the query's Morton leaf ± 1 neighbour leaf
constexpr float kReseed = 0.25f;    // temporal seed unless displacement² > kReseed · previous worst key
// the packet traversal prefetches the stack top's leaf points during a leaf scan (round 6 A/B)
#ifndef IMLS_LEAF_PREFETCH
#define IMLS_LEAF_PREFETCH 1
#endif
#ifndef IMLS_BCAST_SCALAR
#define IMLS_BCAST_SCALAR 1
#endif
#ifndef IMLS_BC_GROUP
#define IMLS_BC_GROUP 4
#endif
__attribute__((unused)) constexpr int kBcGroup = IMLS_BC_GROUP;          // broadcast leaf scan: points per scalar-load group (IMLS_BCAST_SCALAR)
#ifndef IMLS_SPARSE_LANES
#define IMLS_SPARSE_LANES 20
#endif
constexpr int kSparseLanes = IMLS_SPARSE_LANES;    // a leaf wanted by ≤ this many lanes is scanned per lane, not per point
constexpr int kWide = 3;            // binary levels descended per traversal step (8 boxes per step)
constexpr float kBoxSlack = 1.0f + 2e-6f;     // fp32 box / point distance vs exact: ≤ 3.1e-7 rel.
// Round 6: the traversals search radius (1 + skin)·r, not r.  A query with fewer than K map points
// within r ("underfull": the far, sparse part of a scan) relies on EVERY point within r; its list from
// a search of radius r could never be reused (no skin: any move may bring a point inside r), so it
// re-walked the whole r-ball every ICP iteration — the converged iterations' tail.  Searched to
// (1 + skin)·r, its list certifies reuse while the query moves < skin·r / 2 (need = r², verlet_skip).
// Dense queries are unaffected (their bound is the KL-th key ≪ r² after the seed / prefill); k_finish
// still counts only the points within r.
#ifndef IMLS_UNDER_SKIN
#define IMLS_UNDER_SKIN 0.05
#endif
constexpr double kSearchR2 = (1.0 + IMLS_UNDER_SKIN) * (1.0 + IMLS_UNDER_SKIN);   // search r² / r²
constexpr double kCertSlack = 1.0 + 4e-7;
// list length for K ≤ 20 (the shipped K = 20)
#ifndef IMLS_B_KL
#define IMLS_B_KL 22
#endif
#ifndef IMLS_DIST_CHUNK
#define IMLS_DIST_CHUNK 22
#endif
#ifndef IMLS_IMLS_CHUNK
#define IMLS_IMLS_CHUNK 4
#endif

__device__ __forceinline__ bool lessp(double da, int ia, double db, int ib) {
    return da < db || (da == db && ia < ib);
}

// imls_icp.cpp:442-451 / 681-692: acos(ns·n/(|ns||n|))·180/π > threshold; NaN passes (Q8).
// cthr = cos(threshold): away from it (|ca − cthr| > 1e-9, where the evaluated angle is ≥ 5e-8°
// from the threshold — ~6 orders above its rounding error) the comparison is decided without the
// fp64 acos; inside that band, and for NaN or ca < −1 (acos → NaN → passes), as the reference.
__device__ __forceinline__ bool angle_reject(const double ns[3], double n0, double n1, double n2, double thr,
                                             double cthr) {
    // fp32 screen: |ca₃₂ − ca₆₄| ≤ ~1e-6 (inputs rounded to float: 6e-8 each, the dot and the two
    // squared norms ≤ 3 ulp of their term sums, v_rsq ≤ 2 ulp — Cauchy–Schwarz bounds the dot's
    // terms by |ns||n|), so outside ±1e-5 of cos(θ) (and of −1) the fp32 cosine decides what the
    // fp64 evaluation below decides; squared-norm products outside [1e-20, 1e20] (denormal / huge /
    // NaN normals) and the band go to fp64
    {
        const float s0 = (float)ns[0], s1 = (float)ns[1], s2 = (float)ns[2];
        const float m0 = (float)n0, m1 = (float)n1, m2 = (float)n2;
        const float a = __builtin_fmaf(s0, s0, __builtin_fmaf(s1, s1, s2 * s2));
        const float b = __builtin_fmaf(m0, m0, __builtin_fmaf(m1, m1, m2 * m2));
        const float d = __builtin_fmaf(s0, m0, __builtin_fmaf(s1, m1, s2 * m2));
        const float ab = a * b;
        if (ab > 1e-20f && ab < 1e20f) {
            const float ca = d * __builtin_amdgcn_rsqf(ab);
            const float c = (float)cthr;
            if (ca > c + 1e-5f) return false;
            if (ca < c - 1e-5f && ca > -1.0f + 1e-5f) return true;
        }
    }
    double dot = ns[0] * n0;
    dot = dot + ns[1] * n1;
    dot = dot + ns[2] * n2;
    double a = ns[0] * ns[0];
    a = a + ns[1] * ns[1];
    a = a + ns[2] * ns[2];
    double b = n0 * n0;
    b = b + n1 * n1;
    b = b + n2 * n2;
    const double s = sqrt(a) * sqrt(b);
    // the same two decisions without the division: outside ±2e-9 of cthr, dot vs (cthr ± 2e-9)·s
    // decides exactly what ca = dot/s vs cthr ± 1e-9 decides (the division's rounding is ~1e-16
    // relative), and dot ≥ −s(1 − 1e-12) certifies ca ≥ −1; anything else (the bands, zero / ∞ /
    // NaN denominators) takes the reference's own evaluation below
    if (dot > (cthr + 2e-9) * s) return false;
    if (dot < (cthr - 2e-9) * s && dot >= -s * (1.0 - 1e-12)) return true;
    const double ca = dot / s;
    if (ca > cthr + 1e-9) return false;
    if (ca < cthr - 1e-9 && ca >= -1.0) return true;
    const double angle = acos(ca) * 180.0 / M_PI;
    return angle > thr;
}

// Sorted insertion of (d, pos) into the ascending top-KL list; precondition d < lk[KL−1].  With
// c[k] = d < lk[k] (old keys; monotone in k, so the first true c is the insertion point) every slot
// is independent of the others: key k = med3(lk[k−1], d, lk[k]) (= lk[k−1] when c[k−1], else
// min(d, lk[k]): the keys are sorted and never NaN), position k = c[k−1] ? lp[k−1] : (c[k] ? pos :
// lp[k]) — one v_med3 + one compare + two selects per slot, none of fminf's canonicalising maxes.
// Equal keys keep their order (a new key goes after the ones it equals).
template <int KL>
__device__ __forceinline__ void insert_top(float (&lk)[KL], int (&lp)[KL], float d, int pos) {
    bool c[KL];
#pragma unroll
    for (int k = 0; k < KL - 1; ++k) c[k] = d < lk[k];
    c[KL - 1] = true;
#pragma unroll
    for (int k = KL - 1; k >= 1; --k) {
        lp[k] = c[k - 1] ? lp[k - 1] : (c[k] ? pos : lp[k]);
        lk[k] = __builtin_amdgcn_fmed3f(lk[k - 1], d, lk[k]);
    }
    lp[0] = c[0] ? pos : lp[0];
    lk[0] = c[0] ? d : lk[0];
}

// min(a, b) of non-NaN floats (a plain select: fminf canonicalises both operands first)
__device__ __forceinline__ float fmin_nn(float a, float b) { return a < b ? a : b; }

// Keeps a gather where it is issued: the empty asm consumes the loaded registers, so the compiler
// cannot sink the load into the conditional block that uses it (and wait on it there, one
// dependent round trip per gather) — the loads of a chunk all issue before any is waited on.
__device__ __forceinline__ void pin_loaded(const float4& v) { asm volatile("" ::"v"(v.x), "v"(v.y), "v"(v.z)); }

// Keys-only sorted insertion (precondition d < lk[KL−1]): one v_med3 per slot.
template <int KL>
__device__ __forceinline__ void insert_key(float (&lk)[KL], float d) {
#pragma unroll
    for (int k = KL - 1; k >= 1; --k) lk[k] = __builtin_amdgcn_fmed3f(lk[k - 1], d, lk[k]);
    lk[0] = fmin_nn(d, lk[0]);
}

// Gates + ImplicitMLSFunction + projection for one query given its exact neighbour list
// L = (ld[j], lpos[j]) for j ∈ [first, first+cnt) sorted by (d², index) and its NN-1 (d1, p1);
// positions are Morton positions (mpt/mnr: the neighbours of a query share cache lines).
// Returns the reject category or −1 (valid, yf/nf filled).  kq counts the returned neighbours.
// LAZY_D: ld is not read — the one distance the IMLS bandwidth needs (L[target], Q3) is recomputed
// from its point (the same fp64 expression, so the same bits), letting the caller's fp64 list die
// after the certification (k_finish's register budget).
template <int CAP, bool LAZY_D = false>
__device__ int finish_query(const float xf[3], const double ns[3], const double (&ld)[CAP], const int (&lpos)[CAP],
                            int first, int cnt, double d1, int p1, const TreeView& t, const KParams& kp, float yf[3],
                            float nf[3], int& kq, int qi) {
    if (p1 < 0) return IMLS_REJ_TOO_FAR;                      // InvalidIndex → counted as too far (Q18)
    if (d1 > kp.h2) return IMLS_REJ_TOO_FAR;                  // imls_icp.cpp:620
    double nn[3];
    if (kp.tv) {
        // imls_icp.cpp:634-643: the query's own voted normal (tv.hip); a zero tensor has none
        const double4 v = t.tvn[qi];
        if (v.w == 0.0) return IMLS_REJ_NO_NORMAL;
        nn[0] = v.x; nn[1] = v.y; nn[2] = v.z;
    } else {
        if (!kp.get_normals) return IMLS_REJ_INVALID_NORMAL;  // recompute branch under libnabo semantics (Q1)
        const float4 n4 = t.mnr[p1];
        nn[0] = n4.x; nn[1] = n4.y; nn[2] = n4.z;
    }
    if (!(isfinite(nn[0]) && isfinite(nn[1]) && isfinite(nn[2]))) return IMLS_REJ_INVALID_NORMAL;
    if (kp.angle_on && angle_reject(ns, nn[0], nn[1], nn[2], kp.angle_thr_deg, kp.cos_thr)) return IMLS_REJ_NORMAL_CONSTRAINT;
    const double xd[3] = {xf[0], xf[1], xf[2]};
    unsigned long long acc = 0ull;
    int nacc = 0;
    // the normals in chunks of 8 (the loads of a chunk issue together; 24 VGPRs in flight, not 3·CAP)
    constexpr int kChunk = 8;
#pragma unroll
    for (int j0 = 0; j0 < CAP; j0 += kChunk) {
        float4 qn[kChunk];
#pragma unroll
        for (int u = 0; u < kChunk; ++u) {
            const int j = j0 + u;
            const bool inl = j < CAP && j >= first && j < first + cnt;
            qn[u] = t.mnr[inl ? lpos[j < CAP ? j : 0] : p1];
        }
#pragma unroll
        for (int u = 0; u < kChunk; ++u) {
            const int j = j0 + u;
            const bool inl = j < CAP && j >= first && j < first + cnt;
            if (inl) {
                ++kq;
                // get_normals=false without count mode (TV's IMLS neighbours): every normal is ∞ (Q1)
                bool ok = kp.get_normals && isfinite(qn[u].x) && isfinite(qn[u].y) && isfinite(qn[u].z);
                if (ok && kp.angle_on) ok = !angle_reject(ns, qn[u].x, qn[u].y, qn[u].z, kp.angle_thr_deg, kp.cos_thr);
                if (ok) { acc |= 1ull << j; ++nacc; }
            }
        }
    }
    if (nacc < 3) return IMLS_REJ_MLS_FAIL;                   // imls_icp.cpp:463-466
    const int target = first + nacc - 1;                      // Q3: index into L, not into S
    // the accepted neighbours' points and normals in chunks of 8, every load of a chunk issued (and
    // pinned) before any term is formed — the first chunk with the bandwidth point L[target]; a term
    // is added as `accepted ? term : 0`, the same bits as skipping it (both sums start at +0 and so
    // are never −0: s + 0 = s)
    constexpr int kIChunk = IMLS_IMLS_CHUNK;
    float4 qp[kIChunk], qn[kIChunk];
    auto load_chunk = [&](int j0) {
#pragma unroll
        for (int u = 0; u < kIChunk; ++u) {
            const int j = j0 + u;
            const int pj = (j < CAP && (acc & (1ull << j))) ? lpos[j < CAP ? j : 0] : p1;
            qp[u] = t.mpt[pj];
            qn[u] = t.mnr[pj];
        }
    };
    auto pin_chunk = [&]() {
#pragma unroll
        for (int u = 0; u < kIChunk; ++u) {
            pin_loaded(qp[u]);
            pin_loaded(qn[u]);
        }
    };
    double dsel = 0.0;
    if (LAZY_D) {
        int ptg = p1;
#pragma unroll
        for (int j = 0; j < CAP; ++j) ptg = (j == target) ? lpos[j] : ptg;
        const float4 q = t.mpt[ptg];
        load_chunk(0);
        pin_loaded(q);
        pin_chunk();
        dsel = exact_d2(xd, q.x, q.y, q.z);
    } else {
#pragma unroll
        for (int j = 0; j < CAP; ++j) dsel = (j == target) ? ld[j] : dsel;
        load_chunk(0);
        pin_chunk();
    }
    const double hmax = sqrt(dsel) / 3;
    // exp(−‖x−p‖² / h / h) (imls_icp.cpp:470) with one reciprocal per query instead of two divisions
    // per neighbour: w moves by ≤ 2 ulp, y (stored as float) almost never (the 1e-5 y contract)
    const double ih2 = 1.0 / (hmax * hmax);
    double wsum = 0.0, psum = 0.0;
#pragma unroll
    for (int j0 = 0; j0 < CAP; j0 += kIChunk) {
        if (j0 > 0) {
            if (!__ballot((acc >> j0) != 0ull)) break;          // no lane has a later neighbour
            if (!__ballot((acc >> j0) & ((1ull << kIChunk) - 1ull))) continue;     // none in this chunk
            load_chunk(j0);
            pin_chunk();
        }
#pragma unroll
        for (int u = 0; u < kIChunk; ++u) {
            const int j = j0 + u;
            if (j >= CAP) break;
            const bool a = (acc >> j) & 1ull;
            if (!__ballot(a)) continue;                         // wave-uniform
            const double dx = xd[0] - (double)qp[u].x, dy = xd[1] - (double)qp[u].y, dz = xd[2] - (double)qp[u].z;
            double dn = dx * dx;
            dn = dn + dy * dy;
            dn = dn + dz * dz;
            const double w = exp(-dn * ih2);
            double pr = (w * dx) * (double)qn[u].x;
            pr = pr + (w * dy) * (double)qn[u].y;
            pr = pr + (w * dz) * (double)qn[u].z;
            wsum += a ? w : 0.0;
            psum += a ? pr : 0.0;
        }
    }
    const double height = psum / (wsum + 1e-5);               // Q4
    if (isnan(height) || isinf(height)) return IMLS_REJ_NAN_INF_HEIGHT;
    yf[0] = (float)(xd[0] - height * nn[0]);                  // imls_icp.cpp:719-729
    yf[1] = (float)(xd[1] - height * nn[1]);
    yf[2] = (float)(xd[2] - height * nn[2]);
    nf[0] = (float)nn[0]; nf[1] = (float)nn[1]; nf[2] = (float)nn[2];
    return -1;
}

// plane_ICP_proj's loop body after the NN-1 search (laser_odometry.cpp:352-396): unfound → "no
// normal" (the bounds check; no h gate — min_dist is unused) or, in projected-distance mode, an
// empty candidate list → "too far" (336-340); map normal finite, angle gate,
// y = x − ((x−p)·n)·n in double, stored as float.
__device__ int finish_plane(const float xf[3], const double ns[3], int p1, const TreeView& t, const KParams& kp,
                            float yf[3], float nf[3]) {
    if (p1 < 0) return kp.proj ? IMLS_REJ_TOO_FAR : IMLS_REJ_NO_NORMAL;   // empty candidate list: 336-340
    const float4 n4 = t.mnr[p1];
    const double nn[3] = {n4.x, n4.y, n4.z};
    if (!(isfinite(nn[0]) && isfinite(nn[1]) && isfinite(nn[2]))) return IMLS_REJ_INVALID_NORMAL;
    if (kp.angle_on && angle_reject(ns, nn[0], nn[1], nn[2], kp.angle_thr_deg, kp.cos_thr)) return IMLS_REJ_NORMAL_CONSTRAINT;
    const float4 q = t.mpt[p1];
    const double xd[3] = {xf[0], xf[1], xf[2]};
    const double v0 = xd[0] - (double)q.x, v1 = xd[1] - (double)q.y, v2 = xd[2] - (double)q.z;
    double pd = v0 * nn[0];
    pd = pd + v1 * nn[1];
    pd = pd + v2 * nn[2];
    yf[0] = (float)(xd[0] - pd * nn[0]);
    yf[1] = (float)(xd[1] - pd * nn[1]);
    yf[2] = (float)(xd[2] - pd * nn[2]);
    nf[0] = (float)nn[0]; nf[1] = (float)nn[1]; nf[2] = (float)nn[2];
    return -1;
}

// Row of the point-to-plane system for a valid correspondence (solver.cpp:95-103).
__device__ __forceinline__ void plane_row(const float xf[3], const float yf[3], const float nf[3], double a[6], double& b) {
    const double s0 = xf[0], s1 = xf[1], s2 = xf[2];
    const double d0 = yf[0], d1 = yf[1], d2 = yf[2];
    const double n0 = nf[0], n1 = nf[1], n2 = nf[2];
    a[0] = n2 * s1 - n1 * s2;
    a[1] = n0 * s2 - n2 * s0;
    a[2] = n1 * s0 - n0 * s1;
    a[3] = n0; a[4] = n1; a[5] = n2;
    b = n0 * (d0 - s0);
    b = b + n1 * (d1 - s1);
    b = b + n2 * (d2 - s2);
}

// Block-reduce the 28 normal-equation terms into out[0..27] (valid in threads < 28 after return).
template <int NT>
__device__ void block_normeq(const double a[6], double b, double one, double (*red)[kNormEq], double* out) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    int k = 0;
#pragma unroll
    for (int r = 0; r < 6; ++r) {
#pragma unroll
        for (int c = r; c < 6; ++c) {
            const double v = wave_total(a[r] * a[c]);
            if (lane == 63) red[wv][k] = v;
            ++k;
        }
    }
#pragma unroll
    for (int r = 0; r < 6; ++r) {
        const double v = wave_total(a[r] * b);
        if (lane == 63) red[wv][21 + r] = v;
    }
    {
        const double v = wave_total(one);
        if (lane == 63) red[wv][27] = v;
    }
    __syncthreads();
    if (threadIdx.x < kNormEq) {
        double s = 0.0;
#pragma unroll
        for (int w = 0; w < NT / 64; ++w) s += red[w][threadIdx.x];
        out[threadIdx.x] = s;
    }
    __syncthreads();
}

__device__ __forceinline__ void store_result(int i, int cat, const float xf[3], const float yf[3], const float nf[3],
                                             float4* cs, float4* cd, float4* cn) {
    cs[i] = make_float4(xf[0], xf[1], xf[2], cat == -1 ? 1.f : 0.f);
    // y and n are read only behind the valid flag (Rows::get, the RANSAC compaction, imls_project):
    // rejected rows skip them
    if (cat == -1) {
        cd[i] = make_float4(yf[0], yf[1], yf[2], 0.f);
        cn[i] = make_float4(nf[0], nf[1], nf[2], 0.f);
    }
}

// =============================================================================================
// Packet traversal (hot kernel 1): per-query top-KL list positions + worst key
// =============================================================================================
#ifdef IMLS_DEBUG_WAVE_TRACE
constexpr int kDbgWaves = 8192;
__device__ unsigned g_dbg_wave[kDbgWaves][16];
#endif


// Verlet-list reuse (neighbour lists with a skin, as in molecular dynamics): a query's list was
// built at xr.xyz with the guarantee that every map point outside it has fp32 key ≥ xr.w, and
// nr = the key its exact answer relied on there (the K-th key within r, or the NN-1 key if
// larger; ∞ when fewer than K points were within r).  At the new position x, |x − xr| = D:
//   * every point outside the list is at exact distance ≥ √xr.w − D          (lower bound W'),
//   * the answer needs distances ≤ √nr + D (those K points are still there)   (upper bound U),
// so the list — unchanged, not even re-read — still holds the exact answer when U < W'.
// fp32 keys carry ≤ 3.1e-7 relative error and D ≤ 3e-7: the 1e-6 factors and the 1e-5 margin
// cover both; k_finish re-certifies in fp64 against W' (a failure there only costs the exact
// fallback).  Returns true when the traversal can be skipped; w_out = W' (also when the stale
// bound U fails: w_low = W' whenever it is positive, else −1 — the prefilled list, re-measured at x,
// may still certify itself against it, see knn_wave_body).
__device__ __forceinline__ bool verlet_skip(float4 xr, float nr, const float xf[3], float r2s, float& w_out,
                                            float& w_low) {
    const float dx = xf[0] - xr.x, dy = xf[1] - xr.y, dz = xf[2] - xr.z;
    const float D = sqrtf(__builtin_fmaf(dx, dx, __builtin_fmaf(dy, dy, dz * dz))) * (1.0f + 1e-6f) + 1e-6f;
    const float g = sqrtf(xr.w) * (1.0f - 1e-6f) - D;
    w_low = g > 0.f ? fminf(g * g, r2s) : -1.0f;
    if (!(g > 0.f) || !(nr < kInfF)) return false;
    const float u = sqrtf(nr) * (1.0f + 1e-6f) + D;
    const float w = fminf(g * g, r2s);
    w_out = w;
    return u * u * (1.0f + 1e-5f) < w;
}

// The key a fresh list's exact answer relies on (see verlet_skip): max(K-th key within r, NN-1
// key), ∞ when fewer than K keys are within r or no NN-1 exists.  lk ascending.
template <int KL>
__device__ __forceinline__ float need_key(const float (&lk)[KL], float r2, int K) {
    const float r2f = r2 * (1.0f + 1e-6f);
    int cnt_r = 0;
    float dK = kInfF, d1 = kInfF;
#pragma unroll
    for (int j = 0; j < KL; ++j) {
        const bool in = lk[j] <= r2f;
        cnt_r += in ? 1 : 0;
        if (in && d1 == kInfF && lk[j] > 1e-15f) d1 = lk[j];
        if (j == K - 1) dK = lk[j];
    }
    // fewer than K within r: the answer is every point within r (none when no NN-1 exists either)
    return cnt_r >= K ? fmaxf(dK, d1) : (IMLS_UNDER_SKIN > 0 ? r2f : kInfF);
}

// ---------------------------------------------------------------------------------------------
// Slot-id keys (the LDS-list traversal): a lane's top-KL list is its KL keys in registers, kept
// ascending, each key = the fp32 squared distance with its low IDB mantissa bits replaced by the id
// of the LDS slot that holds the point's position.  An insertion evicts the list's last key, whose
// slot takes the new position (one ds_write at a lane-specific address) and whose id the new key
// inherits; the keys move by med3 alone (one VALU per slot) — the positions never move, where the
// register list moves every position with two selects per slot (88 → ~26 VALU per insertion).
//
// Truncation keeps the search exact.  A point is inserted iff trunc(d) < trunc(max key), i.e.
// d < thr = float(bits(max) & ~IDM); thr only falls during the walk, so every point never inserted
// has d ≥ thr_final, and an evicted point's truncated key was ≥ the new maximum's — every point
// outside the final list has d32 ≥ thr_final, which is the W this traversal reports (≤ 2^(IDB−23)
// below the full-precision KL-th key: k_finish's fp64 certificate against W is unchanged).
// Upper bounds taken from a key (need_key_ids, the Verlet reuse) round up: d ≤ float(bits | IDM).
// Empty slots hold finite sentinels kIdSentinel | id (above every real key, never NaN for med3).
// ---------------------------------------------------------------------------------------------
template <int KL>
struct IdKeys {
    static constexpr unsigned IDM = KL <= 32 ? 31u : 63u;
    static constexpr unsigned kSentinel = 0x7F7FFFFFu & ~IDM;
    __device__ static __forceinline__ float lo(float k) { return __uint_as_float(__float_as_uint(k) & ~IDM); }
    __device__ static __forceinline__ float hi(float k) { return __uint_as_float(__float_as_uint(k) | IDM); }
    __device__ static __forceinline__ unsigned id(float k) { return __float_as_uint(k) & IDM; }
    __device__ static __forceinline__ float make(float d, unsigned s) { return __uint_as_float((__float_as_uint(d) & ~IDM) | s); }
    __device__ static __forceinline__ float empty(unsigned s) { return __uint_as_float(kSentinel | s); }
    __device__ static __forceinline__ bool real(float k) { return (__float_as_uint(k) & ~IDM) < kSentinel; }
};

// need_key over slot-id keys: max(K-th key within r, NN-1 key), every bound rounded up (a key's
// point lies in [lo, hi]); ∞ when fewer than K keys are surely within r or no NN-1 exists.
template <int KL>
__device__ __forceinline__ float need_key_ids(const float (&lk)[KL], float r2, int K) {
    using I = IdKeys<KL>;
    const float r2f = r2 * (1.0f + 1e-6f);
    int cnt_r = 0;
    float dK = kInfF, d1 = kInfF;
#pragma unroll
    for (int j = 0; j < KL; ++j) {
        const float up = I::hi(lk[j]);
        const bool in = I::real(lk[j]) && up <= r2f;
        cnt_r += in ? 1 : 0;
        if (in && d1 == kInfF && I::lo(lk[j]) > 1e-15f) d1 = up;
        if (j == K - 1) dK = up;
    }
    return cnt_r >= K ? fmaxf(dK, d1) : (IMLS_UNDER_SKIN > 0 ? r2f : kInfF);   // (need_key)
}

// Slot-id keys in registers, positions in LDS: ~96 VGPRs and ~29 KB of LDS per 4-wave block — 5
// waves/SIMD (round 4: the register list needed 160 VGPRs, 3 waves/SIMD; config B 331 → 406 pairs/s)
#ifndef IMLS_KNN_WAVES
#define IMLS_KNN_WAVES 5
#endif
#define IMLS_KNN_ATTR __attribute__((amdgpu_waves_per_eu(KL <= 26 ? IMLS_KNN_WAVES : 2)))
// MODE (round 6, the later ICP iterations of the packet traversal, use_prev):
//   0  one pass — every lane decides reuse and the packets walk for the lanes that cannot reuse;
//   1  the reuse decision only (Verlet skip, prefill certificate): a reused list is settled here,
//      the block's other slots are compacted, in slot (Morton) order, into the block's own region
//      of cmp, with their count in cmp_count[block];
//   2  the walk over a block's compacted slots, 64 to a packet: fewer packets walk, each full of
//      queries that really re-traverse, from the block's 4·64 Morton-consecutive slots (instead of
//      every packet walking for the few of its lanes that do).  The lane redoes MODE 1's decision
//      (same inputs, same outcome), its prefill included.
//   3  the first ICP iterations' walk with a breadth-first top (k_knn_wave_bfs[b], IMLS_BFS_ITERS):
//      the upper levels expanded against the packet's box, the frontier handed to the depth-first
//      stack.  Measured slower (profiles/r06_bfs_rejected/): off by default, kept for A/B builds.
// (A first version compacted through one atomic counter per frame: packets of runs from anywhere in
// the frame walked 2-6× longer — profiles/r06_compact_rejected/.  Modes 1 and 2 are off as well:
// IMLS_COMPACT.)
template <int KL, int MODE = 0>
__device__ __forceinline__ void knn_wave_body(TreeView t, const float4* __restrict__ spt,
                                                         const unsigned* __restrict__ qperm, int N,
                                                         const double* __restrict__ pose,
                                                         const int* __restrict__ done, KParams kp,
                                                         const double* __restrict__ delta,
                                                         int* __restrict__ lists, float* __restrict__ wlist,
                                                         float4* __restrict__ xref, float* __restrict__ nref,
                                                         int use_prev, unsigned long long* __restrict__ nbr_stats,
                                                         int bx, unsigned* __restrict__ cmp = nullptr,
                                                         unsigned* __restrict__ cmp_count = nullptr) {
    if (done && ld_const(done)) return;
    __shared__ int snode[kWaveBlock / 64][kWaveStack];
    __shared__ float4 sboxa[kWaveBlock / 64][kWaveStack];   // stacked node boxes: lo.xyz, hi.x
    __shared__ float2 sboxb[kWaveBlock / 64][kWaveStack];   //                     hi.yz
    // the list's positions, slot s of thread tid at spos[s][tid] (slot-id keys, IdKeys)
    __shared__ int spos[KL][kWaveBlock];
    const int tid = threadIdx.x, lane = tid & 63;
    int* const mypos = &spos[0][tid];
    using IK = IdKeys<KL>;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    // a wave owns kp.packet Morton-consecutive queries (64; 32 or 16 in the first iterations, where
    // most lanes seed: a smaller packet's union of neighbourhoods is smaller, and the launch lasts
    // as long as its slowest wave); lanes past the packet idle
    const int qp = kp.packet;
    const int pslot = (bx * (kWaveBlock / 64) + wv) * qp + lane;
    int slot = pslot;
    bool active = lane < qp && slot < N;
    if constexpr (MODE == 2) {
        // packet = the block's compacted entries [wv·qp, wv·qp + qp); the count is the prep launch's
        // (no block barrier in this mode: use_prev — a wave past it leaves at once)
        const int cnt = ld_const((const int*)cmp_count + bx);
        if (wv * qp >= cnt) return;
        active = lane < qp && wv * qp + lane < cnt;
        slot = active ? (int)cmp[(size_t)bx * (kWaveBlock / 64) * qp + wv * qp + lane] : 0;
    }
    float xf[3] = {0.f, 0.f, 0.f};
    // the stored list's bound and reference (slot-indexed) load beside the query's point: one round
    // trip after the query index, not one more after the transform
    float w_prev = 0.f, n_prev = 0.f;
    float4 x_prev = make_float4(0.f, 0.f, 0.f, 0.f);
    if (active) {
        double ns[3];
        const int i = (int)qperm[slot];
        const float4 sp4 = spt[i];
        if (use_prev) {
            w_prev = wlist[slot];
            x_prev = xref[slot];
            n_prev = nref[slot];
        }
        transform_query(pose, sp4, make_float4(0.f, 0.f, 0.f, 0.f), 0, xf, ns);
    }
    float lk[KL];
#pragma unroll
    for (int j = 0; j < KL; ++j) lk[j] = IK::empty(j);
    // the slots are cleared here when no seed table is staged; in the first ICP iteration the table
    // aliases spos and they are cleared after the seed search, below
    if (use_prev) {
#pragma unroll
        for (int j = 0; j < KL; ++j) mypos[j * kWaveBlock] = -1;
    }
    // the list behind one interface: thr_ = the strict insertion threshold (a point with key d joins
    // iff d < thr_()), ins_ = sorted insertion (precondition d < thr_()), pos_ = position of slot s
    // (any order), full_ = KL real entries, need_ = need_key (upper-rounded for slot-id keys)
    auto thr_ = [&]() -> float { return IK::lo(lk[KL - 1]); };
    auto full_ = [&]() -> bool { return IK::real(lk[KL - 1]); };
    auto pos_ = [&](int s) -> int { return mypos[s * kWaveBlock]; };
    auto need_ = [&]() -> float { return need_key_ids<KL>(lk, (float)kp.r2, kp.K); };
    auto ins_ = [&](float d, int pos) {
        const unsigned s = IK::id(lk[KL - 1]);
        insert_key<KL>(lk, IK::make(d, s));
        mypos[s * kWaveBlock] = pos;
    };
    const float r2s = (float)(kp.r2 * kSearchR2) * kBoxSlack + 1e-30f;   // the search bound (radius (1 + skin)·r)
    float bnd = active ? r2s : -1.0f;
    const int P = t.P, B = t.B, M = t.M;
#ifdef IMLS_DEBUG_WAVE_TRACE
    const long long dbg_t0 = wall_clock64();
#endif
    bool greedy = active && !use_prev;
    bool skip = false;               // list certified without a traversal (Verlet-list reuse)
    float wskip = kInfF;
    if (active && use_prev) {
        // temporal seed only while the query moved little against its neighbourhood: the last
        // pose increment Δ moves it by at most ‖t‖ + ‖R − I‖_F·‖x‖
        double rf = 0.0;
#pragma unroll
        for (int r = 0; r < 3; ++r)
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                const double e = ld_const(delta + r * 4 + c) - (r == c ? 1.0 : 0.0);
                rf += e * e;
            }
        const double d3 = ld_const(delta + 3), d7 = ld_const(delta + 7), d11 = ld_const(delta + 11);
        const float tn = (float)sqrt(d3 * d3 + d7 * d7 + d11 * d11);
        const float disp = tn + (float)sqrt(rf) * sqrtf(xf[0] * xf[0] + xf[1] * xf[1] + xf[2] * xf[2]);
        greedy = disp * disp > kReseed * w_prev;
    }
    float wlow = -1.0f;              // W' of the stored list at xf (prefill certificate below)
    if (active && !greedy && kp.reuse) skip = verlet_skip(x_prev, n_prev, xf, r2s, wskip, wlow);
    if (active && !greedy && !skip) {
        // prefill from the previous iteration's list re-measured at the new pose: all positions,
        // then all points are loaded before any is consumed (two memory round trips, not 2·KL),
        // and the nearly sorted keys are ordered by an early-exit odd-even transposition sort
        // (the list is full and the bound tight before the traversal starts; a later leaf insert
        // must then skip points already listed).  Slot j keeps entry j's position; its key carries
        // id j (the keys alone get sorted)
        // The points in two chunks, each chunk's loads issued (pinned) before any of its slot writes:
        // in the batched kernel the table's pointers are generic, so a point load after a slot write
        // (an LDS store it might alias) waited for it — one round trip per entry
        int pj[KL];
#pragma unroll
        for (int j = 0; j < KL; ++j) pj[j] = lists[(size_t)j * N + slot];
        constexpr int kPCh = (KL + 1) / 2;
#pragma unroll
        for (int j0 = 0; j0 < KL; j0 += kPCh) {
            float4 q[kPCh];
#pragma unroll
            for (int u = 0; u < kPCh; ++u)
                if (j0 + u < KL) q[u] = t.mpt[max(pj[j0 + u], 0)];
#pragma unroll
            for (int u = 0; u < kPCh; ++u)
                if (j0 + u < KL) pin_loaded(q[u]);
#pragma unroll
            for (int u = 0; u < kPCh; ++u) {
                const int j = j0 + u;
                if (j >= KL) break;
                const float ex = q[u].x - xf[0], ey = q[u].y - xf[1], ez = q[u].z - xf[2];
                const float d32 = __builtin_fmaf(ex, ex, __builtin_fmaf(ey, ey, ez * ez));
                const bool keep = pj[j] >= 0 && d32 <= r2s;
                lk[j] = keep ? IK::make(d32, j) : IK::empty(j);
                mypos[j * kWaveBlock] = keep ? pj[j] : -1;
            }
        }
        bool swapped = true;
        while (swapped) {
            swapped = false;
#pragma unroll
            for (int par = 0; par < 2; ++par) {
#pragma unroll
                for (int j = par; j + 1 < KL; j += 2) {
                    const bool sw = lk[j + 1] < lk[j];
                    const float tk = lk[j];
                    lk[j] = sw ? lk[j + 1] : lk[j];
                    lk[j + 1] = sw ? tk : lk[j + 1];
                    swapped |= sw;
                }
            }
        }
        bnd = fmin_nn(r2s, thr_());
        // prefill certificate: the stored list re-measured at xf holds its answer when the key that
        // answer relies on (max(K-th key within r, NN-1 key), need_key) is below W' — every point
        // outside the list is at least √W' away (verlet_skip) — so the traversal is skipped exactly
        // as for a Verlet reuse; the stale bound √nr + D there is the worst case of this re-measured
        // key.  (fp32 slack as in verlet_skip; k_finish re-certifies the list in fp64 against W'.)
        if (kp.reuse && wlow > 0.f) {
            const float nk = need_();
            if (nk < kInfF && nk * (1.0f + 1e-5f) < wlow) { skip = true; wskip = wlow; }
        }
    }
    if constexpr (MODE == 1) {
        // settle the reused lists; compact the rest for the MODE 2 walk
        if (active && skip) wlist[slot] = wskip;
        const unsigned long long sk = __ballot(skip);
        if (nbr_stats && lane == 0 && sk) atomicAdd(&nbr_stats[kStatSkipped], (unsigned long long)__popcll(sk));
        const bool need = active && !skip;
        const unsigned long long nm = __ballot(need);
        __shared__ int wneed[kWaveBlock / 64];
        if (lane == 0) wneed[wv] = __popcll(nm);
        __syncthreads();              // every wave of the block reaches here (MODE 1 leaves below)
        int off = 0, tot = 0;
#pragma unroll
        for (int w = 0; w < kWaveBlock / 64; ++w) {
            off += w < wv ? wneed[w] : 0;
            tot += wneed[w];
        }
        if (need) cmp[(size_t)bx * (kWaveBlock / 64) * qp + off + __popcll(nm & ((1ull << lane) - 1ull))] = (unsigned)slot;
        if (tid == 0) cmp_count[bx] = (unsigned)tot;
        return;
    }
    // leaf scan shared by the seed pass and the traversal: the lanes in `want` test every point of
    // leaf `leaf` against their bound; `listed`: the leaf may hold points already in a lane's
    // list (prefilled or seeded), which must not be inserted twice
#ifdef IMLS_DEBUG_WAVE_TRACE
    unsigned dbg_ev = 0, dbg_ins = 0;
    unsigned dbg_sparse = 0, dbg_bcast = 0, dbg_sparse_lanes = 0, dbg_sparse_ins = 0;
    unsigned dbg_seed_steps = 0, dbg_seed_pts = 0;   // seed points where any lane inserted / seed points scanned
#endif
    // mine: lane k's point k of the leaf (loaded by the caller; zero past the leaf's count)
    auto scan_leaf = [&](int leaf, unsigned long long want, bool listed, float4 mine) {
        const int base = leaf * B;
        const int cnt = min(B, M - base);
        // points of this leaf already in the lane's list, as a bit mask: one lockstep pass over
        // the list instead of a divergent membership test per point
        unsigned long long inl = 0ull;
        auto listed_mask = [&]() {
#pragma unroll
            for (int k = 0; k < KL; ++k) {
                const unsigned rel = (unsigned)(pos_(k) - base);
                inl |= rel < 64u ? (1ull << rel) : 0ull;
            }
        };
        const bool sparse = __popcll(want) <= kSparseLanes;
#ifdef IMLS_DEBUG_WAVE_TRACE
        if (sparse) { ++dbg_sparse; dbg_sparse_lanes += __popcll(want); } else { ++dbg_bcast; }
#endif
        if (sparse) {
            // few lanes want this leaf (spread-out queries in a dense region): per wanting lane,
            // all leaf points are measured at once (one per lane) and the ones under that lane's
            // bound and not yet listed become its candidate mask; then the lanes insert their own
            // candidates in lockstep, each its lowest pending point per step (index order) fetched
            // by ds_bpermute — max(per-lane candidates) insertion steps instead of one per
            // candidate of every lane.  Per lane, the insertions are exactly the sequential scan's
            // (same order, re-tested at the current bound; a non-candidate was above the
            // leaf-start bound already).
            // Listed points: only their NUMBER in the leaf per lane up front (3 ops per list slot
            // instead of 7).  Every listed point of the leaf is a candidate of its lane (its key,
            // recomputed here bit for bit, is ≤ the lane's candidate bound cb), so a lane with
            // exactly that many candidates has no new one; the mask itself is built only when some
            // lane has more (a leaf with new points).  cb must admit every listed point: slot-id
            // keys truncate, so a listed point can lie up to hi(max key) (the insertion loop
            // re-tests d32 < thr_())
            int nin = 0;
            bool have_inl = !listed;
            if (listed) {
#pragma unroll
                for (int k = 0; k < KL; ++k) nin += (unsigned)(pos_(k) - base) < (unsigned)cnt ? 1 : 0;
            }
            const float cb = fmin_nn(r2s, IK::hi(lk[KL - 1]));
            unsigned long long cm = 0ull;
            unsigned long long m = want;
            while (m) {
                const int q = __builtin_amdgcn_readfirstlane(__builtin_ctzll(m));
                m &= m - 1;
                const float qx = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(xf[0]), q));
                const float qy = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(xf[1]), q));
                const float qz = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(xf[2]), q));
                const float qb = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(cb), q));
                const float ex = mine.x - qx, ey = mine.y - qy, ez = mine.z - qz;
                const float d32 = __builtin_fmaf(ex, ex, __builtin_fmaf(ey, ey, ez * ez));
                unsigned long long pm = __ballot(lane < cnt && d32 <= qb);
                if (!have_inl) {
                    const int nq = __builtin_amdgcn_readlane(nin, q);
                    if (__popcll(pm) > nq) {
                        listed_mask();
                        have_inl = true;
                    } else {
                        pm = 0ull;
                    }
                }
                if (pm) {
                    const unsigned long long inq =
                        ((unsigned long long)(unsigned)__builtin_amdgcn_readlane((int)(unsigned)(inl >> 32), q) << 32) |
                        (unsigned)__builtin_amdgcn_readlane((int)(unsigned)inl, q);
                    pm &= ~inq;
                }
                if (lane == q) cm = pm;
            }
            while (__ballot(cm != 0ull)) {
                // every lane takes part in the permutes (lanes without a candidate read lane 0)
                const int jj = cm ? (int)__builtin_ctzll(cm) : 0;
                const float px = __shfl(mine.x, jj), py = __shfl(mine.y, jj), pz = __shfl(mine.z, jj);
                if (cm) {
                    cm &= cm - 1;
                    const float ex = px - xf[0], ey = py - xf[1], ez = pz - xf[2];
                    const float d32 = __builtin_fmaf(ex, ex, __builtin_fmaf(ey, ey, ez * ez));
                    if (d32 <= bnd && d32 < thr_()) {
#ifdef IMLS_DEBUG_WAVE_TRACE
                        ++dbg_ins;
#endif
                        ins_(d32, base + jj);
                        bnd = fmin_nn(r2s, thr_());
                    }
                }
#ifdef IMLS_DEBUG_WAVE_TRACE
                ++dbg_ev;
#endif
            }
        } else {
            if (listed) listed_mask();
            const bool wants = (want >> lane) & 1ull;
#if IMLS_BCAST_SCALAR
            // broadcast, round 6: the leaf's points come by scalar loads (wave-uniform addresses, a
            // group of kBcGroup points per s_load burst, the next group in flight while this one is
            // measured) and feed the distance VALUs as SGPR operands — no v_readlane per coordinate;
            // a group none of whose points is under any wanting lane's bound (the common case once
            // the bounds are tight) costs one compare and one branch instead of one per point.  The
            // insertion order and the keys are the per-point scan's, bit for bit.
            const kconst_f4* lp = (const kconst_f4*)t.mpt + base;
            kf4v g[kBcGroup];
#pragma unroll
            for (int u = 0; u < kBcGroup; ++u) g[u] = lp[min(u, cnt - 1)];
            for (int j0 = 0; j0 < cnt; j0 += kBcGroup) {
                kf4v nx[kBcGroup];
                const int jn = j0 + kBcGroup;
                if (jn + kBcGroup <= cnt) {   // a whole group: one base address, immediate offsets
                    const kconst_f4* q = lp + jn;
#pragma unroll
                    for (int u = 0; u < kBcGroup; ++u) nx[u] = q[u];
                } else {
#pragma unroll
                    for (int u = 0; u < kBcGroup; ++u) nx[u] = lp[min(jn + u, cnt - 1)];
                }
                float d[kBcGroup];
                float dmin = kInfF;
#pragma unroll
                for (int u = 0; u < kBcGroup; ++u) {
                    const float ex = g[u].x - xf[0], ey = g[u].y - xf[1], ez = g[u].z - xf[2];
                    d[u] = __builtin_fmaf(ex, ex, __builtin_fmaf(ey, ey, ez * ez));
                    dmin = fminf(dmin, d[u]);   // past cnt: a copy of the last point (never inserted)
                }
                if (__ballot(wants && dmin <= bnd)) {
#pragma unroll
                    for (int u = 0; u < kBcGroup; ++u) {
                        const int j = j0 + u;
                        const bool ins = j < cnt && wants && d[u] <= bnd && d[u] < thr_() && !((inl >> j) & 1ull);
                        if (ins) {
                            ins_(d[u], base + j);
                            bnd = fmin_nn(r2s, thr_());
                        }
                    }
                }
#pragma unroll
                for (int u = 0; u < kBcGroup; ++u) g[u] = nx[u];
            }
#else
            // broadcast: each point goes to every lane by v_readlane, every wanting lane tests it
            // against its list
            for (int j = 0; j < cnt; ++j) {
                const float px = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(mine.x), j));
                const float py = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(mine.y), j));
                const float pz = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(mine.z), j));
                const float ex = px - xf[0], ey = py - xf[1], ez = pz - xf[2];
                const float d32 = __builtin_fmaf(ex, ex, __builtin_fmaf(ey, ey, ez * ez));
                const bool ins = wants && d32 <= bnd && d32 < thr_() && !((inl >> j) & 1ull);
#ifdef IMLS_DEBUG_WAVE_TRACE
                const unsigned long long bi = __ballot(ins);
                dbg_ev += bi ? 1 : 0;
                dbg_ins += __popcll(bi);
#endif
                if (ins) {
                    ins_(d32, base + j);
                    bnd = fmin_nn(r2s, thr_());
                }
            }
#endif
        }
    };
    // seed (first ICP iteration, or a lane that moved far): the leaf holding the lane's own Morton
    // key (binary search over the leaves' first keys) ± kSeedHalf, scanned per lane — Morton-near
    // points are mostly space-near, while a greedy box-distance descent goes astray in the heavily
    // overlapping upper-level boxes.  The traversal re-scans these leaves harmlessly (listed points
    // are masked, the rest are not under the bound).
    const unsigned long long gmask = __ballot(greedy);
    // the seed search's leaf: its first ~10 bisection steps run in a coarse table of every S-th
    // leaf key staged in LDS (one coalesced block load), the last ⌈log2 S⌉ in HBM/L2 — instead of
    // ~15 dependent global loads per lane (first ICP iteration only, where every lane seeds: later
    // iterations reseed a few lanes, which would not repay the block barrier).  The table lives in
    // spos, whose slots are not in use yet (cleared after the search)
    static_assert(KL * kWaveBlock * 4 >= kSeedTab * 8, "seed table fits the slot array");
    unsigned long long* const skey = reinterpret_cast<unsigned long long*>(&spos[0][0]);
    const int S = use_prev ? t.L : (t.L + kSeedTab - 1) / kSeedTab;
    const int ntab = S > 0 ? (t.L + S - 1) / S : 0;
    if (!use_prev) {
        for (int k = threadIdx.x; k < ntab; k += kWaveBlock) skey[k] = t.lkeys[(size_t)k * S];
        __syncthreads();
    }
    int seed_leaf = 0;
    if (greedy) {
        const unsigned long long qk = morton48(xf[0], xf[1], xf[2], t.qparams);
        int j = 0, jh = ntab - 1;
        while (j < jh) {
            const int mid = (j + jh + 1) >> 1;
            if (skey[mid] <= qk) j = mid;
            else jh = mid - 1;
        }
        int l = j * S, h = min(t.L, (j + 1) * S) - 1;   // the largest leaf l with lkeys[l] ≤ qk (else 0)
        while (l < h) {
            const int mid = (l + h + 1) >> 1;
            if (t.lkeys[mid] <= qk) l = mid;
            else h = mid - 1;
        }
        seed_leaf = l;
    }
    if (!use_prev) {
        __syncthreads();             // every wave is done with the seed table (it aliases spos)
#pragma unroll
        for (int j = 0; j < KL; ++j) mypos[j * kWaveBlock] = -1;
    }
    if (greedy) {
        const int l = seed_leaf;
        const int p0s = max(0, l - kSeedHalf) * B;
        const int pend = min(M, (min(t.L - 1, l + kSeedHalf) + 1) * B);
        float4 qs[kSeedChunk];
#pragma unroll
        for (int k = 0; k < kSeedChunk; ++k) qs[k] = t.mpt[min(p0s + k, pend - 1)];
        for (int p0 = p0s; p0 < pend; p0 += kSeedChunk) {
            float4 nx[kSeedChunk];   // software pipelined: the next chunk is in flight while this one is consumed
#pragma unroll
            for (int k = 0; k < kSeedChunk; ++k) nx[k] = t.mpt[min(p0 + kSeedChunk + k, pend - 1)];
#pragma unroll
            for (int k = 0; k < kSeedChunk; ++k) {
                const float ex = qs[k].x - xf[0], ey = qs[k].y - xf[1], ez = qs[k].z - xf[2];
                const float d32 = __builtin_fmaf(ex, ex, __builtin_fmaf(ey, ey, ez * ez));
#ifdef IMLS_DEBUG_WAVE_TRACE
                dbg_seed_steps += __ballot(p0 + k < pend && d32 <= bnd && d32 < thr_()) ? 1 : 0;
                ++dbg_seed_pts;
#endif
                if (p0 + k < pend && d32 <= bnd && d32 < thr_()) {
                    ins_(d32, p0 + k);
                    bnd = fmin_nn(r2s, thr_());
                }
            }
#pragma unroll
            for (int k = 0; k < kSeedChunk; ++k) qs[k] = nx[k];
        }
    }
    unsigned n_inner = 0, n_leaf = 0;
#ifdef IMLS_DEBUG_WAVE_TRACE
    const long long dbg_t1 = wall_clock64();
#endif
    if (skip) bnd = -1.0f;           // a certified lane takes no part in the traversal
    int node = 1, sp = 0;
#if IMLS_LEAF_PREFETCH
    int pf_leaf = -1;                 // the leaf whose points `pf` holds (wave-uniform)
    float4 pf = make_float4(0.f, 0.f, 0.f, 0.f);
#endif
    unsigned long long em = __ballot(active && !skip);   // lanes whose bound admits the current node's box
    const unsigned long long skipped = __ballot(skip);
    if (nbr_stats && lane == 0 && skipped) atomicAdd(&nbr_stats[kStatSkipped], (unsigned long long)__popcll(skipped));
    if constexpr (MODE == 3) {
        // Breadth-first top of the walk (round 6, the first ICP iterations, whose waves walk ~55 dependent
        // node / leaf steps): the upper levels are expanded a whole level-step at a time — one lane per
        // frontier node, its 2^sw children tested against the packet's box (the union of the lanes'
        // search balls, a superset of every lane's own test) — while the frontier plus the depth-first
        // pushes still to come below it fit the wave's stack; the frontier then becomes that stack
        // (Morton order on top) and the depth-first walk continues from it, every entry re-checked
        // against the lanes' shrinking bounds at its pop.  Exact either way: nothing a lane's ball
        // reaches is dropped (the box is inflated past fp32 rounding), and k_finish certifies each list.
        if (em) {
            const bool walk = active && !skip;
            const float rr = walk ? sqrtf(bnd * kBoxSlack) * (1.0f + 1e-5f) + 1e-5f : 0.f;
            float plo[3], phi[3];
#pragma unroll
            for (int a = 0; a < 3; ++a) {
                plo[a] = walk ? xf[a] - rr : kInfF;
                phi[a] = walk ? xf[a] + rr : -kInfF;
            }
#pragma unroll
            for (int o = 1; o < 64; o <<= 1)
#pragma unroll
                for (int a = 0; a < 3; ++a) {
                    plo[a] = fminf(plo[a], __shfl_xor(plo[a], o, 64));
                    phi[a] = fmaxf(phi[a], __shfl_xor(phi[a], o, 64));
                }
            int fc = 1, lev = 0;
            if (lane == 0) snode[wv][0] = 1;
            while (lev < t.levels) {
                const int sw = min(kWide, t.levels - lev), nk = 1 << sw;
                const int below = t.levels - lev - sw;
                const int reserve = (kWideMax - 1) * ((below + kWide - 1) / kWide);
                const int n = lane < fc ? snode[wv][lane] : 0;
                const float4* rec = t.nodes + 3 * ((size_t)(n > 0 ? n : 1) << (sw - 1));
                auto child_box = [&](int k, float (&lo)[3], float (&hi)[3]) {
                    const float4 ra = rec[3 * (k >> 1)], rb = rec[3 * (k >> 1) + 1], rc = rec[3 * (k >> 1) + 2];
                    if (k & 1) { lo[0] = rb.z; lo[1] = rb.w; lo[2] = rc.x; hi[0] = rc.y; hi[1] = rc.z; hi[2] = rc.w; }
                    else { lo[0] = ra.x; lo[1] = ra.y; lo[2] = ra.z; hi[0] = ra.w; hi[1] = rb.x; hi[2] = rb.y; }
                };
                unsigned cm = 0u;
                if (lane < fc) {
#pragma unroll
                    for (int k = 0; k < kWideMax; ++k) {
                        if (k >= nk) break;
                        float lo[3], hi[3];
                        child_box(k, lo, hi);
                        const bool ov = lo[0] <= phi[0] && hi[0] >= plo[0] && lo[1] <= phi[1] && hi[1] >= plo[1] &&
                                        lo[2] <= phi[2] && hi[2] >= plo[2];
                        cm |= ov ? (1u << k) : 0u;
                    }
                }
                // exclusive prefix of the lanes' child counts (the next frontier keeps Morton order)
                const int cnt = __popc(cm);
                int inc = cnt;
#pragma unroll
                for (int o = 1; o < 64; o <<= 1) {
                    const int v = __shfl_up(inc, o, 64);
                    if (lane >= o) inc += v;
                }
                const int total = __shfl(inc, 63, 64);
                if (total == 0 || total + reserve > kWaveStack) break;
                int off = inc - cnt;
                if (cm) {
#pragma unroll
                    for (int k = 0; k < kWideMax; ++k) {
                        if (!((cm >> k) & 1u)) continue;
                        float lo[3], hi[3];
                        child_box(k, lo, hi);
                        snode[wv][off] = (n << sw) + k;
                        sboxa[wv][off] = make_float4(lo[0], lo[1], lo[2], hi[0]);
                        sboxb[wv][off] = make_float2(hi[1], hi[2]);
                        ++off;
                    }
                }
                fc = total;
                lev += sw;
                ++n_inner;
            }
            if (lev > 0) {
                // the frontier becomes the depth-first stack, its Morton-first entry on top
                int en = 0;
                float4 ea = make_float4(0.f, 0.f, 0.f, 0.f);
                float2 eb = make_float2(0.f, 0.f);
                if (lane < fc) { en = snode[wv][lane]; ea = sboxa[wv][lane]; eb = sboxb[wv][lane]; }
                if (lane < fc) { snode[wv][fc - 1 - lane] = en; sboxa[wv][fc - 1 - lane] = ea; sboxb[wv][fc - 1 - lane] = eb; }
                sp = fc;
                node = 0;
                while (sp > 0) {
                    --sp;
                    const float4 b0 = sboxa[wv][sp];
                    const float2 b1 = sboxb[wv][sp];
                    const float d = box_d2(xf, b0.x, b0.y, b0.z, b0.w, b1.x, b1.y);
                    em = __ballot(d <= bnd * kBoxSlack);
                    if (em) { node = snode[wv][sp]; break; }
                }
                if (!node) em = 0ull;
            }
        }
    }
    while (em) {
        if (node < P) {
            // one step descends `sw` binary levels at once: the 2^sw descendants' boxes sit in
            // the 2^(sw−1) consecutive records of the intermediate level (one scalar burst of
            // ≤ 192 B), so a root-to-leaf walk costs ⌈levels/3⌉ dependent loads instead of levels
            ++n_inner;
            const int lev = 31 - __builtin_clz(node);
            const int sw = min(kWide, t.levels - lev);
            const int nk = 1 << sw, nrec = nk >> 1;
            // the records are read-only for the whole kernel and the address is wave-uniform: read
            // them through the constant address space so they come by scalar loads into SGPRs (a
            // generic pointer is may-clobbered by the fences / atomics of this kernel and would be
            // fetched by vector loads into 48 VGPRs)
            const int unode = __builtin_amdgcn_readfirstlane(node);
            const kconst_f4* rec = (const kconst_f4*)t.nodes + 3 * ((size_t)unode << (sw - 1));
            float4 R[3 * (kWideMax / 2)];
#pragma unroll
            for (int k = 0; k < 3 * (kWideMax / 2); ++k) {
                const kf4v v = rec[min(k, 3 * nrec - 1)];
                R[k] = make_float4(v.x, v.y, v.z, v.w);
            }
            const float bs = bnd * kBoxSlack;
            unsigned long long m[kWideMax];
            int best = -1;
            float bd = kInfF;
#pragma unroll
            for (int k = 0; k < kWideMax; ++k) {
                const float4 a = R[3 * (k >> 1)], b = R[3 * (k >> 1) + 1], c = R[3 * (k >> 1) + 2];
                const float d = (k & 1) ? box_d2(xf, b.z, b.w, c.x, c.y, c.z, c.w) : box_d2(xf, a.x, a.y, a.z, a.w, b.x, b.y);
                const bool w = k < nk && d <= bs;
                m[k] = __ballot(w);
                if (w && d < bd) { bd = d; best = k; }
            }
            // descend into the child most lanes find nearest; stack the other wanted ones so that
            // they pop in Morton (index) order
            int cstar = -1, vbest = 0;
#pragma unroll
            for (int k = 0; k < kWideMax; ++k) {
                const int v = __popcll(__ballot(best == k));
                if (m[k] && (cstar < 0 || v > vbest)) { cstar = k; vbest = v; }
            }
            if (cstar >= 0) {
#pragma unroll
                for (int k = kWideMax - 1; k >= 0; --k) {
                    if (m[k] && k != cstar) {
                        if (lane == 0) {
                            const float4 a = R[3 * (k >> 1)], b = R[3 * (k >> 1) + 1], c = R[3 * (k >> 1) + 2];
                            snode[wv][sp] = (node << sw) + k;
                            sboxa[wv][sp] = (k & 1) ? make_float4(b.z, b.w, c.x, c.y) : make_float4(a.x, a.y, a.z, a.w);
                            sboxb[wv][sp] = (k & 1) ? make_float2(c.z, c.w) : make_float2(b.x, b.y);
                        }
                        ++sp;
                    }
                }
                em = m[cstar];
                node = (node << sw) + cstar;
                continue;
            }
        } else {
            ++n_leaf;
            const int leaf = node - P;
            float4 mine = make_float4(0.f, 0.f, 0.f, 0.f);
#if IMLS_LEAF_PREFETCH
            // the leaf's points were prefetched when it was the stack's top during the previous leaf
            // scan; else loaded now.  Then the stack's top, when it is a leaf (most often the next node
            // visited: a sibling at the bottom level), has its points in flight during this scan
            if (leaf == pf_leaf) mine = pf;
            else if (lane < min(B, M - leaf * B)) mine = t.mpt[leaf * B + lane];
            pf_leaf = -1;
            if (sp > 0) {
                const int nn = __builtin_amdgcn_readfirstlane(snode[wv][sp - 1]);
                if (nn >= P) {
                    pf_leaf = nn - P;
                    pf = make_float4(0.f, 0.f, 0.f, 0.f);
                    if (lane < min(B, M - pf_leaf * B)) pf = t.mpt[pf_leaf * B + lane];
                }
            }
#else
            // (a broadcast scan reads the leaf by scalar loads: the per-lane copy only for a sparse one)
            if ((!IMLS_BCAST_SCALAR || __popcll(em) <= kSparseLanes) && lane < min(B, M - leaf * B))
                mine = t.mpt[leaf * B + lane];
#endif
            scan_leaf(leaf, em, use_prev || gmask, mine);
        }
        // pop: the stacked node's box is in LDS — re-check it against the shrunken lane bounds
        node = 0;
        while (sp > 0) {
            --sp;
            const float4 b0 = sboxa[wv][sp];
            const float2 b1 = sboxb[wv][sp];
            const float d = box_d2(xf, b0.x, b0.y, b0.z, b0.w, b1.x, b1.y);
            em = __ballot(d <= bnd * kBoxSlack);
            if (em) { node = snode[wv][sp]; break; }
        }
        if (!node) break;
    }
    if (active && skip) wlist[slot] = wskip;   // a reused list stays in place
    if (active && !skip) {
#pragma unroll
        for (int j = 0; j < KL; ++j) lists[(size_t)j * N + slot] = pos_(IK::id(lk[j]));   // ascending keys
        const bool full = full_();
        const float wk = full ? thr_() : kInfF;
        wlist[slot] = wk;
        // reference position + guarantee of a fresh list: every map point outside it has fp32
        // key ≥ the KL-th key's truncation thr_ (full list) or > the search bound (all points
        // within r listed)
        xref[slot] = make_float4(xf[0], xf[1], xf[2], full ? wk : r2s);
        nref[slot] = need_();
    }
#ifdef IMLS_DEBUG_WAVE_TRACE   // debug build only (make DEBUG_WAVE_TRACE=1): insert counters
    if (nbr_stats && lane == 0) {
        atomicAdd(&nbr_stats[6], (unsigned long long)dbg_ev);
        atomicAdd(&nbr_stats[7], (unsigned long long)dbg_ins);
    }
    if (nbr_stats && lane == 0) {
        const long long dbg_t2 = wall_clock64();
        atomicAdd(&nbr_stats[8], (unsigned long long)(dbg_t1 - dbg_t0));
        atomicMax(&nbr_stats[9], (unsigned long long)(dbg_t1 - dbg_t0));
        atomicAdd(&nbr_stats[10], (unsigned long long)(dbg_t2 - dbg_t1));
        atomicMax(&nbr_stats[11], (unsigned long long)(dbg_t2 - dbg_t1));
        atomicAdd(&nbr_stats[12], (unsigned long long)n_leaf);
        atomicMax(&nbr_stats[13], (unsigned long long)n_leaf);
        atomicMax(&nbr_stats[14], (unsigned long long)dbg_ev);
        atomicAdd(&nbr_stats[15], (unsigned long long)__popcll(__ballot(greedy)));
    }
    {
        const unsigned long long gl = __ballot(greedy), wi = __ballot(active && !full_()),
                                 w1 = __ballot(active && full_() && thr_() > 1.0f);
        float wmax = active && full_() ? thr_() : 0.f;
        for (int o = 1; o < 64; o <<= 1) wmax = fmaxf(wmax, __shfl_xor(wmax, o));
        unsigned sins = dbg_sparse_ins;
        for (int o = 1; o < 64; o <<= 1) sins += __shfl_xor(sins, o);
        if (lane == 0) {
            const int w = bx * (kWaveBlock / 64) + wv;
            if (w < kDbgWaves) {
                unsigned* r = g_dbg_wave[w];
                r[0] = (unsigned)(dbg_t1 - dbg_t0); r[1] = (unsigned)(wall_clock64() - dbg_t1);
                r[2] = n_leaf; r[3] = n_inner; r[4] = dbg_ev; r[5] = dbg_sparse; r[6] = dbg_bcast;
                r[7] = __popcll(gl); r[8] = __popcll(wi); r[9] = __popcll(w1); r[10] = __float_as_uint(wmax);
                r[11] = dbg_sparse_lanes; r[12] = sins; r[13] = dbg_ins;
                r[14] = dbg_seed_steps; r[15] = __builtin_amdgcn_readfirstlane(dbg_seed_pts);
            }
        }
    }
#endif
    if (nbr_stats && lane == 0) {
        atomicAdd(&nbr_stats[2], (unsigned long long)n_leaf);
        atomicAdd(&nbr_stats[3], (unsigned long long)n_inner);
        atomicAdd(&nbr_stats[4], 1ull);
    }
}

// =============================================================================================
// One wave per query (sparse query sets, e.g. FPS-sampled scans of the config-C stream): no packet
// union — each query walks only its own neighbourhood — and the top-KL list is spread over the
// lanes (lane k holds entry k, sorted), so every step is wave-uniform: inner nodes are scalar
// loads, a leaf is one coalesced load with one point per lane, an insertion is a ballot + shuffle.
// Output contract identical to k_knn_wave (positions [KL][N], worst key W per query).
// =============================================================================================
// FUSED (k_knn_qwave_f, a small frame alone): the wave goes on to the exact stage of its query
// (finish_q_core) with the list still in its lanes, an uncertified list resolved in the same wave
// (exact_wave_list) — nothing is deferred.  Extra arguments unused otherwise.
template <int KL>
__device__ __forceinline__ void finish_q_core(TreeView t, const float4* __restrict__ spt, const float4* __restrict__ snr,
                                              int i, int slot, const double* __restrict__ pose, const KParams& kp,
                                              int pos, float W, float4* __restrict__ cs, float4* __restrict__ cd,
                                              float4* __restrict__ cn, imls_iter_trace* __restrict__ tr,
                                              unsigned long long* __restrict__ nbr_stats, int* stk_n, float* stk_d);
struct QFinishArgs {
    const float4* snr;
    float4 *cs, *cd, *cn;
    imls_iter_trace* tr;
};
template <int KL, bool FUSED = false>
__device__ __forceinline__ void knn_qwave_body(TreeView t, const float4* __restrict__ spt,
                                                          const unsigned* __restrict__ qperm, int N,
                                                          const double* __restrict__ pose,
                                                          const int* __restrict__ done, KParams kp,
                                                          const double* __restrict__ delta,
                                                          int* __restrict__ lists, float* __restrict__ wlist,
                                                          float4* __restrict__ xref, float* __restrict__ nref,
                                                          int use_prev, unsigned long long* __restrict__ nbr_stats,
                                                          int bx, const QFinishArgs& fa = QFinishArgs{}) {
    static_assert(KL <= 64, "one list entry per lane");
    if (done && ld_const(done)) return;
    __shared__ int snode[kWaveBlock / 64][kWaveStack];
    __shared__ float sdist[kWaveBlock / 64][kWaveStack];
    __shared__ int fnode[kWaveBlock / 64][kFStack];      // frontier traversal
    __shared__ float fdist[kWaveBlock / 64][kFStack];
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int slot = __builtin_amdgcn_readfirstlane(bx * (kWaveBlock / 64) + wv);
    if (slot >= N) return;
#ifdef IMLS_DEBUG_WAVE_TRACE
    const long long dbg_q0 = wall_clock64();
#endif
    float xf[3];
    {
        double ns[3];
        transform_query(pose, spt[qperm[slot]], make_float4(0.f, 0.f, 0.f, 0.f), 0, xf, ns);
    }
    float lkey = kInfF;     // lane k < KL: entry k of the ascending list
    int lpos = -1;
    const float r2s = (float)(kp.r2 * kSearchR2) * kBoxSlack + 1e-30f;   // the search bound (radius (1 + skin)·r)
    // h-gate search (IMLS matcher): a query with no map point within h is rejected as too far
    // whatever lies between h and r (imls_icp.cpp:612-625), so while the list holds nothing within
    // h the traversal bound is h², not r² (27× less volume for isolated queries, the launch's tail);
    // a point found within h re-runs the traversal at the r bound (bounds never grow mid-walk)
    const float h2s = (float)kp.h2 * kBoxSlack + 1e-30f;
    bool hmode = false;
    float bnd = r2s;
    const int P = t.P, B = t.B, M = t.M;
    // insert (c, cp): entries ordered by (key, position); the tail shifts up by one lane
    auto insert = [&](float c, int cp) {
        const unsigned long long before = __ballot(lane < KL && (lkey < c || (lkey == c && lpos < cp)));
        const int at = __popcll(before);
        const float uk = __shfl_up(lkey, 1, 64);
        const int up = __shfl_up(lpos, 1, 64);
        if (lane > at && lane < KL) { lkey = uk; lpos = up; }
        if (lane == at) { lkey = c; lpos = cp; }
        bnd = fminf(hmode ? h2s : r2s, __int_as_float(__builtin_amdgcn_readlane(__float_as_int(lkey), KL - 1)));
    };
    auto worst = [&]() { return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(lkey), KL - 1)); };
    int seed_lo = 0, seed_hi = -1, seed_leaf = -1;
    bool greedy = !use_prev;
    bool skip = false;
    float wskip = kInfF;
    if (use_prev) {
        double rf = 0.0;
#pragma unroll
        for (int r = 0; r < 3; ++r)
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                const double e = ld_const(delta + r * 4 + c) - (r == c ? 1.0 : 0.0);
                rf += e * e;
            }
        const double d3 = ld_const(delta + 3), d7 = ld_const(delta + 7), d11 = ld_const(delta + 11);
        const float tn = (float)sqrt(d3 * d3 + d7 * d7 + d11 * d11);
        const float disp = tn + (float)sqrt(rf) * sqrtf(xf[0] * xf[0] + xf[1] * xf[1] + xf[2] * xf[2]);
        greedy = disp * disp > kReseed * wlist[slot];
    }
    float wlow = -1.0f;
    if (!greedy && kp.reuse) skip = verlet_skip(xref[slot], nref[slot], xf, r2s, wskip, wlow);
    if (skip) {
        // the list stays in place
    } else if (!greedy) {
        // prefill: previous list re-measured at the new pose.  Its ≤ KL distinct points all fit, so
        // inserting them one by one (the list empty, the bound r² until the last) leaves exactly
        // those within r² in (key, position) order: a bitonic sort of the lanes gives that order in
        // log²(KL)/2 exchange steps instead of KL dependent insertions (the re-traversing waves that
        // set a steady iteration's launch time all start here)
        const int pos = lane < KL ? lists[(size_t)lane * N + slot] : -1;
        float d = kInfF;
        if (pos >= 0) {
            const float4 q = t.mpt[pos];
            const float ex = q.x - xf[0], ey = q.y - xf[1], ez = q.z - xf[2];
            d = __builtin_fmaf(ex, ex, __builtin_fmaf(ey, ey, ez * ez));
        }
        const bool in = pos >= 0 && d <= bnd;
        float sk = in ? d : kInfF;
        int sp = in ? pos : -1;
        constexpr int W = KL <= 32 ? 32 : 64;
#pragma unroll
        for (int size = 2; size <= W; size <<= 1) {
#pragma unroll
            for (int stride = size >> 1; stride > 0; stride >>= 1) {
                const float ok = __shfl_xor(sk, stride, 64);
                const int op = __shfl_xor(sp, stride, 64);
                const bool asc = (lane & size) == 0, low = (lane & stride) == 0;
                const bool other_less = ok < sk || (ok == sk && op < sp);
                const bool other_more = sk < ok || (sk == ok && sp < op);
                if (asc == low ? other_less : other_more) { sk = ok; sp = op; }
            }
        }
        if (lane < KL) { lkey = sk; lpos = sp; }
        bnd = fminf(r2s, worst());
    } else {
        // seed: the leaf of the query's own Morton key ± seed_half Morton neighbours
        const unsigned long long qk = morton48(xf[0], xf[1], xf[2], t.qparams);
        int lo = 0, hi = t.L - 1;
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (t.lkeys[mid] <= qk) lo = mid;
            else hi = mid - 1;
        }
        seed_lo = max(0, lo - kSeedHalf);
        seed_hi = min(t.L - 1, lo + kSeedHalf);
        seed_leaf = lo;
        for (int leaf = seed_lo; leaf <= seed_hi; ++leaf) {
            const int base = leaf * B, cnt = min(B, M - base);
            float d = kInfF;
            if (lane < cnt) {
                const float4 q = t.mpt[base + lane];
                const float ex = q.x - xf[0], ey = q.y - xf[1], ez = q.z - xf[2];
                d = __builtin_fmaf(ex, ex, __builtin_fmaf(ey, ey, ez * ez));
            }
            unsigned long long m = __ballot(lane < cnt && d <= bnd);
            while (m) {
                const int j = __builtin_ctzll(m);
                m &= m - 1;
                const float c = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(d), j));
                if (c <= bnd && c < worst()) insert(c, base + j);
            }
        }
    }
    unsigned n_inner = 0, n_leaf = 0;
    if (nbr_stats && lane == 0 && skip) atomicAdd(&nbr_stats[kStatSkipped], 1ull);
    auto nearest = [&]() { return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(lkey))); };
    if (!skip && kp.matcher == IMLS_MATCH_IMLS && !(nearest() <= h2s)) {
        hmode = true;
        bnd = fminf(bnd, h2s);
    }
    for (int pass = 0; pass < 2; ++pass) {
    int node = 0, sp = 0;
    if (!skip) {
        // bottom-up start (round 4): the start leaf — the query's Morton leaf (greedy) or the leaf of
        // its nearest listed point — and the boxes of the siblings along its root path in ONE
        // parallel load (lane k: the sibling of the leaf's ancestor k levels up; a node's box sits in
        // its parent's record).  The leaf and those siblings' subtrees partition the tree, so every
        // sibling within the bound is stacked (nearest level on top) and the walk begins at the leaf:
        // the same leaves are reachable as from the root, without the ⌈levels/3⌉ dependent descent
        const int p0 = __builtin_amdgcn_readfirstlane(lpos);
        const int sl = greedy ? seed_leaf : (p0 >= 0 ? p0 / B : -1);
        node = 1;
        if (sl >= 0) {
            const int ln = P + sl;
            float d = kInfF;
            int sn = 0;
            if (lane < t.levels) {
                sn = (ln >> lane) ^ 1;
                const float4* rec = t.nodes + 3 * (size_t)(sn >> 1);
                const float4 a = rec[0], b = rec[1], c = rec[2];
                d = (sn & 1) ? box_d2(xf, b.z, b.w, c.x, c.y, c.z, c.w) : box_d2(xf, a.x, a.y, a.z, a.w, b.x, b.y);
            }
            const unsigned long long want = __ballot(lane < t.levels && d <= bnd * kBoxSlack);
            if ((want >> lane) & 1ull) {
                const int at = __popcll(want >> (lane + 1));
                snode[wv][at] = sn;
                sdist[wv][at] = d;
            }
            sp = __popcll(want);
            node = ln;
        }
    }
    if (node) {
        // Frontier traversal (round 4): each step takes up to 8 stacked entries within the bound and
        // gives each an 8-lane group — an inner node's group tests the boxes of its descendants
        // `sw` levels down (one record per lane pair), a leaf's group measures its points (B / 8 per
        // lane) — so a query whose ball spans many leaves walks them 8 at a time instead of one
        // dependent step per node (the steady-state iterations' tail: 2 % of the queries, 5-10
        // leaves and 11-16 inner steps each, set the launch time).  Candidates are inserted before
        // the wanted children are stacked (lower lanes on top), so the bound they face is current.
        // The same nodes are pruned by the same test (box d² > bound·slack, the bound only shrinks):
        // exactness is the DFS's.  Near capacity (> kFBatchMax entries) one entry per step keeps the
        // growth to the DFS's depth × 7.
        if (lane < sp) { fnode[wv][lane] = snode[wv][lane]; fdist[wv][lane] = sdist[wv][lane]; }
        if (lane == 0) { fnode[wv][sp] = node; fdist[wv][sp] = 0.0f; }
        int fsp = sp + 1;
        const int ppl = (B + 7) >> 3;
#ifdef IMLS_DEBUG_WAVE_TRACE
        int dbg_steps = 0;
#endif
        while (fsp > 0) {
#ifdef IMLS_DEBUG_WAVE_TRACE
            if (++dbg_steps > 20000 || fsp > kFStack) {
                if (lane == 0)
                    printf("frontier stuck: slot %d pass %d steps %d fsp %d sp0 %d node0 %d bnd %g P %d levels %d B %d M %d\n",
                           slot, pass, dbg_steps, fsp, sp, node, (double)bnd, P, t.levels, B, M);
                break;
            }
#endif
            const int lim = fsp > kFBatchMax ? 1 : 8;
            const int idx = fsp - 1 - lane;
            int en = 0;
            float ed = kInfF;
            if (idx >= 0) { en = fnode[wv][idx]; ed = fdist[wv][idx]; }
            const unsigned long long vm = __ballot(idx >= 0 && ed <= bnd * kBoxSlack);
            unsigned long long rem = vm, taken = 0;
            int gsrc[8];
            int ng = 0;
#pragma unroll
            for (int g = 0; g < 8; ++g) {
                gsrc[g] = 0;
                if (g < lim && rem) {
                    const int b = __builtin_ctzll(rem);
                    gsrc[g] = b;
                    taken |= 1ull << b;
                    rem &= rem - 1;
                    ++ng;
                }
            }
            fsp -= (ng == lim) ? (64 - __builtin_clzll(taken)) : min(fsp, 64);
            if (!ng) continue;
            const int g = lane >> 3, gl = lane & 7;
            int src = gsrc[0];
#pragma unroll
            for (int k = 1; k < 8; ++k) src = g == k ? gsrc[k] : src;
            const int gnode = __shfl(en, src, 64);
            const bool gact = g < ng;
            const bool ginner = gact && gnode < P, gleaf = gact && gnode >= P;
            n_inner += __popcll(__ballot(ginner && gl == 0));
            n_leaf += __popcll(__ballot(gleaf && gl == 0));
            // every lane's loads of the step issue together — its node record (inner groups) and its
            // B / 8 leaf points (leaf groups) — from clamped addresses, the values selected after:
            // loads behind the group / count tests became one branch and one wait per load
            float cdist = kInfF;
            int child = 0;
            int sw = 0;
            if (ginner) sw = min(kWide, t.levels - (31 - __builtin_clz(gnode)));   // ≤ 8 descendants: one per lane
            const bool gbox = ginner && gl < (1 << sw);
            const float4* rec = t.nodes + 3 * (gbox ? (((size_t)gnode << (sw - 1)) + (gl >> 1)) : (size_t)1);
            const float4 ra = rec[0], rb = rec[1], rc = rec[2];
            int lbase = 0, lcnt = 0;
            if (gleaf) {
                const int leaf = gnode - P;
                if (leaf < seed_lo || leaf > seed_hi) {
                    lbase = leaf * B;
                    lcnt = min(B, M - lbase);
                }
            }
            float4 lq[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const int j = gl + 8 * k;
                lq[k] = t.mpt[(k < ppl && j < lcnt) ? lbase + j : 0];
            }
            pin_loaded(ra);
            pin_loaded(rb);
            pin_loaded(rc);
#pragma unroll
            for (int k = 0; k < 8; ++k) pin_loaded(lq[k]);
            if (gbox) {
                cdist = (gl & 1) ? box_d2(xf, rb.z, rb.w, rc.x, rc.y, rc.z, rc.w) : box_d2(xf, ra.x, ra.y, ra.z, ra.w, rb.x, rb.y);
                child = (gnode << sw) + gl;
            }
            float pd[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const int j = gl + 8 * k;
                const float ex = lq[k].x - xf[0], ey = lq[k].y - xf[1], ez = lq[k].z - xf[2];
                const float d = __builtin_fmaf(ex, ex, __builtin_fmaf(ey, ey, ez * ez));
                pd[k] = (k < ppl && j < lcnt) ? d : kInfF;
            }
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                if (k >= ppl) break;
                unsigned long long m = __ballot(pd[k] <= bnd && pd[k] < worst());
                while (m) {
                    const int j = __builtin_ctzll(m);
                    m &= m - 1;
                    const float cd = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(pd[k]), j));
                    const int cp = __builtin_amdgcn_readlane(lbase + gl + 8 * k, j);
                    if (cd <= bnd && cd < worst() && !__ballot(lane < KL && lpos == cp)) insert(cd, cp);
                }
            }
            const unsigned long long want = __ballot(child != 0 && cdist <= bnd * kBoxSlack);
            if ((want >> lane) & 1ull) {
                // rank among the wanted lanes above this one (a 64-bit shift by 64 is not 0 here)
                const int at = fsp + (lane == 63 ? 0 : __popcll(want >> (lane + 1)));
                fnode[wv][at] = child;
                fdist[wv][at] = cdist;
            }
            fsp += __popcll(want);
        }
    }
    if (!hmode) break;
    if (!(nearest() <= h2s)) {
        // no map point within h: too far whatever the rest of the list holds — leave an empty list
        // (k_finish: no NN-1 → "too far"; need_key = ∞ → never reused without a traversal)
        lkey = kInfF;
        lpos = -1;
        break;
    }
    hmode = false;                     // a point within h: the full-r search, from the root
    bnd = fminf(r2s, worst());
    }
    if (skip) {
        if (lane == 0) wlist[slot] = wskip;
    } else {
        if (lane < KL) lists[(size_t)lane * N + slot] = lpos;
        const bool lpos_any = __ballot(lane < KL && lpos >= 0) != 0ull;
        float lkr[KL];   // the list gathered to every lane for the reuse key
#pragma unroll
        for (int k = 0; k < KL; ++k) lkr[k] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(lkey), k));
        // an h-mode list left empty was searched only to h: never reused (need ∞)
        const float nk = lpos_any ? need_key<KL>(lkr, (float)kp.r2, kp.K) : kInfF;
        if (lane == 0) {
            const float wk = worst();
            wlist[slot] = wk;
            xref[slot] = make_float4(xf[0], xf[1], xf[2], wk < kInfF ? wk : r2s);
            nref[slot] = nk;
        }
    }
    if (nbr_stats && lane == 0) {
        atomicAdd(&nbr_stats[2], (unsigned long long)n_leaf);
        atomicAdd(&nbr_stats[3], (unsigned long long)n_inner);
        atomicAdd(&nbr_stats[4], 1ull);
    }
    if constexpr (FUSED) {
#ifdef IMLS_DEBUG_WAVE_TRACE
        const long long dbg_q1 = wall_clock64();
#endif
        // the list as k_finish_q reads it: in the lanes, or (Verlet skip) still in memory
        const int pos = lane < KL ? (skip ? lists[(size_t)lane * N + slot] : lpos) : -1;
        finish_q_core<KL>(t, spt, fa.snr, (int)qperm[slot], slot, pose, kp, pos, skip ? wskip : worst(), fa.cs, fa.cd,
                          fa.cn, fa.tr, nbr_stats, snode[wv], sdist[wv]);
#ifdef IMLS_DEBUG_WAVE_TRACE
        // per-wave record of the last fused launch: start / traversal end / finish end (100 MHz
        // clock, low 32 bits), Verlet skip, leaves, inner steps, hardware id
        if (lane == 0 && slot < kDbgWaves) {
            unsigned* r = g_dbg_wave[slot];
            r[0] = (unsigned)dbg_q0; r[1] = (unsigned)dbg_q1; r[2] = (unsigned)wall_clock64();
            r[3] = skip ? 1u : 0u; r[4] = n_leaf; r[5] = n_inner; r[6] = greedy ? 1u : 0u;
            r[7] = (unsigned)__builtin_amdgcn_s_getreg((23 << 0) | (0 << 6) | (31 << 11));   // HW_ID / HW_ID1
        }
#endif
    }
}

// =============================================================================================
// Exact stage + gates + IMLS (hot kernel 2): one lane per query
// =============================================================================================
// 4 waves/SIMD (≤ 128 VGPRs): the exact stage waits on its gathers, resident waves hide them
#ifndef IMLS_FINISH_WPE
#define IMLS_FINISH_WPE 3
#endif
#define IMLS_FINISH_ATTR __attribute__((amdgpu_waves_per_eu(KL <= 26 ? IMLS_FINISH_WPE : 1)))
template <int KL>
__device__ __forceinline__ void finish_body(TreeView t, const float4* __restrict__ spt,
                                                       const float4* __restrict__ snr,
                                                       const unsigned* __restrict__ qperm, int N,
                                                       const double* __restrict__ pose,
                                                       const int* __restrict__ done, KParams kp,
                                                       const int* __restrict__ lists, const float* __restrict__ wlist,
                                                       float4* __restrict__ cs, float4* __restrict__ cd,
                                                       float4* __restrict__ cn, double* __restrict__ partial1,
                                                       imls_iter_trace* __restrict__ tr,
                                                       unsigned long long* __restrict__ nbr_stats,
                                                       unsigned* __restrict__ fb_list, unsigned* __restrict__ fb_count,
                                                       int bx) {
    if (done && ld_const(done)) return;
    __shared__ double red[kWaveBlock / 64][kNormEq];
    __shared__ double out[kNormEq];
    __shared__ unsigned rej_s[IMLS_NUM_REJ + 3];
    const int tid = threadIdx.x;
    if (tid < IMLS_NUM_REJ + 3) rej_s[tid] = 0;
    __syncthreads();
    const int slot = bx * kWaveBlock + tid;
    const bool active = slot < N;
    const int i = active ? (int)qperm[slot] : 0;
    float xf[3] = {0.f, 0.f, 0.f};
    double ns[3] = {0, 0, 0};
    int cat = -2, kq = 0, i1 = -1, p1 = -1;
    float yf[3] = {0, 0, 0}, nf[3] = {0, 0, 0};
    if (active) {
        // the query's point and normal, then the list (and its bound) beside them: one round trip
        // for both after the query index (the list depends on the slot only)
        const float4 sp4 = spt[i], sn4 = snr[i];
        double ed[KL];
        int ep[KL];
#pragma unroll
        for (int j = 0; j < KL; ++j) ep[j] = lists[(size_t)j * N + slot];
        const float W = wlist[slot];
        transform_query(pose, sp4, sn4, kp.transform_normal, xf, ns);
        const double xd[3] = {xf[0], xf[1], xf[2]};
        // the points in two chunks whose loads all issue before any is consumed (the list's round
        // trip, then two).  The loads are unconditional and pinned (pin_loaded): with
        // `ep ≥ 0 ? exact_d2(…) : ∞` the compiler sank each load into its own branch and waited on
        // it there — 22 dependent round trips per lane, most of this kernel's time
        constexpr int kCh = IMLS_DIST_CHUNK;
#pragma unroll
        for (int j0 = 0; j0 < KL; j0 += kCh) {
            float4 q[kCh];
#pragma unroll
            for (int u = 0; u < kCh; ++u)
                if (j0 + u < KL) q[u] = t.mpt[max(ep[j0 + u], 0)];
#pragma unroll
            for (int u = 0; u < kCh; ++u)
                if (j0 + u < KL) pin_loaded(q[u]);
#pragma unroll
            for (int u = 0; u < kCh; ++u) {
                const int j = j0 + u;
                if (j < KL) ed[j] = exact_d2(xd, q[u].x, q[u].y, q[u].z) + (ep[j] >= 0 ? 0.0 : kInfD);
            }
        }
        // odd-even transposition sort by (d², index); the fp32 order is already nearly exact.  The
        // index (the filtered index in mpt[].w, libnabo's tie order) is read only for an exact tie
        // of two distances (duplicate points): not carried in registers
        auto oidx = [&](int pos) -> int { return pos >= 0 ? (int)__float_as_uint(t.mpt[pos].w) : 0x7fffffff; };
        bool swapped = true;
        while (swapped) {
            swapped = false;
#pragma unroll
            for (int par = 0; par < 2; ++par) {
#pragma unroll
                for (int j = par; j + 1 < KL; j += 2) {
                    bool sw = ed[j + 1] < ed[j];
                    if (ed[j + 1] == ed[j] && ed[j] < kInfD) sw = oidx(ep[j + 1]) < oidx(ep[j]);
                    const double td = ed[j];
                    const int tp = ep[j];
                    ed[j] = sw ? ed[j + 1] : ed[j];
                    ep[j] = sw ? ep[j + 1] : ep[j];
                    ed[j + 1] = sw ? td : ed[j + 1];
                    ep[j + 1] = sw ? tp : ep[j + 1];
                    swapped |= sw;
                }
            }
        }
        const double r2 = kp.r2;
        const int K = kp.K;
        int cnt_r = 0;
        double d1 = kInfD, dK = 0.0;
#pragma unroll
        for (int j = 0; j < KL; ++j) {
            const bool in = ed[j] <= r2;
            cnt_r += in ? 1 : 0;
            if (in && i1 < 0 && ed[j] > DBL_EPSILON) { d1 = ed[j]; i1 = j; p1 = ep[j]; }
            if (j == K - 1) dK = ed[j];
        }
        const bool full = W < kInfF;
        double need = cnt_r >= K ? dK : r2;
        bool cert = true;
        if (full) {
            // no NN-1 in the list: certified only if no map point within r lies outside it (round 6:
            // before, never — a reused list of an isolated query went to the exact fallback)
            need = i1 < 0 ? r2 : fmax(need, d1);
            cert = cert && (need < (double)W / kCertSlack);
        }
        if (kp.force_fb && slot % kp.force_fb == 0) cert = false;   // test hook (IMLS_OPT_FORCE_FALLBACK)
        if (!cert) {
            // deferred to k_project_lane: listed in slot order in this wave's own region
            // fb_list[w·64, …) (its count in fb_count[w], below) — no atomics, so the fallback's rows
            // (and its slab sums) do not depend on timing
            const unsigned long long dm = __ballot(true);     // the wave's deferring lanes
            const int lanei = tid & 63;
            fb_list[((size_t)bx * kWaveBlock + (tid & ~63)) + __popcll(dm & ((1ull << lanei) - 1ull))] = (unsigned)i;
            cat = -3;
            // the list's own bound for the exact re-run: its points are real, so the exact answer
            // needs no point beyond max(K-th listed key within r, listed NN-1) (r² when either is
            // missing) — the fallback's search ball, instead of the whole radius r
            const double lb = i1 < 0 ? r2 : fmax(cnt_r >= K ? dK : r2, d1);
            cs[i] = make_float4(0.f, 0.f, 0.f, (float)(fmin(lb, r2) * (1.0 + 1e-6)));
        } else {
            cat = kp.matcher ? finish_plane(xf, ns, p1, t, kp, yf, nf)
                             : finish_query<KL, true>(xf, ns, ed, ep, 0, min(K, cnt_r), d1, p1, t, kp, yf, nf, kq, i);
            store_result(i, cat, xf, yf, nf, cs, cd, cn);
        }
    }
    if (cat >= 0) atomicAdd(&rej_s[cat], 1u);
    if (active && cat != -3) {
        if (kq) atomicAdd(&rej_s[IMLS_NUM_REJ], (unsigned)kq);
        if (i1 >= 0) atomicAdd(&rej_s[IMLS_NUM_REJ + 1], 1u);
    }
    if (cat == -3) atomicAdd(&rej_s[IMLS_NUM_REJ + 2], 1u);
    {
        const unsigned long long dm = __ballot(cat == -3);
        if ((tid & 63) == 0) fb_count[bx * (kWaveBlock / 64) + (tid >> 6)] = (unsigned)__popcll(dm);
    }
    __syncthreads();                  // rej_s complete (the slab reduction below may be skipped)
    // pass-1 slabs only for the grid solve chain (frames of ≤ kSmallRows rows: k_solve_small forms
    // pass 1 from the rows); N is block-uniform
    if (N > kSmallRows) {
        double a[6] = {0, 0, 0, 0, 0, 0}, bb = 0.0, one = 0.0;
        if (cat == -1) { plane_row(xf, yf, nf, a, bb); one = 1.0; }
        block_normeq<kWaveBlock>(a, bb, one, red, out);
        if (tid < kNormEq) partial1[(size_t)bx * kNormEq + tid] = out[tid];
    }
    if (tid < IMLS_NUM_REJ && rej_s[tid]) atomicAdd((unsigned long long*)&tr->reject[tid], (unsigned long long)rej_s[tid]);
    if (nbr_stats && tid >= IMLS_NUM_REJ && tid < IMLS_NUM_REJ + 2 && rej_s[tid])
        atomicAdd(&nbr_stats[tid - IMLS_NUM_REJ], (unsigned long long)rej_s[tid]);
    if (nbr_stats && tid == IMLS_NUM_REJ + 2 && rej_s[tid]) atomicAdd(&nbr_stats[5], (unsigned long long)rej_s[tid]);
}

// =============================================================================================
// Exact stage, one QUAD per query (round 6, the large frames' k_finish): 4 lanes per query, list
// entry j in lane j & 3, slot j >> 2 (S = ⌈KL/4⌉ slots per lane).  The one-lane form ran ~12
// dependent round trips per lane (list → 22 point gathers → sort → NN-1 normal → 3 normal chunks →
// up to 6 IMLS point + normal chunks → store) with ≤ 1.9 waves per SIMD resident; here every
// entry's point AND normal are gathered once, together (one round trip after the list), and stay in
// the lanes: 44 gathers per query instead of ~83, 4× the waves.  Cross-lane work uses quad DPP
// permutes (VALU, no LDS).  Same values as finish_body / finish_query, bit for bit:
//   * order: the traversal writes the list by ascending fp32 key, which is nearly the exact (d²,
//     index) order — one adjacency check (entry j vs j + 1) certifies it; a wave with a misordered
//     pair (near-equal keys: slot-id keys drop 5 mantissa bits) sorts its quads by odd-even
//     transposition across the lanes and re-gathers (rare);
//   * count within r, NN-1 (first entry in order with d² > DBL_EPSILON), the K-th, the certificate,
//     the gates, target = L[|S| − 1] (Q3), and the IMLS sums accumulated in list order (each
//     term broadcast from its lane in turn) — the reference's evaluation order;
//   * pass-1 slab per block of 64 queries: each quad's row split over its lanes (7 of the 28 terms
//     each), reduced over the wave's quads (DPP row shifts + two xor exchanges) and the 4 waves.
// Deferred (uncertified) queries: the block is one 64-slot region of fb_list (slot order), as the
// one-lane kernel's waves were.
// =============================================================================================
constexpr int kQuadSwap1 = 0xB1;   // quad_perm [1,0,3,2]
constexpr int kQuadSwap2 = 0x4E;   // [2,3,0,1]
constexpr int kQuadRev = 0x1B;     // [3,2,1,0]
constexpr int kQuadNext = 0x39;    // [1,2,3,0]
template <int CTRL>
__device__ __forceinline__ int qperm_i(int v) { return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xf, 0xf, true); }
template <int CTRL>
__device__ __forceinline__ float qperm_f(float v) { return __int_as_float(qperm_i<CTRL>(__float_as_int(v))); }
template <int CTRL>
__device__ __forceinline__ double qperm_d(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = qperm_i<CTRL>((int)(unsigned)(unsigned long long)b);
    const int hi = qperm_i<CTRL>((int)(unsigned)((unsigned long long)b >> 32));
    return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}
// a value held by one lane of the quad (zero bits in the others) → every lane of the quad
__device__ __forceinline__ __attribute__((unused)) int quad_or(int v) {
    v |= qperm_i<kQuadSwap1>(v);
    return v | qperm_i<kQuadSwap2>(v);
}
__device__ __forceinline__ __attribute__((unused)) double quad_or_d(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = quad_or((int)(unsigned)(unsigned long long)b);
    const int hi = quad_or((int)(unsigned)((unsigned long long)b >> 32));
    return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}
__device__ __forceinline__ __attribute__((unused)) int quad_sum(int v) {
    v += qperm_i<kQuadSwap1>(v);
    return v + qperm_i<kQuadSwap2>(v);
}
__device__ __forceinline__ __attribute__((unused)) int quad_min(int v) {
    v = min(v, qperm_i<kQuadSwap1>(v));
    return min(v, qperm_i<kQuadSwap2>(v));
}

constexpr int kFinishQ = kWaveBlock / 4;   // queries per quad-kernel block (= one pass-1 slab, one fb region)
#define IMLS_FINISH4_ATTR __attribute__((amdgpu_waves_per_eu(KL <= 26 ? 4 : 2)))

template <int KL>
__device__ __forceinline__ void finish4_body(TreeView t, const float4* __restrict__ spt, const float4* __restrict__ snr,
                                             const unsigned* __restrict__ qperm, int N, const double* __restrict__ pose,
                                             const int* __restrict__ done, KParams kp, const int* __restrict__ lists,
                                             const float* __restrict__ wlist, float4* __restrict__ cs,
                                             float4* __restrict__ cd, float4* __restrict__ cn,
                                             double* __restrict__ partial1, imls_iter_trace* __restrict__ tr,
                                             unsigned long long* __restrict__ nbr_stats, unsigned* __restrict__ fb_list,
                                             unsigned* __restrict__ fb_count, int bx) {
    if (done && ld_const(done)) return;
    constexpr int S = (KL + 3) / 4;
    __shared__ double red[kWaveBlock / 64][kNormEq];
    __shared__ unsigned rej_s[IMLS_NUM_REJ + 3];
    __shared__ unsigned fbc[kWaveBlock / 64];
    const int tid = threadIdx.x, lane = tid & 63, g = lane & 3, wv = tid >> 6;
    if (tid < IMLS_NUM_REJ + 3) rej_s[tid] = 0;
    __syncthreads();
    const int slot = bx * kFinishQ + (tid >> 2);
    const bool active = slot < N;              // quad-uniform
    const int i = active ? (int)qperm[slot] : 0;
    float xf[3] = {0.f, 0.f, 0.f}, yf[3] = {0.f, 0.f, 0.f}, nf[3] = {0.f, 0.f, 0.f};
    double ns[3] = {0.0, 0.0, 0.0};
    int cat = -2, kq = 0, i1 = -1;
    if (active) {
        const float4 sp4 = spt[i], sn4 = snr[i];
        int pos[S];
#pragma unroll
        for (int s = 0; s < S; ++s) {
            const int j = g + 4 * s;
            const int v = lists[(size_t)min(j, KL - 1) * N + slot];
            pos[s] = j < KL ? v : -1;
        }
        const float W = wlist[slot];
        transform_query(pose, sp4, sn4, kp.transform_normal, xf, ns);
        const double xd[3] = {xf[0], xf[1], xf[2]};
        // every entry's point and normal in one round trip (pinned: not sunk into their uses)
        float4 pt[S], nm[S];
        auto gather = [&]() {
#pragma unroll
            for (int s = 0; s < S; ++s) pt[s] = t.mpt[max(pos[s], 0)];
            if (!kp.matcher) {
#pragma unroll
                for (int s = 0; s < S; ++s) nm[s] = t.mnr[max(pos[s], 0)];
            } else {
#pragma unroll
                for (int s = 0; s < S; ++s) nm[s] = make_float4(0.f, 0.f, 0.f, 0.f);
            }
#pragma unroll
            for (int s = 0; s < S; ++s) {
                pin_loaded(pt[s]);
                pin_loaded(nm[s]);
            }
        };
        gather();
        double ed[S];
        int eid[S];
#pragma unroll
        for (int s = 0; s < S; ++s) {
            ed[s] = pos[s] >= 0 ? exact_d2(xd, pt[s].x, pt[s].y, pt[s].z) : kInfD;
            eid[s] = pos[s] >= 0 ? (int)__float_as_uint(pt[s].w) : 0x7fffffff;   // libnabo's tie order
        }
        // order check: entry j = (g, s) against j + 1 = (g + 1, s), or (0, s + 1) for g = 3
        bool bad = false;
        {
            double rd[S];
            int ri[S];
#pragma unroll
            for (int s = 0; s < S; ++s) {
                rd[s] = qperm_d<kQuadNext>(ed[s]);
                ri[s] = qperm_i<kQuadNext>(eid[s]);
            }
#pragma unroll
            for (int s = 0; s < S; ++s) {
                double nd = rd[s];
                int ni = ri[s];
                if (g == 3) {
                    nd = s + 1 < S ? rd[s + 1 < S ? s + 1 : 0] : kInfD;
                    ni = s + 1 < S ? ri[s + 1 < S ? s + 1 : 0] : 0x7fffffff;
                }
                bad |= lessp(nd, ni, ed[s], eid[s]);
            }
        }
        if (__ballot(bad)) {
            // odd-even transposition across the quad's entries until a pass swaps nothing, then the
            // moved entries' points and normals are gathered again
            bool swapped = true;
            while (__ballot(swapped)) {
                swapped = false;
                // even phase: (4s, 4s+1), (4s+2, 4s+3) — partner lane g ^ 1, same slot
#pragma unroll
                for (int s = 0; s < S; ++s) {
                    const double od = qperm_d<kQuadSwap1>(ed[s]);
                    const int oi = qperm_i<kQuadSwap1>(eid[s]), op = qperm_i<kQuadSwap1>(pos[s]);
                    const bool lower = (g & 1) == 0;
                    const bool take = lower ? lessp(od, oi, ed[s], eid[s]) : lessp(ed[s], eid[s], od, oi);
                    if (take) { ed[s] = od; eid[s] = oi; pos[s] = op; }
                    swapped |= take;
                }
                // odd phase: (4s+1, 4s+2) lanes 1 ↔ 2, and (4s+3, 4s+4) lane 3 slot s ↔ lane 0 slot s+1
                double rd[S];
                int ri[S], rp[S];
#pragma unroll
                for (int s = 0; s < S; ++s) {
                    rd[s] = qperm_d<kQuadRev>(ed[s]);
                    ri[s] = qperm_i<kQuadRev>(eid[s]);
                    rp[s] = qperm_i<kQuadRev>(pos[s]);
                }
#pragma unroll
                for (int s = 0; s < S; ++s) {
                    double od = rd[s];
                    int oi = ri[s], op = rp[s];
                    bool has = g == 1 || g == 2;
                    if (g == 3 && s + 1 < S) { od = rd[s + 1 < S ? s + 1 : 0]; oi = ri[s + 1 < S ? s + 1 : 0]; op = rp[s + 1 < S ? s + 1 : 0]; has = true; }
                    if (g == 0 && s > 0) { od = rd[s > 0 ? s - 1 : 0]; oi = ri[s > 0 ? s - 1 : 0]; op = rp[s > 0 ? s - 1 : 0]; has = true; }
                    const bool lower = g == 1 || g == 3;
                    const bool take = has && (lower ? lessp(od, oi, ed[s], eid[s]) : lessp(ed[s], eid[s], od, oi));
                    if (take) { ed[s] = od; eid[s] = oi; pos[s] = op; }
                    swapped |= take;
                }
            }
            gather();
        }
        const double r2 = kp.r2;
        const int K = kp.K;
        int cr = 0, j1 = 0x7fffffff;
#pragma unroll
        for (int s = 0; s < S; ++s) {
            const bool in = ed[s] <= r2;
            cr += in ? 1 : 0;
            if (in && ed[s] > DBL_EPSILON) j1 = min(j1, g + 4 * s);
        }
        const int cnt_r = quad_sum(cr);
        j1 = quad_min(j1);
        // entry j's values, from its lane (the others contribute zero bits)
        auto pick_d = [&](const double (&v)[S], int j) -> double {
            double m = 0.0;
#pragma unroll
            for (int s = 0; s < S; ++s) m = (j == g + 4 * s) ? v[s] : m;
            return quad_or_d(m);
        };
        auto pick_i = [&](const int (&v)[S], int j) -> int {
            int m = 0;
#pragma unroll
            for (int s = 0; s < S; ++s) m = (j == g + 4 * s) ? v[s] : m;
            return quad_or(m);
        };
        const bool has1 = j1 != 0x7fffffff;
        const double d1 = has1 ? pick_d(ed, j1) : kInfD;
        const int p1 = has1 ? pick_i(pos, j1) : -1;
        i1 = has1 ? j1 : -1;
        const double dK = pick_d(ed, K - 1);
        const bool full = W < kInfF;
        double need = cnt_r >= K ? dK : r2;
        bool cert = true;
        if (full) {
            // no NN-1 in the list: certified only if no map point within r lies outside it (round 6:
            // before, never — a reused list of an isolated query went to the exact fallback)
            need = i1 < 0 ? r2 : fmax(need, d1);
            cert = cert && (need < (double)W / kCertSlack);
        }
        if (kp.force_fb && slot % kp.force_fb == 0) cert = false;   // test hook (IMLS_OPT_FORCE_FALLBACK)
        if (!cert) {
            cat = -3;
            // the exact re-run's search ball: the list's own bound (finish_body)
            const double lb = i1 < 0 ? r2 : fmax(cnt_r >= K ? dK : r2, d1);
            if (g == 0) cs[i] = make_float4(0.f, 0.f, 0.f, (float)(fmin(lb, r2) * (1.0 + 1e-6)));
        } else if (kp.matcher) {
            cat = finish_plane(xf, ns, p1, t, kp, yf, nf);
        } else {
            // finish_query over L = entries 0 … cnt−1 (imls_icp.cpp:612-729)
            const int cnt = min(K, cnt_r);
            double nn[3] = {0.0, 0.0, 0.0};
            cat = -1;
            if (p1 < 0 || d1 > kp.h2) {
                cat = IMLS_REJ_TOO_FAR;                             // imls_icp.cpp:612-625 (Q18)
            } else if (kp.tv) {
                const double4 v = t.tvn[i];
                if (v.w == 0.0) cat = IMLS_REJ_NO_NORMAL;
                nn[0] = v.x; nn[1] = v.y; nn[2] = v.z;
            } else if (!kp.get_normals) {
                cat = IMLS_REJ_INVALID_NORMAL;
            } else {
                float m0 = 0.f, m1 = 0.f, m2 = 0.f;
#pragma unroll
                for (int s = 0; s < S; ++s)
                    if (j1 == g + 4 * s) { m0 = nm[s].x; m1 = nm[s].y; m2 = nm[s].z; }
                nn[0] = __int_as_float(quad_or(__float_as_int(m0)));
                nn[1] = __int_as_float(quad_or(__float_as_int(m1)));
                nn[2] = __int_as_float(quad_or(__float_as_int(m2)));
            }
            if (cat == -1 && !(isfinite(nn[0]) && isfinite(nn[1]) && isfinite(nn[2]))) cat = IMLS_REJ_INVALID_NORMAL;
            if (cat == -1 && kp.angle_on && angle_reject(ns, nn[0], nn[1], nn[2], kp.angle_thr_deg, kp.cos_thr))
                cat = IMLS_REJ_NORMAL_CONSTRAINT;
            if (cat == -1) {
                kq = cnt;
                bool ok[S];
                int na = 0;
#pragma unroll
                for (int s = 0; s < S; ++s) {
                    const bool inl = g + 4 * s < cnt;
                    bool o = inl && kp.get_normals && isfinite(nm[s].x) && isfinite(nm[s].y) && isfinite(nm[s].z);
                    if (o && kp.angle_on) o = !angle_reject(ns, nm[s].x, nm[s].y, nm[s].z, kp.angle_thr_deg, kp.cos_thr);
                    ok[s] = o;
                    na += o ? 1 : 0;
                }
                const int nacc = quad_sum(na);
                if (nacc < 3) {
                    cat = IMLS_REJ_MLS_FAIL;                        // imls_icp.cpp:463-466
                } else {
                    const double hmax = sqrt(pick_d(ed, nacc - 1)) / 3;   // Q3: L[|S| − 1]
                    const double ih2 = 1.0 / (hmax * hmax);             // as finish_query
                    double w[S], pr[S];
#pragma unroll
                    for (int s = 0; s < S; ++s) {
                        const double dx = xd[0] - (double)pt[s].x, dy = xd[1] - (double)pt[s].y, dz = xd[2] - (double)pt[s].z;
                        double dn = dx * dx;
                        dn = dn + dy * dy;
                        dn = dn + dz * dz;
                        const double ww = exp(-dn * ih2);
                        double p = (ww * dx) * (double)nm[s].x;
                        p = p + (ww * dy) * (double)nm[s].y;
                        p = p + (ww * dz) * (double)nm[s].z;
                        w[s] = ok[s] ? ww : 0.0;
                        pr[s] = ok[s] ? p : 0.0;
                    }
                    // Σ in list order (entry j = lane j & 3, slot j >> 2), as finish_query accumulates
                    double wsum = 0.0, psum = 0.0;
#pragma unroll
                    for (int s = 0; s < S; ++s) {
                        wsum += qperm_d<0x00>(w[s]);
                        psum += qperm_d<0x00>(pr[s]);
                        wsum += qperm_d<0x55>(w[s]);
                        psum += qperm_d<0x55>(pr[s]);
                        wsum += qperm_d<0xAA>(w[s]);
                        psum += qperm_d<0xAA>(pr[s]);
                        wsum += qperm_d<0xFF>(w[s]);
                        psum += qperm_d<0xFF>(pr[s]);
                    }
                    const double height = psum / (wsum + 1e-5);     // Q4
                    if (isnan(height) || isinf(height)) {
                        cat = IMLS_REJ_NAN_INF_HEIGHT;
                    } else {
                        yf[0] = (float)(xd[0] - height * nn[0]);    // imls_icp.cpp:719-729
                        yf[1] = (float)(xd[1] - height * nn[1]);
                        yf[2] = (float)(xd[2] - height * nn[2]);
                        nf[0] = (float)nn[0]; nf[1] = (float)nn[1]; nf[2] = (float)nn[2];
                    }
                }
            }
        }
        if (g == 0 && cat != -3) store_result(i, cat, xf, yf, nf, cs, cd, cn);
    }
    const bool lead = g == 0;
    if (lead && cat >= 0) atomicAdd(&rej_s[cat], 1u);
    if (lead && active && cat != -3) {
        if (kq) atomicAdd(&rej_s[IMLS_NUM_REJ], (unsigned)kq);
        if (i1 >= 0) atomicAdd(&rej_s[IMLS_NUM_REJ + 1], 1u);
    }
    if (lead && cat == -3) atomicAdd(&rej_s[IMLS_NUM_REJ + 2], 1u);
    // deferred queries of the block (one 64-slot region), in slot order: no atomics, so the
    // fallback's rows and slabs do not depend on timing
    const unsigned long long dm = __ballot(lead && cat == -3);
    if (lane == 0) fbc[wv] = (unsigned)__popcll(dm);
    __syncthreads();                  // rej_s and fbc complete
    if (lead && cat == -3) {
        unsigned off = (unsigned)__popcll(dm & ((1ull << lane) - 1ull));
#pragma unroll
        for (int w = 0; w < kWaveBlock / 64; ++w) off += w < wv ? fbc[w] : 0u;
        fb_list[(size_t)bx * kFinishQ + off] = (unsigned)i;
    }
    if (tid == 0) {
        unsigned tot = 0;
#pragma unroll
        for (int w = 0; w < kWaveBlock / 64; ++w) tot += fbc[w];
        fb_count[bx] = tot;
    }
    // pass-1 slab of the block's 64 queries (grid solve chain only: N > kSmallRows, block-uniform)
    if (N > kSmallRows) {
        double a[6] = {0, 0, 0, 0, 0, 0}, bb = 0.0, one = 0.0;
        if (cat == -1) { plane_row(xf, yf, nf, a, bb); one = 1.0; }
        double prod[kNormEq];
        int k = 0;
#pragma unroll
        for (int r = 0; r < 6; ++r)
#pragma unroll
            for (int c = r; c < 6; ++c) prod[k++] = a[r] * a[c];
#pragma unroll
        for (int r = 0; r < 6; ++r) prod[21 + r] = a[r] * bb;
        prod[27] = one;
        // lane g of a quad sums terms 7g … 7g+6 over the wave's 16 quads: row shifts by 4 and 8 leave
        // each 16-lane row's sum in lane 12 + g, two xor exchanges add the rows (fixed association)
        double v[7];
#pragma unroll
        for (int u = 0; u < 7; ++u) {
            double x = g == 0 ? prod[u] : (g == 1 ? prod[7 + u] : (g == 2 ? prod[14 + u] : prod[21 + u]));
            x = dpp_add_f64<0x114, 0xf>(x);    // row_shr:4
            x = dpp_add_f64<0x118, 0xf>(x);    // row_shr:8 → lanes 12..15 of each row
            x = x + xor_f64(x, 16);
            x = x + xor_f64(x, 32);
            v[u] = x;
        }
        if (lane >= 12 && lane < 16) {
#pragma unroll
            for (int u = 0; u < 7; ++u) red[wv][7 * g + u] = v[u];
        }
        __syncthreads();
        if (tid < kNormEq) {
            double sum = 0.0;
#pragma unroll
            for (int w = 0; w < kWaveBlock / 64; ++w) sum += red[w][tid];
            partial1[(size_t)bx * kNormEq + tid] = sum;
        }
    }
    if (tid < IMLS_NUM_REJ && rej_s[tid]) atomicAdd((unsigned long long*)&tr->reject[tid], (unsigned long long)rej_s[tid]);
    if (nbr_stats && tid >= IMLS_NUM_REJ && tid < IMLS_NUM_REJ + 2 && rej_s[tid])
        atomicAdd(&nbr_stats[tid - IMLS_NUM_REJ], (unsigned long long)rej_s[tid]);
    if (nbr_stats && tid == IMLS_NUM_REJ + 2 && rej_s[tid]) atomicAdd(&nbr_stats[5], (unsigned long long)rej_s[tid]);
}

// =============================================================================================
// Exact stage, one WAVE per query (a small frame registered alone — the config C/D deployment
// shape, ≤ kSmallRows queries — where k_finish's one-lane-per-query latency chain (~30 µs per
// launch for 2000 queries in 8 blocks) sets the frame latency): lane j holds list entry j, so the
// gathers, the exact distances, the gates and the IMLS weights run across the lanes.  Every value is
// computed by the same expression as k_finish's lane code, the list order is the same (d², index)
// total order (each lane's rank by counting), the IMLS sums accumulate in that order (lane 0 reads
// each term in turn) — the correspondences are the lane kernel's bit for bit.  Rejects are counted
// by integer atomics (order-free).  No pass-1 slabs: frames of ≤ kSmallRows rows are solved by
// k_solve_small, which forms pass 1 from the rows (the same order for every small frame, batched
// or alone, whichever exact stage produced its rows).
// =============================================================================================
__device__ __forceinline__ double rl_f64(double x, int l) {
    const long long b = __double_as_longlong(x);
    const int lo = __builtin_amdgcn_readlane((int)(unsigned)(b & 0xffffffffll), l);
    const int hi = __builtin_amdgcn_readlane((int)(unsigned)((unsigned long long)b >> 32), l);
    return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}

// query i (slot `slot`) from its list: lane k < KL holds entry k's map position `pos` (−1 empty),
// W is the list's bound (the traversal's worst key).  Run by k_finish_q, and by k_knn_qwave_f
// straight after the traversal of the same wave (round 4: one launch per iteration fewer)
__device__ __forceinline__ double shfl_up_f64(double x) {
    const long long b = __double_as_longlong(x);
    const int lo = __shfl_up((int)(unsigned)(b & 0xffffffffll), 1, 64);
    const int hi = __shfl_up((int)(unsigned)((unsigned long long)b >> 32), 1, 64);
    return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}

// The exact list of one query by one wave, for a query whose float list failed its certificate
// (round 4: the fused lone-frame path resolves it in place instead of deferring it to the fallback
// launch): project_lane_body's search — the K nearest map points by (exact d², original index) with
// d² ≤ r², NN-1 = the first with d² > DBL_EPSILON, boxes and points pruned by the float bound
// min(cap, max(K-th, NN-1))·slack — with the list in lanes 0..K−1 instead of registers.  Returns
// lane k's entry position (−1 empty); an NN-1 outside the K entries (more than K points within
// DBL_EPSILON of the query) rides in lane K.  stk_n / stk_d: the wave's LDS stack (kWaveStack).
template <int KL>
__device__ int exact_wave_list(const TreeView& t, const KParams& kp, const double xd[3], const float xf[3], double cap,
                               int* stk_n, float* stk_d) {
    static_assert(KL <= 64, "one list entry per lane");
    const int lane = threadIdx.x & 63;
    const int K = kp.K;
    const double r2 = kp.r2;
    double ek = kInfD;
    int eo = 0x7fffffff, ep = -1;
    double d1 = kInfD;
    int o1 = 0x7fffffff, p1 = -1;
    float bf = (float)cap * kBoxSlack + 1e-30f;
    const int P = t.P, B = t.B, M = t.M;
    int node = 1, sp = 0;
    while (true) {
        if (node < P) {
            const int lev = 31 - __builtin_clz(node);
            const int sw = min(kWide, t.levels - lev);
            const int nk = 1 << sw;
            float d = kInfF;
            if (lane < nk) {
                const float4* rec = t.nodes + 3 * (((size_t)node << (sw - 1)) + (lane >> 1));
                const float4 a = rec[0], b = rec[1], c = rec[2];
                d = (lane & 1) ? box_d2(xf, b.z, b.w, c.x, c.y, c.z, c.w) : box_d2(xf, a.x, a.y, a.z, a.w, b.x, b.y);
            }
            const unsigned long long want = __ballot(lane < nk && d <= bf);
            if (want) {
                const int km = __builtin_ctzll(want);
                unsigned long long rest = want & (want - 1);
                while (rest) {
                    const int kk = 63 - __builtin_clzll(rest);
                    rest &= ~(1ull << kk);
                    const float dk = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(d), kk));
                    if (lane == 0) { stk_n[sp] = (node << sw) + kk; stk_d[sp] = dk; }
                    ++sp;
                }
                node = (node << sw) + km;
                continue;
            }
        } else {
            const int base = (node - P) * B, cnt = min(B, M - base);
            double d2 = kInfD;
            int oi = 0x7fffffff;
            bool c = false;
            if (lane < cnt) {
                const float4 q = t.mpt[base + lane];
                const float ex = q.x - xf[0], ey = q.y - xf[1], ez = q.z - xf[2];
                const float d32 = __builtin_fmaf(ex, ex, __builtin_fmaf(ey, ey, ez * ez));
                if (d32 <= bf) {
                    d2 = exact_d2(xd, q.x, q.y, q.z);
                    oi = (int)__float_as_uint(q.w);
                    c = d2 <= r2;
                }
            }
            unsigned long long m = __ballot(c);
            while (m) {
                const int j = __builtin_ctzll(m);
                m &= m - 1;
                const double cdd = rl_f64(d2, j);
                const int co = __builtin_amdgcn_readlane(oi, j);
                bool changed = false;
                if (cdd > DBL_EPSILON && (cdd < d1 || (cdd == d1 && co < o1))) {
                    d1 = cdd; o1 = co; p1 = base + j;
                    changed = true;
                }
                const double wk = rl_f64(ek, K - 1);
                const int wo = __builtin_amdgcn_readlane(eo, K - 1);
                if (cdd < wk || (cdd == wk && co < wo)) {
                    const int at = __popcll(__ballot(lane < K && (ek < cdd || (ek == cdd && eo < co))));
                    const double uk = shfl_up_f64(ek);
                    const int uo = __shfl_up(eo, 1, 64), up = __shfl_up(ep, 1, 64);
                    if (lane > at && lane < K) { ek = uk; eo = uo; ep = up; }
                    if (lane == at) { ek = cdd; eo = co; ep = base + j; }
                    changed = true;
                }
                if (changed) bf = (float)fmin(cap, fmax(rl_f64(ek, K - 1), d1)) * kBoxSlack + 1e-30f;
            }
        }
        node = 0;
        while (sp > 0) {
            --sp;
            if (stk_d[sp] <= bf) { node = stk_n[sp]; break; }
        }
        if (!node) break;
    }
    if (p1 >= 0 && !__ballot(lane < K && ep == p1) && lane == K) ep = p1;
    return lane <= K ? ep : -1;
}

// query i (slot `slot`) from its list: lane k < KL holds entry k's map position `pos` (−1 empty),
// W is the list's bound (the traversal's worst key).  Run by k_knn_qwave_f straight after the
// traversal of the same wave (round 4: one launch per iteration fewer); an uncertified query gets its
// exact list in place (exact_wave_list, with the wave's LDS stack stk_n / stk_d) — nothing is deferred.
template <int KL>
__device__ __forceinline__ void finish_q_core(TreeView t, const float4* __restrict__ spt, const float4* __restrict__ snr,
                                              int i, int slot, const double* __restrict__ pose, const KParams& kp,
                                              int pos, float W, float4* __restrict__ cs, float4* __restrict__ cd,
                                              float4* __restrict__ cn, imls_iter_trace* __restrict__ tr,
                                              unsigned long long* __restrict__ nbr_stats, int* stk_n, float* stk_d) {
    static_assert(KL <= 64, "one list entry per lane");
    const int lane = threadIdx.x & 63;
    float xf[3];
    double ns[3];
    transform_query(pose, spt[i], snr[i], kp.transform_normal, xf, ns);
    const double xd[3] = {xf[0], xf[1], xf[2]};
    const bool ent = lane < KL;
    const double r2 = kp.r2;
    const int K = kp.K;
    float4 q;
    double ed, d1, dK;
    int eo, rank, cnt_r, l1, p1, lK;
    bool in;
    auto lane_of_rank = [&](int r) -> int {
        const unsigned long long m = __ballot(ent && rank == r);
        return m ? (int)__builtin_ctzll(m) : -1;
    };
    // the list's exact keys, its (d², index) order (k_finish's sort; empty entries after the real
    // ones, by lane), the count within r, the NN-1 and the K-th
    auto analyse = [&]() {
        q = make_float4(0.f, 0.f, 0.f, 0.f);
        ed = kInfD;
        eo = 0x7fffffff;
        if (pos >= 0) {
            q = t.mpt[pos];
            ed = exact_d2(xd, q.x, q.y, q.z);
            eo = (int)__float_as_uint(q.w);
        }
        rank = 0;
#pragma unroll
        for (int k = 0; k < KL; ++k) {
            const double dk = rl_f64(ed, k);
            const int ok = __builtin_amdgcn_readlane(eo, k);
            rank += (dk < ed || (dk == ed && (ok < eo || (ok == eo && k < lane)))) ? 1 : 0;
        }
        in = ent && ed <= r2;
        cnt_r = __popcll(__ballot(in));
        // NN-1: the first entry in order within r with d² > DBL_EPSILON (no self match)
        int r1 = (in && ed > DBL_EPSILON) ? rank : 0x7fffffff;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) r1 = min(r1, __shfl_xor(r1, o, 64));
        l1 = r1 < 0x7fffffff ? lane_of_rank(r1) : -1;
        d1 = l1 >= 0 ? rl_f64(ed, l1) : kInfD;
        p1 = l1 >= 0 ? __builtin_amdgcn_readlane(pos, l1) : -1;
        lK = lane_of_rank(K - 1);
        dK = lK >= 0 ? rl_f64(ed, lK) : 0.0;
    };
    analyse();
    const bool full = W < kInfF;
    double need = cnt_r >= K ? dK : r2;
    bool cert = true;
    if (full) {
        // no NN-1 in the list: certified only if no map point within r lies outside it (round 6:
        // before, never — a reused list of an isolated query went to the exact fallback)
        need = l1 < 0 ? r2 : fmax(need, d1);
        cert = cert && (need < (double)W / kCertSlack);
    }
    if (kp.force_fb && slot % kp.force_fb == 0) cert = false;   // test hook (IMLS_OPT_FORCE_FALLBACK)
    int cat = -1, kq = 0;
    float yf[3] = {0.f, 0.f, 0.f}, nf[3] = {0.f, 0.f, 0.f};
    if (!cert) {
        // the exact search ball: the list's bound (its points are real, the exact answer needs
        // nothing farther — the bound k_project_lane gets from k_finish through cs.w)
        const double lb = l1 < 0 ? r2 : fmax(cnt_r >= K ? dK : r2, d1);
        const float capf = (float)(fmin(lb, r2) * (1.0 + 1e-6));
        pos = exact_wave_list<KL>(t, kp, xd, xf, fmin(r2, (double)capf), stk_n, stk_d);
        analyse();
        if (nbr_stats && lane == 0) atomicAdd(&nbr_stats[5], 1ull);
    }
    if (kp.matcher) {
        cat = finish_plane(xf, ns, p1, t, kp, yf, nf);
    } else {
        // finish_query, entry j of the ordered list = the lane of rank j
        const int cnt = min(K, cnt_r);
        double nn[3] = {0.0, 0.0, 0.0};
        if (p1 < 0 || d1 > kp.h2) {
            cat = IMLS_REJ_TOO_FAR;                             // imls_icp.cpp:612-625 (Q18)
        } else if (kp.tv) {
            const double4 v = t.tvn[i];
            if (v.w == 0.0) cat = IMLS_REJ_NO_NORMAL;
            nn[0] = v.x; nn[1] = v.y; nn[2] = v.z;
        } else if (!kp.get_normals) {
            cat = IMLS_REJ_INVALID_NORMAL;
        } else {
            const float4 n4 = t.mnr[p1];
            nn[0] = n4.x; nn[1] = n4.y; nn[2] = n4.z;
        }
        if (cat == -1 && !(isfinite(nn[0]) && isfinite(nn[1]) && isfinite(nn[2]))) cat = IMLS_REJ_INVALID_NORMAL;
        if (cat == -1 && kp.angle_on && angle_reject(ns, nn[0], nn[1], nn[2], kp.angle_thr_deg, kp.cos_thr))
            cat = IMLS_REJ_NORMAL_CONSTRAINT;
        if (cat == -1) {
            const bool inl = ent && rank < cnt;
            kq = cnt;
            float4 qn = make_float4(0.f, 0.f, 0.f, 0.f);
            if (inl) qn = t.mnr[pos];
            bool ok = inl && kp.get_normals && isfinite(qn.x) && isfinite(qn.y) && isfinite(qn.z);
            if (ok && kp.angle_on) ok = !angle_reject(ns, qn.x, qn.y, qn.z, kp.angle_thr_deg, kp.cos_thr);
            const unsigned long long accm = __ballot(ok);
            const int nacc = __popcll(accm);
            if (nacc < 3) {
                cat = IMLS_REJ_MLS_FAIL;                        // imls_icp.cpp:463-466
            } else {
                const int lt = lane_of_rank(nacc - 1);          // Q3: L[|S| − 1]
                const double hmax = sqrt(rl_f64(ed, lt)) / 3;
                const double ih2 = 1.0 / (hmax * hmax);          // as finish_query
                double w = 0.0, pr = 0.0;
                if (ok) {
                    const double dx = xd[0] - (double)q.x, dy = xd[1] - (double)q.y, dz = xd[2] - (double)q.z;
                    double dn = dx * dx;
                    dn = dn + dy * dy;
                    dn = dn + dz * dz;
                    w = exp(-dn * ih2);
                    pr = (w * dx) * (double)qn.x;
                    pr = pr + (w * dy) * (double)qn.y;
                    pr = pr + (w * dz) * (double)qn.z;
                }
                // Σ in list order, as the lane code accumulates
                double wsum = 0.0, psum = 0.0;
                for (int r = 0; r < cnt; ++r) {
                    const int l = lane_of_rank(r);
                    if ((accm >> l) & 1ull) {
                        wsum += rl_f64(w, l);
                        psum += rl_f64(pr, l);
                    }
                }
                const double height = psum / (wsum + 1e-5);     // Q4
                if (isnan(height) || isinf(height)) {
                    cat = IMLS_REJ_NAN_INF_HEIGHT;
                } else {
                    yf[0] = (float)(xd[0] - height * nn[0]);    // imls_icp.cpp:719-729
                    yf[1] = (float)(xd[1] - height * nn[1]);
                    yf[2] = (float)(xd[2] - height * nn[2]);
                    nf[0] = (float)nn[0]; nf[1] = (float)nn[1]; nf[2] = (float)nn[2];
                }
            }
        }
    }
    if (lane == 0) {
        store_result(i, cat, xf, yf, nf, cs, cd, cn);
        if (cat >= 0) atomicAdd((unsigned long long*)&tr->reject[cat], 1ull);   // integer: order-free
        if (nbr_stats) {
            if (kq) atomicAdd(&nbr_stats[0], (unsigned long long)kq);
            if (l1 >= 0) atomicAdd(&nbr_stats[1], 1ull);
        }
    }
}

// =============================================================================================
// Per-lane exact traversal (fallback for uncertified queries; IMLS_TRAVERSAL_LANE mode)
// =============================================================================================
template <int KCAP>
__device__ __forceinline__ void project_lane_body(TreeView t, const float4* __restrict__ spt,
                                                             const float4* __restrict__ snr,
                                                             const unsigned* __restrict__ qlist,
                                                             const unsigned* __restrict__ qcount, int N,
                                                             const double* __restrict__ pose,
                                                             const int* __restrict__ done, KParams kp,
                                                             float4* __restrict__ cs, float4* __restrict__ cd,
                                                             float4* __restrict__ cn, double* __restrict__ partial1,
                                                             imls_iter_trace* __restrict__ tr,
                                                             unsigned long long* __restrict__ nbr_stats, int nlog) {
    // (done: the k_finish launch that listed the deferred queries left at once too)
    if (done && ld_const(done)) return;
    __shared__ uint2 stack[kStackDepth][kProjBlock];
    __shared__ double red[kProjBlock / 64][kNormEq];
    __shared__ double out[kNormEq];
    __shared__ unsigned rej_s[IMLS_NUM_REJ + 3];
    const int tid = threadIdx.x;
    if (tid < IMLS_NUM_REJ + 3) rej_s[tid] = 0;
    __syncthreads();
    // nlog logical blocks (one pass-1 slab each) taken by the physical blocks in turn: the slabs do
    // not depend on the physical grid.  A logical block lb works in rounds of kProjBlock queries:
    // every query (lane mode, qlist null) — rows lb·128 + k·nlog·128; deferred queries — the regions
    // k_finish's waves lb, lb + nlog, … listed (qlist[w·64 …], qcount[w] entries each), in wave order
    const int nfb = (N + 63) / 64;
    for (int lb = blockIdx.x; lb < nlog; lb += gridDim.x) {
    double acc_out = 0.0;   // thread tid < 28 accumulates its normal-equation term over rounds
    int fbk = lb, off = 0, base = lb * kProjBlock;
    // deferred queries are rare: the logical block's region counts are read in parallel first, and a
    // block with none writes its zero slab without the region walk (a chain of ~nfb/nlog dependent
    // count loads: ~13 µs per launch on config B with no query deferred)
    bool empty = false;
    if (qlist) {
        int any = 0;
        for (int k = tid; lb + k * nlog < nfb; k += kProjBlock) any |= qcount[lb + k * nlog] != 0u;
        empty = !__syncthreads_or(any);
    }
    for (; !empty;) {
        int q, total;
        size_t at;
        if (qlist) {
            while (fbk < nfb && off >= (int)qcount[fbk]) { fbk += nlog; off = 0; }
            if (fbk >= nfb) break;
            q = off + tid;
            total = (int)qcount[fbk];
            at = (size_t)fbk * 64 + q;
            off += kProjBlock;
        } else {
            if (base >= N) break;
            q = base + tid;
            total = N;
            at = (size_t)q;
            base += nlog * kProjBlock;
        }
        const bool active = q < total;
        const int i = active ? (qlist ? (int)qlist[at] : q) : 0;
        int cat = -2, kq = 0, nn_found = 0;
        float xf[3] = {0, 0, 0}, yf[3] = {0, 0, 0}, nf[3] = {0, 0, 0};
        if (active) {
            double ns[3];
            transform_query(pose, spt[i], snr[i], kp.transform_normal, xf, ns);
            const double xd[3] = {xf[0], xf[1], xf[2]};
            const int K = kp.K;
            double ld[KCAP];
            int li[KCAP];
#pragma unroll
            for (int j = 0; j < KCAP; ++j) {
                const bool sentinel = j < KCAP - K;           // capacity K inside KCAP registers
                ld[j] = sentinel ? -1.0 : kInfD;
                li[j] = sentinel ? -1 : 0x7fffffff;
            }
            double d1 = kInfD;
            int i1 = 0x7fffffff;
            // projected-distance mode (imls_icp.cpp:338-369, 563-596; laser_odometry.cpp:316-341):
            // candidates are the points with ‖p−x‖ < gate_dist and ‖(p−x)×n_s‖ < gate_proj, ranked by
            // the projected distance — the tree only bounds the ‖p−x‖ ball, the list key is proj
            const bool proj = kp.proj != 0;
            const double r2 = proj ? kp.gate_dist * kp.gate_dist : kp.r2;
            // a query deferred by k_finish carries its list's bound in cs[i].w (the search ball cap)
            const double cap = (qlist && !proj) ? fmin(r2, (double)cs[i].w) : r2;
            float bf = (float)cap * kBoxSlack + 1e-30f;
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
                    const int s0 = (node - P) * B, e0 = min(s0 + B, M);
                    for (int k = s0; k < e0; ++k) {
                        const float4 q4 = t.mpt[k];
                        const float ex = q4.x - xf[0], ey = q4.y - xf[1], ez = q4.z - xf[2];
                        const float d32 = __builtin_fmaf(ex, ex, __builtin_fmaf(ey, ey, ez * ez));
                        if (d32 > bf) continue;
                        const int oi = (int)__float_as_uint(q4.w);
                        if (proj) {
                            const double dx = (double)q4.x - xd[0], dy = (double)q4.y - xd[1], dz = (double)q4.z - xd[2];
                            const double cx = dy * ns[2] - dz * ns[1], cy = dz * ns[0] - dx * ns[2], cz = dx * ns[1] - dy * ns[0];
                            const double pr = sqrt((cx * cx + cy * cy) + cz * cz);
                            const double dn = sqrt((dx * dx + dy * dy) + dz * dz);
                            if (!(dn < kp.gate_dist && pr < kp.gate_proj)) continue;
                            if (lessp(pr, oi, ld[KCAP - 1], li[KCAP - 1])) {
                                bool prev = true;
#pragma unroll
                                for (int j = KCAP - 1; j >= 0; --j) {
                                    const bool sh = (j > 0) ? lessp(pr, oi, ld[(j > 0) ? j - 1 : 0], li[(j > 0) ? j - 1 : 0]) : false;
                                    const double nd = sh ? ld[(j > 0) ? j - 1 : 0] : (prev ? pr : ld[j]);
                                    const int ni = sh ? li[(j > 0) ? j - 1 : 0] : (prev ? oi : li[j]);
                                    ld[j] = nd;
                                    li[j] = ni;
                                    prev = sh;
                                }
                            }
                            continue;   // fixed bound: every point of the ball is a candidate
                        }
                        const double d2 = exact_d2(xd, q4.x, q4.y, q4.z);
                        if (!(d2 <= r2)) continue;
                        bool changed = false;
                        if (d2 > DBL_EPSILON && lessp(d2, oi, d1, i1)) { d1 = d2; i1 = oi; changed = true; }
                        if (lessp(d2, oi, ld[KCAP - 1], li[KCAP - 1])) {
                            bool prev = true;
#pragma unroll
                            for (int j = KCAP - 1; j >= 0; --j) {
                                const bool sh = (j > 0) ? lessp(d2, oi, ld[(j > 0) ? j - 1 : 0], li[(j > 0) ? j - 1 : 0]) : false;
                                const double nd = sh ? ld[(j > 0) ? j - 1 : 0] : (prev ? d2 : ld[j]);
                                const int ni = sh ? li[(j > 0) ? j - 1 : 0] : (prev ? oi : li[j]);
                                ld[j] = nd;
                                li[j] = ni;
                                prev = sh;
                            }
                            changed = true;
                        }
                        if (changed) bf = (float)fmin(cap, fmax(ld[KCAP - 1], d1)) * kBoxSlack + 1e-30f;
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
            int cnt = 0;
#pragma unroll
            for (int j = 0; j < KCAP; ++j) cnt += (j >= KCAP - K && ld[j] < kInfD) ? 1 : 0;
            if (proj) {
                // NN = the minimum projected distance (min_dist = proj², imls_icp.cpp:585-588); the
                // IMLS list holds proj² as its distances (361-365) — same candidates, same order
                i1 = li[KCAP - K];
                d1 = ld[KCAP - K] * ld[KCAP - K];
#pragma unroll
                for (int j = 0; j < KCAP; ++j) ld[j] = (j >= KCAP - K && ld[j] < kInfD) ? ld[j] * ld[j] : ld[j];
            }
            nn_found = i1 != 0x7fffffff;
            int lpos[KCAP];
#pragma unroll
            for (int j = 0; j < KCAP; ++j) lpos[j] = (li[j] >= 0 && li[j] != 0x7fffffff) ? (int)t.ipos[li[j]] : 0;
            const int p1 = nn_found ? (int)t.ipos[i1] : -1;
            cat = kp.matcher ? finish_plane(xf, ns, p1, t, kp, yf, nf)
                             : finish_query<KCAP>(xf, ns, ld, lpos, KCAP - K, cnt, d1, p1, t, kp, yf, nf, kq, i);
            store_result(i, cat, xf, yf, nf, cs, cd, cn);
        }
        if (cat >= 0) atomicAdd(&rej_s[cat], 1u);
        if (active) {
            if (kq) atomicAdd(&rej_s[IMLS_NUM_REJ], (unsigned)kq);
            if (nn_found) atomicAdd(&rej_s[IMLS_NUM_REJ + 1], 1u);
        }
        if (N > kSmallRows) {           // slabs for the grid solve chain only (see finish_body)
            double a[6] = {0, 0, 0, 0, 0, 0}, bb = 0.0, one = 0.0;
            if (cat == -1) { plane_row(xf, yf, nf, a, bb); one = 1.0; }
            block_normeq<kProjBlock>(a, bb, one, red, out);
            if (tid < kNormEq) acc_out += out[tid];
        }
    }
    if (N > kSmallRows && tid < kNormEq) partial1[(size_t)lb * kNormEq + tid] = acc_out;
    }
    __syncthreads();
    if (tid < IMLS_NUM_REJ && rej_s[tid]) atomicAdd((unsigned long long*)&tr->reject[tid], (unsigned long long)rej_s[tid]);
    if (nbr_stats && tid >= IMLS_NUM_REJ && tid < IMLS_NUM_REJ + 2 && rej_s[tid])
        atomicAdd(&nbr_stats[tid - IMLS_NUM_REJ], (unsigned long long)rej_s[tid]);
}

// ---------------------------------------------------------------------------------------------
// Kernels: one frame (arguments by value) and batched (frame = tab[blockIdx.y]; blocks past the
// frame's own grid leave at once).  Both run the same bodies.
// ---------------------------------------------------------------------------------------------
template <int KL>
__global__ __launch_bounds__(kWaveBlock) IMLS_KNN_ATTR void k_knn_wave(
        TreeView t, const float4* __restrict__ spt, const unsigned* __restrict__ qperm, int N,
        const double* __restrict__ pose, const int* __restrict__ done, KParams kp, const double* __restrict__ delta,
        int* __restrict__ lists, float* __restrict__ wlist, float4* __restrict__ xref, float* __restrict__ nref,
        int use_prev, unsigned long long* __restrict__ nbr_stats) {
    knn_wave_body<KL>(t, spt, qperm, N, pose, done, kp, delta, lists, wlist, xref, nref, use_prev, nbr_stats,
                      (int)blockIdx.x);
}

template <int KL>
__global__ __launch_bounds__(kWaveBlock) IMLS_KNN_ATTR void k_knn_wave_bfs(
        TreeView t, const float4* __restrict__ spt, const unsigned* __restrict__ qperm, int N,
        const double* __restrict__ pose, const int* __restrict__ done, KParams kp, const double* __restrict__ delta,
        int* __restrict__ lists, float* __restrict__ wlist, float4* __restrict__ xref, float* __restrict__ nref,
        int use_prev, unsigned long long* __restrict__ nbr_stats) {
    knn_wave_body<KL, 3>(t, spt, qperm, N, pose, done, kp, delta, lists, wlist, xref, nref, use_prev, nbr_stats,
                         (int)blockIdx.x);
}

template <int KL, int MODE>
__global__ __launch_bounds__(kWaveBlock) IMLS_KNN_ATTR void k_knn_wave_m(
        TreeView t, const float4* __restrict__ spt, const unsigned* __restrict__ qperm, int N,
        const double* __restrict__ pose, const int* __restrict__ done, KParams kp, const double* __restrict__ delta,
        int* __restrict__ lists, float* __restrict__ wlist, float4* __restrict__ xref, float* __restrict__ nref,
        unsigned long long* __restrict__ nbr_stats) {
    knn_wave_body<KL, MODE>(t, spt, qperm, N, pose, done, kp, delta, lists, wlist, xref, nref, 1, nbr_stats,
                            (int)blockIdx.x, cmp_of(lists, N), cmp_count_of(lists, N));
}

template <int KL>
__global__ __launch_bounds__(kWaveBlock) void k_knn_qwave(
        TreeView t, const float4* __restrict__ spt, const unsigned* __restrict__ qperm, int N,
        const double* __restrict__ pose, const int* __restrict__ done, KParams kp, const double* __restrict__ delta,
        int* __restrict__ lists, float* __restrict__ wlist, float4* __restrict__ xref, float* __restrict__ nref,
        int use_prev, unsigned long long* __restrict__ nbr_stats) {
    knn_qwave_body<KL>(t, spt, qperm, N, pose, done, kp, delta, lists, wlist, xref, nref, use_prev, nbr_stats,
                       (int)blockIdx.x);
}

template <int KL>
__global__ __launch_bounds__(kWaveBlock) void k_knn_qwave_f(
        TreeView t, const float4* __restrict__ spt, const unsigned* __restrict__ qperm, int N,
        const double* __restrict__ pose, const int* __restrict__ done, KParams kp, const double* __restrict__ delta,
        int* __restrict__ lists, float* __restrict__ wlist, float4* __restrict__ xref, float* __restrict__ nref,
        int use_prev, unsigned long long* __restrict__ nbr_stats, QFinishArgs fa) {
    knn_qwave_body<KL, true>(t, spt, qperm, N, pose, done, kp, delta, lists, wlist, xref, nref, use_prev, nbr_stats,
                             (int)blockIdx.x, fa);
}

#if IMLS_FINISH_QUAD
#undef IMLS_FINISH_ATTR
#define IMLS_FINISH_ATTR IMLS_FINISH4_ATTR
#endif
template <int KL>
__global__ __launch_bounds__(kWaveBlock) IMLS_FINISH_ATTR void k_finish(
        TreeView t, const float4* __restrict__ spt, const float4* __restrict__ snr, const unsigned* __restrict__ qperm,
        int N, const double* __restrict__ pose, const int* __restrict__ done, KParams kp, const int* __restrict__ lists,
        const float* __restrict__ wlist, float4* __restrict__ cs, float4* __restrict__ cd, float4* __restrict__ cn,
        double* __restrict__ partial1, imls_iter_trace* __restrict__ tr, unsigned long long* __restrict__ nbr_stats,
        unsigned* __restrict__ fb_list, unsigned* __restrict__ fb_count) {
#if IMLS_FINISH_QUAD
    finish4_body<KL>(t, spt, snr, qperm, N, pose, done, kp, lists, wlist, cs, cd, cn, partial1, tr, nbr_stats, fb_list,
                     fb_count, (int)blockIdx.x);
#else
    finish_body<KL>(t, spt, snr, qperm, N, pose, done, kp, lists, wlist, cs, cd, cn, partial1, tr, nbr_stats, fb_list,
                    fb_count, (int)blockIdx.x);
#endif
}

template <int KCAP>
__global__ __launch_bounds__(kProjBlock) void k_project_lane(
        TreeView t, const float4* __restrict__ spt, const float4* __restrict__ snr, const unsigned* __restrict__ qlist,
        const unsigned* __restrict__ qcount, int N, const double* __restrict__ pose, const int* __restrict__ done,
        KParams kp, float4* __restrict__ cs, float4* __restrict__ cd, float4* __restrict__ cn,
        double* __restrict__ partial1, imls_iter_trace* __restrict__ tr, unsigned long long* __restrict__ nbr_stats) {
    project_lane_body<KCAP>(t, spt, snr, qlist, qcount, N, pose, done, kp, cs, cd, cn, partial1, tr, nbr_stats,
                            kFallbackBlocks);
}

// k_finish blocks of a frame (one pass-1 slab each, before the kFallbackBlocks fallback slabs)
__host__ __device__ __forceinline__ int finish_blocks_of(int N) { return (N + kFinishPerBlock - 1) / kFinishPerBlock; }
// traversal blocks for packets of qp queries per wave
__host__ __device__ __forceinline__ int knn_blocks_of(int N, int qp) {
    const int per = qp * (kWaveBlock / 64);
    return (N + per - 1) / per;
}
// traversal choice (launch_wave): one wave per query for sparse query sets, packets otherwise
__host__ __device__ __forceinline__ bool use_qwave(const KParams& kp, int N) {
    return kp.qwave > 0 || (kp.qwave < 0 && N <= kQwaveAutoN);
}
// one-frame launches of a small frame (≤ kSmallRows queries, solved by k_solve_small from its rows):
// the exact stage fused into the wave-per-query traversal (k_knn_qwave_f), nothing deferred — one
// projection launch per ICP iteration
__host__ __forceinline__ bool fused_stage(const KParams& kp, int N) { return use_qwave(kp, N) && N <= kSmallRows; }
// the list block of a frame (see launch_wave): positions [KL][N], worst keys [N], xref, nref
template <int KL>
__device__ __forceinline__ float* wlist_of(int* lists, int N) { return reinterpret_cast<float*>(lists + (size_t)KL * N); }
__device__ __forceinline__ float4* xref_dev(int* lists, int N) {
    return reinterpret_cast<float4*>(reinterpret_cast<char*>(lists) + ((size_t)(kMaxKL + 1) * N * 4 + 255) / 256 * 256);
}

// The (frame, block) a batched block works on.  xcd: blocks are dealt round-robin over the 8 XCDs
// (b and b + 8 share one, MI355X_MICROARCH.md §Workgroup dispatch), so frame f takes the blocks of
// one round-robin slot (f mod 8) — its blocks share that XCD's L2 (a frame's map and tree),
// instead of every frame being spread over all eight.  grid.y is then padded to a multiple of 8.
__device__ __forceinline__ void batch_block(int xcd, int& frame, int& bx) {
    if (!xcd) {
        frame = (int)blockIdx.y;
        bx = (int)blockIdx.x;
        return;
    }
    const unsigned nx = gridDim.x;
    const unsigned p = blockIdx.x + blockIdx.y * nx;
    const unsigned s = p >> 3;
    frame = (int)((p & 7u) + 8u * (s / nx));
    bx = (int)(s % nx);
}

template <int KL>
__global__ __launch_bounds__(kWaveBlock) IMLS_KNN_ATTR void k_knn_wave_b(const PairDev* __restrict__ tab, KParams kp,
                                                                          int use_prev, int npairs) {
    int f, bx;
    batch_block(kp.xcd, f, bx);
    if (f >= npairs) return;
    const PairDev A = device_view(tab + f);
    if (use_qwave(kp, A.N) || bx >= knn_blocks_of(A.N, kp.packet)) return;
    float4* xref = xref_dev(A.lists, A.N);
    knn_wave_body<KL>(A.t, A.spt, A.qperm, A.N, A.st.pose, A.st.done, kp, A.st.delta, A.lists,
                                wlist_of<KL>(A.lists, A.N), xref, reinterpret_cast<float*>(xref + A.N), use_prev, A.stats,
                                bx);
}

template <int KL>
__global__ __launch_bounds__(kWaveBlock) IMLS_KNN_ATTR void k_knn_wave_bfsb(const PairDev* __restrict__ tab, KParams kp,
                                                                             int use_prev, int npairs) {
    int f, bx;
    batch_block(kp.xcd, f, bx);
    if (f >= npairs) return;
    const PairDev A = device_view(tab + f);
    if (use_qwave(kp, A.N) || bx >= knn_blocks_of(A.N, kp.packet)) return;
    float4* xref = xref_dev(A.lists, A.N);
    knn_wave_body<KL, 3>(A.t, A.spt, A.qperm, A.N, A.st.pose, A.st.done, kp, A.st.delta, A.lists,
                         wlist_of<KL>(A.lists, A.N), xref, reinterpret_cast<float*>(xref + A.N), use_prev, A.stats, bx);
}

template <int KL, int MODE>
__global__ __launch_bounds__(kWaveBlock) IMLS_KNN_ATTR void k_knn_wave_mb(const PairDev* __restrict__ tab, KParams kp,
                                                                           int npairs) {
    int f, bx;
    batch_block(kp.xcd, f, bx);
    if (f >= npairs) return;
    const PairDev A = device_view(tab + f);
    if (use_qwave(kp, A.N) || bx >= knn_blocks_of(A.N, kp.packet)) return;
    float4* xref = xref_dev(A.lists, A.N);
    knn_wave_body<KL, MODE>(A.t, A.spt, A.qperm, A.N, A.st.pose, A.st.done, kp, A.st.delta, A.lists,
                            wlist_of<KL>(A.lists, A.N), xref, reinterpret_cast<float*>(xref + A.N), 1, A.stats, bx,
                            cmp_of(A.lists, A.N), cmp_count_of(A.lists, A.N));
}

template <int KL>
__global__ __launch_bounds__(kWaveBlock) void k_knn_qwave_b(const PairDev* __restrict__ tab, KParams kp, int use_prev,
                                                            int npairs) {
    int f, bx;
    batch_block(kp.xcd, f, bx);
    if (f >= npairs) return;
    const PairDev A = device_view(tab + f);
    if (!use_qwave(kp, A.N) || bx * (kWaveBlock / 64) >= A.N) return;
    float4* xref = xref_dev(A.lists, A.N);
    knn_qwave_body<KL>(A.t, A.spt, A.qperm, A.N, A.st.pose, A.st.done, kp, A.st.delta, A.lists, wlist_of<KL>(A.lists, A.N),
                       xref, reinterpret_cast<float*>(xref + A.N), use_prev, A.stats, bx);
}

template <int KL>
__global__ __launch_bounds__(kWaveBlock) IMLS_FINISH_ATTR void k_finish_b(const PairDev* __restrict__ tab, KParams kp,
                                                                           int it, int npairs) {
    int f, bx;
    batch_block(kp.xcd, f, bx);
    if (f >= npairs) return;
    const PairDev A = device_view(tab + f);
    if (bx >= finish_blocks_of(A.N)) return;
#if IMLS_FINISH_QUAD
    finish4_body<KL>(A.t, A.spt, A.snr, A.qperm, A.N, A.st.pose, A.st.done, kp, A.lists, wlist_of<KL>(A.lists, A.N), A.cs,
                     A.cd, A.cn, A.st.partial1, A.trace + it, A.stats, A.fb_list, A.fb_count, bx);
#else
    finish_body<KL>(A.t, A.spt, A.snr, A.qperm, A.N, A.st.pose, A.st.done, kp, A.lists, wlist_of<KL>(A.lists, A.N), A.cs,
                    A.cd, A.cn, A.st.partial1, A.trace + it, A.stats, A.fb_list, A.fb_count, bx);
#endif
}

template <int KCAP>
__global__ __launch_bounds__(kProjBlock) void k_project_lane_b(const PairDev* __restrict__ tab, KParams kp, int it) {
    const PairDev A = device_view(tab + blockIdx.y);
    project_lane_body<KCAP>(A.t, A.spt, A.snr, A.fb_list, A.fb_count, A.N, A.st.pose, A.st.done, kp, A.cs, A.cd, A.cn,
                            A.st.partial1 + (size_t)finish_blocks_of(A.N) * kNormEq, A.trace + it, A.stats,
                            kFallbackBlocks);
}

template <int KL>
void launch_wave_batch(hipStream_t s, const PairDev* tab, int npairs, int maxN, bool any_small, bool any_large,
                       const KParams& kp, int it, int use_prev) {
    const int wb = finish_blocks_of(maxN);
    const int gy = kp.xcd ? (npairs + 7) / 8 * 8 : npairs;
    if (any_small) {
        const int n = kp.qwave > 0 ? maxN : std::min(maxN, kQwaveAutoN);
        k_knn_qwave_b<KL><<<dim3((n + kWaveBlock / 64 - 1) / (kWaveBlock / 64), gy), kWaveBlock, 0, s>>>(tab, kp, use_prev, npairs);
    }
    if (any_large) {
        const int kb = knn_blocks_of(maxN, kp.packet);
        if (it < IMLS_BFS_ITERS) {
            k_knn_wave_bfsb<KL><<<dim3(kb, gy), kWaveBlock, 0, s>>>(tab, kp, use_prev, npairs);
        } else if (use_prev && IMLS_COMPACT) {
            k_knn_wave_mb<KL, 1><<<dim3(kb, gy), kWaveBlock, 0, s>>>(tab, kp, npairs);
            k_knn_wave_mb<KL, 2><<<dim3(kb, gy), kWaveBlock, 0, s>>>(tab, kp, npairs);
        } else {
            k_knn_wave_b<KL><<<dim3(kb, gy), kWaveBlock, 0, s>>>(tab, kp, use_prev, npairs);
        }
    }
    k_finish_b<KL><<<dim3(wb, gy), kWaveBlock, 0, s>>>(tab, kp, it, npairs);
}

template <int KCAP>
void launch_lane(hipStream_t s, int blocks, const TreeView& t, const float4* spt, const float4* snr, const unsigned* qlist,
                 const unsigned* qcount, int N, const double* pose, const int* done, const KParams& kp, float4* cs,
                 float4* cd, float4* cn, double* partial1, imls_iter_trace* tr, unsigned long long* stats) {
    k_project_lane<KCAP><<<blocks, kProjBlock, 0, s>>>(t, spt, snr, qlist, qcount, N, pose, done, kp, cs, cd, cn, partial1,
                                                       tr, stats);
}


// The lone small frame's list (k_knn_qwave_f): entry k in lane k, so a longer list costs the wave no
// registers — K + 12 entries instead of K + 2 give the Verlet certificate a longer skin (√W − √need:
// the 32nd vs the 20th neighbour's distance instead of the 22nd), so fewer steady-iteration queries
// re-traverse (the slowest 2 % set each launch's length).  The list is read only by the same kernel.
#ifndef IMLS_LONE_EXTRA
#define IMLS_LONE_EXTRA 10
#endif
template <int KL>
constexpr int lone_kl() { return KL + IMLS_LONE_EXTRA <= kMaxKL ? KL + IMLS_LONE_EXTRA : kMaxKL; }

template <int KL>
void launch_wave(hipStream_t s, int blocks, const TreeView& t, const float4* spt, const float4* snr, const unsigned* qperm,
                 int N, const double* pose, const int* done, const KParams& kp, float4* cs, float4* cd, float4* cn,
                 double* partial1, imls_iter_trace* tr, unsigned long long* stats, unsigned* fb_list, unsigned* fb_count,
                 const double* delta, int* lists, int use_prev, hipEvent_t* marks) {
    float* wlist = reinterpret_cast<float*>(lists + (size_t)KL * N);
    float4* xref = xref_of(lists, N);
    float* nref = reinterpret_cast<float*>(xref + N);
    if (marks) (void)hipEventRecord(marks[0], s);
    // sparse query sets (≤ kQwaveAutoN queries, e.g. FPS-sampled frames): one wave per query, with the
    // exact stage in the same kernel for ≤ kSmallRows; dense scans: packets of 64 Morton-coherent
    // queries, then k_finish
    const bool fused = fused_stage(kp, N);
    if (fused)
        k_knn_qwave_f<lone_kl<KL>()><<<(N + kWaveBlock / 64 - 1) / (kWaveBlock / 64), kWaveBlock, 0, s>>>(
            t, spt, qperm, N, pose, done, kp, delta, lists, reinterpret_cast<float*>(lists + (size_t)lone_kl<KL>() * N), xref,
            nref, use_prev, stats, QFinishArgs{snr, cs, cd, cn, tr});
    else if (use_qwave(kp, N))
        k_knn_qwave<KL><<<(N + kWaveBlock / 64 - 1) / (kWaveBlock / 64), kWaveBlock, 0, s>>>(t, spt, qperm, N, pose, done, kp,
                                                                                          delta, lists, wlist, xref, nref, use_prev, stats);
    else if (kp.bfs && IMLS_BFS_ITERS > 0)
        k_knn_wave_bfs<KL><<<knn_blocks_of(N, kp.packet), kWaveBlock, 0, s>>>(t, spt, qperm, N, pose, done, kp, delta, lists,
                                                                              wlist, xref, nref, use_prev, stats);
    else if (use_prev && IMLS_COMPACT) {
        // later iterations: reuse decided per lane, then packets of the compacted re-traversing slots
        k_knn_wave_m<KL, 1><<<knn_blocks_of(N, kp.packet), kWaveBlock, 0, s>>>(t, spt, qperm, N, pose, done, kp, delta, lists,
                                                                               wlist, xref, nref, stats);
        k_knn_wave_m<KL, 2><<<knn_blocks_of(N, kp.packet), kWaveBlock, 0, s>>>(t, spt, qperm, N, pose, done, kp, delta, lists,
                                                                               wlist, xref, nref, stats);
    } else
        k_knn_wave<KL><<<knn_blocks_of(N, kp.packet), kWaveBlock, 0, s>>>(t, spt, qperm, N, pose, done, kp, delta, lists, wlist,
                                                                          xref, nref, use_prev, stats);
    if (marks) (void)hipEventRecord(marks[1], s);
    if (!fused)
        k_finish<KL><<<blocks, kWaveBlock, 0, s>>>(t, spt, snr, qperm, N, pose, done, kp, lists, wlist, cs, cd, cn, partial1,
                                                   tr, stats, fb_list, fb_count);
    if (marks) (void)hipEventRecord(marks[2], s);
}

}  // namespace

void launch_project_batch(hipStream_t s, const PairDev* tab, const int* n_host, int npairs, const KParams& kp0, int it,
                          int use_prev) {
    // auto traversal choice for a batch: the wave-per-query kernel wins on one small frame (latency:
    // few waves), packets win once the batch's queries fill the GPU (measured on the config-C-like
    // stream, 32 frames of ~1900 queries per launch: 546 → 320 µs).  Either gives the exact answer.
    KParams kp = kp_at(kp0, kp0.pk_batch ? it : -1);
    long long total = 0;
    for (int k = 0; k < npairs; ++k) total += n_host[k];
    if (kp.qwave < 0 && total > kQwaveAutoN) kp.qwave = 0;
    // XCD-grouped frames for batches of many frames (their maps together outgrow the L2s)
    if (kp.xcd < 0) kp.xcd = npairs >= 16 ? 1 : 0;
    // tensor voting: every frame's voted normals at its current pose first (imls_icp.cpp:514-546)
    if (kp.tv) launch_tv_vote_batch(s, tab, n_host, npairs, kp, use_prev);
    int maxN = 0;
    bool any_small = false, any_large = false;
    for (int k = 0; k < npairs; ++k) {
        maxN = std::max(maxN, n_host[k]);
        (use_qwave(kp, n_host[k]) ? any_small : any_large) = true;
    }
    if (npairs <= 0 || maxN <= 0) return;
    const int K = kp.K;
    if (K <= 8) launch_wave_batch<12>(s, tab, npairs, maxN, any_small, any_large, kp, it, use_prev);
    else if (K <= 16) launch_wave_batch<20>(s, tab, npairs, maxN, any_small, any_large, kp, it, use_prev);
    else if (K <= 20) launch_wave_batch<IMLS_B_KL>(s, tab, npairs, maxN, any_small, any_large, kp, it, use_prev);
    else launch_wave_batch<36>(s, tab, npairs, maxN, any_small, any_large, kp, it, use_prev);
    // exact fallback for uncertified queries: every frame's kFallbackBlocks slabs are written, by
    // fewer physical blocks per frame when many frames share the launch (uncertified queries are
    // rare; a grid of 64 mostly idle blocks per frame cost ~130 µs at 512 frames)
    const dim3 g(npairs >= 16 ? kFallbackBlocksBatched : kFallbackBlocks, npairs);
    if (K <= 8) k_project_lane_b<8><<<g, kProjBlock, 0, s>>>(tab, kp, it);
    else if (K <= 16) k_project_lane_b<16><<<g, kProjBlock, 0, s>>>(tab, kp, it);
    else if (K <= 20) k_project_lane_b<20><<<g, kProjBlock, 0, s>>>(tab, kp, it);
    else k_project_lane_b<32><<<g, kProjBlock, 0, s>>>(tab, kp, it);
}

int project_blocks(int N) { return finish_blocks_of(N) + kFallbackBlocks; }

void launch_project(hipStream_t s, const TreeView& t, const float4* spt, const float4* snr, const unsigned* qperm,
                    int N, const double* pose, const int* done, const KParams& kp, float4* cs, float4* cd, float4* cn,
                    double* partial1, imls_iter_trace* tr, unsigned long long* stats, unsigned* fb_list,
                    unsigned* fb_count, int lane_mode, const double* delta, int* lists, int use_prev, hipEvent_t* marks) {
    const int wblocks = finish_blocks_of(N);
    double* p_fb = partial1 + (size_t)wblocks * kNormEq;
    const int K = kp.K;
    // tensor voting: every source point's voted normal at this pose first (imls_icp.cpp:514-546)
    if (kp.tv) launch_tv_vote(s, t, spt, N, pose, done, kp, const_cast<double4*>(t.tvn), use_prev);
    if (lane_mode || kp.proj) {
        // reference mode: every query through the exact per-lane kernel (grid-stride over the
        // fallback slabs); the wave slabs are zeroed
        (void)hipMemsetAsync(partial1, 0, (size_t)wblocks * kNormEq * sizeof(double), s);
        if (K <= 8) launch_lane<8>(s, kFallbackBlocks, t, spt, snr, nullptr, nullptr, N, pose, done, kp, cs, cd, cn, p_fb, tr, stats);
        else if (K <= 16) launch_lane<16>(s, kFallbackBlocks, t, spt, snr, nullptr, nullptr, N, pose, done, kp, cs, cd, cn, p_fb, tr, stats);
        else if (K <= 20) launch_lane<20>(s, kFallbackBlocks, t, spt, snr, nullptr, nullptr, N, pose, done, kp, cs, cd, cn, p_fb, tr, stats);
        else launch_lane<32>(s, kFallbackBlocks, t, spt, snr, nullptr, nullptr, N, pose, done, kp, cs, cd, cn, p_fb, tr, stats);
        return;
    }
    if (K <= 8) launch_wave<12>(s, wblocks, t, spt, snr, qperm, N, pose, done, kp, cs, cd, cn, partial1, tr, stats, fb_list, fb_count, delta, lists, use_prev, marks);
    else if (K <= 16) launch_wave<20>(s, wblocks, t, spt, snr, qperm, N, pose, done, kp, cs, cd, cn, partial1, tr, stats, fb_list, fb_count, delta, lists, use_prev, marks);
    // K ≤ 20 (the shipped 20): two slack entries certify every query on config B (KL 21 left a few
    // uncertified → the slow exact fallback, −30 %; KL 22 vs 24 measured +6.7 % pairs/s, 4 in flight)
    else if (K <= 20) launch_wave<IMLS_B_KL>(s, wblocks, t, spt, snr, qperm, N, pose, done, kp, cs, cd, cn, partial1, tr, stats, fb_list, fb_count, delta, lists, use_prev, marks);
    else launch_wave<36>(s, wblocks, t, spt, snr, qperm, N, pose, done, kp, cs, cd, cn, partial1, tr, stats, fb_list, fb_count, delta, lists, use_prev, marks);
    // exact fallback for uncertified queries (usually none; the launch exits at once then); the
    // fused small-frame kernel resolves them in place
    if (fused_stage(kp, N)) return;
    if (K <= 8) launch_lane<8>(s, kFallbackBlocks, t, spt, snr, fb_list, fb_count, N, pose, done, kp, cs, cd, cn, p_fb, tr, stats);
    else if (K <= 16) launch_lane<16>(s, kFallbackBlocks, t, spt, snr, fb_list, fb_count, N, pose, done, kp, cs, cd, cn, p_fb, tr, stats);
    else if (K <= 20) launch_lane<20>(s, kFallbackBlocks, t, spt, snr, fb_list, fb_count, N, pose, done, kp, cs, cd, cn, p_fb, tr, stats);
    else launch_lane<32>(s, kFallbackBlocks, t, spt, snr, fb_list, fb_count, N, pose, done, kp, cs, cd, cn, p_fb, tr, stats);
}

}  // namespace imlsgpu

#ifdef IMLS_DEBUG_WAVE_TRACE
// debug build only: per-wave records of the last k_knn_wave launch (16 u32 per wave)
extern "C" int imls_debug_waves(unsigned* out, int nwaves) {
    const int n = nwaves < imlsgpu::kDbgWaves ? nwaves : imlsgpu::kDbgWaves;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(imlsgpu::g_dbg_wave), (size_t)n * 64) == hipSuccess ? n : -1;
}
#endif
