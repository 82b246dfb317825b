// index.hip — per-frame spatial index of the target map (replaces the libnabo kd-tree built by
// IMLSICPMatcher::setTargetPointCloud, imls_icp.cpp:80-103) and the source loader
// (setSourcePointCloud, imls_icp.cpp:74-78).
//
// Build = NaN filter + order-preserving compaction (RemoveNANandINFData, imls_icp.cpp:58-72)
//       → bbox → 48-bit Morton keys → radix sort (key, filtered index) → Morton-ordered float4
//       points → B-point buckets as the leaves of an implicit complete binary tree of AABBs.
// All kernels are HBM-streaming: coalesced float loads, float4 stores.
#include <hipcub/hipcub.hpp>

#include "internal.h"

namespace imlsgpu {
namespace {

template <typename T>
T* carve(char*& p, size_t n) {
    T* r = reinterpret_cast<T*>(p);
    p += ((n * sizeof(T) + 255) / 256) * 256;
    return r;
}

bool ensure(DevBuf& b, size_t bytes, std::string& err) {
    if (b.bytes >= bytes) return true;
    if (b.p) (void)hipFree(b.p);
    b.p = nullptr;
    b.bytes = 0;
    size_t want = bytes + bytes / 4 + 4096;
    if (hipMalloc(&b.p, want) != hipSuccess) {
        err = "hipMalloc failed (" + std::to_string(want) + " bytes)";
        return false;
    }
    b.bytes = want;
    return true;
}

__global__ void k_flag_finite(const float* __restrict__ soa, size_t n, unsigned* __restrict__ flag) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float x = soa[i], y = soa[n + i], z = soa[2 * n + i];
    flag[i] = (isfinite(x) && isfinite(y) && isfinite(z)) ? 1u : 0u;
}

// scatter kept points to float4 records; pos = exclusive prefix sum of flags
__global__ void k_compact(const float* __restrict__ soa, size_t n, const unsigned* __restrict__ flag,
                          const unsigned* __restrict__ pos, float4* __restrict__ pt, float4* __restrict__ nr,
                          unsigned* __restrict__ kept_index, int* __restrict__ count) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    if (i == n - 1) *count = (int)(pos[i] + flag[i]);
    if (!flag[i]) return;
    unsigned o = pos[i];
    pt[o] = make_float4(soa[i], soa[n + i], soa[2 * n + i], 0.f);
    nr[o] = make_float4(soa[3 * n + i], soa[4 * n + i], soa[5 * n + i], 0.f);
    if (kept_index) kept_index[o] = (unsigned)i;
}

__global__ void k_bbox_partial(const float4* __restrict__ pt, const int* __restrict__ count, float* __restrict__ part) {
    __shared__ float red[6][kBlock];
    int M = *count;
    float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < M; i += gridDim.x * blockDim.x) {
        float4 p = pt[i];
        lo[0] = fminf(lo[0], p.x); lo[1] = fminf(lo[1], p.y); lo[2] = fminf(lo[2], p.z);
        hi[0] = fmaxf(hi[0], p.x); hi[1] = fmaxf(hi[1], p.y); hi[2] = fmaxf(hi[2], p.z);
    }
    for (int d = 0; d < 3; ++d) { red[d][threadIdx.x] = lo[d]; red[3 + d][threadIdx.x] = hi[d]; }
    __syncthreads();
    for (int s = kBlock / 2; s > 0; s >>= 1) {
        if (threadIdx.x < s)
            for (int d = 0; d < 3; ++d) {
                red[d][threadIdx.x] = fminf(red[d][threadIdx.x], red[d][threadIdx.x + s]);
                red[3 + d][threadIdx.x] = fmaxf(red[3 + d][threadIdx.x], red[3 + d][threadIdx.x + s]);
            }
        __syncthreads();
    }
    if (threadIdx.x < 6) part[blockIdx.x * 6 + threadIdx.x] = red[threadIdx.x][0];
}

__global__ void k_bbox_final(const float* __restrict__ part, int nparts, float* __restrict__ bbox) {
    __shared__ float red[6][kBlock];
    float r[6] = {INFINITY, INFINITY, INFINITY, -INFINITY, -INFINITY, -INFINITY};
    for (int b = threadIdx.x; b < nparts; b += kBlock)
        for (int d = 0; d < 3; ++d) {
            r[d] = fminf(r[d], part[b * 6 + d]);
            r[3 + d] = fmaxf(r[3 + d], part[b * 6 + 3 + d]);
        }
    for (int d = 0; d < 6; ++d) red[d][threadIdx.x] = r[d];
    __syncthreads();
    for (int st = kBlock / 2; st > 0; st >>= 1) {
        if (threadIdx.x < st)
            for (int d = 0; d < 3; ++d) {
                red[d][threadIdx.x] = fminf(red[d][threadIdx.x], red[d][threadIdx.x + st]);
                red[3 + d][threadIdx.x] = fmaxf(red[3 + d][threadIdx.x], red[3 + d][threadIdx.x + st]);
            }
        __syncthreads();
    }
    if (threadIdx.x < 6) bbox[threadIdx.x] = red[threadIdx.x][0];
}

__global__ void k_qparams(const float* __restrict__ bbox, float* __restrict__ qp) {
    if (threadIdx.x) return;
    const float ext = fmaxf(fmaxf(fmaxf(bbox[3] - bbox[0], bbox[4] - bbox[1]), bbox[5] - bbox[2]), 1e-6f);
    qp[0] = bbox[0]; qp[1] = bbox[1]; qp[2] = bbox[2];
    qp[3] = 65535.f / ext;
}

__global__ void k_morton(const float4* __restrict__ pt, const int* __restrict__ count, const float* __restrict__ qp,
                         unsigned long long* __restrict__ key, unsigned* __restrict__ val) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    int M = *count;
    if (i >= M) return;
    float4 p = pt[i];
    key[i] = morton48(p.x, p.y, p.z, qp);
    val[i] = (unsigned)i;
}

__global__ void k_leaf_keys(const unsigned long long* __restrict__ sorted, int M, int B, unsigned long long* __restrict__ lk) {
    int l = blockIdx.x * blockDim.x + threadIdx.x;
    if (l * B < M) lk[l] = sorted[(size_t)l * B];
}

// Morton-ordered copies: mpt (xyz + original index), mnr (normals), and ipos (original → Morton)
__global__ void k_gather(const float4* __restrict__ pt, const float4* __restrict__ nr, const unsigned* __restrict__ perm,
                         int M, float4* __restrict__ mpt, float4* __restrict__ mnr, unsigned* __restrict__ ipos) {
    int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= M) return;
    unsigned j = perm[k];
    float4 p = pt[j];
    mpt[k] = make_float4(p.x, p.y, p.z, __uint_as_float(j));
    mnr[k] = nr[j];
    ipos[j] = (unsigned)k;
}

struct Box { float lo[3], hi[3]; };

__device__ __forceinline__ Box box_union(const Box& a, const Box& b) {
    Box r;
    for (int d = 0; d < 3; ++d) { r.lo[d] = fminf(a.lo[d], b.lo[d]); r.hi[d] = fmaxf(a.hi[d], b.hi[d]); }
    return r;
}

// leaf boxes: one thread per bucket b < P; buckets ≥ L are empty (inverted box, never visited)
__global__ void k_leaf_boxes(const float4* __restrict__ mpt, int M, int B, int P, float* __restrict__ leafbox) {
    int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= P) return;
    Box bx = {{INFINITY, INFINITY, INFINITY}, {-INFINITY, -INFINITY, -INFINITY}};
    int s = b * B, e = min(s + B, M);
    for (int k = s; k < e; ++k) {
        float4 p = mpt[k];
        bx.lo[0] = fminf(bx.lo[0], p.x); bx.lo[1] = fminf(bx.lo[1], p.y); bx.lo[2] = fminf(bx.lo[2], p.z);
        bx.hi[0] = fmaxf(bx.hi[0], p.x); bx.hi[1] = fmaxf(bx.hi[1], p.y); bx.hi[2] = fmaxf(bx.hi[2], p.z);
    }
    for (int d = 0; d < 3; ++d) { leafbox[b * 6 + d] = bx.lo[d]; leafbox[b * 6 + 3 + d] = bx.hi[d]; }
}

// One block reduces 2^s (≤ 256) consecutive boxes of depth D into their subtree: writes the
// internal-node records of depths D−1 … D−s and the subtree root box to roots[blockIdx].
__global__ void k_subtree(const float* __restrict__ in, int count, int D, float4* __restrict__ nodes, float* __restrict__ roots) {
    __shared__ Box sb[kBlock];
    int t = threadIdx.x;
    int width = min(count, kBlock);
    int base = blockIdx.x * width;
    if (t < width) {
        const float* q = in + (size_t)(base + t) * 6;
        for (int d = 0; d < 3; ++d) { sb[t].lo[d] = q[d]; sb[t].hi[d] = q[3 + d]; }
    }
    __syncthreads();
    int n = width, depth = D;
    while (n > 1) {
        n >>= 1;
        --depth;
        Box u;
        bool act = t < n;
        if (act) {
            Box l = sb[2 * t], r = sb[2 * t + 1];
            int id = (1 << depth) + (base >> (D - depth)) + t;
            float4* rec = nodes + 3 * (size_t)id;
            rec[0] = make_float4(l.lo[0], l.lo[1], l.lo[2], l.hi[0]);
            rec[1] = make_float4(l.hi[1], l.hi[2], r.lo[0], r.lo[1]);
            rec[2] = make_float4(r.lo[2], r.hi[0], r.hi[1], r.hi[2]);
            u = box_union(l, r);
        }
        __syncthreads();
        if (act) sb[t] = u;
        __syncthreads();
    }
    if (t == 0 && roots) {
        for (int d = 0; d < 3; ++d) { roots[blockIdx.x * 6 + d] = sb[0].lo[d]; roots[blockIdx.x * 6 + 3 + d] = sb[0].hi[d]; }
    }
}

inline unsigned grid_for(size_t n, int b = kBlock) { return (unsigned)((n + b - 1) / b); }

}  // namespace

// NaN filter + order-keeping compaction, asynchronous: the kept count lands in *h_count (pinned
// host memory) by an async copy behind the compaction — valid once the stream has passed it.
int filter_async(hipStream_t s, const float* d_soa6, size_t n_in, DevBuf& pt, DevBuf& nr, DevBuf& scratch,
                 unsigned* d_kept, int* h_count, std::string& err) {
    size_t cub_bytes = 0;
    if (hipcub::DeviceScan::ExclusiveSum(nullptr, cub_bytes, (unsigned*)nullptr, (unsigned*)nullptr, (int)n_in, s) != hipSuccess) {
        err = "hipcub scan size query failed";
        return IMLS_ERR_DEVICE;
    }
    size_t need = 2 * (((n_in * 4 + 255) / 256) * 256) + ((cub_bytes + 255) / 256) * 256 + 512;
    if (!ensure(scratch, need, err) || !ensure(pt, n_in * 16 + 16, err) || !ensure(nr, n_in * 16 + 16, err)) return IMLS_ERR_DEVICE;
    char* p = (char*)scratch.p;
    unsigned* flag = carve<unsigned>(p, n_in);
    unsigned* pos = carve<unsigned>(p, n_in);
    int* cnt = carve<int>(p, 64);
    void* cub_tmp = carve<char>(p, cub_bytes);
    k_flag_finite<<<grid_for(n_in), kBlock, 0, s>>>(d_soa6, n_in, flag);
    hipcub::DeviceScan::ExclusiveSum(cub_tmp, cub_bytes, flag, pos, (int)n_in, s);
    k_compact<<<grid_for(n_in), kBlock, 0, s>>>(d_soa6, n_in, flag, pos, (float4*)pt.p, (float4*)nr.p, d_kept, cnt);
    if (hipMemcpyAsync(h_count, cnt, sizeof(int), hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipGetLastError() != hipSuccess) {
        err = "filter/compact launch failed";
        return IMLS_ERR_DEVICE;
    }
    return IMLS_OK;
}

namespace {

// Permutation (sorted → input index) of n float4 points by 48-bit Morton code over their bbox.
// With lkeys: also the first key of each B-point leaf and the quantisation (seed search).
int morton_perm(hipStream_t s, const float4* pts, int n, DevBuf& scratch, DevBuf& perm, std::string& err,
                DevBuf* lkeys = nullptr, int B = 0) {
    size_t cub_bytes = 0;
    hipcub::DeviceRadixSort::SortPairs(nullptr, cub_bytes, (unsigned long long*)nullptr, (unsigned long long*)nullptr,
                                       (unsigned*)nullptr, (unsigned*)nullptr, n, 0, 48, s);
    const int bb_parts = 512;
    size_t need = 2 * (((size_t)n * 8 + 255) / 256 * 256) + (((size_t)n * 4 + 255) / 256 * 256) +
                  ((cub_bytes + 255) / 256) * 256 + bb_parts * 24 + 1024;
    if (!ensure(scratch, need, err) || !ensure(perm, (size_t)n * 4 + 16, err)) return IMLS_ERR_DEVICE;
    char* p = (char*)scratch.p;
    unsigned long long* k0 = carve<unsigned long long>(p, n);
    unsigned long long* k1 = carve<unsigned long long>(p, n);
    unsigned* v0 = carve<unsigned>(p, n);
    void* cub_tmp = carve<char>(p, cub_bytes);
    float* bbpart = carve<float>(p, bb_parts * 6);
    float* bbox = carve<float>(p, 8);
    float* qp = carve<float>(p, 4);
    int* cnt = carve<int>(p, 4);
    const int L = B > 0 ? (n + B - 1) / B : 0;
    if (lkeys && !ensure(*lkeys, (size_t)L * 8 + 16, err)) return IMLS_ERR_DEVICE;
    if (lkeys) qp = (float*)((unsigned long long*)lkeys->p + L);   // qparams live after the keys
    hipMemcpyAsync(cnt, &n, sizeof(int), hipMemcpyHostToDevice, s);
    int nb = std::min(bb_parts, (int)grid_for(n));
    k_bbox_partial<<<nb, kBlock, 0, s>>>(pts, cnt, bbpart);
    k_bbox_final<<<1, kBlock, 0, s>>>(bbpart, nb, bbox);
    k_qparams<<<1, 64, 0, s>>>(bbox, qp);
    k_morton<<<grid_for(n), kBlock, 0, s>>>(pts, cnt, qp, k0, v0);
    hipcub::DeviceRadixSort::SortPairs(cub_tmp, cub_bytes, k0, k1, v0, (unsigned*)perm.p, n, 0, 48, s);
    if (lkeys) k_leaf_keys<<<grid_for(L), kBlock, 0, s>>>(k1, n, B, (unsigned long long*)lkeys->p);
    if (hipGetLastError() != hipSuccess) { err = "morton sort launch failed"; return IMLS_ERR_DEVICE; }
    return IMLS_OK;
}

}  // namespace

int build_target_tree(hipStream_t s, int M, int bucket, DevBuf& lkeys, DevBuf& tpt, DevBuf& tnr, DevBuf& mpt,
                      DevBuf& nodes, DevBuf& scratch, DevBuf& treescratch, DevBuf& permbuf, int* P_out, int* levels_out,
                      std::string& err) {
    if (M <= 0) { *P_out = 0; *levels_out = 0; return IMLS_OK; }
    const int B = bucket;
    int L = (M + B - 1) / B;
    int P = 1, levels = 0;
    while (P < L) { P <<= 1; ++levels; }
    if (levels > kStackDepth - 1) { err = "tree too deep for the traversal stack"; return IMLS_ERR_CAPACITY; }
    int rc = morton_perm(s, (const float4*)tpt.p, M, scratch, permbuf, err, &lkeys, B);
    if (rc) return rc;
    size_t need = ((size_t)P * 24 + 255) / 256 * 256 + 2 * (((size_t)P / kBlock + 1) * 24 + 256) + 1024;
    if (!ensure(treescratch, need, err) || !ensure(mpt, (size_t)M * 36 + 64, err) ||
        !ensure(nodes, (size_t)(P + 1) * 48, err))
        return IMLS_ERR_DEVICE;
    char* p = (char*)treescratch.p;
    float* leafbox = carve<float>(p, (size_t)P * 6);
    float* rootsA = carve<float>(p, ((size_t)P / kBlock + 1) * 6);
    float* rootsB = carve<float>(p, ((size_t)P / kBlock + 1) * 6);
    k_gather<<<grid_for(M), kBlock, 0, s>>>((const float4*)tpt.p, (const float4*)tnr.p, (const unsigned*)permbuf.p, M,
                                            (float4*)mpt.p, (float4*)mpt.p + M, (unsigned*)((float4*)mpt.p + 2 * (size_t)M));
    k_leaf_boxes<<<grid_for(P), kBlock, 0, s>>>((const float4*)mpt.p, M, B, P, leafbox);
    // bottom-up subtree reduction, 256 boxes per block per launch
    const float* in = leafbox;
    float* outs[2] = {rootsA, rootsB};
    int count = P, D = levels, which = 0;
    while (count > 1) {
        int width = std::min(count, kBlock);
        int lg = 0;
        while ((1 << lg) < width) ++lg;
        int blocks = count / width;
        k_subtree<<<blocks, kBlock, 0, s>>>(in, count, D, (float4*)nodes.p, outs[which]);
        in = outs[which];
        which ^= 1;
        count = blocks;
        D -= lg;
    }
    if (hipGetLastError() != hipSuccess) { err = "index build launch failed"; return IMLS_ERR_DEVICE; }
    *P_out = P;
    *levels_out = levels;
    return IMLS_OK;
}

int source_order(hipStream_t s, int N, DevBuf& spt, DevBuf& scratch, DevBuf& qperm, std::string& err) {
    if (N <= 0) return IMLS_OK;
    return morton_perm(s, (const float4*)spt.p, N, scratch, qperm, err);
}

}  // namespace imlsgpu
