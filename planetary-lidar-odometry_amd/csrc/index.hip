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
    // a replaced buffer is retired behind the work that may still read it (internal.h devbuf_grow)
    if (devbuf_grow(b, bytes, bytes + bytes / 4 + 4096)) return true;
    err = "hipMalloc failed (" + std::to_string(bytes + bytes / 4 + 4096) + " bytes)";
    return false;
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
                          unsigned* __restrict__ kept_index, int* __restrict__ count, int* __restrict__ h_count) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    if (i == n - 1) {
        const int c = (int)(pos[i] + flag[i]);
        *count = c;
        *h_count = c;   // pinned host memory, written directly (no copy launch per filter)
    }
    if (!flag[i]) return;
    unsigned o = pos[i];
    pt[o] = make_float4(soa[i], soa[n + i], soa[2 * n + i], 0.f);
    nr[o] = make_float4(soa[3 * n + i], soa[4 * n + i], soa[5 * n + i], 0.f);
    if (kept_index) kept_index[o] = (unsigned)i;
}

__global__ void k_bbox_partial(const float4* __restrict__ pt, int M, float* __restrict__ part) {
    __shared__ float red[6][kBlock];
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

__global__ void k_bbox_final(const float* __restrict__ part, int nparts, float* __restrict__ bbox, float* __restrict__ qp) {
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
    if (threadIdx.x == 0) {    // the quantisation (k_qparams' arithmetic), one launch fewer
        const float ext = fmaxf(fmaxf(fmaxf(red[3][0] - red[0][0], red[4][0] - red[1][0]), red[5][0] - red[2][0]), 1e-6f);
        qp[0] = red[0][0]; qp[1] = red[1][0]; qp[2] = red[2][0];
        qp[3] = 65535.f / ext;
    }
}

__global__ void k_morton(const float4* __restrict__ pt, int M, const float* __restrict__ qp,
                         unsigned long long* __restrict__ key, unsigned* __restrict__ val) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
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

// NaN filter + order-keeping compaction, asynchronous: the kept count lands in *h_count (pinned,
// device-visible host memory) from the compaction kernel itself — valid once the stream has passed it.
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
    k_compact<<<grid_for(n_in), kBlock, 0, s>>>(d_soa6, n_in, flag, pos, (float4*)pt.p, (float4*)nr.p, d_kept, cnt, h_count);
    if (hipGetLastError() != hipSuccess) {
        err = "filter/compact launch failed";
        return IMLS_ERR_DEVICE;
    }
    return IMLS_OK;
}

// ---------------------------------------------------------------------------------------------
// Batched NaN filters (imls_register_frames): every pending filter of a batch's members in three
// launches — per 256-point block counts, one scan block per job (its kept count also to the
// job's pinned host word), order-keeping scatter.  Same output as filter_async, frame by frame.
// ---------------------------------------------------------------------------------------------
namespace {

struct FilterJobDev {
    const float* soa;                 // SoA6 input [6][n]
    size_t n;
    float4 *pt, *nr;                  // kept points / normals
    unsigned* kept;                   // kept → input index, or null
    int* d_count;
    int* h_count;                     // pinned host word
    int* blk;                         // [nb] block counts → offsets
};

__device__ __forceinline__ bool finite_at(const float* soa, size_t n, size_t i) {
    return isfinite(soa[i]) && isfinite(soa[n + i]) && isfinite(soa[2 * n + i]);
}

__global__ __launch_bounds__(kBlock) void k_filter_count_b(const FilterJobDev* __restrict__ jobs) {
    const FilterJobDev& J = jobs[blockIdx.y];
    const size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x;
    if ((size_t)blockIdx.x * kBlock >= J.n) return;
    const bool keep = i < J.n && finite_at(J.soa, J.n, i);
    __shared__ int wc[kBlock / 64];
    const unsigned long long m = __ballot(keep);
    if ((threadIdx.x & 63) == 0) wc[threadIdx.x >> 6] = __popcll(m);
    __syncthreads();
    if (threadIdx.x == 0) {
        int c = 0;
        for (int k = 0; k < kBlock / 64; ++k) c += wc[k];
        J.blk[blockIdx.x] = c;
    }
}

__global__ __launch_bounds__(1024) void k_filter_scan_b(const FilterJobDev* __restrict__ jobs) {
    const FilterJobDev& J = jobs[blockIdx.x];
    const int nb = (int)((J.n + kBlock - 1) / kBlock);
    __shared__ int sc[1024];
    int carry = 0;
    for (int base = 0; base < nb; base += 1024) {
        const int b = base + threadIdx.x;
        const int v = b < nb ? J.blk[b] : 0;
        sc[threadIdx.x] = v;
        __syncthreads();
        for (int off = 1; off < 1024; off <<= 1) {
            const int t = threadIdx.x >= off ? sc[threadIdx.x - off] : 0;
            __syncthreads();
            sc[threadIdx.x] += t;
            __syncthreads();
        }
        if (b < nb) J.blk[b] = carry + sc[threadIdx.x] - v;
        __syncthreads();
        carry += sc[1023];
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        *J.d_count = carry;
        *J.h_count = carry;
    }
}

__global__ __launch_bounds__(kBlock) void k_filter_scatter_b(const FilterJobDev* __restrict__ jobs) {
    const FilterJobDev& J = jobs[blockIdx.y];
    if ((size_t)blockIdx.x * kBlock >= J.n) return;
    const size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x;
    const bool keep = i < J.n && finite_at(J.soa, J.n, i);
    __shared__ int wc[kBlock / 64];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const unsigned long long m = __ballot(keep);
    if (lane == 0) wc[wv] = __popcll(m);
    __syncthreads();
    if (!keep) return;
    int o = J.blk[blockIdx.x];
    for (int k = 0; k < wv; ++k) o += wc[k];
    o += __popcll(m & ((1ull << lane) - 1ull));
    const float* s = J.soa;
    const size_t n = J.n;
    J.pt[o] = make_float4(s[i], s[n + i], s[2 * n + i], 0.f);
    J.nr[o] = make_float4(s[3 * n + i], s[4 * n + i], s[5 * n + i], 0.f);
    if (J.kept) J.kept[o] = (unsigned)i;
}

}  // namespace

size_t filter_job_bytes() { return sizeof(FilterJobDev); }

int filter_batch(hipStream_t s, const std::vector<FilterJob>& jobs, DevBuf& scratch, DevBuf& table, void* h_table,
                 size_t h_table_bytes, std::string& err) {
    const int nj = (int)jobs.size();
    if (nj == 0) return IMLS_OK;
    if ((size_t)nj * sizeof(FilterJobDev) > h_table_bytes) { err = "filter table too small"; return IMLS_ERR_CAPACITY; }
    if (nj > 65535) { err = "too many filter jobs"; return IMLS_ERR_CAPACITY; }
    size_t blocks = 0, maxn = 1;
    for (const auto& f : jobs) {
        blocks += (f.n + kBlock - 1) / kBlock + 64;
        maxn = std::max(maxn, f.n);
    }
    if (!ensure(scratch, blocks * 4 + (size_t)nj * 256 + 4096, err) ||
        !ensure(table, (size_t)nj * sizeof(FilterJobDev) + 256, err))
        return IMLS_ERR_DEVICE;
    char* p = (char*)scratch.p;
    FilterJobDev* J = (FilterJobDev*)h_table;
    for (int q = 0; q < nj; ++q) {
        const FilterJob& f = jobs[q];
        if (!ensure(*f.pt, f.n * 16 + 16, err) || !ensure(*f.nr, f.n * 16 + 16, err)) return IMLS_ERR_DEVICE;
        FilterJobDev d{};
        d.soa = f.soa;
        d.n = f.n;
        d.pt = (float4*)f.pt->p;
        d.nr = (float4*)f.nr->p;
        d.kept = f.kept;
        d.d_count = carve<int>(p, 16);
        d.h_count = f.h_count;
        d.blk = carve<int>(p, (f.n + kBlock - 1) / kBlock + 1);
        J[q] = d;
    }
    const FilterJobDev* jd = (const FilterJobDev*)table.p;
    hipMemcpyAsync(table.p, h_table, (size_t)nj * sizeof(FilterJobDev), hipMemcpyHostToDevice, s);
    const unsigned gx = grid_for(maxn);
    k_filter_count_b<<<dim3(gx, nj), kBlock, 0, s>>>(jd);
    k_filter_scan_b<<<nj, 1024, 0, s>>>(jd);
    k_filter_scatter_b<<<dim3(gx, nj), kBlock, 0, s>>>(jd);
    if (hipGetLastError() != hipSuccess) { err = "batched filter launch failed"; return IMLS_ERR_DEVICE; }
    return IMLS_OK;
}

namespace {

// ---------------------------------------------------------------------------------------------
// Stable (key, index) pair sort for the index builds' ≤ 256k-point sorts (round 6: the source's and a
// FIFO run's Morton order — hipcub's radix sort runs a merge sort there, ~14 launches and ~100 µs per
// 126k keys with their gaps).  The values are the input positions (k_morton / k_morton_fq), so
// ordering the distinct (key, value) pairs is the stable radix sort's order, bit for bit.
//   k_tile_sort: 4096-pair tiles bitonic-sorted in LDS by 512 threads;
//   k_merge_pass: sorted runs of w merged pairwise, 2048 outputs per block — the block's two
//   merge-path splits by a 128-ary search (128 threads per diagonal, 3 rounds for runs ≤ 2M), both
//   input segments staged in LDS, each thread's 8 outputs merged sequentially.
// ---------------------------------------------------------------------------------------------
constexpr int kSortTile = 4096;
constexpr int kSortTileThreads = 512;
// measured slower than hipcub's merge sort (k_tile_sort 61.7 µs + 5 merge passes of 9.8 µs per 126k keys;
// FIFO index 0.218-0.221 vs 0.170-0.188 ms per registration, profiles/r06_sort_rejected/): off
#ifndef IMLS_SMALL_SORT
#define IMLS_SMALL_SORT 0
#endif
constexpr int kSortSmallMax = IMLS_SMALL_SORT ? 1 << 18 : 0;
constexpr int kMergeOut = 2048;
constexpr int kMergeOutPer = kMergeOut / kBlock;

__device__ __forceinline__ bool pair_less(unsigned long long ka, unsigned va, unsigned long long kb, unsigned vb) {
    return ka < kb || (ka == kb && va < vb);
}

__global__ __launch_bounds__(kSortTileThreads) void k_tile_sort(const unsigned long long* __restrict__ key,
                                                               const unsigned* __restrict__ val, int n,
                                                               unsigned long long* __restrict__ okey,
                                                               unsigned* __restrict__ oval) {
    __shared__ unsigned long long sk[kSortTile];
    __shared__ unsigned sv[kSortTile];
    const int base = blockIdx.x * kSortTile;
    for (int e = threadIdx.x; e < kSortTile; e += kSortTileThreads) {
        const int g = base + e;
        sk[e] = g < n ? key[g] : ~0ull;     // padding sorts last (keys are < 2^48)
        sv[e] = g < n ? val[g] : ~0u;
    }
    for (int size = 2; size <= kSortTile; size <<= 1)
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            __syncthreads();
            for (int e = threadIdx.x; e < kSortTile / 2; e += kSortTileThreads) {
                const int i = ((e & ~(stride - 1)) << 1) | (e & (stride - 1)), j = i + stride;
                const bool up = (i & size) == 0;
                const unsigned long long ki = sk[i], kj = sk[j];
                const unsigned vi = sv[i], vj = sv[j];
                if (pair_less(kj, vj, ki, vi) == up) { sk[i] = kj; sk[j] = ki; sv[i] = vj; sv[j] = vi; }
            }
        }
    __syncthreads();
    for (int e = threadIdx.x; e < kSortTile; e += kSortTileThreads) {
        const int g = base + e;
        if (g < n) { okey[g] = sk[e]; oval[g] = sv[e]; }
    }
}

__global__ __launch_bounds__(kBlock) void k_merge_pass(const unsigned long long* __restrict__ key,
                                                       const unsigned* __restrict__ val, int n, int w,
                                                       unsigned long long* __restrict__ okey,
                                                       unsigned* __restrict__ oval) {
    __shared__ unsigned long long sk[kMergeOut];
    __shared__ unsigned sv[kMergeOut];
    __shared__ int scnt[2][kBlock / 64];
    __shared__ int ssplit[2];
    const long long o0 = (long long)blockIdx.x * kMergeOut;
    if (o0 >= n) return;                                   // block-uniform
    const long long o1 = std::min(o0 + kMergeOut, (long long)n);
    const long long ps = o0 / (2ll * w) * (2ll * w);       // the pair of runs holding this block's outputs
    const int na = (int)std::min((long long)w, n - ps);
    const int nb = (int)std::max(0ll, std::min((long long)w, n - ps - w));
    const unsigned long long* ak = key + ps;
    const unsigned* av = val + ps;
    const unsigned long long* bk = key + ps + na;
    const unsigned* bv = val + ps + na;
    // the splits of the block's two diagonals: A's entries among the first d outputs, P(a) = A[a] < B[d−1−a]
    // holds exactly below the split; 128 samples per round narrow [lo, hi] below ⌈span / 128⌉
    const int g = threadIdx.x >> 7, lt = threadIdx.x & 127, wv = threadIdx.x >> 6;
    const long long d = g ? o1 - ps : o0 - ps;
    int lo = (int)std::max(0ll, d - nb), hi = (int)std::min(d, (long long)na);
#pragma unroll
    for (int round = 0; round < 3; ++round) {
        const int span = hi - lo;
        const int step = (span + 127) / 128;
        const int pos = lo + lt * step;
        const bool smp = span > 0 && pos < hi;
        const bool pt = smp && pair_less(ak[pos], av[pos], bk[d - 1 - pos], bv[d - 1 - pos]);
        const unsigned long long bt = __ballot(pt), bs = __ballot(smp);
        if ((threadIdx.x & 63) == 0) { scnt[0][wv] = __popcll(bt); scnt[1][wv] = __popcll(bs); }
        __syncthreads();
        const int k = scnt[0][2 * g] + scnt[0][2 * g + 1], ns = scnt[1][2 * g] + scnt[1][2 * g + 1];
        __syncthreads();
        if (span > 0) {
            if (k == 0) {
                hi = lo;
            } else {
                const int last = lo + (k - 1) * step;
                hi = k < ns ? lo + k * step : hi;
                lo = last + 1;
            }
        }
    }
    if (lt == 0) ssplit[g] = lo;
    __syncthreads();
    const int i0 = ssplit[0], i1 = ssplit[1];
    const int j0 = (int)(o0 - ps - i0), j1 = (int)(o1 - ps - i1);
    const int la = i1 - i0, lb = j1 - j0;
    for (int e = threadIdx.x; e < la; e += kBlock) { sk[e] = ak[i0 + e]; sv[e] = av[i0 + e]; }
    for (int e = threadIdx.x; e < lb; e += kBlock) { sk[la + e] = bk[j0 + e]; sv[la + e] = bv[j0 + e]; }
    __syncthreads();
    const int q = threadIdx.x * kMergeOutPer, m = la + lb;
    if (q >= m) return;
    int x0 = std::max(0, q - lb), x1 = std::min(q, la);
    while (x0 < x1) {
        const int mid = (x0 + x1) >> 1;
        if (pair_less(sk[mid], sv[mid], sk[la + q - 1 - mid], sv[la + q - 1 - mid])) x0 = mid + 1;
        else x1 = mid;
    }
    int x = x0, y = q - x0;
    const int qe = std::min(q + kMergeOutPer, m);
    for (int r = q; r < qe; ++r) {
        const bool takeA = y >= lb || (x < la && pair_less(sk[x], sv[x], sk[la + y], sv[la + y]));
        const int src = takeA ? x : la + y;
        okey[o0 + r] = sk[src];
        oval[o0 + r] = sv[src];
        x += takeA ? 1 : 0;
        y += takeA ? 0 : 1;
    }
}

// The pairs of (k0, v0) sorted; returns 1 when the result is in (k1, v1), 0 when in (k0, v0).
int small_sort_pairs(hipStream_t s, unsigned long long* k0, unsigned* v0, unsigned long long* k1, unsigned* v1, int n) {
    const int tiles = (n + kSortTile - 1) / kSortTile;
    k_tile_sort<<<tiles, kSortTileThreads, 0, s>>>(k0, v0, n, k1, v1);
    int cur = 1;
    const int blocks = (n + kMergeOut - 1) / kMergeOut;
    for (long long w = kSortTile; w < n; w *= 2) {
        if (cur) k_merge_pass<<<blocks, kBlock, 0, s>>>(k1, v1, n, (int)w, k0, v0);
        else k_merge_pass<<<blocks, kBlock, 0, s>>>(k0, v0, n, (int)w, k1, v1);
        cur ^= 1;
    }
    return cur;
}

// The sort orders the full 48-bit Morton codes.  Sorting their top 32 bits only (two radix passes
// fewer, the lone frame's index build ~15 µs shorter) coarsens the order inside 1/1625-extent cells:
// config B's leaves and packets lose coherence, 423.7 → 397.5 pairs/s (round 4, profiles/r04_final3)
constexpr int kMortonSortLo = 0;

// Permutation (sorted → input index) of n float4 points by 48-bit Morton code over their bbox.
// With lkeys: also the first key of each B-point leaf and the quantisation (seed search).  The sort
// is double-buffered (round 6: the plain form ended in two copy-back launches of keys and values);
// *perm_out = the buffer holding the permutation — perm's own storage when the caller needs it there
// (need_in_perm: one device copy if the sort left it in scratch), else possibly scratch.
int morton_perm(hipStream_t s, const float4* pts, int n, DevBuf& scratch, DevBuf& perm, std::string& err,
                DevBuf* lkeys = nullptr, int B = 0, const unsigned** perm_out = nullptr) {
    size_t cub_bytes = 0;
    {
        hipcub::DoubleBuffer<unsigned long long> kq(nullptr, nullptr);
        hipcub::DoubleBuffer<unsigned> vq(nullptr, nullptr);
        hipcub::DeviceRadixSort::SortPairs(nullptr, cub_bytes, kq, vq, n, kMortonSortLo, 48, s);
    }
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
    (void)cnt;
    int nb = std::min(bb_parts, (int)grid_for(n));
    k_bbox_partial<<<nb, kBlock, 0, s>>>(pts, n, bbpart);
    k_bbox_final<<<1, kBlock, 0, s>>>(bbpart, nb, bbox, qp);
    k_morton<<<grid_for(n), kBlock, 0, s>>>(pts, n, qp, k0, v0);
    unsigned long long* kcur;
    unsigned* vcur;
    if (n <= kSortSmallMax && kMortonSortLo == 0) {
        const int r = small_sort_pairs(s, k0, v0, k1, (unsigned*)perm.p, n);
        kcur = r ? k1 : k0;
        vcur = r ? (unsigned*)perm.p : v0;
    } else {
        hipcub::DoubleBuffer<unsigned long long> kb(k0, k1);
        hipcub::DoubleBuffer<unsigned> vb(v0, (unsigned*)perm.p);
        hipcub::DeviceRadixSort::SortPairs(cub_tmp, cub_bytes, kb, vb, n, kMortonSortLo, 48, s);
        kcur = kb.Current();
        vcur = vb.Current();
    }
    if (lkeys) k_leaf_keys<<<grid_for(L), kBlock, 0, s>>>(kcur, n, B, (unsigned long long*)lkeys->p);
    if (perm_out) {
        *perm_out = vcur;
    } else if (vcur != (unsigned*)perm.p) {
        (void)hipMemcpyAsync(perm.p, vcur, (size_t)n * 4, hipMemcpyDeviceToDevice, s);
    }
    if (hipGetLastError() != hipSuccess) { err = "morton sort launch failed"; return IMLS_ERR_DEVICE; }
    return IMLS_OK;
}

}  // namespace

void tree_rounds(hipStream_t s, const float4* mpt, int M, int B, int P, int levels, float4* nodes, float* leafbox,
                 float* rootsA, float* rootsB);
void subtree_rounds(hipStream_t s, const float* leafbox, int P, int levels, float4* nodes, float* rootsA, float* rootsB);

int build_target_tree(hipStream_t s, int M, int bucket, DevBuf& lkeys, DevBuf& tpt, DevBuf& tnr, DevBuf& mpt,
                      DevBuf& nodes, DevBuf& scratch, DevBuf& treescratch, DevBuf& permbuf, int* P_out, int* levels_out,
                      std::string& err) {
    if (M <= 0) { *P_out = 0; *levels_out = 0; return IMLS_OK; }
    const int B = bucket;
    int L = (M + B - 1) / B;
    int P = 1, levels = 0;
    while (P < L) { P <<= 1; ++levels; }
    if (levels > kStackDepth - 1) { err = "tree too deep for the traversal stack"; return IMLS_ERR_CAPACITY; }
    const unsigned* perm = nullptr;
    int rc = morton_perm(s, (const float4*)tpt.p, M, scratch, permbuf, err, &lkeys, B, &perm);
    if (rc) return rc;
    size_t need = ((size_t)P * 24 + 255) / 256 * 256 + 2 * (((size_t)P / kBlock + 1) * 24 + 256) + 1024;
    if (!ensure(treescratch, need, err) || !ensure(mpt, (size_t)M * 36 + 64, err) ||
        !ensure(nodes, (size_t)(P + 1) * 48, err))
        return IMLS_ERR_DEVICE;
    char* p = (char*)treescratch.p;
    float* leafbox = carve<float>(p, (size_t)P * 6);
    float* rootsA = carve<float>(p, ((size_t)P / kBlock + 1) * 6);
    float* rootsB = carve<float>(p, ((size_t)P / kBlock + 1) * 6);
    k_gather<<<grid_for(M), kBlock, 0, s>>>((const float4*)tpt.p, (const float4*)tnr.p, perm, M,
                                            (float4*)mpt.p, (float4*)mpt.p + M, (unsigned*)((float4*)mpt.p + 2 * (size_t)M));
    tree_rounds(s, (const float4*)mpt.p, M, B, P, levels, (float4*)nodes.p, leafbox, rootsA, rootsB);
    if (hipGetLastError() != hipSuccess) { err = "index build launch failed"; return IMLS_ERR_DEVICE; }
    *P_out = P;
    *levels_out = levels;
    return IMLS_OK;
}

// leaf boxes of the Morton-ordered points, then the bottom-up subtree reduction, 256 boxes per block
// per launch (the node records of every internal level)
void tree_rounds(hipStream_t s, const float4* mpt, int M, int B, int P, int levels, float4* nodes, float* leafbox,
                 float* rootsA, float* rootsB) {
    k_leaf_boxes<<<grid_for(P), kBlock, 0, s>>>(mpt, M, B, P, leafbox);
    subtree_rounds(s, leafbox, P, levels, nodes, rootsA, rootsB);
}

// the internal levels from P leaf boxes (k_subtree rounds, 256 boxes per block per round)
void subtree_rounds(hipStream_t s, const float* leafbox, int P, int levels, float4* nodes, float* rootsA, float* rootsB) {
    const float* in = leafbox;
    float* outs[2] = {rootsA, rootsB};
    int count = P, D = levels, which = 0;
    while (count > 1) {
        int width = std::min(count, kBlock);
        int lg = 0;
        while ((1 << lg) < width) ++lg;
        int blocks = count / width;
        k_subtree<<<blocks, kBlock, 0, s>>>(in, count, D, nodes, outs[which]);
        in = outs[which];
        which ^= 1;
        count = blocks;
        D -= lg;
    }
}

namespace {
// The source order of a small frame (≤ kSmallOrderN points) in ONE launch: the bbox and quantisation
// (k_bbox_partial / k_bbox_final's min / max and arithmetic), the 48-bit Morton keys, and a bitonic
// sort of (key, index) in LDS — the permutation the stable radix sort gives (equal keys keep index
// order), where morton_perm / the batched build take 6-8 launches (a lone frame's critical path:
// the source is ordered after its filter's count arrives, before the first traversal)
__global__ __launch_bounds__(kSmallOrderN / 2) void k_small_order(const float4* __restrict__ pt, int n,
                                                                unsigned* __restrict__ perm) {
    constexpr int T = kSmallOrderN / 2;
    __shared__ unsigned long long sk[kSmallOrderN];
    __shared__ unsigned sv[kSmallOrderN];
    __shared__ float red[6][T];
    __shared__ float qp[4];
    const int t = threadIdx.x;
    float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    float4 p[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        const int i = t + u * T;
        p[u] = i < n ? pt[i] : make_float4(0.f, 0.f, 0.f, 0.f);
        if (i < n) {
            lo[0] = fminf(lo[0], p[u].x); lo[1] = fminf(lo[1], p[u].y); lo[2] = fminf(lo[2], p[u].z);
            hi[0] = fmaxf(hi[0], p[u].x); hi[1] = fmaxf(hi[1], p[u].y); hi[2] = fmaxf(hi[2], p[u].z);
        }
    }
    for (int d = 0; d < 3; ++d) { red[d][t] = lo[d]; red[3 + d][t] = hi[d]; }
    __syncthreads();
    for (int st = T / 2; st > 0; st >>= 1) {
        if (t < st)
            for (int d = 0; d < 3; ++d) {
                red[d][t] = fminf(red[d][t], red[d][t + st]);
                red[3 + d][t] = fmaxf(red[3 + d][t], red[3 + d][t + st]);
            }
        __syncthreads();
    }
    if (t == 0) {                     // k_bbox_final's quantisation
        const float ext = fmaxf(fmaxf(fmaxf(red[3][0] - red[0][0], red[4][0] - red[1][0]), red[5][0] - red[2][0]), 1e-6f);
        qp[0] = red[0][0]; qp[1] = red[1][0]; qp[2] = red[2][0];
        qp[3] = 65535.f / ext;
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        const int i = t + u * T;
        sk[i] = i < n ? morton48(p[u].x, p[u].y, p[u].z, qp) : ~0ull;
        sv[i] = i < n ? (unsigned)i : ~0u;
    }
    __syncthreads();
    for (int size = 2; size <= kSmallOrderN; size <<= 1)
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            const int i = ((t & ~(stride - 1)) << 1) | (t & (stride - 1)), j = i + stride;
            const unsigned long long ki = sk[i], kj = sk[j];
            const unsigned vi = sv[i], vj = sv[j];
            const bool gt = ki > kj || (ki == kj && vi > vj);
            if (gt == ((i & size) == 0)) { sk[i] = kj; sk[j] = ki; sv[i] = vj; sv[j] = vi; }
            __syncthreads();
        }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        const int i = t + u * T;
        if (i < n) perm[i] = sv[i];
    }
}
}  // namespace

int small_source_order(hipStream_t s, const float4* pts, int N, unsigned* perm, std::string& err) {
    if (N <= 0) return IMLS_OK;
    if (N > kSmallOrderN) { err = "small source order: too many points"; return IMLS_ERR_CAPACITY; }
    k_small_order<<<1, kSmallOrderN / 2, 0, s>>>(pts, N, perm);
    if (hipGetLastError() != hipSuccess) { err = "source order launch failed"; return IMLS_ERR_DEVICE; }
    return IMLS_OK;
}

int source_order(hipStream_t s, int N, DevBuf& spt, DevBuf& scratch, DevBuf& qperm, std::string& err) {
    if (N <= 0) return IMLS_OK;
    if (N <= kSmallOrderN) {
        if (!ensure(qperm, (size_t)N * 4 + 16, err)) return IMLS_ERR_DEVICE;
        return small_source_order(s, (const float4*)spt.p, N, (unsigned*)qperm.p, err);
    }
    return morton_perm(s, (const float4*)spt.p, N, scratch, qperm, err);
}

// ---------------------------------------------------------------------------------------------
// Batched builds (imls_register_frames): the target trees and source orders of many frames in one
// launch sequence — per-frame bbox partials, Morton keys with the job index above bit 48 (one radix
// sort orders every frame's points at once; stable, so each frame's permutation is exactly its own
// sort's), the Morton-ordered copies / leaf keys / permutations, leaf boxes and the subtree rounds.
// Every step computes what the per-frame build computes, in the same float operations.
// ---------------------------------------------------------------------------------------------
namespace {

constexpr int kBBoxParts = 64;          // bbox partial blocks per job (grid-stride)
constexpr int kSubRounds = 4;           // subtree rounds: ⌈levels / 8⌉ ≤ 3 for levels ≤ 23

struct JobDev {
    const float4* pts;                  // filtered points (xyz, 0)
    const float4* nrm;                  // filtered normals (targets)
    int n, off;                         // points; offset in the concatenated key array
    int B, L, P, levels;                // targets: bucket, leaves, padded leaves, tree levels (B = 0: source)
    float* qp;                          // [4] quantisation (targets: after the leaf keys)
    unsigned long long* lkeys;          // targets: first key of each leaf
    float4 *mpt, *mnr;                  // targets: Morton-ordered copies
    unsigned* ipos;                     // targets: input → Morton position
    float4* nodes;                      // targets: node records
    unsigned* perm;                     // sources: sorted → input index
    float* bbpart;                      // [kBBoxParts × 6]
    float* leafbox;                     // targets: [P × 6]
    const float* sub_in[kSubRounds];    // subtree round r: input boxes, count, depth, output roots
    float* sub_out[kSubRounds];
    int sub_count[kSubRounds], sub_D[kSubRounds];
};

__global__ __launch_bounds__(kBlock) void k_bbox_b(const JobDev* __restrict__ jobs) {
    const JobDev& J = jobs[blockIdx.y];
    __shared__ float red[6][kBlock];
    const int M = J.n;
    const int nb = min(kBBoxParts, (int)((M + kBlock - 1) / kBlock));
    if ((int)blockIdx.x >= nb) return;
    float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (int i = blockIdx.x * kBlock + threadIdx.x; i < M; i += nb * kBlock) {
        const float4 p = J.pts[i];
        lo[0] = fminf(lo[0], p.x); lo[1] = fminf(lo[1], p.y); lo[2] = fminf(lo[2], p.z);
        hi[0] = fmaxf(hi[0], p.x); hi[1] = fmaxf(hi[1], p.y); hi[2] = fmaxf(hi[2], p.z);
    }
    for (int d = 0; d < 3; ++d) { red[d][threadIdx.x] = lo[d]; red[3 + d][threadIdx.x] = hi[d]; }
    __syncthreads();
    for (int st = kBlock / 2; st > 0; st >>= 1) {
        if (threadIdx.x < st)
            for (int d = 0; d < 3; ++d) {
                red[d][threadIdx.x] = fminf(red[d][threadIdx.x], red[d][threadIdx.x + st]);
                red[3 + d][threadIdx.x] = fmaxf(red[3 + d][threadIdx.x], red[3 + d][threadIdx.x + st]);
            }
        __syncthreads();
    }
    if (threadIdx.x < 6) J.bbpart[blockIdx.x * 6 + threadIdx.x] = red[threadIdx.x][0];
}

// bbox (min / max are exact in any order) → quantisation (k_qparams' arithmetic), one wave per job
__global__ __launch_bounds__(64) void k_qparams_b(const JobDev* __restrict__ jobs) {
    const JobDev& J = jobs[blockIdx.x];
    const int M = J.n;
    if (M <= 0) return;
    const int nb = min(kBBoxParts, (int)((M + kBlock - 1) / kBlock));
    const int t = threadIdx.x;
    float b[6] = {INFINITY, INFINITY, INFINITY, -INFINITY, -INFINITY, -INFINITY};
    if (t < nb)
        for (int d = 0; d < 3; ++d) { b[d] = J.bbpart[t * 6 + d]; b[3 + d] = J.bbpart[t * 6 + 3 + d]; }
    for (int o = 32; o > 0; o >>= 1)
        for (int d = 0; d < 3; ++d) {
            b[d] = fminf(b[d], __shfl_xor(b[d], o, 64));
            b[3 + d] = fmaxf(b[3 + d], __shfl_xor(b[3 + d], o, 64));
        }
    if (t == 0) {
        const float ext = fmaxf(fmaxf(fmaxf(b[3] - b[0], b[4] - b[1]), b[5] - b[2]), 1e-6f);
        J.qp[0] = b[0]; J.qp[1] = b[1]; J.qp[2] = b[2];
        J.qp[3] = 65535.f / ext;
    }
}

// keys tagged with the job index above bit 48
__global__ __launch_bounds__(kBlock) void k_morton_b(const JobDev* __restrict__ jobs, unsigned long long* __restrict__ key,
                                                     unsigned* __restrict__ val) {
    const JobDev& J = jobs[blockIdx.y];
    const int i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= J.n) return;
    const float4 p = J.pts[i];
    key[(size_t)J.off + i] = ((unsigned long long)blockIdx.y << 48) | morton48(p.x, p.y, p.z, J.qp);
    val[(size_t)J.off + i] = (unsigned)i;
}

// sorted segment of a job → targets: Morton copies, input → Morton positions, leaf first keys;
// sources: the permutation
__global__ __launch_bounds__(kBlock) void k_place_b(const JobDev* __restrict__ jobs, const unsigned long long* __restrict__ key,
                                                    const unsigned* __restrict__ val) {
    const JobDev& J = jobs[blockIdx.y];
    const int k = blockIdx.x * kBlock + threadIdx.x;
    if (k >= J.n) return;
    const unsigned j = val[(size_t)J.off + k];
    if (J.B == 0) {
        J.perm[k] = j;
        return;
    }
    const float4 p = J.pts[j];
    J.mpt[k] = make_float4(p.x, p.y, p.z, __uint_as_float(j));
    J.mnr[k] = J.nrm[j];
    J.ipos[j] = (unsigned)k;
    if (k % J.B == 0) J.lkeys[k / J.B] = key[(size_t)J.off + k] & 0xFFFFFFFFFFFFull;
}

__global__ __launch_bounds__(kBlock) void k_leaf_boxes_b(const JobDev* __restrict__ jobs) {
    const JobDev& J = jobs[blockIdx.y];
    const int b = blockIdx.x * kBlock + threadIdx.x;
    if (J.B == 0 || b >= J.P) return;
    Box bx = {{INFINITY, INFINITY, INFINITY}, {-INFINITY, -INFINITY, -INFINITY}};
    const int s = b * J.B, e = min(s + J.B, J.n);
    for (int k = s; k < e; ++k) {
        const float4 p = J.mpt[k];
        bx.lo[0] = fminf(bx.lo[0], p.x); bx.lo[1] = fminf(bx.lo[1], p.y); bx.lo[2] = fminf(bx.lo[2], p.z);
        bx.hi[0] = fmaxf(bx.hi[0], p.x); bx.hi[1] = fmaxf(bx.hi[1], p.y); bx.hi[2] = fmaxf(bx.hi[2], p.z);
    }
    for (int d = 0; d < 3; ++d) { J.leafbox[b * 6 + d] = bx.lo[d]; J.leafbox[b * 6 + 3 + d] = bx.hi[d]; }
}

// subtree round r of every job (k_subtree's reduction; a job past its last round leaves)
__global__ __launch_bounds__(kBlock) void k_subtree_b(const JobDev* __restrict__ jobs, int r) {
    const JobDev& J = jobs[blockIdx.y];
    if (J.B == 0) return;
    const int count = J.sub_count[r];
    if (count <= 1) return;
    const int width = min(count, kBlock);
    if ((int)blockIdx.x >= count / width) return;
    const int D = J.sub_D[r];
    __shared__ Box sb[kBlock];
    const int t = threadIdx.x;
    const int base = blockIdx.x * width;
    if (t < width) {
        const float* q = J.sub_in[r] + (size_t)(base + t) * 6;
        for (int d = 0; d < 3; ++d) { sb[t].lo[d] = q[d]; sb[t].hi[d] = q[3 + d]; }
    }
    __syncthreads();
    int n = width, depth = D;
    while (n > 1) {
        n >>= 1;
        --depth;
        Box u;
        const bool act = t < n;
        if (act) {
            const Box l = sb[2 * t], rr = sb[2 * t + 1];
            const int id = (1 << depth) + (base >> (D - depth)) + t;
            float4* rec = J.nodes + 3 * (size_t)id;
            rec[0] = make_float4(l.lo[0], l.lo[1], l.lo[2], l.hi[0]);
            rec[1] = make_float4(l.hi[1], l.hi[2], rr.lo[0], rr.lo[1]);
            rec[2] = make_float4(rr.lo[2], rr.hi[0], rr.hi[1], rr.hi[2]);
            u = box_union(l, rr);
        }
        __syncthreads();
        if (act) sb[t] = u;
        __syncthreads();
    }
    if (t == 0)
        for (int d = 0; d < 3; ++d) { J.sub_out[r][blockIdx.x * 6 + d] = sb[0].lo[d]; J.sub_out[r][blockIdx.x * 6 + 3 + d] = sb[0].hi[d]; }
}

}  // namespace

size_t build_job_bytes() { return sizeof(JobDev); }

int build_batch(hipStream_t s, std::vector<BuildJob>& jobs, DevBuf& scratch, DevBuf& table, void* h_table,
                size_t h_table_bytes, std::string& err) {
    const int nj = (int)jobs.size();
    if (nj == 0) return IMLS_OK;
    if ((size_t)nj * sizeof(JobDev) > h_table_bytes) { err = "build table too small"; return IMLS_ERR_CAPACITY; }
    if (nj > 65535) { err = "too many build jobs"; return IMLS_ERR_CAPACITY; }
    size_t total = 0, leaf_floats = 0, root_floats = 0;
    int maxn = 1, maxP = 1;
    for (auto& b : jobs) {
        if (b.n <= 0) continue;
        total += (size_t)b.n;
        maxn = std::max(maxn, b.n);
        if (b.B > 0) {
            const int L = (b.n + b.B - 1) / b.B;
            int P = 1, levels = 0;
            while (P < L) { P <<= 1; ++levels; }
            if (levels > kStackDepth - 1) { err = "tree too deep for the traversal stack"; return IMLS_ERR_CAPACITY; }
            b.P = P;
            b.levels = levels;
            maxP = std::max(maxP, P);
            leaf_floats += ((size_t)P * 6 + 63) / 64 * 64;
            root_floats += 2 * (((size_t)P / kBlock + 1) * 6 + 63) / 64 * 64;
        }
    }
    int end_bit = 48;
    while ((1ll << (end_bit - 48)) < nj) ++end_bit;
    // double-buffered sort (round 6: the plain form copied keys and values back at its end)
    size_t cub_bytes = 0;
    {
        hipcub::DoubleBuffer<unsigned long long> kq(nullptr, nullptr);
        hipcub::DoubleBuffer<unsigned> vq(nullptr, nullptr);
        hipcub::DeviceRadixSort::SortPairs(nullptr, cub_bytes, kq, vq, (int)std::max<size_t>(total, 1), kMortonSortLo, end_bit, s);
    }
    const size_t need = 2 * ((total * 8 + 255) / 256 * 256) + 2 * ((total * 4 + 255) / 256 * 256) +
                        (cub_bytes + 255) / 256 * 256 + (size_t)nj * (kBBoxParts * 6 * 4 + 256) + (leaf_floats + root_floats) * 4 +
                        (size_t)nj * 4 * 256 + 4096;
    if (!ensure(scratch, need, err) || !ensure(table, (size_t)nj * sizeof(JobDev) + 256, err)) return IMLS_ERR_DEVICE;
    char* p = (char*)scratch.p;
    unsigned long long* k0 = carve<unsigned long long>(p, total);
    unsigned long long* k1 = carve<unsigned long long>(p, total);
    unsigned* v0 = carve<unsigned>(p, total);
    unsigned* v1 = carve<unsigned>(p, total);
    void* cub_tmp = carve<char>(p, cub_bytes);
    JobDev* J = (JobDev*)h_table;
    size_t off = 0;
    for (int q = 0; q < nj; ++q) {
        const BuildJob& b = jobs[q];
        JobDev d{};
        d.pts = b.pts;
        d.nrm = b.nrm;
        d.n = std::max(b.n, 0);
        d.off = (int)off;
        off += (size_t)d.n;
        d.bbpart = carve<float>(p, kBBoxParts * 6);
        if (b.B > 0 && b.n > 0) {
            d.B = b.B;
            d.L = (b.n + b.B - 1) / b.B;
            d.P = b.P;
            d.levels = b.levels;
            d.lkeys = b.lkeys;
            d.qp = (float*)(b.lkeys + d.L);          // the quantisation lives after the leaf keys
            d.mpt = b.mpt;
            d.mnr = b.mpt + b.n;
            d.ipos = (unsigned*)(b.mpt + 2 * (size_t)b.n);
            d.nodes = b.nodes;
            d.leafbox = carve<float>(p, (size_t)b.P * 6);
            float* ra = carve<float>(p, ((size_t)b.P / kBlock + 1) * 6);
            float* rb = carve<float>(p, ((size_t)b.P / kBlock + 1) * 6);
            // the rounds of the per-frame bottom-up reduction, precomputed
            const float* in = d.leafbox;
            float* outs[2] = {ra, rb};
            int count = b.P, D = b.levels, which = 0;
            for (int r = 0; r < kSubRounds; ++r) {
                d.sub_in[r] = in;
                d.sub_out[r] = outs[which];
                d.sub_count[r] = count;
                d.sub_D[r] = D;
                if (count <= 1) continue;
                const int width = std::min(count, kBlock);
                int lg = 0;
                while ((1 << lg) < width) ++lg;
                in = outs[which];
                which ^= 1;
                count /= width;
                D -= lg;
            }
            if (count > 1) { err = "tree too deep for the batched build"; return IMLS_ERR_CAPACITY; }
        } else {
            d.B = 0;
            d.qp = carve<float>(p, 4);
            d.perm = b.perm;
        }
        J[q] = d;
    }
    const JobDev* jd = (const JobDev*)table.p;
    hipMemcpyAsync(table.p, h_table, (size_t)nj * sizeof(JobDev), hipMemcpyHostToDevice, s);
    const unsigned gx = grid_for((size_t)maxn);
    k_bbox_b<<<dim3(std::min<unsigned>(kBBoxParts, gx), nj), kBlock, 0, s>>>(jd);
    k_qparams_b<<<nj, 64, 0, s>>>(jd);
    k_morton_b<<<dim3(gx, nj), kBlock, 0, s>>>(jd, k0, v0);
    hipcub::DoubleBuffer<unsigned long long> kb(k0, k1);
    hipcub::DoubleBuffer<unsigned> vb(v0, v1);
    if (total > 0) hipcub::DeviceRadixSort::SortPairs(cub_tmp, cub_bytes, kb, vb, (int)total, kMortonSortLo, end_bit, s);
    k_place_b<<<dim3(gx, nj), kBlock, 0, s>>>(jd, kb.Current(), vb.Current());
    bool any_tree = false;
    for (auto& b : jobs) any_tree |= b.B > 0 && b.n > 0;
    if (any_tree) {
        k_leaf_boxes_b<<<dim3(grid_for((size_t)maxP), nj), kBlock, 0, s>>>(jd);
        for (int r = 0, cnt = maxP; r < kSubRounds && cnt > 1; ++r) {
            const int width = std::min(cnt, kBlock);
            k_subtree_b<<<dim3(cnt / width, nj), kBlock, 0, s>>>(jd, r);
            cnt /= width;
        }
    }
    if (hipGetLastError() != hipSuccess) { err = "batched index build launch failed"; return IMLS_ERR_DEVICE; }
    return IMLS_OK;
}


// =============================================================================================
// Incremental index of the map FIFO (accumulateTargetCloud, laser_odometry.cpp:116-136: the last
// max_queue_size filtered scans, oldest first; setTargetPointCloud rebuilds libnabo's tree over
// their concatenation every frame, imls_icp.cpp:80-103).  With a quantisation frame fixed for the
// FIFO, a scan's Morton keys never change: each scan is sorted ONCE (a run, fifo_run_build), and a
// registration only merges — the previous merged order minus the evicted scans (a stable
// compaction), merged with the new runs (merge path, older entries first on equal keys).  That is
// exactly the stable sort of the concatenation by key, i.e. the order the full build gives under
// the same quantisation; the records then get their concatenated filtered index (the libnabo tie
// order, mpt[].w), ipos, the leaf keys and the tree (fifo_index).
// =============================================================================================
namespace {

constexpr int kMergeTile = 2048;            // outputs per merge block (12 B each in LDS)

// keys under the fixed quantisation fq; points outside its cube (clamped: still exact, the tree's
// boxes come from the points) are counted, so the host can re-frame the FIFO at its next build
__global__ void k_morton_fq(const float4* __restrict__ pt, int n, const float* __restrict__ fq,
                            unsigned long long* __restrict__ key, unsigned* __restrict__ val, unsigned* __restrict__ clamp) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    bool out = false;
    if (i < n) {
        const float4 p = pt[i];
        key[i] = morton48(p.x, p.y, p.z, fq);
        val[i] = (unsigned)i;
        const float sc = fq[3], qmax = 65535.f;
        const float u = (p.x - fq[0]) * sc, v = (p.y - fq[1]) * sc, w = (p.z - fq[2]) * sc;
        out = !(u >= 0.f && u <= qmax && v >= 0.f && v <= qmax && w >= 0.f && w <= qmax);
    }
    const unsigned long long m = __ballot(out);
    if ((threadIdx.x & 63) == 0 && m) atomicAdd(clamp, (unsigned)__popcll(m));
}

// a run's Morton-ordered records: rpt = (xyz, bits(local filtered index)), rnr, and its sorted keys
// (from wherever the double-buffered sort left them: no copy-back launches)
__global__ void k_run_gather(const float4* __restrict__ pt, const float4* __restrict__ nr, const unsigned* __restrict__ perm,
                             const unsigned long long* __restrict__ skey, int n, float4* __restrict__ rpt,
                             float4* __restrict__ rnr, unsigned long long* __restrict__ rkey) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    const unsigned j = perm[k];
    const float4 p = pt[j];
    rpt[k] = make_float4(p.x, p.y, p.z, __uint_as_float(j));
    rnr[k] = nr[j];
    rkey[k] = skey[k];
}

// the FIFO quantisation frame: a cube of side 2 × the runs' largest bbox extent, its origin half an
// extent below their bbox on every axis (later scans of a moving sensor stay inside; the host
// re-frames if one does not).  Side and offset are powers of two times the full build's cell
// (origin = bbox min, side = extent): the grid lines are the full build's, one level up, so the
// Morton order — and the tree — is the full build's up to the top-level block order and the last
// bit (on config B's map the query-ball overlaps of leaves / nodes are 8.03 / 74.1 per query vs the
// full build's 7.80 / 73.5; a 1.5× cube centred on the bbox gave 8.85 / 86.4:
// tools/fifo_frame_probe.py)
__global__ void k_fifo_frame(const float* __restrict__ part, int nparts, float* __restrict__ fq) {
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
    if (threadIdx.x == 0) {
        float ext = 1e-6f;
        for (int d = 0; d < 3; ++d) ext = fmaxf(ext, red[3 + d][0] - red[d][0]);
        const float side = 2.0f * ext;
        for (int d = 0; d < 3; ++d) fq[d] = red[d][0] - 0.5f * ext;
        fq[3] = 65535.f / side;
    }
}

// stable compaction of the merged order: entries whose run id (val >> 27) is live.  Two launches
// (round 6: count + scan + scatter and the scan's init were four): tiles of kKeepTile entries, 16 per
// thread in order; the scatter block sums the earlier tiles' counts itself (≤ a few hundred words)
// instead of a device-wide scan launch
__device__ __forceinline__ bool live_entry(unsigned v, unsigned live) { return (live >> (v >> 27)) & 1u; }
constexpr int kKeepPer = 16;
constexpr int kKeepTile = kBlock * kKeepPer;   // entries per block: kKeepPer rounds of kBlock, coalesced
__global__ __launch_bounds__(kBlock) void k_keep_count(const unsigned* __restrict__ val, int n, unsigned live, int* __restrict__ blk) {
    __shared__ int wc[kBlock / 64];
    const int base = blockIdx.x * kKeepTile + threadIdx.x;
    int c = 0;
#pragma unroll
    for (int k = 0; k < kKeepPer; ++k) {
        const int i = base + k * kBlock;
        c += (i < n && live_entry(val[i], live)) ? 1 : 0;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
    if ((threadIdx.x & 63) == 0) wc[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
        int t = 0;
        for (int k = 0; k < kBlock / 64; ++k) t += wc[k];
        blk[blockIdx.x] = t;
    }
}
__global__ __launch_bounds__(kBlock) void k_keep_scatter(const unsigned long long* __restrict__ key, const unsigned* __restrict__ val,
                                                         int n, unsigned live, const int* __restrict__ blk,
                                                         unsigned long long* __restrict__ okey, unsigned* __restrict__ oval) {
    __shared__ int wsum[kKeepPer][kBlock / 64];
    __shared__ int s_off;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    // this tile's output offset: Σ of the earlier tiles' counts
    int pre = 0;
    for (int b = tid; b < (int)blockIdx.x; b += kBlock) pre += blk[b];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) pre += __shfl_xor(pre, o, 64);
    if (lane == 0) wsum[0][wv] = pre;
    __syncthreads();
    if (tid == 0) {
        int t = 0;
        for (int k = 0; k < kBlock / 64; ++k) t += wsum[0][k];
        s_off = t;
    }
    __syncthreads();
    // every round's wave counts first (one barrier), then each entry's rank in tile order
    const int base = blockIdx.x * kKeepTile + tid;
    unsigned long long m[kKeepPer];
#pragma unroll
    for (int k = 0; k < kKeepPer; ++k) {
        const int i = base + k * kBlock;
        m[k] = __ballot(i < n && live_entry(val[i], live));
        if (lane == 0) wsum[k][wv] = __popcll(m[k]);
    }
    __syncthreads();
    int run = s_off;
#pragma unroll
    for (int k = 0; k < kKeepPer; ++k) {
        int before = 0, tot = 0;
#pragma unroll
        for (int w = 0; w < kBlock / 64; ++w) {
            before += w < wv ? wsum[k][w] : 0;
            tot += wsum[k][w];
        }
        if ((m[k] >> lane) & 1ull) {
            const int i = base + k * kBlock;
            const int o = run + before + __popcll(m[k] & ((1ull << lane) - 1ull));
            okey[o] = key[i];
            oval[o] = val[i];
        }
        run += tot;
    }
}

// merge path: the entries of A among the first d outputs of merge(A, B), A first on equal keys
// (A: the older entries)
__device__ __forceinline__ int merge_split_at(const unsigned long long* __restrict__ a, int na,
                                              const unsigned long long* __restrict__ b, int nb, long long d) {
    int lo = (int)std::max(0ll, d - nb), hi = (int)std::min<long long>(d, na);
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (a[mid] <= b[d - 1 - mid]) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}
// one output tile of kMergeTile: its two splits by binary search on the diagonals (threads 0 / 1;
// round 6: a separate split launch before), both input segments in LDS; then each thread finds its own
// diagonal split of the tile (one binary search in LDS) and merges its kMergePer consecutive outputs
// sequentially (round 6: one binary search per output before), A first on equal keys.  B's values
// are (bid << 27) | index (a run's entries in its sorted order)
constexpr int kMergePer = kMergeTile / kBlock;
__global__ __launch_bounds__(kBlock) void k_merge_tile(const unsigned long long* __restrict__ a, const unsigned* __restrict__ av,
                                                       int na, const unsigned long long* __restrict__ b, unsigned bid, int nb,
                                                       unsigned long long* __restrict__ okey, unsigned* __restrict__ oval) {
    __shared__ unsigned long long sk[kMergeTile];
    __shared__ unsigned sv[kMergeTile];
    __shared__ int ssplit[2];
    const int t = blockIdx.x;
    const long long d0 = (long long)t * kMergeTile, d1 = std::min(d0 + kMergeTile, (long long)na + nb);
    if (threadIdx.x < 2) ssplit[threadIdx.x] = merge_split_at(a, na, b, nb, threadIdx.x ? d1 : d0);
    __syncthreads();
    const int i0 = ssplit[0], i1 = ssplit[1];
    const int j0 = (int)(d0 - i0), j1 = (int)(d1 - i1);
    const int la = i1 - i0, lb = j1 - j0;
    for (int k = threadIdx.x; k < la; k += kBlock) { sk[k] = a[i0 + k]; sv[k] = av[i0 + k]; }
    for (int k = threadIdx.x; k < lb; k += kBlock) { sk[la + k] = b[j0 + k]; sv[la + k] = (bid << 27) | (unsigned)(j0 + k); }
    __syncthreads();
    // this thread's outputs [q, q + kMergePer) of the tile: x of A's entries before output q
    const int q = threadIdx.x * kMergePer, n = la + lb;
    if (q >= n) return;
    int lo = max(0, q - lb), hi = min(q, la);
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (sk[mid] <= sk[la + q - 1 - mid]) lo = mid + 1;
        else hi = mid;
    }
    int x = lo, y = q - lo;
    const int qe = min(q + kMergePer, n);
    for (int r = q; r < qe; ++r) {
        const bool takeA = y >= lb || (x < la && sk[x] <= sk[la + y]);
        const int src = takeA ? x : la + y;
        okey[d0 + r] = sk[src];
        oval[d0 + r] = sv[src];
        x += takeA ? 1 : 0;
        y += takeA ? 0 : 1;
    }
}

// the index records from the merged order: mpt (xyz, bits(concatenated filtered index)), mnr, ipos,
// every B-th key (the leaves' first keys, for the seed search) — and, fused in (round 6: four launches
// fewer — k_leaf_boxes, and three small copies), each leaf's box (a segmented min / max over the B
// lanes of its points: the same values as k_leaf_boxes' serial loop, min / max being exact), the
// padded leaves' empty boxes, the quantisation after the leaf keys (TreeView::qparams) and this
// build's clamp count into the host's coherent word.  The run table comes by value.
__global__ __launch_bounds__(kBlock) void k_fifo_gather(const unsigned long long* __restrict__ mkey,
                                                        const unsigned* __restrict__ mval, int M, FifoRunTable runs, int B,
                                                        int L, int P, const float* __restrict__ fq,
                                                        const unsigned* __restrict__ clamp, unsigned* __restrict__ h_clamp,
                                                        float4* __restrict__ mpt, float4* __restrict__ mnr,
                                                        unsigned* __restrict__ ipos, unsigned long long* __restrict__ lkeys,
                                                        float* __restrict__ leafbox) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    if (k < M) {
        const unsigned v = mval[k];
        const FifoRun r = runs.r[v >> 27];
        const unsigned pos = v & ((1u << 27) - 1u);
        const float4 p = r.rpt[pos];
        const unsigned w = r.off + __float_as_uint(p.w);
        mpt[k] = make_float4(p.x, p.y, p.z, __uint_as_float(w));
        mnr[k] = r.rnr[pos];
        ipos[w] = (unsigned)k;
        if (k % B == 0) lkeys[k / B] = mkey[k];
        lo[0] = hi[0] = p.x; lo[1] = hi[1] = p.y; lo[2] = hi[2] = p.z;
    }
    // leaf k / B = lanes [k − k % B, … + B) of this wave (B divides 64)
    for (int o = 1; o < B; o <<= 1) {
#pragma unroll
        for (int d = 0; d < 3; ++d) {
            lo[d] = fminf(lo[d], __shfl_xor(lo[d], o, 64));
            hi[d] = fmaxf(hi[d], __shfl_xor(hi[d], o, 64));
        }
    }
    if (k < M && k % B == 0) {
        float* q = leafbox + (size_t)(k / B) * 6;
        q[0] = lo[0]; q[1] = lo[1]; q[2] = lo[2]; q[3] = hi[0]; q[4] = hi[1]; q[5] = hi[2];
    }
    if (k < P - L) {                           // padded leaves L … P−1: empty boxes
        float* q = leafbox + (size_t)(L + k) * 6;
        q[0] = q[1] = q[2] = INFINITY;
        q[3] = q[4] = q[5] = -INFINITY;
    }
    if (k < 4) reinterpret_cast<float*>(lkeys + L)[k] = fq[k];
    if (k == 0) *h_clamp = *clamp;
}

}  // namespace

size_t fifo_scratch_bytes(int max_run, int nruns, int M) {
    size_t sort_b = 0, scan_b = 0;
    const int nb = (int)grid_for((size_t)std::max(M, 1));
    {
        hipcub::DoubleBuffer<unsigned long long> kq(nullptr, nullptr);
        hipcub::DoubleBuffer<unsigned> vq(nullptr, nullptr);
        hipcub::DeviceRadixSort::SortPairs(nullptr, sort_b, kq, vq, std::max(max_run, 1), 0, 48);
    }
    hipcub::DeviceScan::ExclusiveSum(nullptr, scan_b, (int*)nullptr, (int*)nullptr, nb);
    const size_t n = (size_t)std::max(max_run, 1);
    const size_t run = 2 * ((n * 8 + 255) / 256 * 256) + 2 * ((n * 4 + 255) / 256 * 256) + (sort_b + 255) / 256 * 256 + 1024;
    const size_t frame = (size_t)std::max(nruns, 1) * 64 * 24 + 1024;
    const size_t keep = 2 * (((size_t)nb * 4 + 255) / 256 * 256) + scan_b + 1024;
    const size_t merge = ((size_t)M / kMergeTile + 2) * 4 + 256;
    return std::max(std::max(run, frame), std::max(keep, merge));
}

int fifo_frame(hipStream_t s, const std::vector<std::pair<const float4*, int>>& runs, float* fq, DevBuf& scratch,
               std::string& err) {
    const int per = 64;                         // bbox partial blocks per run
    if (!ensure(scratch, runs.size() * per * 24 + 1024, err)) return IMLS_ERR_DEVICE;
    float* part = (float*)scratch.p;
    int np = 0;
    for (const auto& r : runs) {
        if (r.second <= 0) continue;
        const int nb = std::min(per, (int)grid_for(r.second));
        k_bbox_partial<<<nb, kBlock, 0, s>>>(r.first, r.second, part + (size_t)np * 6);
        np += nb;
    }
    if (np == 0) return IMLS_OK;
    k_fifo_frame<<<1, kBlock, 0, s>>>(part, np, fq);
    if (hipGetLastError() != hipSuccess) { err = "FIFO frame launch failed"; return IMLS_ERR_DEVICE; }
    return IMLS_OK;
}

int fifo_run_build(hipStream_t s, const float4* fpt, const float4* fnr, int n, const float* fq, unsigned* clamp,
                   DevBuf& run, DevBuf& scratch, std::string& err) {
    if (n <= 0) return IMLS_OK;
    if (n >= (1 << 27)) { err = "scan too large for the FIFO index"; return IMLS_ERR_CAPACITY; }
    // double-buffered sort (round 6: the plain form ended in two copy-back launches, ~14 µs with their
    // gaps on a 126k-point scan); k_run_gather takes the keys from the current buffer
    size_t cub_bytes = 0;
    {
        hipcub::DoubleBuffer<unsigned long long> kq(nullptr, nullptr);
        hipcub::DoubleBuffer<unsigned> vq(nullptr, nullptr);
        hipcub::DeviceRadixSort::SortPairs(nullptr, cub_bytes, kq, vq, n, 0, 48, s);
    }
    const size_t need = 2 * (((size_t)n * 8 + 255) / 256 * 256) + 2 * (((size_t)n * 4 + 255) / 256 * 256) +
                        ((cub_bytes + 255) / 256) * 256 + 1024;
    if (!ensure(scratch, need, err) || !ensure(run, fifo_run_bytes(n), err)) return IMLS_ERR_DEVICE;
    char* p = (char*)scratch.p;
    unsigned long long* k0 = carve<unsigned long long>(p, n);
    unsigned long long* k1 = carve<unsigned long long>(p, n);
    unsigned* v0 = carve<unsigned>(p, n);
    unsigned* v1 = carve<unsigned>(p, n);
    void* cub_tmp = carve<char>(p, cub_bytes);
    k_morton_fq<<<grid_for(n), kBlock, 0, s>>>(fpt, n, fq, k0, v0, clamp);
    unsigned long long* kcur;
    unsigned* vcur;
    if (n <= kSortSmallMax) {
        const int r = small_sort_pairs(s, k0, v0, k1, v1, n);
        kcur = r ? k1 : k0;
        vcur = r ? v1 : v0;
    } else {
        hipcub::DoubleBuffer<unsigned long long> kb(k0, k1);
        hipcub::DoubleBuffer<unsigned> vb(v0, v1);
        hipcub::DeviceRadixSort::SortPairs(cub_tmp, cub_bytes, kb, vb, n, 0, 48, s);
        kcur = kb.Current();
        vcur = vb.Current();
    }
    k_run_gather<<<grid_for(n), kBlock, 0, s>>>(fpt, fnr, vcur, kcur, n, fifo_run_pts(run.p, n),
                                                fifo_run_nrm(run.p, n), fifo_run_keys(run.p, n));
    if (hipGetLastError() != hipSuccess) { err = "FIFO run build launch failed"; return IMLS_ERR_DEVICE; }
    return IMLS_OK;
}

int fifo_keep(hipStream_t s, const unsigned long long* key, const unsigned* val, int n, unsigned live,
              unsigned long long* okey, unsigned* oval, DevBuf& scratch, std::string& err) {
    if (n <= 0) return IMLS_OK;
    const int nb = (n + kKeepTile - 1) / kKeepTile;
    if (!ensure(scratch, ((size_t)nb * 4 + 255) / 256 * 256 + 1024, err)) return IMLS_ERR_DEVICE;
    int* blk = (int*)scratch.p;
    k_keep_count<<<nb, kBlock, 0, s>>>(val, n, live, blk);
    k_keep_scatter<<<nb, kBlock, 0, s>>>(key, val, n, live, blk, okey, oval);
    if (hipGetLastError() != hipSuccess) { err = "FIFO compaction launch failed"; return IMLS_ERR_DEVICE; }
    return IMLS_OK;
}

int fifo_merge(hipStream_t s, const unsigned long long* a, const unsigned* av, int na, const unsigned long long* b,
               unsigned bid, int nb, unsigned long long* okey, unsigned* oval, DevBuf& scratch, std::string& err) {
    (void)scratch;
    (void)err;
    const int tiles = (int)(((long long)na + nb + kMergeTile - 1) / kMergeTile);
    if (tiles == 0) return IMLS_OK;
    k_merge_tile<<<tiles, kBlock, 0, s>>>(a, av, na, b, bid, nb, okey, oval);
    if (hipGetLastError() != hipSuccess) { err = "FIFO merge launch failed"; return IMLS_ERR_DEVICE; }
    return IMLS_OK;
}

int fifo_index(hipStream_t s, const unsigned long long* mkey, const unsigned* mval, int M, const FifoRunTable& runs,
               const float* fq, const unsigned* clamp, unsigned* h_clamp, int B, DevBuf& lkeys, DevBuf& mpt, DevBuf& nodes,
               DevBuf& treescratch, int* P_out, int* levels_out, std::string& err) {
    if (M <= 0) { *P_out = 0; *levels_out = 0; return IMLS_OK; }
    const int L = (M + B - 1) / B;
    int P = 1, levels = 0;
    while (P < L) { P <<= 1; ++levels; }
    if (levels > kStackDepth - 1) { err = "tree too deep for the traversal stack"; return IMLS_ERR_CAPACITY; }
    const size_t need = ((size_t)P * 24 + 255) / 256 * 256 + 2 * (((size_t)P / kBlock + 1) * 24 + 256) + 1024;
    if (!ensure(treescratch, need, err) || !ensure(mpt, (size_t)M * 36 + 64, err) || !ensure(nodes, (size_t)(P + 1) * 48, err) ||
        !ensure(lkeys, (size_t)L * 8 + 16, err))
        return IMLS_ERR_DEVICE;
    char* p = (char*)treescratch.p;
    float* leafbox = carve<float>(p, (size_t)P * 6);
    float* rootsA = carve<float>(p, ((size_t)P / kBlock + 1) * 6);
    float* rootsB = carve<float>(p, ((size_t)P / kBlock + 1) * 6);
    float4* mp = (float4*)mpt.p;
    k_fifo_gather<<<grid_for(M), kBlock, 0, s>>>(mkey, mval, M, runs, B, L, P, fq, clamp, h_clamp, mp, mp + M,
                                                 (unsigned*)(mp + 2 * (size_t)M), (unsigned long long*)lkeys.p, leafbox);
    subtree_rounds(s, leafbox, P, levels, (float4*)nodes.p, rootsA, rootsB);
    if (hipGetLastError() != hipSuccess) { err = "FIFO index launch failed"; return IMLS_ERR_DEVICE; }
    *P_out = P;
    *levels_out = levels;
    return IMLS_OK;
}

}  // namespace imlsgpu
