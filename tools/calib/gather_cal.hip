// gather_cal.hip — calibrates rocprofv3's FETCH_SIZE for the access patterns of the projection
// kernels (16-B gathers of float4 map records), on gfx950.  MI355X_MICROARCH.md §HBM: FETCH_SIZE
// reports ½ of the bytes of a wide coalesced streaming read; other widths are uncalibrated.  Each
// kernel below reads a KNOWN number of bytes with one pattern, so FETCH_SIZE ÷ known bytes is that
// pattern's factor:
//   stream   : coalesced float4 sweep (16 B per lane, consecutive lanes consecutive rows) — the guide's
//              reference case (expect ½)
//   rand16   : one float4 row per lane per step at a uniformly random row — the k_finish gather of a
//              list point whose line is not shared with the wave's other lanes
//   pair_s   : two rows per step in one 32-B sector (rows r, r^1): a pair that shares a sector
//   pair_h   : rows r and r^4: one 128-B line, different 64-B halves — separates 64-B from 128-B fetch
//              granularity
//   pair_l   : rows r and r^8: two different 128-B lines
// on two tables: 512 MiB (beyond the 256-MiB Infinity Cache: misses go to HBM) and 40 MB (the size of
// config B's Morton map: resident in the Infinity Cache, so FETCH_SIZE counts fabric requests that the
// Infinity Cache serves).  Every lane writes one float4 (WRITE_SIZE exact for 16-B stores).
// Row indices come from a per-lane hash (no index array traffic).  Prints one line per launch:
//   pattern table_bytes rows_read known_read_bytes known_write_bytes ms
// Run under rocprofv3 --pmc FETCH_SIZE (and WRITE_SIZE in a separate pass) with --kernel-trace.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

namespace {
constexpr int kThreads = 256;
constexpr int kSteps = 32;                 // gathers (pairs) per lane

__device__ __forceinline__ unsigned hash32(unsigned x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x;
}

// mode 0 stream, 1 rand16, 2 pair_s (r^1), 3 pair_h (r^4), 4 pair_l (r^8)
__global__ __launch_bounds__(kThreads) void k_gather(const float4* __restrict__ tab, unsigned rows, int mode,
                                                     float4* __restrict__ out, unsigned seed) {
    const unsigned gid = blockIdx.x * kThreads + threadIdx.x;
    const unsigned nthreads = gridDim.x * kThreads;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    unsigned h = hash32(gid * 2654435761u + seed);
#pragma unroll 4
    for (int k = 0; k < kSteps; ++k) {
        if (mode == 0) {
            const float4 v = tab[(gid + (unsigned)k * nthreads) % rows];
            acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
        } else {
            h = hash32(h + (unsigned)k);
            const unsigned r = h % rows;
            const float4 v = tab[r];
            acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
            if (mode >= 2) {
                const unsigned x = mode == 2 ? 1u : (mode == 3 ? 4u : 8u);
                const float4 u = tab[(r ^ x) % rows];
                acc.x += u.x; acc.y += u.y; acc.z += u.z; acc.w += u.w;
            }
        }
    }
    out[gid] = acc;
}

__global__ void k_fill(float4* __restrict__ tab, size_t rows) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < rows; i += (size_t)gridDim.x * blockDim.x)
        tab[i] = make_float4((float)(i & 1023), 1.f, 2.f, 3.f);
}
}  // namespace

int main() {
    const size_t big = (size_t)512 << 20, small = (size_t)40 << 20;
    float4* tab = nullptr;
    float4* out = nullptr;
    const int blocks = 2048;                 // 8 blocks per CU: 524,288 lanes
    const size_t lanes = (size_t)blocks * kThreads;
    if (hipMalloc(&tab, big) != hipSuccess || hipMalloc(&out, lanes * 16) != hipSuccess) {
        std::fprintf(stderr, "hipMalloc failed\n");
        return 1;
    }
    k_fill<<<4096, 256>>>(tab, big / 16);
    (void)hipDeviceSynchronize();
    const char* names[5] = {"stream", "rand16", "pair_s", "pair_h", "pair_l"};
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    for (size_t tb : {big, small}) {
        const unsigned rows = (unsigned)(tb / 16);
        for (int mode = 0; mode < 5; ++mode) {
            for (int rep = 0; rep < 3; ++rep) {
                (void)hipEventRecord(a);
                k_gather<<<blocks, kThreads>>>(tab, rows, mode, out, 17u * (unsigned)rep + 1u);
                (void)hipEventRecord(b);
                (void)hipEventSynchronize(b);
                float ms = 0.f;
                (void)hipEventElapsedTime(&ms, a, b);
                const double per = mode >= 2 ? 2.0 : 1.0;
                const double nrows = (double)lanes * kSteps * per;
                std::printf("%s %zu %.0f %.0f %.0f %.4f\n", names[mode], tb, nrows, nrows * 16.0, (double)lanes * 16.0, ms);
            }
        }
    }
    if (hipGetLastError() != hipSuccess) { std::fprintf(stderr, "launch failed\n"); return 1; }
    (void)hipFree(tab);
    (void)hipFree(out);
    return 0;
}
