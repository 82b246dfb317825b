// front.hip — the upstream producer's front end on gfx950 (scan_registration.cpp:laserCloudHandler):
// NaN filter (pcl::removeNaNFromPointCloud, 862: a cloud flagged is_dense is copied unchanged), the
// range filter removeClosedPointCloud (87-115, 863), and the scan-ring assignment with the
// per-point relative time (898-1058): ring id from the vertical angle (16 / 32 / 64 lines),
// azimuth unwrapped against the first and last points with the sequential `halfPassed` switch,
// intensity = ring + scanPeriod·relTime, then laserCloud = the rings concatenated in ring order,
// each in input order (1064-1069).
//
// The sequential loop becomes four streaming passes over the sweep (one thread per point):
//   k_front_valid  the two filters; first / last surviving point (startOri / endOri);
//   k_front_ring   ring id, the azimuth as the !halfPassed branch adjusts it, and the switch test —
//                  halfPassed flips at the FIRST ring-valid point whose adjusted azimuth passes
//                  startOri + π (an atomicMin), so every point up to it takes that branch and every
//                  later one the halfPassed branch: the sequential state machine, exactly;
//   k_front_emit   the branch's azimuth, relTime, intensity, (x, y, z, intensity) records, ring keys;
//   hipcub radix sort by ring (stable: input order kept within a ring) → k_front_gather.
// Arithmetic follows the reference's mixed float / double evaluation (float sums and products,
// comparisons and the ±2π steps against M_PI in double, x86 float→int truncation with INT_MIN for
// NaN / out of range); atan, atan2 and sqrt are correctly rounded float values taken through fp64
// (glibc's atanf / atan2f are within an ulp of them: see DESIGN §3).
// Roofline: HBM streaming, ~60 B per input point over the passes; latency-bound at one sweep.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <climits>
#include <string>
#include <vector>

#include "internal.h"

namespace imlsgpu {
namespace {

constexpr int kFrontBlock = 256;
constexpr unsigned kNoRing = 127u;      // sort key of a point without a ring (sorted last, not emitted)
constexpr double kPi = 3.14159265358979323846;

// static_cast<int>(double) as x86-64 evaluates it (cvttsd2si): truncation, INT_MIN ("integer
// indefinite") for NaN and out-of-range values
__device__ __forceinline__ int x86_d2i(double v) {
    if (!(v > -2147483649.0 && v < 2147483648.0)) return INT_MIN;
    return (int)v;
}
__device__ __forceinline__ float atanf_cr(float t) { return (float)atan((double)t); }
__device__ __forceinline__ float atan2f_cr(float y, float x) { return (float)atan2((double)y, (double)x); }
__device__ __forceinline__ float sqrtf_cr(float s) { return (float)sqrt((double)s); }

// scan_registration.cpp:963-967 (VLP-32C table; the HDL-32 one is commented out there)
__constant__ float kVlp32Angles[27] = {-25.000f, -15.639f, -11.310f, -8.843f, -7.254f, -6.148f, -5.333f,
                                       -4.667f,  -4.000f,  -3.667f,  -3.333f, -3.000f, -2.667f, -2.333f,
                                       -2.000f,  -1.667f,  -1.333f,  -1.000f, -0.667f, -0.333f, 0.000f,
                                       0.333f,   0.667f,   1.000f,   1.333f,  1.667f,  2.333f};

// The ring of a point (scan_registration.cpp:940-1011), or −1 when the reference drops it.
__device__ int ring_of(float x, float y, float z, int n_scans) {
    const float range = sqrtf_cr(x * x + y * y);                       // 942
    const float vertical_angle = atanf_cr(z / range);                  // 943
    const float angle = (float)((double)(vertical_angle * 180.0f) / kPi);   // 944: float·int, then / M_PI in double
    if (n_scans == 16) {
        const int s = x86_d2i((double)((angle + 15.0f) / 2.0f) + 0.5);     // 950
        return (s > n_scans - 1 || s < 0) ? -1 : s;
    }
    if (n_scans == 32) {
        float min_diff = 3.402823466e+38f;                             // numeric_limits<float>::max()
        int s = 0;
        for (int j = 0; j < 27; ++j) {                                 // 976-984: first minimum
            const float diff = fabsf(angle - kVlp32Angles[j]);
            if (diff < min_diff) { min_diff = diff; s = j; }
        }
        return (s > n_scans - 1 || s < 0) ? -1 : s;
    }
    // 64 (992-1003): upperBound 2, lowerBound −24.33 (927-928)
    const float upper = 2.0f, lower = -24.33f;
    int s;
    if ((double)angle >= -8.83) s = x86_d2i((double)(upper - angle) * 3.0 + 0.5);
    else s = (int)((unsigned)(n_scans / 2) + (unsigned)x86_d2i((-8.83 - (double)angle) * 2.0 + 0.5));   // x86 wrap
    if (angle > upper || angle < lower || s > 50 || s < 0) return -1;
    return s;
}

// Input: xyz SoA [3][n]; ok[i]: survives both filters; ints[0] = first, ints[1] = last survivor.
__global__ __launch_bounds__(kFrontBlock) void k_front_valid(const float* __restrict__ xyz, int n, int is_dense,
                                                            float minr, float maxr, unsigned char* __restrict__ ok,
                                                            int* __restrict__ ints) {
    const int i = blockIdx.x * kFrontBlock + threadIdx.x;
    if (i >= n) return;
    const float x = xyz[i], y = xyz[n + i], z = xyz[2 * (size_t)n + i];
    bool v = is_dense || (isfinite(x) && isfinite(y) && isfinite(z));       // removeNaNFromPointCloud
    const float r2 = x * x + y * y + z * z;                                   // ((x² + y²) + z²), float
    if (r2 < minr * minr || r2 > maxr * maxr) v = false;                      // 101-103 (NaN passes)
    ok[i] = v ? 1 : 0;
    if (v) {
        atomicMin(&ints[0], i);
        atomicMax(&ints[1], i);
    }
}

struct Oris {
    float start, end;
};
__device__ __forceinline__ Oris start_end(const float* xyz, int n, const int* ints) {
    const int f = ints[0], l = ints[1];
    Oris o;
    o.start = -atan2f_cr(xyz[n + f], xyz[f]);                                           // 900
    o.end = (float)((double)(-atan2f_cr(xyz[n + l], xyz[l])) + 2 * kPi);               // 901-903
    if ((double)(o.end - o.start) > 3 * kPi) o.end = (float)((double)o.end - 2 * kPi);        // 905-908
    else if ((double)(o.end - o.start) < kPi) o.end = (float)((double)o.end + 2 * kPi);      // 909-912
    return o;
}

// ring id (−1: dropped), the !halfPassed azimuth, and the halfPassed switch point (ints[2]).
__global__ __launch_bounds__(kFrontBlock) void k_front_ring(const float* __restrict__ xyz, int n, int n_scans,
                                                           const unsigned char* __restrict__ ok, int* __restrict__ ints,
                                                           int* __restrict__ ring, float* __restrict__ ori_a) {
    const int i = blockIdx.x * kFrontBlock + threadIdx.x;
    if (i >= n) return;
    int r = -1;
    if (ok[i]) {
        const float x = xyz[i], y = xyz[n + i], z = xyz[2 * (size_t)n + i];
        r = ring_of(x, y, z, n_scans);
        if (r >= 0) {
            const Oris so = start_end(xyz, n, ints);
            float ori = -atan2f_cr(y, x);                                                  // 1017
            if ((double)ori < (double)so.start - kPi / 2) ori = (float)((double)ori + 2 * kPi);          // 1020-1023
            else if ((double)ori > (double)so.start + kPi * 3 / 2) ori = (float)((double)ori - 2 * kPi); // 1024-1027
            ori_a[i] = ori;
            if ((double)(ori - so.start) > kPi) atomicMin(&ints[2], i);                    // 1029-1032
        }
    }
    ring[i] = r;
}

// The point's azimuth under its branch, relTime, intensity; its record and ring key; ring counts.
__global__ __launch_bounds__(kFrontBlock) void k_front_emit(const float* __restrict__ xyz, int n, float scan_period,
                                                           const int* __restrict__ ints, const int* __restrict__ ring,
                                                           const float* __restrict__ ori_a, float4* __restrict__ rec,
                                                           unsigned* __restrict__ key, unsigned* __restrict__ val,
                                                           int* __restrict__ counts) {
    __shared__ int cnt[64];
    if (threadIdx.x < 64) cnt[threadIdx.x] = 0;
    __syncthreads();
    const int i = blockIdx.x * kFrontBlock + threadIdx.x;
    if (i < n) {
        const int r = ring[i];
        unsigned k = kNoRing;
        if (r >= 0) {
            const Oris so = start_end(xyz, n, ints);
            const float x = xyz[i], y = xyz[n + i], z = xyz[2 * (size_t)n + i];
            float ori;
            if (i <= ints[2]) {
                ori = ori_a[i];                                           // !halfPassed branch (incl. the switch point)
            } else {
                ori = (float)((double)(-atan2f_cr(y, x)) + 2 * kPi);      // 1036
                if ((double)ori < (double)so.end - kPi * 3 / 2) ori = (float)((double)ori + 2 * kPi);       // 1037-1040
                else if ((double)ori > (double)so.end + kPi / 2) ori = (float)((double)ori - 2 * kPi);      // 1041-1044
            }
            const float rel = (ori - so.start) / (so.end - so.start);    // 1047
            rec[i] = make_float4(x, y, z, (float)r + scan_period * rel);  // 1048
            k = (unsigned)r;
            atomicAdd(&cnt[r], 1);
        }
        key[i] = k;
        val[i] = (unsigned)i;
    }
    __syncthreads();
    if (threadIdx.x < 64 && cnt[threadIdx.x]) atomicAdd(&counts[threadIdx.x], cnt[threadIdx.x]);
}

__global__ __launch_bounds__(kFrontBlock) void k_front_gather(const float4* __restrict__ rec, const unsigned* __restrict__ perm,
                                                             int m, float4* __restrict__ out, unsigned* __restrict__ index) {
    const int k = blockIdx.x * kFrontBlock + threadIdx.x;
    if (k >= m) return;
    const unsigned i = perm[k];
    out[k] = rec[i];
    index[k] = i;
}

__global__ void k_front_init(int* ints, int n) {
    const int t = threadIdx.x;
    if (t == 0) { ints[0] = INT_MAX; ints[1] = -1; ints[2] = INT_MAX; }
    if (t < 64) ints[8 + t] = 0;
    (void)n;
}

template <typename T>
T* carve(char*& p, size_t n) {
    T* r = reinterpret_cast<T*>(p);
    p += ((n * sizeof(T) + 255) / 256) * 256;
    return r;
}

}  // namespace

int front_end_run(hipStream_t s, const imls_front_params& p, const float* xyz_host, size_t stride, size_t n_in,
                  DevBuf& mem, float* out_xyzi, uint32_t* out_index, int32_t* ring_sizes, size_t* n_out,
                  std::string& err) {
    *n_out = 0;
    if (p.n_scans != 16 && p.n_scans != 32 && p.n_scans != 64) { err = "scan_line must be 16, 32 or 64"; return IMLS_ERR_ARG; }
    for (int r = 0; r < p.n_scans; ++r) ring_sizes[r] = 0;
    if (n_in == 0) return IMLS_OK;
    if (n_in > (size_t)0x3fffffff || stride < 3) { err = "bad sweep size / stride"; return IMLS_ERR_ARG; }
    const int n = (int)n_in;
    size_t cub_bytes = 0;
    hipcub::DeviceRadixSort::SortPairs(nullptr, cub_bytes, (unsigned*)nullptr, (unsigned*)nullptr, (unsigned*)nullptr,
                                       (unsigned*)nullptr, n, 0, 7, s);
    const size_t nn = (size_t)n;
    const size_t need = 3 * nn * 4 + nn + nn * 4 + nn * 4 + 2 * nn * 16 + 4 * nn * 4 + nn * 4 + cub_bytes + 128 * 4 + 16 * 256;
    if (!devbuf_grow(mem, need, need + need / 4)) { err = "hipMalloc (front end)"; return IMLS_ERR_DEVICE; }
    char* q = (char*)mem.p;
    float* xyz = carve<float>(q, 3 * nn);
    unsigned char* ok = carve<unsigned char>(q, nn);
    int* ring = carve<int>(q, nn);
    float* ori_a = carve<float>(q, nn);
    float4* rec = carve<float4>(q, nn);
    float4* out = carve<float4>(q, nn);
    unsigned* key = carve<unsigned>(q, nn);
    unsigned* val = carve<unsigned>(q, nn);
    unsigned* key2 = carve<unsigned>(q, nn);
    unsigned* val2 = carve<unsigned>(q, nn);
    unsigned* idx = carve<unsigned>(q, nn);
    int* ints = carve<int>(q, 128);
    void* cub_tmp = carve<char>(q, cub_bytes);
    // the sweep as SoA xyz (host pack: the reference's PointXYZ message records, any stride)
    std::vector<float> h(3 * nn);
    for (size_t i = 0; i < nn; ++i) {
        const float* r = xyz_host + i * stride;
        h[i] = r[0]; h[nn + i] = r[1]; h[2 * nn + i] = r[2];
    }
    const unsigned g = (unsigned)((n + kFrontBlock - 1) / kFrontBlock);
    hipMemcpyAsync(xyz, h.data(), 3 * nn * 4, hipMemcpyHostToDevice, s);
    k_front_init<<<1, 64, 0, s>>>(ints, n);
    k_front_valid<<<g, kFrontBlock, 0, s>>>(xyz, n, p.is_dense, p.minimum_range, p.maximum_range, ok, ints);
    k_front_ring<<<g, kFrontBlock, 0, s>>>(xyz, n, p.n_scans, ok, ints, ring, ori_a);
    k_front_emit<<<g, kFrontBlock, 0, s>>>(xyz, n, p.scan_period, ints, ring, ori_a, rec, key, val, ints + 8);
    hipcub::DeviceRadixSort::SortPairs(cub_tmp, cub_bytes, key, key2, val, val2, n, 0, 7, s);
    int hc[64 + 8];
    hipMemcpyAsync(hc, ints, (8 + 64) * 4, hipMemcpyDeviceToHost, s);
    if (hipStreamSynchronize(s) != hipSuccess) { err = "front end failed"; return IMLS_ERR_DEVICE; }
    if (hc[1] < 0) return IMLS_OK;                  // nothing survives the filters (the reference indexes an empty cloud)
    size_t m = 0;
    for (int r = 0; r < p.n_scans; ++r) { ring_sizes[r] = hc[8 + r]; m += (size_t)hc[8 + r]; }
    if (m > 0) {
        k_front_gather<<<(unsigned)((m + kFrontBlock - 1) / kFrontBlock), kFrontBlock, 0, s>>>(rec, val2, (int)m, out, idx);
        hipMemcpyAsync(out_xyzi, out, m * 16, hipMemcpyDeviceToHost, s);
        if (out_index) hipMemcpyAsync(out_index, idx, m * 4, hipMemcpyDeviceToHost, s);
        if (hipStreamSynchronize(s) != hipSuccess) { err = "front end failed"; return IMLS_ERR_DEVICE; }
    }
    *n_out = m;
    return IMLS_OK;
}

}  // namespace imlsgpu
