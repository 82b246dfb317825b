// micro-benchmark: single-thread latency of the 6x6 solve and delta_from_x (solve_common.h)
#include <cstdio>
#include "../../planetary-lidar-odometry_amd/csrc/solve_common.h"
using namespace imlsgpu;
__global__ void k(const double* ne, double* out, long long* t) {
    double x[6], D[16];
    long long t0 = wall_clock64();
    solve6(ne, x);
    long long t1 = wall_clock64();
    delta_from_x(x, D);
    long long t2 = wall_clock64();
    for (int i = 0; i < 6; ++i) out[i] = x[i];
    for (int i = 0; i < 16; ++i) out[6 + i] = D[i];
    t[0] = t1 - t0; t[1] = t2 - t1;
}
int main() {
    double h[28];
    // a well-conditioned SPD system: J^T J of a few random rows
    double A[6][6] = {}, g[6] = {};
    unsigned s = 1;
    for (int r = 0; r < 50; ++r) {
        double a[6]; for (int k = 0; k < 6; ++k) { s = s * 1103515245 + 12345; a[k] = (s >> 16) / 65536.0 - 0.5; }
        for (int i = 0; i < 6; ++i) { for (int j = 0; j < 6; ++j) A[i][j] += a[i] * a[j]; g[i] += a[i] * 0.01; }
    }
    int q = 0; for (int i = 0; i < 6; ++i) for (int j = i; j < 6; ++j) h[q++] = A[i][j];
    for (int i = 0; i < 6; ++i) h[21 + i] = g[i];
    h[27] = 50;
    double *dne, *dout; long long* dt;
    hipMalloc(&dne, 28 * 8); hipMalloc(&dout, 32 * 8); hipMalloc(&dt, 16);
    hipMemcpy(dne, h, 28 * 8, hipMemcpyHostToDevice);
    for (int rep = 0; rep < 3; ++rep) {
        hipLaunchKernelGGL(k, 1, 1, 0, 0, dne, dout, dt);
        long long t[2]; hipMemcpy(t, dt, 16, hipMemcpyDeviceToHost);
        printf("solve6 %.2f us  delta_from_x %.2f us (100 MHz ticks %lld %lld)\n", t[0] / 100.0, t[1] / 100.0, t[0], t[1]);
    }
    return 0;
}
