// geom.h — device geometry shared by the matching kernels (project.hip, tv.hip): the fp32 box
// distance used for pruning, the exact libnabo metric and the per-iteration source transform.
#pragma once
#include "internal.h"

namespace imlsgpu {
namespace {

__device__ __forceinline__ float box_d2(const float q[3], float lx, float ly, float lz, float hx, float hy, float hz) {
    const float vx = fmaxf(fmaxf(lx - q[0], q[0] - hx), 0.f);
    const float vy = fmaxf(fmaxf(ly - q[1], q[1] - hy), 0.f);
    const float vz = fmaxf(fmaxf(lz - q[2], q[2] - hz), 0.f);
    return __builtin_fmaf(vx, vx, __builtin_fmaf(vy, vy, vz * vz));
}

// exact libnabo metric on float storage
__device__ __forceinline__ double exact_d2(const double xd[3], float px, float py, float pz) {
    const double dx = xd[0] - (double)px, dy = xd[1] - (double)py, dz = xd[2] - (double)pz;
    double d2 = dx * dx;
    d2 = d2 + dy * dy;
    d2 = d2 + dz * dz;
    return d2;
}

// x = float(rPose·[p;1]) and the (optionally rotated) source normal (laser_odometry.cpp:527-549)
__device__ __forceinline__ void transform_query(const double* __restrict__ pose, float4 p, float4 nsv, int rot_normal,
                                                float xf[3], double ns[3]) {
    // the pose through the constant address space: one set of scalar loads for the wave (a pointer
    // read from the batched kernels' frame table is generic, and was loaded per lane, 96 B each)
    typedef __attribute__((address_space(4))) const double kconst_d;
    const kconst_d* cp = (const kconst_d*)pose;
    double T[12];
#pragma unroll
    for (int k = 0; k < 12; ++k) T[k] = cp[k];
    const double pd[3] = {p.x, p.y, p.z};
#pragma unroll
    for (int r = 0; r < 3; ++r) {
        double v = T[r * 4 + 0] * pd[0];
        v = v + T[r * 4 + 1] * pd[1];
        v = v + T[r * 4 + 2] * pd[2];
        v = v + T[r * 4 + 3] * 1.0;
        xf[r] = (float)v;
    }
    if (rot_normal) {
        const double nd[3] = {nsv.x, nsv.y, nsv.z};
#pragma unroll
        for (int r = 0; r < 3; ++r) {
            double v = T[r * 4 + 0] * nd[0];
            v = v + T[r * 4 + 1] * nd[1];
            v = v + T[r * 4 + 2] * nd[2];
            ns[r] = (double)(float)v;
        }
    } else {
        ns[0] = nsv.x; ns[1] = nsv.y; ns[2] = nsv.z;
    }
}

}  // namespace
}  // namespace imlsgpu
