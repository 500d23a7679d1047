// bqp_plant.hip — the true plant of the reference's closed loops, stepped on the GPU between
// batched solves (bqp_closed_loop_ocp_device).
//
// Moore-Greitzer compressor (examples/DMS_tracking_LMPC_casadi.m:215-221, `system`; the same
// model as models/trueModel.m:32-41) integrated by one classical RK4 step of length delta
// (`dynamic`, :297-304).  One thread per instance: the plant is 4 states, the solve dominates.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "bqp_internal.h"

namespace bqp {

__device__ __forceinline__ void mg_system(const double (&x)[4], double u, double (&f)[4]) {
    f[0] = -x[1] + 1.0 + 3.0 * (x[0] / 2.0) - (x[0] * x[0] * x[0] / 2.0);   // mass flow rate
    f[1] = (x[0] + 1.0 - x[2] * sqrt(x[1]));                              // pressure rise rate
    f[2] = x[3];                                                          // throttle opening rate
    f[3] = -1000.0 * x[2] - 2.0 * sqrt(500.0) * x[3] + 1000.0 * u;        // throttle acceleration
}

__device__ __forceinline__ void mg_rk4(double delta, double (&x)[4], double u) {
    double k1[4], k2[4], k3[4], k4[4], y[4];
    mg_system(x, u, k1);
#pragma unroll
    for (int i = 0; i < 4; ++i) y[i] = x[i] + delta / 2.0 * k1[i];
    mg_system(y, u, k2);
#pragma unroll
    for (int i = 0; i < 4; ++i) y[i] = x[i] + delta / 2.0 * k2[i];
    mg_system(y, u, k3);
#pragma unroll
    for (int i = 0; i < 4; ++i) y[i] = x[i] + delta * k3[i];
    mg_system(y, u, k4);
#pragma unroll
    for (int i = 0; i < 4; ++i) x[i] = x[i] + delta / 6.0 * (k1[i] + 2.0 * k2[i] + 2.0 * k3[i] + k4[i]);
}

// s (deviation state fed to the solver) = x_init - x_eq; X[:, 0] = x_init
__global__ void closed_loop_init_kernel(int batch, int nx, int steps, const double* xinit,
                                        const double* xeq, double* s, double* X) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= batch) return;
    for (int i = 0; i < nx; ++i) {
        const double v = xinit[(int64_t)b * nx + i];
        s[(int64_t)b * nx + i] = v - xeq[i];
        X[(int64_t)b * (steps + 1) * nx + i] = v;
    }
}

// apply u_0 of the step-t solve to the plant: u = u_eq + du_0, x+ = RK4(x, u)
__global__ void mg_plant_kernel(int batch, int N, int steps, int t, double delta,
                                const double* uo, const int* fl, const double* xeq,
                                const double* ueq, double* s, double* X, double* U, int* flags) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= batch) return;
    double x[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) x[i] = s[(int64_t)b * 4 + i] + xeq[i];
    const double u = uo[(int64_t)b * N] + ueq[0];
    mg_rk4(delta, x, u);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        s[(int64_t)b * 4 + i] = x[i] - xeq[i];
        X[((int64_t)b * (steps + 1) + t + 1) * 4 + i] = x[i];
    }
    U[(int64_t)b * steps + t] = u;
    if (flags) flags[(int64_t)b * steps + t] = fl[b];
}

hipError_t launch_closed_loop_init(int batch, int nx, int steps, const double* xinit,
                                   const double* xeq, double* s, double* X, hipStream_t st) {
    hipLaunchKernelGGL(closed_loop_init_kernel, dim3((batch + 255) / 256), dim3(256), 0, st, batch,
                       nx, steps, xinit, xeq, s, X);
    return hipGetLastError();
}

hipError_t launch_mg_plant(int batch, int N, int steps, int t, double delta, const double* uo,
                           const int* fl, const double* xeq, const double* ueq, double* s,
                           double* X, double* U, int* flags, hipStream_t st) {
    hipLaunchKernelGGL(mg_plant_kernel, dim3((batch + 255) / 256), dim3(256), 0, st, batch, N,
                       steps, t, delta, uo, fl, xeq, ueq, s, X, U, flags);
    return hipGetLastError();
}

}  // namespace bqp
