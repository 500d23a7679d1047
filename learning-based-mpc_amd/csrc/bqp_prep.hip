// bqp_prep.hip — device-side preparation of the shared tables of the structured OCP kernel and
// the per-instance output finalisation.  Runs on the caller's stream (no host round trip), so
// the *_device entry point stays asynchronous.
#include <hip/hip_runtime.h>
#include <math.h>

#include <algorithm>

#include "../../include/bqp.h"
#include "bqp_internal.h"

namespace bqp {

// internal index [x; theta; u] -> external [x; u; theta]
__device__ __forceinline__ int ext_index(int i, int nx, int nu, int np) {
    const int ns = nx + np;
    if (i < nx) return i;
    if (i < ns) return nx + nu + (i - nx);
    return nx + (i - ns);
}

__global__ void ocp_prep_kernel(const double* __restrict__ W, const double* __restrict__ Fp,
                                int nx, int nu, int np, int N, int mp, int kp, int hstride,
                                int mpad, double* __restrict__ Hout, double* __restrict__ Fout,
                                int* __restrict__ qzero) {
    const int nv = nx + nu + np, ns = nx + np;
    // the structured launches' work-queue counters (OcpKernelArgs::queue), one per launch
    if (qzero && blockIdx.x == 0 && threadIdx.x < OCP_QUEUES) qzero[threadIdx.x] = 0;
    const int nH = (N + 1) * hstride;
    const int nF = nv * mpad;
    for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < nH + nF; t += gridDim.x * blockDim.x) {
        if (t < nH) {
            const int k = t / hstride, e = t % hstride;
            double v = 0.0;
            if (e < nv * nv) {
                const int i = e / nv, j = e % nv;  // row-major internal
                const int ei = ext_index(i, nx, nu, np), ej = ext_index(j, nx, nu, np);
                v = W[(size_t)k * nv * nv + (size_t)ej * nv + ei];  // column-major external
                if (k == N && (i >= ns || j >= ns)) v = 0.0;
            }
            Hout[t] = v;
        } else {
            const int q = t - nH;
            const int c = q / mpad, r = q % mpad;
            double v = 0.0;
            if (r < mp) {
                v = Fp[(size_t)ext_index(c, nx, nu, np) * mp + r];
                if (kp == N && c >= ns) v = 0.0;
            }
            Fout[q] = v;
        }
    }
}

hipError_t launch_ocp_prep(const double* W, const double* Fp, int nx, int nu, int np, int N,
                           int mp, int kp, int hstride, int mpad, double* Hout, double* Fout,
                           int* qzero, hipStream_t st) {
    const int total = (N + 1) * hstride + (nx + nu + np) * mpad;
    const int blocks = (total + 255) / 256;
    hipLaunchKernelGGL(ocp_prep_kernel, dim3(blocks), dim3(256), 0, st, W, Fp, nx, nu, np, N,
                       mp, kp, hstride, mpad, Hout, Fout, qzero);
    return hipGetLastError();
}

// per-instance stage-cost tables (bqp_ocp_data.sW != 0): batch x (N+1) x hstride, same layout
// as the shared table of ocp_prep_kernel
__global__ void ocp_prep_h_kernel(const double* __restrict__ W, int64_t sW, int batch, int nx,
                                  int nu, int np, int N, int hstride, double* __restrict__ Hout) {
    const int nv = nx + nu + np, ns = nx + np;
    const int64_t per = (int64_t)(N + 1) * hstride;
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < per * batch;
         t += (int64_t)gridDim.x * blockDim.x) {
        const int64_t b = t / per;
        const int q = (int)(t - b * per);
        const int k = q / hstride, e = q % hstride;
        double v = 0.0;
        if (e < nv * nv) {
            const int i = e / nv, j = e % nv;
            const int ei = ext_index(i, nx, nu, np), ej = ext_index(j, nx, nu, np);
            v = W[b * sW + (int64_t)k * nv * nv + (int64_t)ej * nv + ei];
            if (k == N && (i >= ns || j >= ns)) v = 0.0;
        }
        Hout[t] = v;
    }
}

hipError_t launch_ocp_prep_h(const double* W, int64_t sW, int batch, int nx, int nu, int np,
                             int N, int hstride, double* Hout, hipStream_t st) {
    const int64_t total = (int64_t)(N + 1) * hstride * batch;
    const int blocks = (int)std::min<int64_t>((total + 255) / 256, 65536);
    hipLaunchKernelGGL(ocp_prep_h_kernel, dim3(blocks), dim3(256), 0, st, W, sW, batch, nx, nu, np,
                       N, hstride, Hout);
    return hipGetLastError();
}

__global__ void finalize_kernel(const double* __restrict__ stats, int batch, bqp_output* out) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= batch) return;
    const double* s = stats + (size_t)b * STATS_W;
    bqp_output o;
    o.iterations = (int)s[0];
    o.firstorderopt = s[1];
    o.constrviolation = s[2];
    o.mu = s[3];
    o.kkt[0] = s[1];
    o.kkt[1] = s[4];
    o.kkt[2] = s[5];
    o.kkt[3] = s[3];
    o.polished = (int)s[6];
    out[b] = o;
}

hipError_t launch_ocp_finalize(const double* stats, int batch, void* out, hipStream_t st) {
    hipLaunchKernelGGL(finalize_kernel, dim3((batch + 255) / 256), dim3(256), 0, st, stats, batch,
                       (bqp_output*)out);
    return hipGetLastError();
}

}  // namespace bqp
