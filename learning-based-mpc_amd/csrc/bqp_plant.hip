// bqp_plant.hip — the true plant of the reference's closed loops, stepped on the GPU between
// batched solves (bqp_closed_loop_ocp_device).
//
// Moore-Greitzer compressor (examples/DMS_tracking_LMPC_casadi.m:215-221, `system`; the same
// model as models/trueModel.m:32-41) integrated over one sampling period delta by
//   BQP_PLANT_MG_RK4    one classical RK4 step (`dynamic`, :297-304) - the CasADi scripts;
//   BQP_PLANT_MG_ODE23  MATLAB's ode23 with its default options (trueModel.m:14/48,
//                       simulate_cont) - the fmincon loops ocpLMPC.m / ocpLBMPC.m through
//                       transitionTrue.m.
// One thread per instance: the plant is 4 states, the solve dominates.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "../../include/bqp.h"
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

// MATLAB ode23 over [0, T] from y with the input held: the Bogacki-Shampine 3(2) pair with
// first-same-as-last, local extrapolation and the step-size control of the MATLAB ODE suite
// (Shampine & Reichelt 1997) at the defaults RelTol 1e-3, AbsTol 1e-6 (threshold AbsTol/RelTol),
// MaxStep 0.1 T; initial step min(MaxStep, T) capped by 0.8 RelTol^(1/3) / |f0 / max(|y|, thr)|;
// a step within 10 % of the end is stretched to it.  Error estimate
// err = h |f E ./ max(|y|, |ynew|, thr)|_inf with E = [-5/72 1/12 1/9 -1/8]; a failed step
// shrinks h by max(0.5, 0.8 (RelTol/err)^(1/3)) the first time, by 0.5 after; a step without
// failure grows h by 1 / (1.25 (err/RelTol)^(1/3)), at most 5x.  The restatement
// (oracle/mg_model.py mg_ode23) reproduces every stored transition x_k -> x_{k+1} of the
// reference's fmincon runs (LMPC_N20/40/50, LBMPC_N40/50_sys_full.mat) to 1.4e-15.
__device__ void mg_ode23(double T, double (&y)[4], double u) {
    constexpr double rtol = 1e-3, thr = 1e-6 / 1e-3;
    constexpr double E0 = -5.0 / 72.0, E1 = 1.0 / 12.0, E2 = 1.0 / 9.0, E3 = -1.0 / 8.0;
    const double pw = 1.0 / 3.0, hmax = 0.1 * T;
    double F0[4], F1[4], F2[4], F3[4], ys[4], yn[4];
    mg_system(y, u, F0);
    double absh = fmin(hmax, T), rh = 0.0;
#pragma unroll
    for (int i = 0; i < 4; ++i) rh = fmax(rh, fabs(F0[i] / fmax(fabs(y[i]), thr)));
    rh /= 0.8 * pow(rtol, pw);
    if (absh * rh > 1.0) absh = 1.0 / rh;
    double t = 0.0;
    bool done = false;
    // at most 4096 step attempts (the MG plant takes 10-14 per 0.01 s sampling period)
    for (int guard = 0; !done && guard < 4096; ++guard) {
        const double hmin = 16.0 * (nextafter(t, INFINITY) - t);
        absh = fmin(hmax, fmax(hmin, absh));
        double h = absh;
        if (1.1 * absh >= fabs(T - t)) {
            h = T - t;
            absh = fabs(h);
            done = true;
        }
        bool nofailed = true;
        double err = 0.0;
        for (;; ++guard) {
            const double h1 = h * 0.5, h2 = h * 0.75;
#pragma unroll
            for (int i = 0; i < 4; ++i) ys[i] = y[i] + F0[i] * h1;
            mg_system(ys, u, F1);
#pragma unroll
            for (int i = 0; i < 4; ++i) ys[i] = y[i] + F1[i] * h2;
            mg_system(ys, u, F2);
            const double tnew = done ? T : t + h;
            h = tnew - t;
            const double b0 = h * (2.0 / 9.0), b1 = h * (1.0 / 3.0), b2 = h * (4.0 / 9.0);
#pragma unroll
            for (int i = 0; i < 4; ++i) yn[i] = y[i] + (F0[i] * b0 + F1[i] * b1 + F2[i] * b2);
            mg_system(yn, u, F3);
            double e = 0.0;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const double fe = F0[i] * E0 + F1[i] * E1 + F2[i] * E2 + F3[i] * E3;
                e = fmax(e, fabs(fe / fmax(fmax(fabs(y[i]), fabs(yn[i])), thr)));
            }
            err = absh * e;
            if (!(err > rtol)) {
                t = tnew;
                break;
            }
            if (absh <= hmin || guard >= 4096) {   // MATLAB warns and returns here
                done = true;
                t = tnew;
                break;
            }
            absh = nofailed ? fmax(hmin, absh * fmax(0.5, 0.8 * pow(rtol / err, pw)))
                            : fmax(hmin, 0.5 * absh);
            nofailed = false;
            h = absh;
            done = false;
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            y[i] = yn[i];
            F0[i] = F3[i];
        }
        if (!done && nofailed) {
            const double temp = 1.25 * pow(err / rtol, pw);
            absh = temp > 0.2 ? absh / temp : 5.0 * absh;
        }
    }
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

// apply u_0 of the step-t solve to the plant: u = u_eq + du_0, x+ = RK4(x, u) or ode23
__global__ void mg_plant_kernel(int plant, int batch, int N, int steps, int t, double delta,
                                const double* uo, const int* fl, const double* xeq,
                                const double* ueq, double* s, double* X, double* U, int* flags) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= batch) return;
    double x[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) x[i] = s[(int64_t)b * 4 + i] + xeq[i];
    const double u = uo[(int64_t)b * N] + ueq[0];
    if (plant == BQP_PLANT_MG_ODE23) mg_ode23(delta, x, u);
    else mg_rk4(delta, x, u);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        s[(int64_t)b * 4 + i] = x[i] - xeq[i];
        X[((int64_t)b * (steps + 1) + t + 1) * 4 + i] = x[i];
    }
    U[(int64_t)b * steps + t] = u;
    if (flags) flags[(int64_t)b * steps + t] = fl[b];
}

// ------------------------------------------------------------------------------------------
// LBMPC data window (DMS_LBMPC_casadi.m:198-207, utilities/get_data.m, functions/casadiL2NW.m):
// after the plant step t (iteration it = t + 1 of the reference loop) one wave per instance
//   - forms the learned one-step prediction of the step, with the window BEFORE its update,
//       xl = x_eq + A dx + B du + g(xi),  g = sum_i Y_i k_i / (lambda + sum_j k_j v_j),
//       k_i = exp(-|X_i - xi|^2 / h^2),  xi = [dx1; dx2; du]   (casadiL2NW.m:14-28)
//   - appends the sample X = [dx1; dx2; du], Y = (x+ - x_eq) - (A dx + B du) with v = 1.
// The window is a ring of q points, 8 doubles each ([X; Y; v], the 8 x q layout of the reference
// with its columns in ring order): iteration it writes point it mod q, which is exactly the
// column get_data.m fills (it < q) or the oldest one it drops (it >= q).  The NW sum does not
// depend on the column order.  lanes run over the points; the sums are wave reductions.
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ double wave_sum64(double v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

__global__ void lbmpc_window_kernel(int batch, int steps, int t, int q, double hinv2, double lam,
                                    const double* A, int64_t sA, const double* B, int64_t sB,
                                    const double* xeq, const double* ueq, const double* X,
                                    const double* U, double* win, double* XL) {
    const int lane = threadIdx.x & 63;
    const int b = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (b >= batch) return;
    const double* xt = X + ((int64_t)b * (steps + 1) + t) * 4;
    double dx[4], x1[4], nom[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) { dx[i] = xt[i] - xeq[i]; x1[i] = xt[4 + i]; }
    const double du = U[(int64_t)b * steps + t] - ueq[0];
    const double* Ab = A + (int64_t)b * sA;
    const double* Bb = B + (int64_t)b * sB;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        double v = Bb[i] * du;
#pragma unroll
        for (int j = 0; j < 4; ++j) v += Ab[j * 4 + i] * dx[j];   // column-major A
        nom[i] = v;
    }
    const double xi0 = dx[0], xi1 = dx[1], xi2 = du;
    double* w = win + (int64_t)b * q * 8;
    double sy0 = 0, sy1 = 0, sy2 = 0, sy3 = 0, sk = 0;
    for (int i = lane; i < q; i += 64) {
        const double* pt = w + (int64_t)i * 8;
        const double e0 = pt[0] - xi0, e1 = pt[1] - xi1, e2 = pt[2] - xi2;
        const double k = exp(-(e0 * e0 + e1 * e1 + e2 * e2) * hinv2);
        sy0 += pt[3] * k; sy1 += pt[4] * k; sy2 += pt[5] * k; sy3 += pt[6] * k;
        sk += k * pt[7];
    }
    sy0 = wave_sum64(sy0); sy1 = wave_sum64(sy1); sy2 = wave_sum64(sy2); sy3 = wave_sum64(sy3);
    sk = wave_sum64(sk);
    if (lane == 0) {
        const double den = lam + sk;
        const double g[4] = {sy0 / den, sy1 / den, sy2 / den, sy3 / den};
        double* xl = XL + ((int64_t)b * (steps + 1) + t + 1) * 4;
#pragma unroll
        for (int i = 0; i < 4; ++i) xl[i] = xeq[i] + nom[i] + g[i];
        // get_data.m: the sample of iteration t + 1 into ring slot (t + 1) mod q
        double* pt = w + (int64_t)((t + 1) % q) * 8;
        pt[0] = xi0; pt[1] = xi1; pt[2] = xi2;
#pragma unroll
        for (int i = 0; i < 4; ++i) pt[3 + i] = (x1[i] - xeq[i]) - nom[i];
        pt[7] = 1.0;
    }
}

// initial window: zeros; validity 1 on the first point only (DMS_LBMPC_casadi.m:160-161) or on
// every point (mask = 0: the 7-row window of hybrid_LBMPC_casadi.m:160, no validity row);
// XL[:, 0] = x_init
__global__ void lbmpc_window_init_kernel(int batch, int steps, int q, int mask,
                                         const double* xinit, double* win, double* XL) {
    const int b = blockIdx.x;
    if (b >= batch) return;
    double* w = win + (int64_t)b * q * 8;
    for (int i = threadIdx.x; i < q * 8; i += blockDim.x)
        w[i] = ((i & 7) == 7 && (!mask || i == 7)) ? 1.0 : 0.0;
    if (threadIdx.x < 4) XL[(int64_t)b * (steps + 1) * 4 + threadIdx.x] = xinit[(int64_t)b * 4 + threadIdx.x];
}

// ------------------------------------------------------------------------------------------
// learned-model NLP loop glue (bqp_closed_loop_sqp_device).  One workgroup per instance.
// prep: bin = bin0 + Bx s (the condensed nominal constraints at the measured deviation state s,
// Bx column-major m x nx) and, with shift, the warm start z <- [z_1 .. z_{nv-1}, 0, theta]
// (DMS_LBMPC_casadi.m:209-213 with Kstabil's tail move 0; nu = 1, nv = N moves then theta)
// ------------------------------------------------------------------------------------------
__global__ void sqp_loop_prep_kernel(int nx, int n, int m, int nv, int shift, const double* s,
                                     const double* bin0, const double* Bx, double* bin, double* z) {
    const int b = blockIdx.x;
    const double* sb = s + (int64_t)b * nx;
    double* bb = bin + (int64_t)b * m;
    for (int r = threadIdx.x; r < m; r += blockDim.x) {
        double v = bin0[r];
        for (int j = 0; j < nx; ++j) v += Bx[(int64_t)j * m + r] * sb[j];
        bb[r] = v;
    }
    if (shift) {
        double* zb = z + (int64_t)b * n;
        // read all moves before any write (one pass per thread block, n <= a few hundred)
        double v[4];
        int cnt = 0;
        for (int j = threadIdx.x; j < nv && cnt < 4; j += blockDim.x, ++cnt)
            v[cnt] = (j + 1 < nv) ? zb[j + 1] : 0.0;
        __syncthreads();
        cnt = 0;
        for (int j = threadIdx.x; j < nv && cnt < 4; j += blockDim.x, ++cnt) zb[j] = v[cnt];
    }
}

// u_0 = K s + z_0 (deviation) for the plant kernel (stride 1); log z and the iteration count
__global__ void sqp_loop_u0_kernel(int batch, int nx, int n, const double* K, const double* s,
                                   const double* z, double* uo, const int* it, int steps, int t,
                                   double* Zlog, int* itlog) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= batch) return;
    double u = z[(int64_t)b * n];
    for (int j = 0; j < nx; ++j) u += K[j] * s[(int64_t)b * nx + j];
    uo[b] = u;
    if (itlog) itlog[(int64_t)b * steps + t] = it[b];
    if (Zlog)
        for (int j = 0; j < n; ++j) Zlog[((int64_t)b * steps + t) * n + j] = z[(int64_t)b * n + j];
}

// ------------------------------------------------------------------------------------------
// asynchronous learned-model loop (bqp_closed_loop_sqp_device, round 5): every instance runs at
// its own closed-loop step ts[b].  After each SQP iteration of the batch, an instance whose SQP has
// finished (done[b] = 1) and still has steps to go advances here, in one workgroup: u_0 = K s +
// z_0 and the logs (sqp_loop_u0_kernel), the plant step (mg_plant_kernel), the data window
// (lbmpc_window_kernel: the learned prediction with the window before the sample, then the
// sample), and unless that was its last step the next step's constraints and warm start
// (sqp_loop_prep_kernel) with its SQP state reset (done, iterations) - the same operations, in the
// same order per instance, as the step-synchronous loop, whose SQP launches ran until the
// slowest instance of the batch had converged while the others idled.  At its last step the
// instance stays done and nfin counts it.
// ------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) sqp_loop_advance_kernel(SqpAdvanceArgs a) {
    const int b = blockIdx.x;
    if (b >= a.batch || !a.done[b] || a.ts[b] >= a.steps) return;     // uniform per workgroup
    const int t = a.ts[b], tid = threadIdx.x, lane = tid & 63;
    const int nx = a.nx, n = a.n, m = a.m, steps = a.steps, q = a.q;
    __shared__ double sh[8];
    double* sb = a.s + (int64_t)b * nx;
    double* zb = a.z + (int64_t)b * n;
    // u_0 and the logs (sqp_loop_u0_kernel)
    if (a.Zlog)
        for (int j = tid; j < n; j += blockDim.x) a.Zlog[((int64_t)b * steps + t) * n + j] = zb[j];
    if (tid == 0) {
        double u = zb[0];
        for (int j = 0; j < nx; ++j) u += a.K[j] * sb[j];
        if (a.itlog) a.itlog[(int64_t)b * steps + t] = a.iters[b];
        // plant step (mg_plant_kernel)
        double x[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) x[i] = sb[i] + a.xeq[i];
        const double uu = u + a.ueq[0];
        if (a.plant == BQP_PLANT_MG_ODE23) mg_ode23(a.delta, x, uu);
        else mg_rk4(a.delta, x, uu);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            sh[i] = x[i] - a.xeq[i];
            a.X[((int64_t)b * (steps + 1) + t + 1) * 4 + i] = x[i];
        }
        a.U[(int64_t)b * steps + t] = uu;
        if (a.flags) a.flags[(int64_t)b * steps + t] = a.flag[b];
    }
    __syncthreads();
    // data window (lbmpc_window_kernel), wave 0
    if (tid < 64) {
        const double* xt = a.X + ((int64_t)b * (steps + 1) + t) * 4;
        double dx[4], x1[4], nom[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) { dx[i] = xt[i] - a.xeq[i]; x1[i] = xt[4 + i]; }
        const double du = a.U[(int64_t)b * steps + t] - a.ueq[0];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            double v = a.Bm[i] * du;
#pragma unroll
            for (int j = 0; j < 4; ++j) v += a.A[j * 4 + i] * dx[j];   // column-major A
            nom[i] = v;
        }
        const double xi0 = dx[0], xi1 = dx[1], xi2 = du;
        double* w = a.win + (int64_t)b * q * 8;
        double sy0 = 0, sy1 = 0, sy2 = 0, sy3 = 0, sk = 0;
        for (int i = lane; i < q; i += 64) {
            const double* pt = w + (int64_t)i * 8;
            const double e0 = pt[0] - xi0, e1 = pt[1] - xi1, e2 = pt[2] - xi2;
            const double k = exp(-(e0 * e0 + e1 * e1 + e2 * e2) * a.hinv2);
            sy0 += pt[3] * k; sy1 += pt[4] * k; sy2 += pt[5] * k; sy3 += pt[6] * k;
            sk += k * pt[7];
        }
        sy0 = wave_sum64(sy0); sy1 = wave_sum64(sy1); sy2 = wave_sum64(sy2); sy3 = wave_sum64(sy3);
        sk = wave_sum64(sk);
        if (lane == 0) {
            const double den = a.lam + sk;
            const double g[4] = {sy0 / den, sy1 / den, sy2 / den, sy3 / den};
            double* xl = a.XL + ((int64_t)b * (steps + 1) + t + 1) * 4;
#pragma unroll
            for (int i = 0; i < 4; ++i) xl[i] = a.xeq[i] + nom[i] + g[i];
            double* pt = w + (int64_t)((t + 1) % q) * 8;
            pt[0] = xi0; pt[1] = xi1; pt[2] = xi2;
#pragma unroll
            for (int i = 0; i < 4; ++i) pt[3 + i] = (x1[i] - a.xeq[i]) - nom[i];
            pt[7] = 1.0;
        }
    }
    if (tid < nx) sb[tid] = sh[tid];      // the new measured deviation state
    __syncthreads();
    if (t + 1 < steps) {
        // the next step's constraints and warm start (sqp_loop_prep_kernel)
        double* bb = a.bin + (int64_t)b * m;
        for (int r = tid; r < m; r += blockDim.x) {
            double v = a.bin0[r];
            for (int j = 0; j < nx; ++j) v += a.Bx[(int64_t)j * m + r] * sh[j];
            bb[r] = v;
        }
        double v[4];
        int cnt = 0;
        for (int j = tid; j < n && cnt < 4; j += blockDim.x, ++cnt)
            v[cnt] = !a.warm ? 0.0 : (j < a.nv ? ((j + 1 < a.nv) ? zb[j + 1] : 0.0) : zb[j]);
        __syncthreads();
        cnt = 0;
        for (int j = tid; j < n && cnt < 4; j += blockDim.x, ++cnt) zb[j] = v[cnt];
        if (tid == 0) { a.iters[b] = 0; a.hused[b] = 0; a.ts[b] = t + 1; a.done[b] = 0; }
    } else if (tid == 0) {
        a.ts[b] = steps;
        atomicAdd(a.nfin, 1);
    }
}

hipError_t launch_sqp_loop_advance(const SqpAdvanceArgs& a, hipStream_t st) {
    // the kernel is written for the MG plant shape (x[4], one input: RK4 / ode23 of
    // models/trueModel.m, K x + c with K 1 x 4)
    if (a.n > 4 * 256 || a.nx != 4 || a.nu != 1) return hipErrorInvalidValue;
    hipLaunchKernelGGL(sqp_loop_advance_kernel, dim3(a.batch), dim3(256), 0, st, a);
    return hipGetLastError();
}

hipError_t launch_sqp_loop_prep(int batch, int nx, int n, int m, int nv, int shift, const double* s,
                                const double* bin0, const double* Bx, double* bin, double* z,
                                hipStream_t st) {
    if (nv > 4 * 256) return hipErrorInvalidValue;
    hipLaunchKernelGGL(sqp_loop_prep_kernel, dim3(batch), dim3(256), 0, st, nx, n, m, nv, shift, s,
                       bin0, Bx, bin, z);
    return hipGetLastError();
}

hipError_t launch_sqp_loop_u0(int batch, int nx, int n, const double* K, const double* s,
                              const double* z, double* uo, const int* it, int steps, int t,
                              double* Zlog, int* itlog, hipStream_t st) {
    hipLaunchKernelGGL(sqp_loop_u0_kernel, dim3((batch + 255) / 256), dim3(256), 0, st, batch, nx,
                       n, K, s, z, uo, it, steps, t, Zlog, itlog);
    return hipGetLastError();
}

hipError_t launch_lbmpc_window_init(int batch, int steps, int q, int mask, const double* xinit,
                                    double* win, double* XL, hipStream_t st) {
    hipLaunchKernelGGL(lbmpc_window_init_kernel, dim3(batch), dim3(256), 0, st, batch, steps, q,
                       mask, xinit, win, XL);
    return hipGetLastError();
}

hipError_t launch_lbmpc_window(int batch, int steps, int t, int q, double bw, double lam,
                               const double* A, int64_t sA, const double* B, int64_t sB,
                               const double* xeq, const double* ueq, const double* X,
                               const double* U, double* win, double* XL, hipStream_t st) {
    hipLaunchKernelGGL(lbmpc_window_kernel, dim3((batch + 3) / 4), dim3(256), 0, st, batch, steps,
                       t, q, 1.0 / (bw * bw), lam, A, sA, B, sB, xeq, ueq, X, U, win, XL);
    return hipGetLastError();
}

hipError_t launch_closed_loop_init(int batch, int nx, int steps, const double* xinit,
                                   const double* xeq, double* s, double* X, hipStream_t st) {
    hipLaunchKernelGGL(closed_loop_init_kernel, dim3((batch + 255) / 256), dim3(256), 0, st, batch,
                       nx, steps, xinit, xeq, s, X);
    return hipGetLastError();
}

hipError_t launch_mg_plant(int plant, int batch, int N, int steps, int t, double delta,
                           const double* uo, const int* fl, const double* xeq, const double* ueq,
                           double* s, double* X, double* U, int* flags, hipStream_t st) {
    hipLaunchKernelGGL(mg_plant_kernel, dim3((batch + 255) / 256), dim3(256), 0, st, plant, batch, N,
                       steps, t, delta, uo, fl, xeq, ueq, s, X, U, flags);
    return hipGetLastError();
}

}  // namespace bqp
