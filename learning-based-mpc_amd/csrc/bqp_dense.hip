// bqp_dense.hip — batched dense Mehrotra predictor-corrector IPM with MATLAB quadprog semantics
// (bqp_quadprog_batched):  min 0.5 x'Hx + f'x  s.t.  A x <= b, Aeq x = beq, lb <= x <= ub.
//
// One 256-thread workgroup per instance.  Per iteration: residuals (row- and column-parallel
// mat-vecs), K = H + A'DA + diag(bounds) (one thread per upper-triangle entry, A streamed in
// 32-row LDS tiles), right-looking Cholesky of K in the instance's global workspace (L2
// resident), equality Schur complement S = Aeq K^{-1} Aeq', then two solves (predictor,
// corrector) that reuse the factors.  Same step rules as the structured kernel (bqp_ocp.hip):
// CVXOPT-style unit-scaled start, sigma = (mu_aff/mu)^3, fraction-to-boundary tau.
// Fixed variables (lb == ub) must be passed as equality rows (the Python/MEX shims do that).
//
// quadprog exit flags (algorithm statement with the same rules: oracle/dense_ipm.py):
//    1 converged;  0 iteration limit;
//   -6 non-convex: H + CONVEX_EPS max(1, max H_ii) I has no Cholesky factor (tested once);
//   -8 non-finite residuals;
//   -3 unbounded: |z|_inf > Z_BIG (1 + data scale) - the iterates run along a recession
//      direction (K keeps a static pivot floor, so it always factors on a convex problem);
//   -2 primal infeasible: mu grew MU_BLOWUP-fold over its minimum with the primal residual
//      stalled (the structured kernel's rule, bqp_ocp.hip).
#include <hip/hip_runtime.h>
#include <math.h>

#include "bqp_internal.h"
#include "bqp_wave.h"

namespace bqp {

#define DT 256
#define TILE 32
#define DQ_PIV_FLOOR 1e-14    // static pivot floor of K, relative to its largest diagonal entry
#define DQ_CONVEX_EPS 1e-10   // shift of the convexity test (relative)
#define DQ_MU_BLOWUP 1e6
#define DQ_Z_BIG 1e12

struct DWork {
    int64_t K, Y, S, z, y, q, w, dz, dy, rd, re, tA, lA, riA, rcA, dtA, dlA, tB, lB, riB, rcB, dtB, dlB, total;
    __host__ __device__ static DWork make(int n, int m, int me) {
        DWork o;
        int64_t c = 0;
        o.K = c; c += (int64_t)n * n;
        o.Y = c; c += (int64_t)n * me;
        o.S = c; c += (int64_t)me * me;
        o.z = c; c += n; o.y = c; c += me; o.q = c; c += n; o.w = c; c += n;
        o.dz = c; c += n; o.dy = c; c += me; o.rd = c; c += n; o.re = c; c += me;
        o.tA = c; c += m; o.lA = c; c += m; o.riA = c; c += m; o.rcA = c; c += m;
        o.dtA = c; c += m; o.dlA = c; c += m;
        // bound rows: 2n (upper: 0..n-1, lower: n..2n-1)
        o.tB = c; c += 2 * n; o.lB = c; c += 2 * n; o.riB = c; c += 2 * n; o.rcB = c; c += 2 * n;
        o.dtB = c; c += 2 * n; o.dlB = c; c += 2 * n;
        o.total = (c + 7) & ~7;
        return o;
    }
};

int dense_work_doubles(int n, int m, int me) { return (int)DWork::make(n, m, me).total; }

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

struct Red {
    double* sc;  // LDS scratch, >= 4 doubles
    __device__ double sum(double v) {
        v = wave_sum(v);
        const int w = threadIdx.x >> 6;
        __syncthreads();
        if ((threadIdx.x & 63) == 0) sc[w] = v;
        __syncthreads();
        double r = sc[0] + sc[1] + sc[2] + sc[3];
        return r;
    }
    __device__ double max(double v) {
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o));
        const int w = threadIdx.x >> 6;
        __syncthreads();
        if ((threadIdx.x & 63) == 0) sc[w] = v;
        __syncthreads();
        return fmax(fmax(sc[0], sc[1]), fmax(sc[2], sc[3]));
    }
    __device__ double min(double v) {
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) v = fmin(v, __shfl_xor(v, o));
        const int w = threadIdx.x >> 6;
        __syncthreads();
        if ((threadIdx.x & 63) == 0) sc[w] = v;
        __syncthreads();
        return fmin(fmin(sc[0], sc[1]), fmin(sc[2], sc[3]));
    }
};

// in-place lower Cholesky of an n x n column-major matrix (global/L2).  fl >= 0: every pivot is
// floored at fl (static pivoting; never fails on finite input); fl < 0: returns false at the
// first non-positive pivot (the convexity test)
__device__ bool block_cholesky(double* K, int n, double* sc, double fl) {
    const int tid = threadIdx.x;
    for (int j = 0; j < n; ++j) {
        if (tid == 0) {
            double d = K[(int64_t)j * n + j];
            if (fl >= 0.0 && !(d > fl)) d = fl;
            sc[8] = d;
            K[(int64_t)j * n + j] = (d > 0.0) ? sqrt(d) : d;
        }
        __syncthreads();
        const double dj = sc[8];
        if (!(dj > 0.0)) return false;
        const double ljj = sqrt(dj);
        for (int i = j + 1 + tid; i < n; i += DT) K[(int64_t)j * n + i] /= ljj;
        __syncthreads();
        // trailing update of the lower triangle: K[c][r] -= L[j][r] * L[j][c], r >= c > j
        const int rem = n - j - 1;
        const int64_t cnt = (int64_t)rem * (rem + 1) / 2;
        for (int64_t e = tid; e < cnt; e += DT) {
            // map e -> (c, r) with c <= r in the trailing block (column-wise packing)
            int c = (int)((2 * rem + 1 - sqrt((double)(2 * rem + 1) * (2 * rem + 1) - 8.0 * e)) / 2);
            if (c < 0) c = 0;
            while ((int64_t)c * (2 * rem - c + 1) / 2 > e) --c;
            while ((int64_t)(c + 1) * (2 * rem - c) / 2 <= e) ++c;
            const int r = (int)(e - (int64_t)c * (2 * rem - c + 1) / 2) + c;
            const int cc = j + 1 + c, rr = j + 1 + r;
            K[(int64_t)cc * n + rr] -= K[(int64_t)j * n + rr] * K[(int64_t)j * n + cc];
        }
        __syncthreads();
    }
    return true;
}

// solve L L' x = b in place (x in LDS vector xs of length n), thread-parallel dot products
__device__ void chol_solve_vec(const double* L, int n, double* xs, Red& red) {
    // forward L y = b
    for (int i = 0; i < n; ++i) {
        double part = 0.0;
        for (int k = threadIdx.x; k < i; k += DT) part += L[(int64_t)k * n + i] * xs[k];
        const double s = red.sum(part);
        if (threadIdx.x == 0) xs[i] = (xs[i] - s) / L[(int64_t)i * n + i];
        __syncthreads();
    }
    // backward L' x = y
    for (int i = n - 1; i >= 0; --i) {
        double part = 0.0;
        for (int k = i + 1 + threadIdx.x; k < n; k += DT) part += L[(int64_t)i * n + k] * xs[k];
        const double s = red.sum(part);
        if (threadIdx.x == 0) xs[i] = (xs[i] - s) / L[(int64_t)i * n + i];
        __syncthreads();
    }
}

// sequential per-thread solve of L L' x = b for column vectors stored with stride (one per thread)
__device__ void chol_solve_col(const double* L, int n, double* x) {
    for (int i = 0; i < n; ++i) {
        double v = x[i];
        for (int k = 0; k < i; ++k) v -= L[(int64_t)k * n + i] * x[k];
        x[i] = v / L[(int64_t)i * n + i];
    }
    for (int i = n - 1; i >= 0; --i) {
        double v = x[i];
        for (int k = i + 1; k < n; ++k) v -= L[(int64_t)i * n + k] * x[k];
        x[i] = v / L[(int64_t)i * n + i];
    }
}

__global__ void __launch_bounds__(DT) dense_ipm_kernel(DenseKernelArgs a) {
    const int inst = blockIdx.x;
    if (inst >= a.batch) return;
    const int n = a.n, m = a.m, me = a.me, tid = threadIdx.x;
    __shared__ double sc[16];
    __shared__ double tileA[TILE * 257];
    Red red{sc};
    const DWork L = DWork::make(n, m, me);
    double* W = a.work + (int64_t)inst * a.work_stride;
    const double* H = a.H + (int64_t)inst * a.sH;
    const double* f = a.f + (int64_t)inst * a.sf;
    const double* A = a.A ? a.A + (int64_t)inst * a.sA : nullptr;
    const double* b = a.b ? a.b + (int64_t)inst * a.sb : nullptr;
    const double* E = a.Aeq ? a.Aeq + (int64_t)inst * a.sAeq : nullptr;
    const double* e = a.beq ? a.beq + (int64_t)inst * a.sbeq : nullptr;
    const double* lb = a.lb ? a.lb + (int64_t)inst * a.slb : nullptr;
    const double* ub = a.ub ? a.ub + (int64_t)inst * a.sub : nullptr;
    double *z = W + L.z, *y = W + L.y, *q = W + L.q, *w = W + L.w, *dz = W + L.dz, *dy = W + L.dy;
    double *rd = W + L.rd, *re = W + L.re;
    double *tA = W + L.tA, *lA = W + L.lA, *riA = W + L.riA, *rcA = W + L.rcA, *dtA = W + L.dtA, *dlA = W + L.dlA;
    double *tB = W + L.tB, *lB = W + L.lB, *riB = W + L.riB, *rcB = W + L.rcB, *dtB = W + L.dtB, *dlB = W + L.dlB;
    double* K = W + L.K;
    double* Y = W + L.Y;
    double* S = W + L.S;
    auto up_present = [&](int j) -> bool { return ub && isfinite(ub[j]); };
    auto lo_present = [&](int j) -> bool { return lb && isfinite(lb[j]); };
    // row count
    double cnt = 0.0;
    for (int j = tid; j < n; j += DT) cnt += (up_present(j) ? 1.0 : 0.0) + (lo_present(j) ? 1.0 : 0.0);
    const double mtot = red.sum(cnt) + (double)m;
    const double minv = 1.0 / fmax(mtot, 1.0);

    // ---------------------------------------------------------------- residuals
    auto residuals = [&](double& stat, double& feq, double& fin, double& csum, double& gscale, double& zmax) {
        double fe = 0.0, fq = 0.0, cs = 0.0, st = 0.0, gs = 0.0, zm = 0.0;
        for (int r = tid; r < m; r += DT) {
            double v = tA[r] - b[r];
            for (int j = 0; j < n; ++j) v += A[(int64_t)j * m + r] * z[j];
            riA[r] = v;
            fe = fmax(fe, fabs(v));
            cs += tA[r] * lA[r];
        }
        for (int r = tid; r < me; r += DT) {
            double v = -e[r];
            for (int j = 0; j < n; ++j) v += E[(int64_t)j * me + r] * z[j];
            re[r] = v;
            fq = fmax(fq, fabs(v));
        }
        for (int j = tid; j < n; j += DT) {
            double v = f[j];
            for (int i = 0; i < n; ++i) v += H[(int64_t)j * n + i] * z[i];
            gs = fmax(gs, fabs(v));
            for (int r = 0; r < me; ++r) v += E[(int64_t)j * me + r] * y[r];
            for (int r = 0; r < m; ++r) v += A[(int64_t)j * m + r] * lA[r];
            riB[j] = 0.0; riB[n + j] = 0.0;
            if (up_present(j)) {
                v += lB[j];
                riB[j] = z[j] + tB[j] - ub[j];
                cs += tB[j] * lB[j];
            }
            if (lo_present(j)) {
                v -= lB[n + j];
                riB[n + j] = -z[j] + tB[n + j] + lb[j];
                cs += tB[n + j] * lB[n + j];
            }
            fe = fmax(fe, fmax(fabs(riB[j]), fabs(riB[n + j])));
            rd[j] = v;
            st = fmax(st, fabs(v));
            zm = fmax(zm, fabs(z[j]));
        }
        stat = red.max(st);
        fin = red.max(fe);
        feq = red.max(fq);
        csum = red.sum(cs);
        gscale = red.max(gs);
        zmax = red.max(zm);
    };

    // ---------------------------------------------------------------- factorisation
    auto factor = [&]() -> bool {
        // K upper entries (i <= j) = H_ij + sum_r A_ri D_r A_rj (+ bound diagonal)
        const int ne = n * (n + 1) / 2;
        double dmx = 0.0;                 // largest diagonal entry (pivot floor scale)
        for (int base = 0; base < ne; base += DT * 8) {
            double acc[8];
            int ii[8], jj[8];
#pragma unroll
            for (int q2 = 0; q2 < 8; ++q2) {
                const int e2 = base + tid + q2 * DT;
                acc[q2] = 0.0;
                ii[q2] = -1; jj[q2] = -1;
                if (e2 < ne) {
                    // column-wise packing of the upper triangle: e2 -> (i <= j)
                    int j = (int)((sqrt(8.0 * e2 + 1.0) - 1.0) / 2.0);
                    while ((int64_t)j * (j + 1) / 2 > e2) --j;
                    while ((int64_t)(j + 1) * (j + 2) / 2 <= e2) ++j;
                    const int i = e2 - j * (j + 1) / 2;
                    ii[q2] = i; jj[q2] = j;
                    acc[q2] = H[(int64_t)j * n + i];
                }
            }
            for (int r0 = 0; r0 < m; r0 += TILE) {
                const int rows = min(TILE, m - r0);
                __syncthreads();
                for (int t2 = tid; t2 < rows * n; t2 += DT) {
                    const int rr = t2 % rows, j = t2 / rows;
                    tileA[rr * 257 + j] = A[(int64_t)j * m + r0 + rr];
                }
                if (tid < rows) tileA[tid * 257 + 256] = lA[r0 + tid] / tA[r0 + tid];
                __syncthreads();
#pragma unroll
                for (int q2 = 0; q2 < 8; ++q2) {
                    if (ii[q2] < 0) continue;
                    double s = 0.0;
                    for (int rr = 0; rr < rows; ++rr)
                        s += tileA[rr * 257 + ii[q2]] * tileA[rr * 257 + 256] * tileA[rr * 257 + jj[q2]];
                    acc[q2] += s;
                }
            }
#pragma unroll
            for (int q2 = 0; q2 < 8; ++q2) {
                if (ii[q2] < 0) continue;
                double v = acc[q2];
                if (ii[q2] == jj[q2]) {
                    const int j = jj[q2];
                    if (up_present(j)) v += lB[j] / tB[j];
                    if (lo_present(j)) v += lB[n + j] / tB[n + j];
                    dmx = fmax(dmx, fabs(v));
                }
                K[(int64_t)ii[q2] * n + jj[q2]] = v;   // lower part (row jj, col ii) col-major
                K[(int64_t)jj[q2] * n + ii[q2]] = v;
            }
        }
        const double kfl = DQ_PIV_FLOOR * fmax(red.max(dmx), 1e-300);
        if (!block_cholesky(K, n, sc, kfl)) return false;
        // Y = K^{-1} Aeq' (one thread per equality row), S = Aeq Y
        for (int r = tid; r < me; r += DT) {
            double* yc = Y + (int64_t)r * n;
            for (int j = 0; j < n; ++j) yc[j] = E[(int64_t)j * me + r];
            chol_solve_col(K, n, yc);
        }
        __syncthreads();
        double smx = 0.0;
        for (int t2 = tid; t2 < me * me; t2 += DT) {
            const int r1 = t2 % me, r2 = t2 / me;
            double s = 0.0;
            for (int j = 0; j < n; ++j) s += E[(int64_t)j * me + r1] * Y[(int64_t)r2 * n + j];
            S[(int64_t)r2 * me + r1] = s;
            if (r1 == r2) smx = fmax(smx, fabs(s));
        }
        const double sfl = DQ_PIV_FLOOR * fmax(red.max(smx), 1e-300);
        if (me > 0 && !block_cholesky(S, me, sc, sfl)) return false;
        return true;
    };

    // ---------------------------------------------------------------- solve (rc given)
    double* xs = tileA;  // LDS vector workspace (n <= 256 and me <= 256)
    auto solve = [&]() {
        // q = rd + A'((lam riA - rcA)/tA) + bound terms ; w = -K^{-1} q
        for (int j = tid; j < n; j += DT) {
            double v = rd[j];
            for (int r = 0; r < m; ++r) v += A[(int64_t)j * m + r] * ((lA[r] * riA[r] - rcA[r]) / tA[r]);
            if (up_present(j)) v += (lB[j] * riB[j] - rcB[j]) / tB[j];
            if (lo_present(j)) v -= (lB[n + j] * riB[n + j] - rcB[n + j]) / tB[n + j];
            q[j] = v;
        }
        __syncthreads();
        for (int j = tid; j < n; j += DT) xs[j] = -q[j];
        __syncthreads();
        chol_solve_vec(K, n, xs, red);
        for (int j = tid; j < n; j += DT) w[j] = xs[j];
        __syncthreads();
        if (me > 0) {
            // dy = S^{-1}(Aeq w + re)
            for (int r = tid; r < me; r += DT) {
                double v = re[r];
                for (int j = 0; j < n; ++j) v += E[(int64_t)j * me + r] * w[j];
                xs[r] = v;
            }
            __syncthreads();
            chol_solve_vec(S, me, xs, red);
            for (int r = tid; r < me; r += DT) dy[r] = xs[r];
            __syncthreads();
        }
        for (int j = tid; j < n; j += DT) {
            double v = w[j];
            for (int r = 0; r < me; ++r) v -= Y[(int64_t)r * n + j] * dy[r];
            dz[j] = v;
        }
        __syncthreads();
        for (int r = tid; r < m; r += DT) {
            double v = 0.0;
            for (int j = 0; j < n; ++j) v += A[(int64_t)j * m + r] * dz[j];
            dtA[r] = -riA[r] - v;
            dlA[r] = (-rcA[r] - lA[r] * dtA[r]) / tA[r];
        }
        for (int j = tid; j < n; j += DT) {
            dtB[j] = dlB[j] = dtB[n + j] = dlB[n + j] = 0.0;
            if (up_present(j)) { dtB[j] = -riB[j] - dz[j]; dlB[j] = (-rcB[j] - lB[j] * dtB[j]) / tB[j]; }
            if (lo_present(j)) { dtB[n + j] = -riB[n + j] + dz[j]; dlB[n + j] = (-rcB[n + j] - lB[n + j] * dtB[n + j]) / tB[n + j]; }
        }
        __syncthreads();
    };

    auto max_step = [&]() -> double {
        double al = 1.0;
#define DQ_RATIO(v, dv) if ((dv) < 0.0) al = fmin(al, -(v) / (dv));
        for (int r = tid; r < m; r += DT) { DQ_RATIO(tA[r], dtA[r]); DQ_RATIO(lA[r], dlA[r]); }
        for (int j = tid; j < n; j += DT) {
            if (up_present(j)) { DQ_RATIO(tB[j], dtB[j]); DQ_RATIO(lB[j], dlB[j]); }
            if (lo_present(j)) { DQ_RATIO(tB[n + j], dtB[n + j]); DQ_RATIO(lB[n + j], dlB[n + j]); }
        }
#undef DQ_RATIO
        return red.min(al);
    };
    auto comp_after = [&](double al) -> double {
        double c = 0.0;
        for (int r = tid; r < m; r += DT) c += (tA[r] + al * dtA[r]) * (lA[r] + al * dlA[r]);
        for (int j = tid; j < n; j += DT) {
            if (up_present(j)) c += (tB[j] + al * dtB[j]) * (lB[j] + al * dlB[j]);
            if (lo_present(j)) c += (tB[n + j] + al * dtB[n + j]) * (lB[n + j] + al * dlB[n + j]);
        }
        return red.sum(c);
    };

    // ---------------------------------------------------------------- initial point
    for (int j = tid; j < n; j += DT) {
        z[j] = 0.0;
        tB[j] = tB[n + j] = 1.0;
        lB[j] = up_present(j) ? 1.0 : 0.0;
        lB[n + j] = lo_present(j) ? 1.0 : 0.0;
        rcB[j] = rcB[n + j] = 1.0;
        if (!up_present(j)) rcB[j] = 0.0;
        if (!lo_present(j)) rcB[n + j] = 0.0;
    }
    for (int r = tid; r < me; r += DT) y[r] = 0.0;
    for (int r = tid; r < m; r += DT) { tA[r] = 1.0; lA[r] = 1.0; rcA[r] = 1.0; }
    // bound rows take part in the unit-scaled start like the structured kernel (lam = 1)
    for (int j = tid; j < n; j += DT) {
        if (up_present(j)) lB[j] = 1.0;
        if (lo_present(j)) lB[n + j] = 1.0;
    }
    __syncthreads();
    // primal data scale for the relative feasibility test
    double bsl = 0.0;
    for (int r = tid; r < m; r += DT) bsl = fmax(bsl, fabs(b[r]));
    for (int r = tid; r < me; r += DT) bsl = fmax(bsl, fabs(e[r]));
    for (int j = tid; j < n; j += DT) {
        if (up_present(j)) bsl = fmax(bsl, fabs(ub[j]));
        if (lo_present(j)) bsl = fmax(bsl, fabs(lb[j]));
    }
    const double bscale = red.max(bsl);
    double fmx = 0.0;
    for (int j = tid; j < n; j += DT) fmx = fmax(fmx, fabs(f[j]));
    const double zbig = DQ_Z_BIG * (1.0 + bscale + red.max(fmx));
    int flag = 0;
    {
        // convexity test: Cholesky of H + CONVEX_EPS max(1, max H_ii) I without pivot floor
        double hd = 0.0;
        for (int j = tid; j < n; j += DT) hd = fmax(hd, fabs(H[(int64_t)j * n + j]));
        const double sh = DQ_CONVEX_EPS * fmax(1.0, red.max(hd));
        for (int e2 = tid; e2 < n * n; e2 += DT) {
            const int i = e2 % n, j = e2 / n;
            K[e2] = H[e2] + (i == j ? sh : 0.0);
        }
        __syncthreads();
        if (!block_cholesky(K, n, sc, -1.0)) flag = -6;
    }
    double stat = 0.0, feq = 0.0, fin = 0.0, csum = 0.0, gscale = 0.0, zmax = 0.0;
    residuals(stat, feq, fin, csum, gscale, zmax);
    if (flag == 0 && !factor()) flag = -8;
    if (flag == 0) {
        solve();
        double tmin = INFINITY, tmax = -INFINITY;
        for (int j = tid; j < n; j += DT) z[j] += dz[j];
        for (int r = tid; r < me; r += DT) y[r] += dy[r];
        for (int r = tid; r < m; r += DT) { const double t = 1.0 + dtA[r]; tmin = fmin(tmin, t); tmax = fmax(tmax, t); }
        for (int j = tid; j < n; j += DT) {
            if (up_present(j)) { const double t = 1.0 + dtB[j]; tmin = fmin(tmin, t); tmax = fmax(tmax, t); }
            if (lo_present(j)) { const double t = 1.0 + dtB[n + j]; tmin = fmin(tmin, t); tmax = fmax(tmax, t); }
        }
        tmin = red.min(tmin);
        tmax = red.max(tmax);
        const double shp = (tmin <= 0.0) ? 1.0 - tmin : 0.0;
        const double shd = (tmax >= 0.0) ? 1.0 + tmax : 0.0;
        for (int r = tid; r < m; r += DT) { const double t = 1.0 + dtA[r]; tA[r] = t + shp; lA[r] = -t + shd; }
        for (int j = tid; j < n; j += DT) {
            const double tu = 1.0 + dtB[j], tl = 1.0 + dtB[n + j];
            tB[j] = up_present(j) ? tu + shp : 1.0; lB[j] = up_present(j) ? -tu + shd : 0.0;
            tB[n + j] = lo_present(j) ? tl + shp : 1.0; lB[n + j] = lo_present(j) ? -tl + shd : 0.0;
        }
        __syncthreads();
    }
    // ---------------------------------------------------------------- main loop
    int it = 0;
    double mu = 0.0, mu_min = INFINITY;
    if (flag == 0) {
        for (it = 0; it <= a.max_iter; ++it) {
            residuals(stat, feq, fin, csum, gscale, zmax);
            const double feas = fmax(feq, fin);
            mu = csum * minv;
            if (stat <= a.tol_stat * (1.0 + gscale) && feas <= a.tol_feas * (1.0 + bscale) &&
                mu <= a.tol_comp) { flag = 1; break; }
            if (!(isfinite(stat) && isfinite(feas) && isfinite(mu))) { flag = -8; break; }
            if (zmax > zbig) { flag = -3; break; }
            if (mu > DQ_MU_BLOWUP * mu_min && feas > 1e-6 * (1.0 + bscale)) { flag = -2; break; }
            mu_min = fmin(mu_min, mu);
            if (it == a.max_iter) break;
            if (!factor()) { flag = -8; break; }
            for (int r = tid; r < m; r += DT) rcA[r] = tA[r] * lA[r];
            for (int j = tid; j < 2 * n; j += DT) rcB[j] = tB[j] * lB[j];
            __syncthreads();
            solve();
            double al = max_step();
            const double mua = comp_after(al) * minv;
            double sg = mua / mu;
            sg = sg * sg * sg;
            const double smu = sg * mu;
            for (int r = tid; r < m; r += DT) rcA[r] = tA[r] * lA[r] + dtA[r] * dlA[r] - smu;
            for (int j = tid; j < n; j += DT) {
                rcB[j] = up_present(j) ? tB[j] * lB[j] + dtB[j] * dlB[j] - smu : 0.0;
                rcB[n + j] = lo_present(j) ? tB[n + j] * lB[n + j] + dtB[n + j] * dlB[n + j] - smu : 0.0;
            }
            __syncthreads();
            solve();
            al = fmin(1.0, max_step() * a.tau);
            for (int j = tid; j < n; j += DT) {
                z[j] += al * dz[j];
                if (up_present(j)) { tB[j] += al * dtB[j]; lB[j] += al * dlB[j]; }
                if (lo_present(j)) { tB[n + j] += al * dtB[n + j]; lB[n + j] += al * dlB[n + j]; }
            }
            for (int r = tid; r < me; r += DT) y[r] += al * dy[r];
            for (int r = tid; r < m; r += DT) { tA[r] += al * dtA[r]; lA[r] += al * dlA[r]; }
            __syncthreads();
        }
    }
    // ---------------------------------------------------------------- outputs
    double fv = 0.0;
    for (int j = tid; j < n; j += DT) {
        double hz = 0.0;
        for (int i = 0; i < n; ++i) hz += H[(int64_t)j * n + i] * z[i];
        fv += z[j] * (0.5 * hz + f[j]);
        a.x[(int64_t)inst * n + j] = z[j];
        if (a.lam_lower) a.lam_lower[(int64_t)inst * n + j] = (lo_present(j) && flag != -6) ? lB[n + j] : 0.0;
        if (a.lam_upper) a.lam_upper[(int64_t)inst * n + j] = (up_present(j) && flag != -6) ? lB[j] : 0.0;
    }
    for (int r = tid; r < m; r += DT)
        if (a.lam_ineqlin) a.lam_ineqlin[(int64_t)inst * m + r] = flag != -6 ? lA[r] : 0.0;
    for (int r = tid; r < me; r += DT)
        if (a.lam_eqlin) a.lam_eqlin[(int64_t)inst * me + r] = flag != -6 ? y[r] : 0.0;
    fv = red.sum(fv);
    if (tid == 0) {
        if (a.fval) a.fval[inst] = fv;
        a.exitflag[inst] = flag;
        double* so = a.stats + (int64_t)inst * STATS_W;
        so[0] = (double)it; so[1] = stat; so[2] = fmax(feq, fin); so[3] = mu; so[4] = feq; so[5] = fin;
    }
}

// ==========================================================================================
// small dense QPs (n <= 32, no equality rows): one WAVE per instance, every vector and the
// factor in LDS, DPP wave reductions, readlane-broadcast triangular solves - no workgroup
// barrier anywhere.  Same Mehrotra rules and start as dense_ipm_kernel; used for the LBMPC
// SQP sub-problems (n = N*nu + np = 11 at config C1) and small quadprog calls, where the
// workgroup kernel above is barrier-bound (~130 us per IPM iteration at n = 11).
// ==========================================================================================
#define SW_NMAX 32
#define SW_LDS_MAX (64 * 1024 / 8)   // doubles of dynamic LDS per wave-instance

#define SW_A_LDS_MAX 4096             // A (m x n) staged in LDS when it has at most this many entries

__host__ __device__ inline int small_lds_doubles(int n, int m) {
    return n * n + 4 * n + 12 * n + 7 * m + (m * n <= SW_A_LDS_MAX ? m * n : 0);
}

__global__ void __launch_bounds__(64) dense_wave_kernel(DenseKernelArgs a) {
    const int inst = blockIdx.x;
    if (inst >= a.batch) return;
    const int n = a.n, m = a.m, lane = threadIdx.x;
    extern __shared__ double sm[];
    double* K = sm;                       // n x n column-major; lower Cholesky factor in place
    double* z = K + n * n;
    double* q = z + n;
    double* dz = q + n;
    double* rd = dz + n;
    double* tB = rd + n;                  // bound rows: [upper 0..n-1, lower n..2n-1]
    double* lB = tB + 2 * n;
    double* riB = lB + 2 * n;
    double* rcB = riB + 2 * n;
    double* dtB = rcB + 2 * n;
    double* dlB = dtB + 2 * n;
    double* tA = dlB + 2 * n;             // inequality rows
    double* lA = tA + m;
    double* riA = lA + m;
    double* rcA = riA + m;
    double* dtA = rcA + m;
    double* dlA = dtA + m;
    double* DA = dlA + m;
    const double* H = a.H + (int64_t)inst * a.sH;
    const double* f = a.f + (int64_t)inst * a.sf;
    const double* A = a.A ? a.A + (int64_t)inst * a.sA : nullptr;
    const double* b = a.b ? a.b + (int64_t)inst * a.sb : nullptr;
    const double* lb = a.lb ? a.lb + (int64_t)inst * a.slb : nullptr;
    const double* ub = a.ub ? a.ub + (int64_t)inst * a.sub : nullptr;
    if (A && m * n <= SW_A_LDS_MAX) {             // the rows are re-read ~6x per IPM iteration
        double* As = DA + m;
        for (int i = lane; i < m * n; i += 64) As[i] = A[i];
        wave_sync();
        A = As;
    }
    auto up_present = [&](int j) -> bool { return ub && isfinite(ub[j]); };
    auto lo_present = [&](int j) -> bool { return lb && isfinite(lb[j]); };
    double cnt = 0.0;
    for (int j = lane; j < n; j += 64) cnt += (up_present(j) ? 1.0 : 0.0) + (lo_present(j) ? 1.0 : 0.0);
    const double minv = 1.0 / fmax(wsum(cnt) + (double)m, 1.0);

    auto residuals = [&](double& stat, double& fin, double& csum, double& gscale, double& zmax) {
        double fe = 0.0, cs = 0.0, st = 0.0, gs = 0.0, zm = 0.0;
        for (int r = lane; r < m; r += 64) {
            double v = tA[r] - b[r];
            for (int j = 0; j < n; ++j) v += A[(int64_t)j * m + r] * z[j];
            riA[r] = v;
            fe = fmax(fe, fabs(v));
            cs += tA[r] * lA[r];
        }
        for (int j = lane; j < n; j += 64) {
            double v = f[j];
            for (int i = 0; i < n; ++i) v += H[(int64_t)j * n + i] * z[i];
            gs = fmax(gs, fabs(v));
            for (int r = 0; r < m; ++r) v += A[(int64_t)j * m + r] * lA[r];
            riB[j] = 0.0; riB[n + j] = 0.0;
            if (up_present(j)) { v += lB[j]; riB[j] = z[j] + tB[j] - ub[j]; cs += tB[j] * lB[j]; }
            if (lo_present(j)) { v -= lB[n + j]; riB[n + j] = -z[j] + tB[n + j] + lb[j]; cs += tB[n + j] * lB[n + j]; }
            fe = fmax(fe, fmax(fabs(riB[j]), fabs(riB[n + j])));
            rd[j] = v;
            st = fmax(st, fabs(v));
            zm = fmax(zm, fabs(z[j]));
        }
        stat = wmax(st); fin = wmax(fe); csum = wsum(cs); gscale = wmax(gs); zmax = wmax(zm);
        wave_sync();
    };

    // in-place lower Cholesky of K (lane r owns row r).  fl >= 0: pivots floored at fl (static
    // pivoting); fl < 0: false at the first non-positive pivot (the convexity test)
    auto chol = [&](double fl) -> bool {
        bool ok = true;
        for (int j = 0; j < n; ++j) {
            double d = K[(int64_t)j * n + j];
            if (fl >= 0.0 && !(d > fl)) d = fl;
            if (!(d > 0.0)) { ok = false; break; }
            const double ljj = sqrt(d);
            const double il = 1.0 / ljj;
            if (lane > j && lane < n) K[(int64_t)j * n + lane] *= il;
            if (lane == j) K[(int64_t)j * n + j] = ljj;
            wave_sync();
            if (lane > j && lane < n) {
                const double lrj = K[(int64_t)j * n + lane];
                for (int c = j + 1; c <= lane; ++c) K[(int64_t)c * n + lane] -= lrj * K[(int64_t)j * n + c];
            }
            wave_sync();
        }
        return ok;
    };
    // K = H + A'DA + bound diagonal, factored with the static pivot floor
    auto factor = [&]() -> bool {
        for (int r = lane; r < m; r += 64) DA[r] = lA[r] / tA[r];
        wave_sync();
        const int ne = n * (n + 1) / 2;
        double dmx = 0.0;
        for (int e2 = lane; e2 < ne; e2 += 64) {
            int j = (int)((sqrt(8.0 * e2 + 1.0) - 1.0) / 2.0);
            while (j * (j + 1) / 2 > e2) --j;
            while ((j + 1) * (j + 2) / 2 <= e2) ++j;
            const int i = e2 - j * (j + 1) / 2;          // i <= j
            double v = H[(int64_t)j * n + i];
            for (int r = 0; r < m; ++r) v += A[(int64_t)i * m + r] * DA[r] * A[(int64_t)j * m + r];
            if (i == j) {
                if (up_present(j)) v += lB[j] / tB[j];
                if (lo_present(j)) v += lB[n + j] / tB[n + j];
                dmx = fmax(dmx, fabs(v));
            }
            K[(int64_t)i * n + j] = v;                   // lower: row j, column i
        }
        const double kfl = DQ_PIV_FLOOR * fmax(wmax(dmx), 1e-300);
        wave_sync();
        return chol(kfl);
    };

    // x = -(L L')^{-1} q with lane i holding entry i (n <= 32): column-oriented substitution,
    // the solved entry broadcast by readlane
    auto chol_neg_solve = [&](double* x) {
        double v = (lane < n) ? -q[lane] : 0.0;
        for (int i = 0; i < n; ++i) {                     // L y = -q
            const double yi = rl(v, i) / K[(int64_t)i * n + i];
            if (lane == i) v = yi;
            else if (lane > i && lane < n) v -= K[(int64_t)i * n + lane] * yi;
        }
        for (int i = n - 1; i >= 0; --i) {                // L' x = y
            const double xi = rl(v, i) / K[(int64_t)i * n + i];
            if (lane == i) v = xi;
            else if (lane < i) v -= K[(int64_t)lane * n + i] * xi;
        }
        if (lane < n) x[lane] = v;
        wave_sync();
    };

    auto solve = [&]() {
        for (int r = lane; r < m; r += 64) dlA[r] = (lA[r] * riA[r] - rcA[r]) / tA[r];
        wave_sync();
        for (int j = lane; j < n; j += 64) {
            double v = rd[j];
            for (int r = 0; r < m; ++r) v += A[(int64_t)j * m + r] * dlA[r];
            if (up_present(j)) v += (lB[j] * riB[j] - rcB[j]) / tB[j];
            if (lo_present(j)) v -= (lB[n + j] * riB[n + j] - rcB[n + j]) / tB[n + j];
            q[j] = v;
        }
        wave_sync();
        chol_neg_solve(dz);
        for (int r = lane; r < m; r += 64) {
            double v = 0.0;
            for (int j = 0; j < n; ++j) v += A[(int64_t)j * m + r] * dz[j];
            dtA[r] = -riA[r] - v;
            dlA[r] = (-rcA[r] - lA[r] * dtA[r]) / tA[r];
        }
        for (int j = lane; j < n; j += 64) {
            dtB[j] = dlB[j] = dtB[n + j] = dlB[n + j] = 0.0;
            if (up_present(j)) { dtB[j] = -riB[j] - dz[j]; dlB[j] = (-rcB[j] - lB[j] * dtB[j]) / tB[j]; }
            if (lo_present(j)) { dtB[n + j] = -riB[n + j] + dz[j]; dlB[n + j] = (-rcB[n + j] - lB[n + j] * dtB[n + j]) / tB[n + j]; }
        }
        wave_sync();
    };
    auto max_step = [&]() -> double {
        double al = 1.0;
#define DW_RATIO(v, dv) if ((dv) < 0.0) al = fmin(al, -(v) / (dv));
        for (int r = lane; r < m; r += 64) { DW_RATIO(tA[r], dtA[r]); DW_RATIO(lA[r], dlA[r]); }
        for (int j = lane; j < n; j += 64) {
            if (up_present(j)) { DW_RATIO(tB[j], dtB[j]); DW_RATIO(lB[j], dlB[j]); }
            if (lo_present(j)) { DW_RATIO(tB[n + j], dtB[n + j]); DW_RATIO(lB[n + j], dlB[n + j]); }
        }
#undef DW_RATIO
        return wmin(al);
    };
    auto comp_after = [&](double al) -> double {
        double c = 0.0;
        for (int r = lane; r < m; r += 64) c += (tA[r] + al * dtA[r]) * (lA[r] + al * dlA[r]);
        for (int j = lane; j < n; j += 64) {
            if (up_present(j)) c += (tB[j] + al * dtB[j]) * (lB[j] + al * dlB[j]);
            if (lo_present(j)) c += (tB[n + j] + al * dtB[n + j]) * (lB[n + j] + al * dlB[n + j]);
        }
        return wsum(c);
    };

    // initial point (as dense_ipm_kernel)
    for (int j = lane; j < n; j += 64) {
        z[j] = 0.0;
        tB[j] = tB[n + j] = 1.0;
        lB[j] = up_present(j) ? 1.0 : 0.0;
        lB[n + j] = lo_present(j) ? 1.0 : 0.0;
        rcB[j] = up_present(j) ? 1.0 : 0.0;
        rcB[n + j] = lo_present(j) ? 1.0 : 0.0;
    }
    for (int r = lane; r < m; r += 64) { tA[r] = 1.0; lA[r] = 1.0; rcA[r] = 1.0; }
    wave_sync();
    double bsl = 0.0;
    for (int r = lane; r < m; r += 64) bsl = fmax(bsl, fabs(b[r]));
    for (int j = lane; j < n; j += 64) {
        if (up_present(j)) bsl = fmax(bsl, fabs(ub[j]));
        if (lo_present(j)) bsl = fmax(bsl, fabs(lb[j]));
    }
    const double bscale = wmax(bsl);
    double fmx = 0.0;
    for (int j = lane; j < n; j += 64) fmx = fmax(fmx, fabs(f[j]));
    const double zbig = DQ_Z_BIG * (1.0 + bscale + wmax(fmx));
    int flag = 0;
    {
        // convexity test: Cholesky of H + CONVEX_EPS max(1, max H_ii) I without pivot floor
        double hd = 0.0;
        for (int j = lane; j < n; j += 64) hd = fmax(hd, fabs(H[(int64_t)j * n + j]));
        const double sh = DQ_CONVEX_EPS * fmax(1.0, wmax(hd));
        for (int e2 = lane; e2 < n * n; e2 += 64) {
            const int i = e2 % n, j = e2 / n;
            K[e2] = H[e2] + (i == j ? sh : 0.0);
        }
        wave_sync();
        if (!chol(-1.0)) flag = -6;
    }
    const double feq = 0.0;                 // no equality rows on this path
    double stat = 0.0, fin = 0.0, csum = 0.0, gscale = 0.0, zmax = 0.0;
    residuals(stat, fin, csum, gscale, zmax);
    if (flag == 0 && !factor()) flag = -8;
    if (flag == 0) {
        solve();
        double tmin = INFINITY, tmax = -INFINITY;
        for (int j = lane; j < n; j += 64) z[j] += dz[j];
        for (int r = lane; r < m; r += 64) { const double t = 1.0 + dtA[r]; tmin = fmin(tmin, t); tmax = fmax(tmax, t); }
        for (int j = lane; j < n; j += 64) {
            if (up_present(j)) { const double t = 1.0 + dtB[j]; tmin = fmin(tmin, t); tmax = fmax(tmax, t); }
            if (lo_present(j)) { const double t = 1.0 + dtB[n + j]; tmin = fmin(tmin, t); tmax = fmax(tmax, t); }
        }
        tmin = wmin(tmin);
        tmax = wmax(tmax);
        const double shp = (tmin <= 0.0) ? 1.0 - tmin : 0.0;
        const double shd = (tmax >= 0.0) ? 1.0 + tmax : 0.0;
        for (int r = lane; r < m; r += 64) { const double t = 1.0 + dtA[r]; tA[r] = t + shp; lA[r] = -t + shd; }
        for (int j = lane; j < n; j += 64) {
            const double tu = 1.0 + dtB[j], tl = 1.0 + dtB[n + j];
            tB[j] = up_present(j) ? tu + shp : 1.0; lB[j] = up_present(j) ? -tu + shd : 0.0;
            tB[n + j] = lo_present(j) ? tl + shp : 1.0; lB[n + j] = lo_present(j) ? -tl + shd : 0.0;
        }
        wave_sync();
    }
    int it = 0;
    double mu = 0.0, mu_min = INFINITY;
    if (flag == 0) {
        for (it = 0; it <= a.max_iter; ++it) {
            residuals(stat, fin, csum, gscale, zmax);
            const double feas = fin;
            mu = csum * minv;
            if (stat <= a.tol_stat * (1.0 + gscale) && feas <= a.tol_feas * (1.0 + bscale) &&
                mu <= a.tol_comp) { flag = 1; break; }
            if (!(isfinite(stat) && isfinite(feas) && isfinite(mu))) { flag = -8; break; }
            if (zmax > zbig) { flag = -3; break; }
            if (mu > DQ_MU_BLOWUP * mu_min && feas > 1e-6 * (1.0 + bscale)) { flag = -2; break; }
            mu_min = fmin(mu_min, mu);
            if (it == a.max_iter) break;
            if (!factor()) { flag = -8; break; }
            for (int r = lane; r < m; r += 64) rcA[r] = tA[r] * lA[r];
            for (int j = lane; j < 2 * n; j += 64) rcB[j] = tB[j] * lB[j];
            wave_sync();
            solve();
            double al = max_step();
            const double mua = comp_after(al) * minv;
            double sg = mua / mu;
            sg = sg * sg * sg;
            const double smu = sg * mu;
            for (int r = lane; r < m; r += 64) rcA[r] = tA[r] * lA[r] + dtA[r] * dlA[r] - smu;
            for (int j = lane; j < n; j += 64) {
                rcB[j] = up_present(j) ? tB[j] * lB[j] + dtB[j] * dlB[j] - smu : 0.0;
                rcB[n + j] = lo_present(j) ? tB[n + j] * lB[n + j] + dtB[n + j] * dlB[n + j] - smu : 0.0;
            }
            wave_sync();
            solve();
            al = fmin(1.0, max_step() * a.tau);
            for (int j = lane; j < n; j += 64) {
                z[j] += al * dz[j];
                if (up_present(j)) { tB[j] += al * dtB[j]; lB[j] += al * dlB[j]; }
                if (lo_present(j)) { tB[n + j] += al * dtB[n + j]; lB[n + j] += al * dlB[n + j]; }
            }
            for (int r = lane; r < m; r += 64) { tA[r] += al * dtA[r]; lA[r] += al * dlA[r]; }
            wave_sync();
        }
    }
    double fv = 0.0;
    for (int j = lane; j < n; j += 64) {
        double hz = 0.0;
        for (int i = 0; i < n; ++i) hz += H[(int64_t)j * n + i] * z[i];
        fv += z[j] * (0.5 * hz + f[j]);
        a.x[(int64_t)inst * n + j] = z[j];
        if (a.lam_lower) a.lam_lower[(int64_t)inst * n + j] = (lo_present(j) && flag != -6) ? lB[n + j] : 0.0;
        if (a.lam_upper) a.lam_upper[(int64_t)inst * n + j] = (up_present(j) && flag != -6) ? lB[j] : 0.0;
    }
    for (int r = lane; r < m; r += 64)
        if (a.lam_ineqlin) a.lam_ineqlin[(int64_t)inst * m + r] = flag != -6 ? lA[r] : 0.0;
    fv = wsum(fv);
    if (lane == 0) {
        if (a.fval) a.fval[inst] = fv;
        a.exitflag[inst] = flag;
        double* so = a.stats + (int64_t)inst * STATS_W;
        so[0] = (double)it; so[1] = stat; so[2] = fmax(feq, fin); so[3] = mu; so[4] = feq; so[5] = fin;
    }
}

hipError_t launch_dense(const DenseKernelArgs& a, hipStream_t st) {
    if (a.n > 256 || a.me > 256) return hipErrorInvalidValue;
    if (a.me == 0 && a.n <= SW_NMAX && small_lds_doubles(a.n, a.m) <= SW_LDS_MAX) {
        hipLaunchKernelGGL(dense_wave_kernel, dim3(a.batch), dim3(64),
                           sizeof(double) * small_lds_doubles(a.n, a.m), st, a);
        return hipGetLastError();
    }
    hipLaunchKernelGGL(dense_ipm_kernel, dim3(a.batch), dim3(DT), 0, st, a);
    return hipGetLastError();
}

}  // namespace bqp
