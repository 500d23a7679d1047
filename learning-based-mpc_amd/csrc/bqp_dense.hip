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
#include <stdlib.h>

#include "bqp_internal.h"
#include "bqp_wave.h"

namespace bqp {

#define DT 256
#define TILE 32
#define DQ_THL 256   // A row-tile bounds kept in LDS (m <= 8192 rows)
#define DQ_RPT 4     // rows per thread of the register-resident row state (m <= DQ_RPT * DT)
typedef double dbl4 __attribute__((ext_vector_type(4)));
#define DQ_PIV_FLOOR 1e-14    // static pivot floor of K, relative to its largest diagonal entry
#define DQ_CONVEX_EPS 1e-10   // shift of the convexity test (relative)
#define DQ_MU_BLOWUP 1e6
#define DQ_Z_BIG 1e12
// round-3 safeguards, as the structured kernel (bqp_ocp.hip) and oracle/dense_ipm.py:
#define DQ_FEAS_GUARD 1e-8    // -2 needs the primal residual above this (relative)
#define DQ_CMAX_K 100.0       // convergence also needs every row's t lam <= CMAX_K tol_comp
#define DQ_SOC_ALPHA 0.1      // predictor step below this on a primal-feasible iterate: no SOC term
#define DQ_RES_SHORT 0.5      // a step shorter than this: the next residuals evaluated exactly
#define DQ_RES_EVERY 8        // and at least every 8th iteration (else the (1 - al) recurrence)
#define DQ_POL_ROUNDS 4       // active-set corrections of the polish
#define DQ_POL_KLDS (16 * 1024) // doubles of K the polish kernel keeps in LDS (n <= 128)

// polish mode of an instance: the launch's, or 2 once the instance's own SQP iteration count has
// reached pol_stall (DenseKernelArgs.pol_it)
__device__ __forceinline__ int pol_mode(const DenseKernelArgs& a, int inst) {
    return (a.pol_it && a.pol_it[inst] >= a.pol_stall) ? 2 : a.polish;
}

struct DWork {
    int64_t K, Y, S, z, y, q, w, dz, dy, rd, re, tA, lA, riA, rcA, dtA, dlA, tB, lB, riB, rcB, dtB, dlB, hr, th,
        total;
    __host__ __device__ static DWork make(int n, int m, int me) {
        DWork o;
        int64_t c = 0;
        // Y / S also hold the polish's [Aeq; active rows] (at most max(me, n) of them)
        const int64_t ne = me > n ? me : n;
        o.K = c; c += (int64_t)n * n;
        o.Y = c; c += (int64_t)n * ne;
        o.S = c; c += ne * ne;
        o.z = c; c += n; o.y = c; c += me; o.q = c; c += n; o.w = c; c += n;
        o.dz = c; c += n; o.dy = c; c += me; o.rd = c; c += n; o.re = c; c += me;
        o.tA = c; c += m; o.lA = c; c += m; o.riA = c; c += m; o.rcA = c; c += m;
        o.dtA = c; c += m; o.dlA = c; c += m;
        // bound rows: 2n (upper: 0..n-1, lower: n..2n-1)
        o.tB = c; c += 2 * n; o.lB = c; c += 2 * n; o.riB = c; c += 2 * n; o.rcB = c; c += 2 * n;
        o.dtB = c; c += 2 * n; o.dlB = c; c += 2 * n;
        // nonzero column bound of each row of A and of each TILE-row tile (dense_ipm_kernel)
        o.hr = c; c += m; o.th = c; c += (m + 31) / 32;
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
    // forceinline: as calls, sc became a generic pointer (flat accesses) and each reduction a call
    __device__ __forceinline__ double sum(double v) {
        v = wave_sum(v);
        const int w = threadIdx.x >> 6;
        __syncthreads();
        if ((threadIdx.x & 63) == 0) sc[w] = v;
        __syncthreads();
        double r = sc[0] + sc[1] + sc[2] + sc[3];
        return r;
    }
    __device__ __forceinline__ double max(double v) {
        v = wmax(v);                    // DPP (was six ds_bpermute shuffles)
        const int w = threadIdx.x >> 6;
        __syncthreads();
        if ((threadIdx.x & 63) == 0) sc[w] = v;
        __syncthreads();
        return fmax(fmax(sc[0], sc[1]), fmax(sc[2], sc[3]));
    }
    __device__ __forceinline__ double min(double v) {
        v = wmin(v);
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
template <int NTH = DT>
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
        // column j of L, and its transpose into the (dead) upper triangle: row j of L' is then
        // contiguous for the backward substitution of chol_solve_w
        for (int i = j + 1 + tid; i < n; i += NTH) {
            const double v = K[(int64_t)j * n + i] / ljj;
            K[(int64_t)j * n + i] = v;
            K[(int64_t)i * n + j] = v;
        }
        __syncthreads();
        // trailing update of the lower triangle: K[c][r] -= L[j][r] * L[j][c], r >= c > j
        const int rem = n - j - 1;
        if (NTH == 256 && rem <= 128) {
            // 16 x 16 thread grid, 8 x 8 entries per thread: rows j+1 + ty + 16 p, columns
            // j+1 + tx + 16 q (the packed-triangle index map below costs a square root and two
            // corrections per entry).  Loads are unconditional from clamped (valid) addresses and
            // all issued before the first store: guarded loads and in-place read-modify-writes
            // were one memory round trip each (~50 chained latencies per pivot at n = 101)
            if (rem == 0) break;
            const int tx = tid & 15, ty = tid >> 4, nbr = (rem + 15) >> 4;   // nbr: block-uniform
            const double* lj = K + (int64_t)j * n + j + 1;
            double lr[8], lc[8];
#pragma unroll
            for (int p = 0; p < 8; ++p) {
                lr[p] = lc[p] = 0.0;
                if (p < nbr) {
                    lr[p] = lj[min(ty + 16 * p, rem - 1)];
                    lc[p] = lj[min(tx + 16 * p, rem - 1)];
                }
            }
            // blocks (p, q) with q <= p < nbr only (the others are empty or upper); two halves of
            // 4 x 8 (a 64-entry register tile spilled)
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                if (4 * h >= nbr) break;
                double t[4][8];
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int qq = 4 * h + q, cc = min(tx + 16 * qq, rem - 1);
#pragma unroll
                    for (int p = 0; p < 8; ++p)
                        if (p >= qq && p < nbr)
                            t[q][p] = K[(int64_t)(j + 1 + cc) * n + j + 1 + min(ty + 16 * p, rem - 1)];
                }
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int qq = 4 * h + q, cc = tx + 16 * qq;
#pragma unroll
                    for (int p = 0; p < 8; ++p) {
                        const int rr = ty + 16 * p;
                        if (p >= qq && p < nbr && cc < rem && rr < rem && rr >= cc)
                            K[(int64_t)(j + 1 + cc) * n + j + 1 + rr] = t[q][p] - lr[p] * lc[qq];
                    }
                }
            }
            __syncthreads();
            continue;
        }
        const int64_t cnt = (int64_t)rem * (rem + 1) / 2;
        for (int64_t e = tid; e < cnt; e += NTH) {
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

// trailing update of pivot j over NB = ceil(rem / 16) block rows (compile-time, so no uniform
// branch per block: those cost more than the LDS traffic of the update), thread (tx, ty) owning
// rows j+1 + ty + 16 p and columns j+1 + tx + 16 q, blocks q <= p.  Loads clamped and
// unconditional; stores of entries outside the lower trailing triangle go to a per-lane junk
// slot instead of a masked store.  Also writes the scaled column j to the upper triangle.
template <int NB>
__device__ __forceinline__ void chol_upd(double* K, int n, int j, int rem, double inv, double* junk) {
    const int tid = threadIdx.x, tx = tid & 15, ty = tid >> 4;
    const double* lj = K + (int64_t)j * n + j + 1;
    double lr[NB], lc[NB];
#pragma unroll
    for (int p = 0; p < NB; ++p) {
        lr[p] = lj[min(ty + 16 * p, rem - 1)];
        lc[p] = lj[min(tx + 16 * p, rem - 1)];
    }
    double* jk = junk + (tid & 63);
#pragma unroll
    for (int p = 0; p < NB; ++p) { lr[p] *= inv; lc[p] *= inv; }
    if (ty == 0) {
#pragma unroll
        for (int q = 0; q < NB; ++q) {
            const int cc = tx + 16 * q;
            if (cc < rem) K[(int64_t)(j + 1 + cc) * n + j] = lc[q];
        }
    }
    constexpr int NH = (NB + 3) / 4;
#pragma unroll
    for (int h = 0; h < NH; ++h) {
        double t[4][NB];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int qq = 4 * h + q, cc = min(tx + 16 * qq, rem - 1);
#pragma unroll
            for (int p = 0; p < NB; ++p)
                if (qq < NB && p >= qq)
                    t[q][p] = K[(int64_t)(j + 1 + cc) * n + j + 1 + min(ty + 16 * p, rem - 1)];
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int qq = 4 * h + q, cc = tx + 16 * qq;
#pragma unroll
            for (int p = 0; p < NB; ++p) {
                if (qq < NB && p >= qq) {
                    const int rr = ty + 16 * p;
                    double* dst = (cc < rem && rr < rem && rr >= cc) ? K + (int64_t)(j + 1 + cc) * n + j + 1 + rr : jk;
                    *dst = t[q][p] - lr[p] * lc[qq];
                }
            }
        }
    }
}

// Cholesky for n <= 128 on 256 threads with ONE barrier per pivot (block_cholesky has three):
// every thread reads the pivot and column j itself and scales by 1/l_jj in registers; the scaled
// column goes to the upper triangle (row j of L'), which nothing reads during the sweep, and the
// lower triangle is filled from it at the end; l_jj is stored one pivot later (no thread reads
// K[j-1][j-1] at pivot j).  The trailing update is block_cholesky's 16 x 16 grid.  Same result
// layout as block_cholesky (L lower, L' upper).
__device__ __forceinline__ bool chol_1b(double* K, int n, double fl, double* junk) {   // inlined: K stays LDS
    const int tid = threadIdx.x, tx = tid & 15, ty = tid >> 4;
    double lprev = 0.0;
    for (int j = 0; j < n; ++j) {
        double d = K[(int64_t)j * n + j];
        if (fl >= 0.0 && !(d > fl)) d = fl;
        if (!(d > 0.0)) { __syncthreads(); return false; }   // uniform: every thread read d
        const double ljj = sqrt(d), inv = 1.0 / ljj;
        if (tid == 0 && j > 0) K[(int64_t)(j - 1) * n + j - 1] = lprev;
        lprev = ljj;
        const int rem = n - j - 1;
        switch ((rem + 15) >> 4) {      // block-uniform; each case branch-free inside
            case 1: chol_upd<1>(K, n, j, rem, inv, junk); break;
            case 2: chol_upd<2>(K, n, j, rem, inv, junk); break;
            case 3: chol_upd<3>(K, n, j, rem, inv, junk); break;
            case 4: chol_upd<4>(K, n, j, rem, inv, junk); break;
            case 5: chol_upd<5>(K, n, j, rem, inv, junk); break;
            case 6: chol_upd<6>(K, n, j, rem, inv, junk); break;
            case 7: chol_upd<7>(K, n, j, rem, inv, junk); break;
            case 8: chol_upd<8>(K, n, j, rem, inv, junk); break;
            default: break;
        }
        __syncthreads();
    }
    if (tid == 0) K[(int64_t)(n - 1) * n + n - 1] = lprev;
    for (int c = ty; c < n; c += 16)                 // lower <- upper: L(r, c) = K[r n + c]
        for (int r = c + 1 + tx; r < n; r += 16) K[(int64_t)c * n + r] = K[(int64_t)r * n + c];
    __syncthreads();
    return true;
}

// two pivots j, j + 1 per barrier (rank-2 trailing update): L(r, j) = K(r, j) / l_jj and
// L(r, j+1) = (K(r, j+1) - L(r, j) a) / l_{j+1,j+1} (a = L(j+1, j)) formed in registers from
// the unupdated columns, then K(r, c) -= L(r, j) L(c, j) + L(r, j+1) L(c, j+1) over the trailing
// block from row / column j + 2 - one pass over the trailing triangle and one barrier for the
// two pivots (chol_upd: one each).  Same operation order per entry as two chol_upd steps.
template <int NB>
__device__ __forceinline__ void chol_upd2(double* K, int n, int j, int rem2, double inv0, double a,
                                          double inv1, double* junk) {
    const int tid = threadIdx.x, tx = tid & 15, ty = tid >> 4;
    const double* k0 = K + (int64_t)j * n + j + 2;         // column j, rows j + 2 ..
    const double* k1 = K + (int64_t)(j + 1) * n + j + 2;   // column j + 1, rows j + 2 ..
    double r0[NB], c0[NB], r1[NB], c1[NB];
#pragma unroll
    for (int p = 0; p < NB; ++p) {
        const int ir = min(ty + 16 * p, rem2 - 1), ic = min(tx + 16 * p, rem2 - 1);
        r0[p] = k0[ir]; c0[p] = k0[ic];
        r1[p] = k1[ir]; c1[p] = k1[ic];
    }
#pragma unroll
    for (int p = 0; p < NB; ++p) {
        r0[p] *= inv0; c0[p] *= inv0;
        r1[p] = (r1[p] - r0[p] * a) * inv1;
        c1[p] = (c1[p] - c0[p] * a) * inv1;
    }
    if (ty == 0) {             // rows j and j + 1 of L' (upper triangle) from row j + 2 on
#pragma unroll
        for (int q = 0; q < NB; ++q) {
            const int cc = tx + 16 * q;
            if (cc < rem2) {
                K[(int64_t)(j + 2 + cc) * n + j] = c0[q];
                K[(int64_t)(j + 2 + cc) * n + j + 1] = c1[q];
            }
        }
    }
    double* jk = junk + (tid & 63);
    constexpr int NH = (NB + 3) / 4;
#pragma unroll
    for (int h = 0; h < NH; ++h) {
        double t[4][NB];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int qq = 4 * h + q, cc = min(tx + 16 * qq, rem2 - 1);
#pragma unroll
            for (int p = 0; p < NB; ++p)
                if (qq < NB && p >= qq)
                    t[q][p] = K[(int64_t)(j + 2 + cc) * n + j + 2 + min(ty + 16 * p, rem2 - 1)];
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int qq = 4 * h + q, cc = tx + 16 * qq;
#pragma unroll
            for (int p = 0; p < NB; ++p) {
                if (qq < NB && p >= qq) {
                    const int rr = ty + 16 * p;
                    double* dst = (cc < rem2 && rr < rem2 && rr >= cc) ? K + (int64_t)(j + 2 + cc) * n + j + 2 + rr : jk;
                    *dst = (t[q][p] - r0[p] * c0[qq]) - r1[p] * c1[qq];
                }
            }
        }
    }
}

// chol_1b with two pivots per barrier (chol_upd2); a last odd pivot as in chol_1b
__device__ __forceinline__ bool chol_2b(double* K, int n, double fl, double* junk) {   // inlined: K stays LDS
    const int tid = threadIdx.x, tx = tid & 15, ty = tid >> 4;
    double lp0 = 0.0, lp1 = 0.0;
    int jp = -1;                      // the previous step's first pivot (its diagonals are stored late)
    int j = 0;
    for (; j + 1 < n; j += 2) {
        double d0 = K[(int64_t)j * n + j];
        if (fl >= 0.0 && !(d0 > fl)) d0 = fl;
        if (!(d0 > 0.0)) { __syncthreads(); return false; }   // uniform: every thread read d0
        const double l00 = sqrt(d0), inv0 = 1.0 / l00;
        const double a = K[(int64_t)j * n + j + 1] * inv0;     // L(j+1, j)
        double d1 = K[(int64_t)(j + 1) * n + j + 1] - a * a;
        if (fl >= 0.0 && !(d1 > fl)) d1 = fl;
        if (!(d1 > 0.0)) { __syncthreads(); return false; }
        const double l11 = sqrt(d1), inv1 = 1.0 / l11;
        if (tid == 0) {
            if (jp >= 0) {
                K[(int64_t)jp * n + jp] = lp0;
                K[(int64_t)(jp + 1) * n + jp + 1] = lp1;
            }
            K[(int64_t)(j + 1) * n + j] = a;                  // row j of L', entry j + 1
        }
        jp = j; lp0 = l00; lp1 = l11;
        const int rem2 = n - j - 2;
        switch ((rem2 + 15) >> 4) {     // block-uniform; each case branch-free inside
            case 1: chol_upd2<1>(K, n, j, rem2, inv0, a, inv1, junk); break;
            case 2: chol_upd2<2>(K, n, j, rem2, inv0, a, inv1, junk); break;
            case 3: chol_upd2<3>(K, n, j, rem2, inv0, a, inv1, junk); break;
            case 4: chol_upd2<4>(K, n, j, rem2, inv0, a, inv1, junk); break;
            case 5: chol_upd2<5>(K, n, j, rem2, inv0, a, inv1, junk); break;
            case 6: chol_upd2<6>(K, n, j, rem2, inv0, a, inv1, junk); break;
            case 7: chol_upd2<7>(K, n, j, rem2, inv0, a, inv1, junk); break;
            case 8: chol_upd2<8>(K, n, j, rem2, inv0, a, inv1, junk); break;
            default: break;
        }
        __syncthreads();
    }
    if (tid == 0 && jp >= 0) {
        K[(int64_t)jp * n + jp] = lp0;
        K[(int64_t)(jp + 1) * n + jp + 1] = lp1;
    }
    if (j < n) {                      // the last pivot of an odd n (nothing trails it)
        double d = K[(int64_t)j * n + j];
        if (fl >= 0.0 && !(d > fl)) d = fl;
        __syncthreads();              // every thread has read d before thread 0 overwrites it
        if (!(d > 0.0)) return false;
        if (tid == 0) K[(int64_t)j * n + j] = sqrt(d);
    }
    for (int c = ty; c < n; c += 16)                 // lower <- upper: L(r, c) = K[r n + c]
        for (int r = c + 1 + tx; r < n; r += 16) K[(int64_t)c * n + r] = K[(int64_t)r * n + c];
    __syncthreads();
    return true;
}

// ------------------------------------------------------------------------------------------
// Blocked Cholesky on register tiles (round 5, n <= 128).  The lower block triangle of K in 16 x
// 16 tiles is held by the four waves exactly as the MFMA A'DA leaves it: tile t = I (I+1)/2 + J
// (J <= I) on wave t % 4 as acc[t / 4], lane l = 16 k4 + c16, register e holding K(16 I + k4 + 4 e,
// 16 J + c16); a diagonal tile holds the whole symmetric block, padding rows / columns (>= n) the
// identity.  Per block column J: the owner of tile (J, J) factors it in registers (D), the owners
// of the tiles (I, J) below solve them against it (P), and every tile right of column J takes the
// update K_IK -= L_IJ L_KJ' as four v_mfma_f64_16x16x4 (U) with operands read from the factor in
// LDS: two workgroup barriers per block column (chol_2b: one per two pivots, 51 at n = 101).  Per
// entry the in-block updates run in pivot order as chol_2b's; the updates of earlier block columns
// are summed by the matrix cores.  The factor leaves K as chol_2b does: L lower, L' upper, l_jj on
// the diagonal.

// pivot P of a diagonal tile T (one wave): l_PP = sqrt(K_PP) (pivot floor fl >= 0; fl < 0: fail on a
// non-positive pivot), column P scaled by 1 / l_PP - broadcast along each 16-lane row (row
// newbcast: every lane gets L(r, P) of its rows) and, for the lane's own column c16, L(c16, P) =
// K(P, c16) / l_PP from row P (symmetric storage) by row swaps (xrow_bcast) - then the rank-1 update of the
// trailing block; row P of the tile becomes L' (upper), column P L (lower).
template <int P>
__device__ __forceinline__ void dtile_piv(dbl4& T, int k4, int c16, double fl, bool& ok, double& rvl, int lane) {
    constexpr int EP = P >> 2, SRC = 16 * (P & 3) + P;
    double d = rl(T[EP], SRC);
    if (fl >= 0.0 && !(d > fl)) d = fl;
    if (!(d > 0.0)) ok = false;          // wave-uniform
    // 1 / l_PP: the hardware reciprocal square root and two Newton steps (the pivot chain's
    // latency: sqrt then a division were ~25 dependent instructions), l_PP = d / sqrt(d)
    double inv = __builtin_amdgcn_rsq(d);
    inv = inv * fma(-0.5 * d * inv, inv, 1.5);
    inv = inv * fma(-0.5 * d * inv, inv, 1.5);
    const double ljj = d * inv;
    const double xc = xrow_bcast<P & 3>(T[EP]) * inv;
    double xr[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) xr[e] = rbc<P>(T[e]) * inv;
    // branch-free (as selects the per-lane cases were exec-mask branches)
    const bool cg = c16 > P, ce = c16 == P;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        const int r = k4 + 4 * e;
        const double below = cg ? fma(-xr[e], xc, T[e]) : (ce ? xr[e] : T[e]);
        const double onrow = cg ? xc : (ce ? ljj : T[e]);
        T[e] = r > P ? below : (r == P ? onrow : T[e]);
    }
    rvl = (lane == P) ? inv : rvl;       // lane P keeps 1 / l_PP (stored after the 16 pivots)
    if constexpr (P + 1 < 16) dtile_piv<P + 1>(T, k4, c16, fl, ok, rvl, lane);
}

// column P of a panel tile (I, J): L(r, P) = K(r, P) / l_PP reaches the lane's 16-lane row, the
// later columns c16 > P take - L(r, P) L(c16, P); lc = the lane's row of the diagonal factor in LDS
// (L(16 J + c16, 16 J + q) at lc[q n]), rv the reciprocal pivots (both read at the use: held in
// registers across the unrolled tiles they spilled)
template <int P>
__device__ __forceinline__ void ptile_piv(dbl4& T, int c16, const double* lc, int n, const double* rv) {
    const double ri = rv[P], lv = lc[(int64_t)P * n];
    double x[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) x[e] = rbc<P>(T[e]) * ri;
    const bool cg = c16 > P, ce = c16 == P;
#pragma unroll
    for (int e = 0; e < 4; ++e) T[e] = cg ? fma(-x[e], lv, T[e]) : (ce ? x[e] : T[e]);
    if constexpr (P + 1 < 16) ptile_piv<P + 1>(T, c16, lc, n, rv);
}

// the tiles of wave w: slots 0 and 1 the diagonal tiles (J, J) with J = w, w + 4 (the Cholesky's
// diagonal factor then works on a fixed register tile: a runtime slot index put the tiles in
// scratch memory), slots 2 .. 8 the off-diagonal tiles o = 4 (u - 2) + w in row-major order over
// the strictly lower block triangle; I = -1: no tile.  nbk <= 8 (n <= 128): at most 2 + 7 slots.
__device__ __forceinline__ void tile_of(int w, int u, int nbk, int& I, int& J) {
    I = -1; J = 0;
    if (u < 2) {
        const int d = w + 4 * u;
        if (d < nbk) { I = d; J = d; }
        return;
    }
    const int o = 4 * (u - 2) + w;
    if (o >= nbk * (nbk - 1) / 2) return;
    int i = 1;
    while ((i + 1) * i / 2 <= o) ++i;
    I = i;
    J = o - i * (i - 1) / 2;
}

#ifdef BQP_DSTAMPS
#define TST_ARGS , unsigned long long* dacc, unsigned long long& dlast
#define TST_PASS , dst_acc, dst_last
#define TST(id)                                                            \
    do {                                                                   \
        __builtin_amdgcn_s_waitcnt(0);                                     \
        const unsigned long long _t = __builtin_amdgcn_s_memtime();        \
        dacc[id] += _t - dlast;                                            \
        dlast = _t;                                                        \
    } while (0)
// the same without waiting for vector-memory loads in flight (LDS / scalar only): sections
// that overlap a copy; chol_solve_w's stamps (optional pointers: only dense_ipm_kernel passes them)
#define TSTN(acc_, last_, id)                                              \
    do {                                                                   \
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                 \
        const unsigned long long _t = __builtin_amdgcn_s_memtime();        \
        (acc_)[id] += _t - (last_);                                        \
        (last_) = _t;                                                      \
    } while (0)
#define TSW_ARGS , unsigned long long* dacc = nullptr, unsigned long long* dlastp = nullptr
#define TSW_PASS , dst_acc, &dst_last
#define TSW(id) do { if (dacc) TSTN(dacc, *dlastp, id); } while (0)
#else
#define TST_ARGS
#define TST_PASS
#define TST(id) do { } while (0)
#define TSW_ARGS
#define TSW_PASS
#define TSW(id) do { } while (0)
#endif
// the diagonal tile J in registers: symmetric from its lower triangle (the MFMA A'DA forms K(i, j)
// and K(j, i) with different rounding; chol_2b read the lower triangle only - with both, the
// factor of the extreme late-iteration matrices left fp64 range), the 16 pivots, the tile to LDS
__device__ __forceinline__ bool dtile(dbl4& T, int J, double* K, int n, double fl, double* rv, int lane,
                                      int k4, int c16) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        const int r = k4 + 4 * e, i = 16 * J + r, j = 16 * J + c16;
        if (r >= c16 && i < n) K[(int64_t)j * n + i] = T[e];
    }
    wave_sync();
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        const int r = k4 + 4 * e;
        if (r < c16 && 16 * J + c16 < n) T[e] = K[(int64_t)(16 * J + r) * n + 16 * J + c16];
    }
    bool ok = true;
    double rvl = 0.0;
    dtile_piv<0>(T, k4, c16, fl, ok, rvl, lane);
    if (lane < 16) rv[lane] = rvl;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        const int i = 16 * J + k4 + 4 * e, j = 16 * J + c16;
        if (i < n && j < n) K[(int64_t)j * n + i] = T[e];
    }
    return ok;
}

template <int TPW>
__device__ __forceinline__ bool tile_chol(dbl4 (&acc)[TPW], const int (&tI)[TPW], const int (&tJ)[TPW],
                                          double* K, int n, double fl, double* rv TST_ARGS) {
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int c16 = lane & 15, k4 = lane >> 4;
    const int nbk = (n + 15) >> 4;
    // D: the diagonal tile J by its owner (wave J % 4, slot J / 4): the 16 pivots, L_JJ to LDS, the
    // reciprocal pivots and the fail flag to rv
    auto dfac = [&](int J) __attribute__((always_inline)) {
        bool ok = true;
        if (J < 4) ok = dtile(acc[0], J, K, n, fl, rv, lane, k4, c16);
        else       ok = dtile(acc[1], J, K, n, fl, rv, lane, k4, c16);
        if (lane == 0) rv[16] = ok ? 0.0 : 1.0;
    };
    if (wv == 0) dfac(0);
    for (int J = 0; J < nbk; ++J) {
        TST(12);
        __syncthreads();
        TST(13);
        if (rv[16] != 0.0) { __syncthreads(); return false; }   // uniform
        if (J + 1 == nbk) break;
        // ---- P: the tiles (I, J), I > J, against L_JJ ----
        {
            // L(16 J + c16, 16 J + q) at lc[q n] (used for q < c16: the lower triangle)
            const double* lc = K + (int64_t)(16 * J) * n + min(16 * J + c16, n - 1);
#pragma unroll
            for (int u = 0; u < TPW; ++u) {
                if (tI[u] < 0 || tJ[u] != J || tI[u] == J) continue;   // wave-uniform
                ptile_piv<0>(acc[u], c16, lc, n, rv);
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int i = 16 * tI[u] + k4 + 4 * e, j = 16 * J + c16;
                    if (i < n) {
                        K[(int64_t)j * n + i] = acc[u][e];          // L (lower)
                        K[(int64_t)i * n + j] = acc[u][e];          // L' (upper)
                    }
                }
            }
        }
        TST(14);
        __syncthreads();
        TST(15);
        // ---- U: every tile (I, K), K > J: K_IK -= L_IJ L_KJ' on the matrix cores ----
        // Lookahead (round 6): the diagonal tiles (slots 0, 1) first; the owner of tile J + 1 then
        // factors it (D of the next block column) while the other waves are still updating their
        // off-diagonal tiles, instead of all waves waiting at the next barrier for the diagonal
        // pivot chain.  Each tile takes the same operations in the same order as before (the
        // factor is bitwise the same); D writes block (J + 1, J + 1) of K and rv, which the
        // remaining updates of column J do not read.
        auto upd = [&](int u) __attribute__((always_inline)) {
            if (tI[u] < 0 || tJ[u] <= J) return;
            const int rA = 16 * tI[u] + c16, rB = 16 * tJ[u] + c16;
            double av[4], bv[4];
#pragma unroll
            for (int s4 = 0; s4 < 4; ++s4) {
                const int64_t col = (int64_t)(16 * J + 4 * s4 + k4) * n;
                av[s4] = rA < n ? -K[col + rA] : 0.0;
                bv[s4] = rB < n ? K[col + rB] : 0.0;
            }
#pragma unroll
            for (int s4 = 0; s4 < 4; ++s4)
                acc[u] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[s4], bv[s4], acc[u], 0, 0, 0);
        };
        upd(0);
        if constexpr (TPW > 1) upd(1);
        if (((J + 1) & 3) == wv) dfac(J + 1);
#pragma unroll
        for (int u = 2; u < TPW; ++u) upd(u);
        TST(16);
    }
    __syncthreads();
    return true;
}

// solve L L' x = b in place (x in LDS vector xs of length n), thread-parallel dot products
template <int NTH = DT, class R = Red>
__device__ void chol_solve_vec(const double* L, int n, double* xs, R& red) {
    // forward L y = b
    for (int i = 0; i < n; ++i) {
        double part = 0.0;
        for (int k = threadIdx.x; k < i; k += NTH) part += L[(int64_t)k * n + i] * xs[k];
        const double s = red.sum(part);
        if (threadIdx.x == 0) xs[i] = (xs[i] - s) / L[(int64_t)i * n + i];
        __syncthreads();
    }
    // backward L' x = y
    for (int i = n - 1; i >= 0; --i) {
        double part = 0.0;
        for (int k = i + 1 + threadIdx.x; k < n; k += NTH) part += L[(int64_t)i * n + k] * xs[k];
        const double s = red.sum(part);
        if (threadIdx.x == 0) xs[i] = (xs[i] - s) / L[(int64_t)i * n + i];
        __syncthreads();
    }
}

// one 16-entry block of the substitutions: the block's entries sit in one 16-lane row of a slot
// (lane jl of the row holds entry e0 + jl, as its unscaled residual r).  Entry J's value is
// r_J d_J (d_J its reciprocal pivot); it updates the row's later (forward) or earlier (backward)
// entries as r_i -= (L_iJ d_J) r_J with the coefficients L_iJ d_J formed before the chain (zero
// outside the triangle, past n and off the block's row), so each of the 16 dependent steps is one
// DPP row broadcast (v_mov_b64_dpp row_newbcast) and one FMA (round 4's step - broadcast of x and
// of d, product, masked update, select - took ~110 cycles); the entries are scaled after it
template <int JJ>
__device__ __forceinline__ void tri_coef(double (&lcs)[16], const double (&lc)[16], double dv, int jl,
                                         bool inrow, int nval, bool fwd) {
    // the broadcast outside any lane condition (DPP under an exec mask reads 0 from inactive lanes)
    const double db = rbc<JJ>(dv);
    const bool ok = inrow && JJ < nval && (fwd ? jl > JJ : jl < JJ);
    lcs[JJ] = (ok ? -lc[JJ] : 0.0) * db;
    if constexpr (JJ + 1 < 16) tri_coef<JJ + 1>(lcs, lc, dv, jl, inrow, nval, fwd);
}
template <int JJ, bool FWD>
__device__ __forceinline__ void tri_blk(double& rv, const double (&lcs)[16]) {
    constexpr int J = FWD ? JJ : 15 - JJ;
    rv = fma(lcs[J], rbc<J>(rv), rv);
    if constexpr (JJ + 1 < 16) tri_blk<JJ + 1, FWD>(rv, lcs);
}

// solve L L' x = b in place (xs in LDS, n <= 256) by the first wave alone: lane l keeps entries
// l, l + 64, .. in registers.  Blocked substitutions (round 4): 16-entry diagonal blocks solved
// inside one 16-lane row (DPP row broadcasts, no scalar round trip per entry), each solved block
// published through LDS and applied to the remaining entries as a 16-column update (the
// column-at-a-time form spent ~530 cycles per entry on its readlane / load / update chain).  L's
// column j (forward) and row i (backward, the upper triangle block_cholesky leaves) are both at
// [j n + e].  No workgroup barrier inside; every thread calls it.
__device__ __forceinline__ void chol_solve_w_body(const double* L, int n, double* xs TSW_ARGS) {
    if (threadIdx.x < 64 && n > 0) {
        const int l = threadIdx.x, jl = l & 15, rw = l >> 4;
        double xr[4], dr[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int k = min(l + 64 * q, n - 1);
            xr[q] = (l + 64 * q < n) ? xs[l + 64 * q] : 0.0;
            dr[q] = 1.0 / L[(int64_t)k * n + k];   // the pivots' reciprocals
        }
        const int nb = (n + 15) >> 4;
        for (int pass = 0; pass < 2; ++pass) {
            const bool fwd = pass == 0;
            for (int bi = 0; bi < nb; ++bi) {
                const int b = fwd ? bi : nb - 1 - bi;
                const int qb = b >> 2, e0 = 16 * b;
                const bool inrow = rw == (b & 3);
                double xv = 0.0, dv = 0.0;
#pragma unroll
                for (int q = 0; q < 4; ++q) if (q == qb) { xv = xr[q]; dv = dr[q]; }
                // the block's coefficients of this lane's entry e0 + jl: [(e0 + jj) n + e0 + jl]
                double lc[16];
                const int ec = min(e0 + jl, n - 1);
#pragma unroll
                for (int jj = 0; jj < 16; ++jj) lc[jj] = L[(int64_t)min(e0 + jj, n - 1) * n + ec];
                // the last block may be partial: steps past n are skipped (backward: they come
                // first and would reach valid entries)
                double lcs[16];
                tri_coef<0>(lcs, lc, dv, jl, inrow, n - e0, fwd);
                TSW(17);
                if (fwd) tri_blk<0, true>(xv, lcs);
                else     tri_blk<0, false>(xv, lcs);
                if (inrow) xv *= dv;
                TSW(18);
#pragma unroll
                for (int q = 0; q < 4; ++q) if (q == qb) xr[q] = xv;
                // publish the block, then the 16-column update of the entries after (forward) /
                // before (backward) it
                if (inrow) xs[e0 + jl] = xv;
                wave_sync();
                double xb[16];
#pragma unroll
                for (int jj = 0; jj < 16; ++jj) {   // unconditional loads (clamped), then the select
                    const double v = xs[min(e0 + jj, n - 1)];
                    xb[jj] = (e0 + jj < n) ? v : 0.0;
                }
                TSW(19);
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int e = l + 64 * q;
                    const bool upd = e < n && (fwd ? e >= e0 + 16 : e < e0);
                    if (!upd) continue;
                    double ac4[4] = {0.0, 0.0, 0.0, 0.0};   // four chains of 4 FMAs, not one of 16
#pragma unroll
                    for (int jj = 0; jj < 16; ++jj)
                        ac4[jj & 3] = fma(L[(int64_t)min(e0 + jj, n - 1) * n + e], xb[jj], ac4[jj & 3]);
                    xr[q] -= (ac4[0] + ac4[1]) + (ac4[2] + ac4[3]);
                }
                wave_sync();
                TSW(20);
            }
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) if (l + 64 * q < n) xs[l + 64 * q] = xr[q];
    }
    __syncthreads();
}
// The same substitutions on all four waves of the workgroup (round 6; dense_ipm_kernel with the
// factor in LDS, n <= 256): wave w keeps entry l + 64 w of lane l in a register.  Block b's
// 16-step chain runs in its owner wave (w = b / 4, the 16-lane row b % 4), which publishes the
// solved block through LDS; after one workgroup barrier every wave applies the block to its own
// entries.  One chain per block on the critical path and the 16-column updates spread over 256
// lanes instead of four entries per lane on wave 0 while three waves idled; each entry receives
// the same updates in the same order as in chol_solve_w_body (bitwise the same solution).
__device__ __forceinline__ void chol_solve_wg(const double* L, int n, double* xs) {
    const int tid = threadIdx.x, l = tid & 63, w = tid >> 6, jl = l & 15, rw = l >> 4;
    const int e = l + 64 * w;
    double xr = (e < n) ? xs[e] : 0.0;
    const int ek = min(e, n - 1);
    const double dr = 1.0 / L[(int64_t)ek * n + ek];       // the pivots' reciprocals
    const int nb = (n + 15) >> 4;
    for (int pass = 0; pass < 2; ++pass) {
        const bool fwd = pass == 0;
        for (int bi = 0; bi < nb; ++bi) {
            const int b = fwd ? bi : nb - 1 - bi;
            const int e0 = 16 * b;
            if (w == (b >> 2)) {                               // wave-uniform: the block's owner
                const bool inrow = rw == (b & 3);
                double xv = xr;
                double lc[16];
                const int ec = min(e0 + jl, n - 1);
#pragma unroll
                for (int jj = 0; jj < 16; ++jj) lc[jj] = L[(int64_t)min(e0 + jj, n - 1) * n + ec];
                double lcs[16];
                tri_coef<0>(lcs, lc, dr, jl, inrow, n - e0, fwd);
                if (fwd) tri_blk<0, true>(xv, lcs);
                else     tri_blk<0, false>(xv, lcs);
                if (inrow) xv *= dr;
                xr = xv;
                if (inrow) xs[e0 + jl] = xv;                    // publish the block
            }
            __syncthreads();
            double xb[16];
#pragma unroll
            for (int jj = 0; jj < 16; ++jj) {                   // unconditional loads (clamped), then the select
                const double v = xs[min(e0 + jj, n - 1)];
                xb[jj] = (e0 + jj < n) ? v : 0.0;
            }
            const bool upd = e < n && (fwd ? e >= e0 + 16 : e < e0);
            if (upd) {
                double ac4[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
                for (int jj = 0; jj < 16; ++jj)
                    ac4[jj & 3] = fma(L[(int64_t)min(e0 + jj, n - 1) * n + e], xb[jj], ac4[jj & 3]);
                xr -= (ac4[0] + ac4[1]) + (ac4[2] + ac4[3]);
            }
        }
        __syncthreads();                                        // the passes publish the same slots
    }
    if (e < n) xs[e] = xr;
    __syncthreads();
}

// the called form (factor / vector in global memory or generic pointers); dense_ipm_kernel's
// factor in LDS inlines the body, so that L and xs are ds_* accesses (the call made them flat
// loads, ~4 solve-phase round trips slower per block)
__device__ void chol_solve_w(const double* L, int n, double* xs) { chol_solve_w_body(L, n, xs); }

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

// ------------------------------------------------------------------------------------------
// active-set polish after a 0 / -8 exit (oracle/dense_ipm.py::_polish): the rows with lam > t
// join the equality rows and the equality-constrained QP is solved directly from z - K = H +
// rho G_a'G_a (rho = max(1, max H_ii): positive definite whenever the reduced problem is), the
// Schur complement of Ex = [Aeq; G_a], one exact Newton step.  Accepted when stationarity
// <= tol_stat (1 + |Hz + f|), every row and the equalities within 1e-12 (1 + |data|) and no
// active multiplier below -1e-9 (1 + max); otherwise rows with negative multipliers leave,
// violated rows enter (DQ_POL_ROUNDS rounds).  Scratch: the instance's global workspace
// (its IPM vectors are dead by now); the IPM state (z, y, t, lam) is overwritten only on
// acceptance.  Rows r: 0..m-1 the rows of A, m + j the upper bound of j, m + n + j the lower.
struct DPolish {
    int n, m, me;
    const double *H, *f, *A, *b, *E, *e, *lb, *ub;
    double *z, *y, *tA, *lA, *tB, *lB;
    double* W;             // the instance's DWork
    double bscale, tol_stat;
    double* Kl;            // the n x n matrix K in LDS (dense_polish_kernel when it fits), else null:
                           // the workspace's (round 6: the Cholesky and the n-long substitutions of the
                           // Schur columns were L2 round trips, ~65 % of a polish in its stamps)
};

#ifdef BQP_DSTAMPS
// diagnostic build only: s_memtime cycles per phase of the polish (every 16th instance of a launch
// prints its phases at exit)
#define PST_DECL                                                           \
    unsigned long long pst_last = __builtin_amdgcn_s_memtime(), pst_acc[9]; \
    int pst_rounds = 0;                                                    \
    _Pragma("unroll") for (int i_ = 0; i_ < 9; ++i_) pst_acc[i_] = 0
#define PST(id)                                                            \
    do {                                                                   \
        __builtin_amdgcn_s_waitcnt(0);                                     \
        const unsigned long long _t = __builtin_amdgcn_s_memtime();        \
        pst_acc[id] += _t - pst_last;                                      \
        pst_last = _t;                                                     \
    } while (0)
#define PST_RET(v)                                                         \
    do {                                                                   \
        if ((blockIdx.x & 15) == 0 && threadIdx.x == 0)                    \
            printf("PSTAMPS n %d m %d rounds %d ret %d actlist %llu K %llu cholK %llu Y %llu S %llu "    \
                   "cholS %llu mult %llu checks %llu corr %llu\n", n, m, pst_rounds, (int)(v), pst_acc[0], \
                   pst_acc[1], pst_acc[2], pst_acc[3], pst_acc[4], pst_acc[5], pst_acc[6], pst_acc[7],    \
                   pst_acc[8]);                                            \
        return (v);                                                        \
    } while (0)
#define PST_ROUND() (++pst_rounds)
#else
#define PST_DECL do { } while (0)
#define PST(id) do { } while (0)
#define PST_RET(v) return (v)
#define PST_ROUND() do { } while (0)
#endif

template <int NTH, class R>
__device__ bool dense_polish(const DPolish p, double* sc, double* xs) {
    R red{sc};
    PST_DECL;
    const int n = p.n, m = p.m, me = p.me, tid = threadIdx.x;
    const DWork L = DWork::make(n, m, me);
    double *K = p.Kl ? p.Kl : p.W + L.K, *Y = p.W + L.Y, *S = p.W + L.S;
    double *actA = p.W + L.rcA, *actB = p.W + L.rcB, *nuA = p.W + L.dlA, *nuB = p.W + L.dlB;
    double *riA = p.W + L.riA, *riB = p.W + L.riB, *idx = p.W + L.dtB, *zn = p.W + L.dz;
    double *w = p.W + L.w, *mult = p.W + L.rd, *ra = p.W + L.q;
    auto upp = [&](int j) -> bool { return p.ub && isfinite(p.ub[j]); };
    auto lop = [&](int j) -> bool { return p.lb && isfinite(p.lb[j]); };
    // entry i of row r and its right-hand side
    auto g = [&](int r, int i) -> double {
        if (r < m) return p.A[(int64_t)i * m + r];
        if (r < m + n) return (i == r - m) ? 1.0 : 0.0;
        return (i == r - m - n) ? -1.0 : 0.0;
    };
    auto hr = [&](int r) -> double { return r < m ? p.b[r] : (r < m + n ? p.ub[r - m] : -p.lb[r - m - n]); };
    auto gdot = [&](int r, const double* v) -> double {
        if (r < m) {
            double s = 0.0;
            for (int i = 0; i < n; ++i) s += p.A[(int64_t)i * m + r] * v[i];
            return s;
        }
        return r < m + n ? v[r - m] : -v[r - m - n];
    };
    for (int r = tid; r < m; r += NTH) actA[r] = p.lA[r] > p.tA[r] ? 1.0 : 0.0;
    for (int j = tid; j < n; j += NTH) {
        actB[j] = (upp(j) && p.lB[j] > p.tB[j]) ? 1.0 : 0.0;
        actB[n + j] = (lop(j) && p.lB[n + j] > p.tB[n + j]) ? 1.0 : 0.0;
    }
    double hd = 0.0;
    for (int j = tid; j < n; j += NTH) hd = fmax(hd, fabs(p.H[(int64_t)j * n + j]));
    const double rho = fmax(1.0, red.max(hd));
    const double tf = 1e-12 * (1.0 + p.bscale);
    for (int round = 0; round < DQ_POL_ROUNDS; ++round) {
        PST_ROUND();
        __syncthreads();
        if (tid == 0) {             // active row list (serial: a handful of rounds per instance)
            int c = 0;
            bool over = false;
            for (int r = 0; r < m + 2 * n; ++r) {
                const double av = r < m ? actA[r] : actB[r - m];
                if (av != 0.0) {
                    if (me + c < n) idx[c++] = (double)r;
                    else over = true;
                }
            }
            sc[9] = (over || me + c > n) ? -1.0 : (double)c;
        }
        __syncthreads();
        PST(0);
        if (sc[9] < 0.0) PST_RET(false);     // more active rows than variables: degenerate
        const int na = (int)sc[9], ne = me + na;
        // K = H + rho G_a'G_a
        double dmx = 0.0;
        for (int e2 = tid; e2 < n * n; e2 += NTH) {
            const int i = e2 % n, j = e2 / n;
            double v = p.H[e2];
            for (int k = 0; k < na; ++k) {
                const int r = (int)idx[k];
                if (r < m) v += rho * p.A[(int64_t)i * m + r] * p.A[(int64_t)j * m + r];
                else if (i == j && (r - m) % n == i) v += rho;
            }
            K[e2] = v;
            if (i == j) dmx = fmax(dmx, fabs(v));
        }
        const double kfl = DQ_PIV_FLOOR * fmax(red.max(dmx), 1e-300);
        __syncthreads();
        PST(1);
        block_cholesky<NTH>(K, n, sc, kfl);
        PST(2);
        // Y = K^{-1} Ex', S = Ex Y (one thread per row of Ex)
        for (int k = tid; k < ne; k += NTH) {
            double* yc = Y + (int64_t)k * n;
            if (k < me) for (int j = 0; j < n; ++j) yc[j] = p.E[(int64_t)j * me + k];
            else { const int r = (int)idx[k - me]; for (int j = 0; j < n; ++j) yc[j] = g(r, j); }
            chol_solve_col(K, n, yc);
        }
        // ra = G_a z - h_a
        for (int k = tid; k < na; k += NTH) { const int r = (int)idx[k]; ra[k] = gdot(r, p.z) - hr(r); }
        __syncthreads();
        PST(3);
        double smx = 0.0;
        for (int t2 = tid; t2 < ne * ne; t2 += NTH) {
            const int r1 = t2 % ne, r2 = t2 / ne;
            const double* yc = Y + (int64_t)r2 * n;
            double s = 0.0;
            if (r1 < me) for (int j = 0; j < n; ++j) s += p.E[(int64_t)j * me + r1] * yc[j];
            else s = gdot((int)idx[r1 - me], yc);
            S[(int64_t)r2 * ne + r1] = s;
            if (r1 == r2) smx = fmax(smx, fabs(s));
        }
        // w = -K^{-1}(Hz + f + rho G_a' ra)
        for (int j = tid; j < n; j += NTH) {
            double v = p.f[j];
            for (int i = 0; i < n; ++i) v += p.H[(int64_t)i * n + j] * p.z[i];
            for (int k = 0; k < na; ++k) v += rho * g((int)idx[k], j) * ra[k];
            xs[j] = -v;
        }
        const double sfl = DQ_PIV_FLOOR * fmax(red.max(smx), 1e-300);
        __syncthreads();
        PST(4);
        if (ne > 0) block_cholesky<NTH>(S, ne, sc, sfl);
        chol_solve_w(K, n, xs);
        for (int j = tid; j < n; j += NTH) w[j] = xs[j];
        __syncthreads();
        // mult = S^{-1}(Ex w + Ex z - ex)
        for (int k = tid; k < ne; k += NTH) {
            double v;
            if (k < me) {
                v = -p.e[k];
                for (int j = 0; j < n; ++j) v += p.E[(int64_t)j * me + k] * (w[j] + p.z[j]);
            } else {
                const int r = (int)idx[k - me];
                v = gdot(r, w) + ra[k - me];
            }
            xs[k] = v;
        }
        __syncthreads();
        if (ne > 0) chol_solve_w(S, ne, xs);
        for (int k = tid; k < ne; k += NTH) mult[k] = xs[k];
        __syncthreads();
        PST(5);
        for (int j = tid; j < n; j += NTH) {
            double v = p.z[j] + w[j];
            for (int k = 0; k < ne; ++k) v -= Y[(int64_t)k * n + j] * mult[k];
            zn[j] = v;
        }
        for (int r = tid; r < m; r += NTH) nuA[r] = 0.0;
        for (int j = tid; j < 2 * n; j += NTH) nuB[j] = 0.0;
        __syncthreads();
        for (int k = tid; k < na; k += NTH) {
            const int r = (int)idx[k];
            if (r < m) nuA[r] = mult[me + k]; else nuB[r - m] = mult[me + k];
        }
        __syncthreads();
        PST(6);
        // checks at zn.  A' nuA by groups of 16 columns, lanes over the rows (coalesced, 16 loads in
        // flight) and one transposed wave sum per group, into xs (free here); one thread per column
        // running down the m rows waited on every load (round 6)
        if (m > 0) {
            const int lane = tid & 63, wv = tid >> 6;
            for (int g0 = 16 * wv; g0 < n; g0 += 16 * (NTH / 64)) {
                double ac[16];
#pragma unroll
                for (int c = 0; c < 16; ++c) ac[c] = 0.0;
                for (int r = lane; r < m; r += 64) {
                    const double nr = nuA[r];
                    double av[16];
#pragma unroll
                    for (int c = 0; c < 16; ++c) av[c] = p.A[(int64_t)min(g0 + c, n - 1) * m + r];
#pragma unroll
                    for (int c = 0; c < 16; ++c) ac[c] = fma(av[c], nr, ac[c]);
                }
                const double tot = wsum_t(ac, lane);
                if (lane < 16 && g0 + lane < n) xs[g0 + lane] = tot;
            }
            __syncthreads();
        }
        double viol = 0.0, va = 0.0, lmx = 0.0, lneg = 0.0, fe = 0.0, st = 0.0, gs = 0.0;
        for (int r = tid; r < m; r += NTH) {
            const double v = gdot(r, zn) - p.b[r];
            riA[r] = v;
            viol = fmax(viol, v);
            if (actA[r] != 0.0) { va = fmax(va, fabs(v)); lmx = fmax(lmx, nuA[r]); lneg = fmin(lneg, nuA[r]); }
        }
        for (int j = tid; j < n; j += NTH) {
            riB[j] = upp(j) ? zn[j] - p.ub[j] : -INFINITY;
            riB[n + j] = lop(j) ? -zn[j] + p.lb[j] : -INFINITY;
            for (int s2 = 0; s2 < 2; ++s2) {
                const int q2 = s2 * n + j;
                viol = fmax(viol, riB[q2]);
                if (actB[q2] != 0.0) { va = fmax(va, fabs(riB[q2])); lmx = fmax(lmx, nuB[q2]); lneg = fmin(lneg, nuB[q2]); }
            }
            double v = p.f[j];
            for (int i = 0; i < n; ++i) v += p.H[(int64_t)i * n + j] * zn[i];
            gs = fmax(gs, fabs(v));
            for (int k = 0; k < me; ++k) v += p.E[(int64_t)j * me + k] * mult[k];
            if (m > 0) v += xs[j];
            v += nuB[j] - nuB[n + j];
            st = fmax(st, fabs(v));
        }
        for (int k = tid; k < me; k += NTH) {
            double v = -p.e[k];
            for (int j = 0; j < n; ++j) v += p.E[(int64_t)j * me + k] * zn[j];
            fe = fmax(fe, fabs(v));
        }
        const double stat = red.max(st), gsc = red.max(gs), vio = red.max(viol), vac = red.max(va);
        const double lx = red.max(lmx), ln = red.min(lneg), fq = red.max(fe);
        const double td = 1e-9 * (1.0 + lx);
        PST(7);
        if (isfinite(stat) && stat <= p.tol_stat * (1.0 + gsc) && vio <= tf && vac <= tf && ln >= -td && fq <= tf) {
            for (int j = tid; j < n; j += NTH) {
                p.z[j] = zn[j];
                if (upp(j)) { p.lB[j] = fmax(nuB[j], 0.0); p.tB[j] = fmax(-riB[j], 0.0); }
                if (lop(j)) { p.lB[n + j] = fmax(nuB[n + j], 0.0); p.tB[n + j] = fmax(-riB[n + j], 0.0); }
            }
            for (int r = tid; r < m; r += NTH) { p.lA[r] = fmax(nuA[r], 0.0); p.tA[r] = fmax(-riA[r], 0.0); }
            for (int k = tid; k < me; k += NTH) p.y[k] = mult[k];
            if (tid == 0) { sc[10] = stat; sc[11] = fmax(fmax(vio, 0.0), fq); }
            __syncthreads();
            PST_RET(true);
        }
        // set corrections
        double chg = 0.0;
        for (int r = tid; r < m; r += NTH) {
            if (actA[r] != 0.0 && nuA[r] < -td) { actA[r] = 0.0; chg = 1.0; }
            else if (actA[r] == 0.0 && riA[r] > tf) { actA[r] = 1.0; chg = 1.0; }
        }
        for (int q2 = tid; q2 < 2 * n; q2 += NTH) {
            if (actB[q2] != 0.0 && nuB[q2] < -td) { actB[q2] = 0.0; chg = 1.0; }
            else if (actB[q2] == 0.0 && riB[q2] > tf) { actB[q2] = 1.0; chg = 1.0; }
        }
        const bool nochg = red.max(chg) == 0.0;
        PST(8);
        if (nochg) PST_RET(false);
    }
    PST_RET(false);
}

#ifdef BQP_DSTAMPS
// diagnostic build only (tools/gpu_r03_dstamps.sh): s_memtime cycles per phase of instance 0,
// printed by thread 0 at exit; never linked into the product library
#define DST_DECL                                                           \
    unsigned long long dst_last = __builtin_amdgcn_s_memtime(), dst_acc[25]; \
    _Pragma("unroll") for (int i_ = 0; i_ < 25; ++i_) dst_acc[i_] = 0
#define DST(id)                                                            \
    do {                                                                   \
        __builtin_amdgcn_s_waitcnt(0);                                     \
        const unsigned long long _t = __builtin_amdgcn_s_memtime();        \
        dst_acc[id] += _t - dst_last;                                      \
        dst_last = _t;                                                     \
    } while (0)
#define DSTN(id) TSTN(dst_acc, dst_last, id)
#else
#define DST_DECL do { } while (0)
#define DST(id) do { } while (0)
#define DSTN(id) do { } while (0)
#endif

// dense_ipm_kernel LDS: the A row tiles (TILE rows, stride ts = 32 ceil(n/32) + 1 doubles - odd
// in 64-bit words across the rows a tile load writes - column ts - 1 the row weight), then, when
// it fits, the n x n factor K = L (lower) / L' (upper) itself: the Cholesky and the four
// triangular solves per iteration then run on LDS instead of L2 round trips
#define DENSE_LDS_MAX (152 * 1024)
#define DQ_GB 34     // A'DA row-tile buffers filled by global_load_lds: column stride (32 rows + 2:
                     // 16-byte aligned columns, 16 lanes' b128 reads on distinct banks)
__host__ __device__ inline int dense_ts(int n) { return 32 * ((n + 31) / 32) + 1; }
// one A'DA buffer: column-major 32-row tile, columns 0 .. n-1 of A and column n the row weights
// (column n: the row weights d_r; column n + 1: the predictor's A' weights, below)
__host__ __device__ inline int dense_gbuf(int n) { return DQ_GB * (n + 2); }
// the two-buffer A'DA (global_load_lds of tile t + 1 in flight while the MFMAs run on tile t)
// when both buffers and the factor fit in LDS; otherwise the single row-major tile
// (every budget below counts the reduction scratch and the tile bounds, DQ_TAIL doubles at the end)
#define DQ_TAIL (48 + DQ_THL)
#define DQ_NVEC 17   // n-vectors of dense_ipm_kernel RG in LDS (5 of n, 6 of 2n)
__host__ __device__ inline bool dense_glds(int n) {
    const int a = TILE * dense_ts(n), b = 2 * dense_gbuf(n);
    return n <= 128 && (size_t)((a > b ? a : b) + n * n + DQ_TAIL) * sizeof(double) <= DENSE_LDS_MAX;
}
__host__ __device__ inline int dense_tiles(int n) {   // doubles of LDS before the factor
    const int a = TILE * dense_ts(n), b = 2 * dense_gbuf(n);
    return dense_glds(n) && b > a ? b : a;
}
__host__ __device__ inline bool dense_k_lds(int n) {
    return (size_t)(dense_tiles(n) + n * n + DQ_TAIL) * sizeof(double) <= DENSE_LDS_MAX;
}
// + the reduction scratch (16), the tile Cholesky's reciprocal pivots and fail flag (32) and the
// A tile bounds (DQ_THL) at the end: the kernel's only LDS
// object is the dynamic array (a second __shared__ object made hipcc wait for the in-flight
// global_load_lds before every LDS read)
__host__ __device__ inline size_t dense_lds_bytes(int n) {
    return sizeof(double) * (size_t)(dense_tiles(n) + (dense_k_lds(n) ? n * n : 0) + DQ_TAIL);
}

template <bool KL,    // KL: the factor lives in LDS (dense_k_lds(n)); a compile-time choice so that
                     // every access to it is a ds_* instruction (a run-time select made the pointer
                     // generic: flat accesses, ~5k cycles per Cholesky pivot)
          bool RG>   // RG: the row state in registers, the n-vectors in LDS (dense_rows_in_regs)
__global__ void __launch_bounds__(DT) dense_ipm_kernel(DenseKernelArgs a) {
    const int inst = blockIdx.x;
    if (inst >= a.batch || (a.skip && a.skip[inst])) return;
    const int n = a.n, m = a.m, me = a.me, tid = threadIdx.x;
    extern __shared__ __attribute__((aligned(16))) double dlds[];
    double* sc = dlds + dense_tiles(n) + (KL ? n * n : 0);
    double* rvp = sc + 16;           // tile Cholesky: reciprocal pivots, fail flag (tile_chol)
    double* thl = sc + 48;           // tile bounds of A (below)
    const int ts = dense_ts(n), tw = ts - 1;
    double* tileA = dlds;
    Red red{sc};
    DST_DECL;
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
    // RG: the n-vectors of the iteration and the bound rows in LDS as well, after the tail (DQ_NVEC
    // n doubles: z, q, w, dz, rd, then tB, lB, riB, rcB, dtB, dlB of 2n each); the repair launch's
    // start (z, tB, lB) is copied to the workspace at the end
    double* vb = dlds + dense_tiles(n) + (KL ? n * n : 0) + DQ_TAIL;
    double *z = RG ? vb : W + L.z, *y = W + L.y, *q = RG ? vb + n : W + L.q, *w = RG ? vb + 2 * n : W + L.w;
    double *dz = RG ? vb + 3 * n : W + L.dz, *dy = W + L.dy;
    double *rd = RG ? vb + 4 * n : W + L.rd, *re = W + L.re;
    double *tA = W + L.tA, *lA = W + L.lA, *riA = W + L.riA, *rcA = W + L.rcA, *dtA = W + L.dtA, *dlA = W + L.dlA;
    double *tB = RG ? vb + 5 * n : W + L.tB, *lB = RG ? vb + 7 * n : W + L.lB, *riB = RG ? vb + 9 * n : W + L.riB;
    double *rcB = RG ? vb + 11 * n : W + L.rcB, *dtB = RG ? vb + 13 * n : W + L.dtB, *dlB = RG ? vb + 15 * n : W + L.dlB;
    // the row state of the m rows of A - slack t, multiplier lam, residual ri, complementarity rc,
    // the direction dt, dlam - in registers when RG (round 6): row r = tid + DT i in slot i, the
    // mapping of every row pass below; otherwise in the instance's workspace.  In the workspace
    // it was rewritten every iteration and left L2 for HBM (135 MB of writes per 128-instance
    // launch of the learned loop's sub-problem, profiles/pmc_CLL.json of round 5).  The row
    // weights of the A'DA tiles (another mapping) are formed by the threads that hold the rows.
    constexpr int RPT = RG ? DQ_RPT : 1;
    double tAr[RPT], lAr[RPT], riAr[RPT], rcAr[RPT], dtAr[RPT], dlAr[RPT];
#define TA(i, r) (RG ? tAr[RG ? (i) : 0] : tA[r])
#define LA(i, r) (RG ? lAr[RG ? (i) : 0] : lA[r])
#define RIA(i, r) (RG ? riAr[RG ? (i) : 0] : riA[r])
#define RCA(i, r) (RG ? rcAr[RG ? (i) : 0] : rcA[r])
#define DTA(i, r) (RG ? dtAr[RG ? (i) : 0] : dtA[r])
#define DLA(i, r) (RG ? dlAr[RG ? (i) : 0] : dlA[r])
    // the rows of this thread: slot i, row r (unrolled over the DQ_RPT slots when RG)
#define DQ_ROWS(i, r) \
    _Pragma("unroll") for (int i = 0; RG ? (i < RPT) : (tid + i * DT < m); ++i) \
        if (const int r = tid + i * DT; !RG || r < m)
    double* K = KL ? dlds + dense_tiles(n) : W + L.K;   // the factor (LDS when it fits)
    double* Y = W + L.Y;
    double* S = W + L.S;
    auto up_present = [&](int j) -> bool { return ub && isfinite(ub[j]); };
    auto lo_present = [&](int j) -> bool { return lb && isfinite(lb[j]); };
    // rows r0 .. r0 + rows - 1 of A into tileA (row-major, stride ts): 8 clamped loads in flight
    // per thread before the LDS stores (the load -> store loop waited on every load)
    auto load_tile = [&](int r0, int rows, int ncol) {   // columns 0 .. ncol - 1
        const int tot = rows * ncol;
        const bool full = rows == TILE;
        for (int b0 = 0; b0 < tot; b0 += 8 * DT) {
            double v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int t2 = min(b0 + tid + u * DT, tot - 1);
                const int rr = full ? (t2 & (TILE - 1)) : t2 % rows, j = full ? (t2 / TILE) : t2 / rows;
                v[u] = A[(int64_t)j * m + r0 + rr];
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int t2 = b0 + tid + u * DT;
                const int rr = full ? (t2 & (TILE - 1)) : t2 % rows, j = full ? (t2 / TILE) : t2 / rows;
                if (t2 < tot) tileA[rr * ts + j] = v[u];
            }
        }
    };
    // (A v)_r for one row r of column-major A over its nonzero columns j < hr[r] (the skipped
    // products are exact zeros): v staged in LDS (vlds, by stage_v), 16 clamped loads of A in
    // flight per batch and four independent chains (four loads per step with v read from global
    // took one memory round trip per four columns)
    double* hr = W + L.hr;
    double* th = W + L.th;
    // the tile bounds from LDS (the first DQ_THL tiles; later ones are taken as full)
    auto tbound = [&](int t) -> double { return t < DQ_THL ? thl[t] : (double)n; };
    double* vlds = tileA + TILE * ts - n;   // the end of the tile buffer (free around the row products)
    auto stage_v = [&](const double* v) {
        __syncthreads();
        for (int j = tid; j < n; j += DT) vlds[j] = v[j];
        __syncthreads();
    };
    auto arow = [&](int r) -> double {
        const int jm = (int)hr[r];
        const double* pr = A + r;
        double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
        int j0 = 0;
        for (; j0 + 16 <= jm; j0 += 16) {        // whole batches: no clamps or selects
            double av[16];
#pragma unroll
            for (int u = 0; u < 16; ++u) av[u] = pr[(int64_t)(j0 + u) * m];
#pragma unroll
            for (int u = 0; u < 16; u += 4) {
                s0 = fma(av[u], vlds[j0 + u], s0);
                s1 = fma(av[u + 1], vlds[j0 + u + 1], s1);
                s2 = fma(av[u + 2], vlds[j0 + u + 2], s2);
                s3 = fma(av[u + 3], vlds[j0 + u + 3], s3);
            }
        }
        if (j0 < jm) {                           // the tail (clamped, masked)
            double av[16];
#pragma unroll
            for (int u = 0; u < 16; ++u) av[u] = pr[(int64_t)min(j0 + u, jm - 1) * m];
#pragma unroll
            for (int u = 0; u < 16; u += 4) {
                s0 = fma(j0 + u < jm ? av[u] : 0.0, vlds[min(j0 + u, n - 1)], s0);
                s1 = fma(j0 + u + 1 < jm ? av[u + 1] : 0.0, vlds[min(j0 + u + 1, n - 1)], s1);
                s2 = fma(j0 + u + 2 < jm ? av[u + 2] : 0.0, vlds[min(j0 + u + 2, n - 1)], s2);
                s3 = fma(j0 + u + 3 < jm ? av[u + 3] : 0.0, vlds[min(j0 + u + 3, n - 1)], s3);
            }
        }
        return (s0 + s1) + (s2 + s3);
    };
    // A'(w) for a row weight w(r) (every thread calls it): A streamed through LDS row tiles
    // (coalesced along the rows of column-major A, as the factorisation does), thread j < n
    // accumulating column j from LDS; the column loops over all m rows that one thread per
    // column ran before touched 64 cache lines per wave load (m = 1024: ~0.5 ms per product)
    auto atw = [&](auto&& wfun) __attribute__((always_inline)) -> double {
        if (RG || m + n <= TILE * ts) {   // (RG: the host checked that it fits)
            // the row weights into LDS once; wave wv takes column groups 16 g (g = wv, wv + 4,
            // ..): lanes over rows, 16 independent loads per row step, one transposed wave sum
            // (wsum_t) per group; no tile barriers (the tile version waited on a load round
            // trip and two barriers per 32 rows)
            double* wl = tileA;
            double* out = tileA + m;
            __syncthreads();
            DQ_ROWS(i, r) wl[r] = wfun(i, r);
            __syncthreads();
            const int lane = tid & 63, wv = tid >> 6;
            for (int g = wv; 16 * g < n; g += DT / 64) {
                double ac[16];
#pragma unroll
                for (int c = 0; c < 16; ++c) ac[c] = 0.0;
                const double* Ag = A + (int64_t)(16 * g) * m;
                // two 64-row steps per pass: 32 loads in flight
                for (int r = lane; r < m; r += 128) {
                    // rows r - lane .. r - lane + 127 (four tiles) all zero in this column group
                    const int t0 = (r - lane) / TILE;
                    double thm = tbound(t0);
#pragma unroll
                    for (int k = 1; k < 4; ++k) thm = fmax(thm, (t0 + k) * TILE < m ? tbound(t0 + k) : 0.0);
                    if (thm <= 16.0 * g) continue;
                    const int r2 = min(r + 64, m - 1);
                    const double vr = wl[r], vr2 = r + 64 < m ? wl[r2] : 0.0;
                    double a1[16], a2[16];
#pragma unroll
                    for (int c = 0; c < 16; ++c) {
                        const int64_t co = (int64_t)min(c, n - 1 - 16 * g) * m;
                        a1[c] = Ag[co + r];
                        a2[c] = Ag[co + r2];
                    }
#pragma unroll
                    for (int c = 0; c < 16; ++c) ac[c] = fma(a2[c], vr2, fma(a1[c], vr, ac[c]));
                }
                const double sv = wsum_t(ac, lane);
                if (lane < 16 && 16 * g + lane < n) out[16 * g + lane] = sv;
            }
            __syncthreads();
            const double res = tid < n ? out[tid] : 0.0;
            __syncthreads();
            return res;
        }
        double acc = 0.0;
        for (int r0 = 0; r0 < m; r0 += TILE) {
            const int rows = min(TILE, m - r0);
            __syncthreads();
            load_tile(r0, rows, n);
            if (tid < rows) tileA[tid * ts + tw] = wfun(0, r0 + tid);
            __syncthreads();
            if (tid < n)
                for (int rr = 0; rr < rows; ++rr) acc += tileA[rr * ts + tid] * tileA[rr * ts + tw];
        }
        __syncthreads();
        return acc;
    };
    // nonzero column bound of every row of A (1 + its last nonzero column) and of every TILE-row
    // tile (the max over its rows), once per launch: the products skip the columns and tiles past
    // it - exact zeros.  The condensed rows of an MPC problem reach only the inputs up to their
    // stage (the learned-model loop's sub-problem: each row k of the state / input boxes sees
    // u_0 .. u_{k-1}), so A'DA runs on about a third of its tiles there.
    for (int r = tid; r < m; r += DT) {
        int j = n - 1;
        while (j >= 0 && A[(int64_t)j * m + r] == 0.0) --j;
        hr[r] = (double)(j + 1);
    }
    __syncthreads();
    for (int t = tid; t * TILE < m; t += DT) {
        double mx = 0.0;
        for (int rr = t * TILE; rr < min(m, (t + 1) * TILE); ++rr) mx = fmax(mx, hr[rr]);
        th[t] = mx;
        if (t < DQ_THL) thl[t] = mx;
    }
    __syncthreads();
    // row count
    double cnt = 0.0;
    for (int j = tid; j < n; j += DT) cnt += (up_present(j) ? 1.0 : 0.0) + (lo_present(j) ? 1.0 : 0.0);
    const double mtot = red.sum(cnt) + (double)m;
    const double minv = 1.0 / fmax(mtot, 1.0);

    // ---------------------------------------------------------------- residuals
    auto residuals = [&](double& stat, double& feq, double& fin, double& csum, double& gscale, double& zmax,
                         double& cmax) __attribute__((always_inline)) {
        double fe = 0.0, fq = 0.0, cs = 0.0, st = 0.0, gs = 0.0, zm = 0.0, cm = 0.0;
        stage_v(z);
        DQ_ROWS(i, r) {
            const double v = TA(i, r) - b[r] + arow(r);
            RIA(i, r) = v;
            fe = fmax(fe, fabs(v));
            cs += TA(i, r) * LA(i, r);
            cm = fmax(cm, TA(i, r) * LA(i, r));
        }
        // f + H z (z from vlds; row j of H read across the lanes - coalesced, H symmetric as
        // the factorisation assumes; 16 loads in flight) into rd, completed below
        for (int j = tid; j < n; j += DT) {
            double v = f[j];
            for (int i0 = 0; i0 < n; i0 += 16) {
                double hv[16];
#pragma unroll
                for (int u = 0; u < 16; ++u) hv[u] = H[(int64_t)min(i0 + u, n - 1) * n + j];
#pragma unroll
                for (int u = 0; u < 16; ++u)
                    if (i0 + u < n) v = fma(hv[u], vlds[i0 + u], v);
            }
            rd[j] = v;
        }
        DST(0);
        for (int r = tid; r < me; r += DT) {
            double v = -e[r];
            for (int j = 0; j < n; ++j) v += E[(int64_t)j * me + r] * z[j];
            re[r] = v;
            fq = fmax(fq, fabs(v));
        }
        const double alam = atw([&](int i, int r) { return LA(i, r); });   // (A' lam)_tid
        DST(10);
        for (int j = tid; j < n; j += DT) {
            double v = rd[j];
            gs = fmax(gs, fabs(v));
            for (int r = 0; r < me; ++r) v += E[(int64_t)j * me + r] * y[r];
            v += alam;
            riB[j] = 0.0; riB[n + j] = 0.0;
            if (up_present(j)) {
                v += lB[j];
                riB[j] = z[j] + tB[j] - ub[j];
                cs += tB[j] * lB[j];
                cm = fmax(cm, tB[j] * lB[j]);
            }
            if (lo_present(j)) {
                v -= lB[n + j];
                riB[n + j] = -z[j] + tB[n + j] + lb[j];
                cs += tB[n + j] * lB[n + j];
                cm = fmax(cm, tB[n + j] * lB[n + j]);
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
        cmax = red.max(cm);
        DST(11);
    };

    // the residuals after a step of length al from the ones before it: with one step length for
    // every variable, the row residuals r = t - b + A z (bounds alike) of the stepped iterate are
    // exactly (1 - al) r (dt = -r - A dz), and the dual / equality residuals are (1 - al) times
    // theirs up to the accuracy of the Newton solve - so the A z and A' lam passes over A and the
    // H z product (0.88M + 0.60M of ~10M cycles per n = 101, m = 1024 solve) run only where the
    // iteration needs exact values: the first iteration, and every convergence test these scaled
    // residuals pass (residuals() then re-evaluates, and the iteration continues on exact values
    // if they do not pass).  gscale (max |f + H z|, the stationarity tolerance's scale) keeps its
    // last exact value.
    auto scaled_residuals = [&](double s, double& stat, double& feq, double& fin, double& csum, double& zmax,
                                double& cmax) __attribute__((always_inline)) {
        double fe = 0.0, fq = 0.0, cs = 0.0, st = 0.0, zm = 0.0, cm = 0.0;
        DQ_ROWS(i, r) {
            const double v = s * RIA(i, r);
            RIA(i, r) = v;
            fe = fmax(fe, fabs(v));
            const double c = TA(i, r) * LA(i, r);
            cs += c;
            cm = fmax(cm, c);
        }
        for (int r = tid; r < me; r += DT) { const double v = s * re[r]; re[r] = v; fq = fmax(fq, fabs(v)); }
        for (int j = tid; j < n; j += DT) {
            const double v = s * rd[j];
            rd[j] = v;
            st = fmax(st, fabs(v));
            zm = fmax(zm, fabs(z[j]));
            if (up_present(j)) {
                riB[j] *= s;
                const double c = tB[j] * lB[j];
                cs += c;
                cm = fmax(cm, c);
            }
            if (lo_present(j)) {
                riB[n + j] *= s;
                const double c = tB[n + j] * lB[n + j];
                cs += c;
                cm = fmax(cm, c);
            }
            fe = fmax(fe, fmax(fabs(riB[j]), fabs(riB[n + j])));
        }
        stat = red.max(st);
        fin = red.max(fe);
        feq = red.max(fq);
        csum = red.sum(cs);
        zmax = red.max(zm);
        cmax = red.max(cm);
        DST(11);
    };

    // (A' w)_tid of the predictor's right-hand side, w_r = (lam_r riA_r - t_r lam_r) / t_r, formed
    // inside the A'DA pipeline from the row tiles it already has in LDS (aq_ok): one pass over A
    // per iteration less (the predictor's atw, ~0.5M of ~9M cycles per n = 101 solve)
    double aq_pre = 0.0;
    bool aq_ok = false;
    // ---------------------------------------------------------------- factorisation
    auto factor = [&]() __attribute__((always_inline)) -> bool {   // inlined: a call spilled (callee budget)
        aq_ok = false;
        // K = H + sum_r A_r' D_r A_r (+ bound diagonal): lower triangle (n <= 128) or both
        const int ne = n * (n + 1) / 2;
        double dmx = 0.0;                 // largest diagonal entry (pivot floor scale)
        if (n <= 128) {
            // K = H + A'DA on the fp64 matrix cores (v_mfma_f64_16x16x4_f64): the lower block
            // triangle of ceil(n/16)^2 16 x 16 tiles, on wave w the tiles of tile_of (at most 9
            // per wave); each k-step takes 4 rows of A from the LDS row tile - lane l supplies
            // A[r][16 I + l%16] (r = 4 s + l/16) as the A operand and d_r A[r][16 J + l%16] as the
            // B operand, so tile (I, J) accumulates sum_r A[r][16I + i] d_r A[r][16J + j].
            // Columns >= n read a clamped (finite) column and rows past the tile have d = 0:
            // their products land in entries i or j >= n, which are not written back.  (Round 3
            // formed this product with VALU FMAs from 8 x 8 register tiles: ~10 % of the CU's
            // FP64 rate, the largest phase of the learned-model loop's sub-problem.)
            constexpr int TPW = 9;
            const int lane = tid & 63, wv = tid >> 6;
            const int c16 = lane & 15, k4 = lane >> 4;
            const int nbk = (n + 15) >> 4;
            int tI[TPW], tJ[TPW];
#pragma unroll
            for (int u = 0; u < TPW; ++u) tile_of(wv, u, nbk, tI[u], tJ[u]);
            dbl4 acc[TPW];
#pragma unroll
            for (int u = 0; u < TPW; ++u) acc[u] = dbl4{0.0, 0.0, 0.0, 0.0};
            const bool gl = KL && m > 0 && dense_glds(n);   // (m = 0: no rows, A may be null)
            if (gl) {
                // two column-major buffers: tile t + 1 is copied by global_load_lds (no VGPR
                // staging) while the MFMAs consume tile t, one barrier per tile.  One 4-byte
                // load per lane moves one column's 32 rows (256 B) - rows past m read row m - 1,
                // whose weight slot is 0 - so each column lands at its own padded offset.  (The
                // 16-byte form - four columns per wave-instruction, row pairs rotated per column
                // against bank conflicts - issued a quarter of the copies and took the same time
                // per solve: the tile's MFMA chain, not the copy issue, sets the pace.)
                const int ntile = (m + TILE - 1) / TILE;
                const int rowl = lane >> 1;
                // The copy is issued from inline asm (M0 = the column's LDS byte address): with
                // the builtin, hipcc cannot tell the two buffers apart and waited for the copy of
                // tile t + 1 before the first LDS read of tile t.  Its completion is waited for
                // explicitly (vmcnt(0)) before the barrier that hands the buffer over.
                // The column loop runs on scalar registers (wave index, column count and LDS
                // address made wave-uniform: a per-lane loop counter put an exec-mask update and
                // two readfirstlanes on every copy, ~3k cycles per tile)
                const int wvu = __builtin_amdgcn_readfirstlane(wv);
                const int64_t cstr = (int64_t)(DT / 64) * m * sizeof(double);
                auto issue = [&](int t, double* buf) {
                    const int ncol = __builtin_amdgcn_readfirstlane(min(n, 16 * (((int)tbound(t) + 15) / 16)));
                    const char* g = (const char*)(A + min(t * TILE + rowl, m - 1)) + 4 * (lane & 1) +
                                    (int64_t)wvu * m * sizeof(double);
                    unsigned ldsa = __builtin_amdgcn_readfirstlane(
                        (unsigned)(uintptr_t)(__attribute__((address_space(3))) double*)(buf)) +
                        (unsigned)(wvu * DQ_GB * sizeof(double));
                    for (int j = wvu; j < ncol; j += DT / 64, g += cstr, ldsa += (DT / 64) * DQ_GB * sizeof(double)) {
                        unsigned keep;
                        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
                                     "global_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
                                     : "=&s"(keep) : "v"(g), "s"(ldsa) : "memory");
                    }
                };
                auto copy_wait = [] { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); };
                double* gb0 = dlds;
                double* gb1 = dlds + dense_gbuf(n);
                double aw = 0.0;
                {
                    // rows 0 .. TILE - 1: threads 0 .. TILE - 1, slot 0 (RG)
                    const int rd0 = min(tid, min(TILE, m) - 1);
                    const double la = RG ? lAr[0] : lA[rd0], ta = RG ? tAr[0] : tA[rd0], ri = RG ? riAr[0] : riA[rd0];
                    issue(0, gb0);
                    if (tid < TILE) {
                        const bool in = tid < min(TILE, m);
                        gb0[DQ_GB * n + tid] = in ? la / ta : 0.0;
                        gb0[DQ_GB * (n + 1) + tid] = in ? (la * ri - ta * la) / ta : 0.0;
                    }
                }
                copy_wait();
                __syncthreads();
                for (int t = 0; t < ntile; ++t) {
                    double* cur = (t & 1) ? gb1 : gb0;
                    double* nxt = (t & 1) ? gb0 : gb1;
                    const int r0 = t * TILE;
                    const bool more = t + 1 < ntile;
                    double la = 1.0, ta = 1.0, ri = 0.0;
                    const int rows1 = more ? min(TILE, m - r0 - TILE) : 0;
                    // RG: the rows of tile t + 1 are held by threads wb .. wb + TILE - 1 (slot s1)
                    const int wb = (r0 + TILE) % DT, s1 = (r0 + TILE) / DT, tl = RG ? tid - wb : tid;
                    if (more) {
                        if constexpr (RG) {
#pragma unroll
                            for (int i = 0; i < RPT; ++i)
                                if (i == s1) { la = lAr[i]; ta = tAr[i]; ri = riAr[i]; }
                        } else {
                            const int rd1 = r0 + TILE + min(tid, rows1 - 1);
                            la = lA[rd1]; ta = tA[rd1]; ri = riA[rd1];
                        }
                        issue(t + 1, nxt);
                    }
                    DSTN(21);
                    const double thi = tbound(t);
                    // k-step s of lane group k4 takes row 8 k4 + s: each lane's 8 rows of a column
                    // are contiguous, read as four ds_read_b128 (rows past the tile hold finite
                    // copies of row m - 1 and weight 0)
                    double drv[TILE / 4];
                    {
                        const double2* dp = reinterpret_cast<const double2*>(cur + DQ_GB * n + 8 * k4);
#pragma unroll
                        for (int h = 0; h < TILE / 8; ++h) { const double2 v = dp[h]; drv[2 * h] = v.x; drv[2 * h + 1] = v.y; }
                    }
#pragma unroll
                    for (int u = 0; u < TPW; ++u) {
                        if (tI[u] >= 0 && 16.0 * tI[u] < thi) {
                            const int ci = min(16 * tI[u] + c16, n - 1), cj = min(16 * tJ[u] + c16, n - 1);
                            const double2* pa = reinterpret_cast<const double2*>(cur + DQ_GB * ci + 8 * k4);
                            const double2* pb = reinterpret_cast<const double2*>(cur + DQ_GB * cj + 8 * k4);
                            double ai[TILE / 4], aj[TILE / 4];
#pragma unroll
                            for (int h = 0; h < TILE / 8; ++h) {
                                const double2 va = pa[h], vb = pb[h];
                                ai[2 * h] = va.x; ai[2 * h + 1] = va.y;
                                aj[2 * h] = vb.x; aj[2 * h + 1] = vb.y;
                            }
#pragma unroll
                            for (int s4 = 0; s4 < TILE / 4; ++s4)
                                acc[u] = __builtin_amdgcn_mfma_f64_16x16x4f64(ai[s4], drv[s4] * aj[s4], acc[u], 0, 0, 0);
                        }
                    }
                    // the predictor's A' w on the columns this tile reaches: thread tid takes
                    // column tid % 128 over the tile's rows 16 (tid / 128) .. + 15 (all four waves)
                    if ((tid & 127) < min(n, 16 * (((int)thi + 15) / 16))) {
                        const double2* pc = reinterpret_cast<const double2*>(cur + DQ_GB * (tid & 127) + 16 * (tid >> 7));
                        const double2* pw = reinterpret_cast<const double2*>(cur + DQ_GB * (n + 1) + 16 * (tid >> 7));
                        double s0 = 0.0, s1 = 0.0;
#pragma unroll
                        for (int h = 0; h < TILE / 4; ++h) {
                            const double2 av = pc[h], wv2 = pw[h];
                            s0 = fma(av.x, wv2.x, s0);
                            s1 = fma(av.y, wv2.y, s1);
                        }
                        aw += s0 + s1;
                    }
                    DSTN(22);
                    if (more && tl >= 0 && tl < TILE) {
                        nxt[DQ_GB * n + tl] = tl < rows1 ? la / ta : 0.0;
                        nxt[DQ_GB * (n + 1) + tl] = tl < rows1 ? (la * ri - ta * la) / ta : 0.0;
                    }
                    copy_wait();
                    DSTN(23);
                    __syncthreads();
                    DSTN(24);
                }
                // the two row halves of each column (the loop's last barrier has retired gb0)
                if (tid >= 128 && (tid & 127) < n) gb0[tid & 127] = aw;
                __syncthreads();
                aq_pre = tid < n ? aw + gb0[tid] : 0.0;
                aq_ok = true;
                __syncthreads();
            }
            for (int r0 = 0; r0 < ((RG || gl) ? 0 : m); r0 += TILE) {
                const int rows = min(TILE, m - r0);
                __syncthreads();
                // only the columns the tile's rows reach, to the 16-column block (the MFMA operands
                // read columns below 16 (I + 1) <= that of tiles I < thi / 16; the rest are zeros)
                const double thi = tbound(r0 / TILE);
                // the row weights' loads ahead of the tile's (one round trip for both)
                const int rd0 = r0 + min(tid, rows - 1);
                const double la = lA[rd0], ta = tA[rd0];
                load_tile(r0, rows, min(n, 16 * (((int)thi + 15) / 16)));
                if (tid < rows) tileA[tid * ts + tw] = la / ta;
                __syncthreads();
                // per output tile u the 8 k-steps of the row tile: 16 operand reads issued
                // together, then 8 MFMAs on acc[u] (with the k-steps outermost every tile's pair
                // of reads sat in its own branch block, one LDS round trip per MFMA)
                double drv[TILE / 4];
#pragma unroll
                for (int s4 = 0; s4 < TILE / 4; ++s4) {
                    const int rr = 4 * s4 + k4;
                    drv[s4] = rr < rows ? tileA[min(rr, rows - 1) * ts + tw] : 0.0;
                }
#pragma unroll
                for (int u = 0; u < TPW; ++u) {
                    // wave-uniform: the tile exists and the rows reach its column block I (J <= I)
                    if (tI[u] >= 0 && 16.0 * tI[u] < thi) {
                        const int ci = min(16 * tI[u] + c16, n - 1), cj = min(16 * tJ[u] + c16, n - 1);
                        double ai[TILE / 4], aj[TILE / 4];
#pragma unroll
                        for (int s4 = 0; s4 < TILE / 4; ++s4) {
                            const double* Tr = tileA + min(4 * s4 + k4, rows - 1) * ts;
                            ai[s4] = Tr[ci];
                            aj[s4] = Tr[cj];
                        }
#pragma unroll
                        for (int s4 = 0; s4 < TILE / 4; ++s4)
                            acc[u] = __builtin_amdgcn_mfma_f64_16x16x4f64(ai[s4], drv[s4] * aj[s4], acc[u], 0, 0, 0);
                    }
                }
            }
            // tile (I, J), lane l, register e: K(16 I + l/16 + 4 e, 16 J + l%16) = H + A'DA + the
            // bound diagonal.  Factor in LDS (KL): the blocked Cholesky on the tiles (tile_chol;
            // diagonal tiles whole, padding the identity).  Factor in global memory (n > 122):
            // the lower triangle to K and chol_2b there (tile_chol on global K spilled).
#pragma unroll
            for (int u = 0; u < TPW; ++u) {
                if (tI[u] < 0) continue;
#pragma unroll
                for (int e2 = 0; e2 < 4; ++e2) {
                    const int i = 16 * tI[u] + k4 + 4 * e2, j = 16 * tJ[u] + c16;
                    double v = (i == j) ? 1.0 : 0.0;
                    if (i < n && j < n) {
                        v = H[(int64_t)j * n + i] + acc[u][e2];
                        if (i == j) {
                            if (up_present(j)) v += lB[j] / tB[j];
                            if (lo_present(j)) v += lB[n + j] / tB[n + j];
                            dmx = fmax(dmx, fabs(v));
                        }
                        if (!KL && i >= j) K[(int64_t)j * n + i] = v;
                    }
                    acc[u][e2] = v;
                }
            }
            const double kfl = DQ_PIV_FLOOR * fmax(red.max(dmx), 1e-300);
            DST(1);
            if constexpr (KL) {
                if (!tile_chol(acc, tI, tJ, K, n, kfl, rvp TST_PASS)) return false;
            } else {
                if (!chol_2b(K, n, kfl, tileA)) return false;
            }
            DST(2);
        }
        for (int base = 0; base < ((RG || n <= 128) ? 0 : ne); base += DT * 8) {
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
                load_tile(r0, rows, n);
                if (tid < rows) tileA[tid * ts + tw] = lA[r0 + tid] / tA[r0 + tid];
                __syncthreads();
#pragma unroll
                for (int q2 = 0; q2 < 8; ++q2) {
                    if (ii[q2] < 0) continue;
                    double s = 0.0;
                    for (int rr = 0; rr < rows; ++rr)
                        s += tileA[rr * ts + ii[q2]] * tileA[rr * ts + tw] * tileA[rr * ts + jj[q2]];
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
        if (n > 128) {
            const double kfl = DQ_PIV_FLOOR * fmax(red.max(dmx), 1e-300);
            DST(1);
            if (!block_cholesky(K, n, sc, kfl)) return false;
            DST(2);
        }
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
    auto solve = [&]() __attribute__((always_inline)) {
        // q = rd + A'((lam riA - rcA)/tA) + bound terms ; w = -K^{-1} q
        DST(3);
        // the first solve after a factorisation (rc = t lam) takes the A' w formed with A'DA
        const double aq = aq_ok ? aq_pre : atw([&](int i, int r) { return (LA(i, r) * RIA(i, r) - RCA(i, r)) / TA(i, r); });
        aq_ok = false;
        DST(7);
        for (int j = tid; j < n; j += DT) {
            double v = rd[j] + aq;
            if (up_present(j)) v += (lB[j] * riB[j] - rcB[j]) / tB[j];
            if (lo_present(j)) v -= (lB[n + j] * riB[n + j] - rcB[n + j]) / tB[n + j];
            q[j] = v;
        }
        __syncthreads();
        for (int j = tid; j < n; j += DT) xs[j] = -q[j];
        __syncthreads();
        DST(8);
        if constexpr (KL) chol_solve_wg(K, n, xs);
        else chol_solve_w(K, n, xs);
        DST(8);
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
            chol_solve_w(S, me, xs);
            for (int r = tid; r < me; r += DT) dy[r] = xs[r];
            __syncthreads();
        }
        for (int j = tid; j < n; j += DT) {
            double v = w[j];
            for (int r = 0; r < me; ++r) v -= Y[(int64_t)r * n + j] * dy[r];
            dz[j] = v;
        }
        stage_v(dz);
        DQ_ROWS(i, r) {
            const double v = arow(r);
            DTA(i, r) = -RIA(i, r) - v;
            DLA(i, r) = (-RCA(i, r) - LA(i, r) * DTA(i, r)) / TA(i, r);
        }
        for (int j = tid; j < n; j += DT) {
            dtB[j] = dlB[j] = dtB[n + j] = dlB[n + j] = 0.0;
            if (up_present(j)) { dtB[j] = -riB[j] - dz[j]; dlB[j] = (-rcB[j] - lB[j] * dtB[j]) / tB[j]; }
            if (lo_present(j)) { dtB[n + j] = -riB[n + j] + dz[j]; dlB[n + j] = (-rcB[n + j] - lB[n + j] * dtB[n + j]) / tB[n + j]; }
        }
        __syncthreads();
        DST(9);
    };

    auto max_step = [&]() __attribute__((always_inline)) -> double {
        double al = 1.0;
#define DQ_RATIO(v, dv) if ((dv) < 0.0) al = fmin(al, -(v) / (dv));
        DQ_ROWS(i, r) { DQ_RATIO(TA(i, r), DTA(i, r)); DQ_RATIO(LA(i, r), DLA(i, r)); }
        for (int j = tid; j < n; j += DT) {
            if (up_present(j)) { DQ_RATIO(tB[j], dtB[j]); DQ_RATIO(lB[j], dlB[j]); }
            if (lo_present(j)) { DQ_RATIO(tB[n + j], dtB[n + j]); DQ_RATIO(lB[n + j], dlB[n + j]); }
        }
#undef DQ_RATIO
        return red.min(al);
    };
    auto comp_after = [&](double al) __attribute__((always_inline)) -> double {
        double c = 0.0;
        DQ_ROWS(i, r) c += (TA(i, r) + al * DTA(i, r)) * (LA(i, r) + al * DLA(i, r));
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
    DQ_ROWS(i, r) { TA(i, r) = 1.0; LA(i, r) = 1.0; RCA(i, r) = 1.0; RIA(i, r) = 0.0; DTA(i, r) = 0.0; DLA(i, r) = 0.0; }
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
        if (KL && n <= 128) {
            // the same blocked factor on tiles of H + sh I (tile_chol, no pivot floor)
            constexpr int TPW = 9;
            const int lane = tid & 63, wv = tid >> 6, c16 = lane & 15, k4 = lane >> 4;
            int tI[TPW], tJ[TPW];
            dbl4 acc[TPW];
#pragma unroll
            for (int u = 0; u < TPW; ++u) {
                tile_of(wv, u, (n + 15) >> 4, tI[u], tJ[u]);
#pragma unroll
                for (int e2 = 0; e2 < 4; ++e2) {
                    const int i = 16 * tI[u] + k4 + 4 * e2, j = 16 * tJ[u] + c16;
                    double v = (i == j) ? 1.0 : 0.0;
                    if (tI[u] >= 0 && i < n && j < n) v = H[(int64_t)j * n + i] + (i == j ? sh : 0.0);
                    acc[u][e2] = v;
                }
            }
            if (!tile_chol(acc, tI, tJ, K, n, -1.0, rvp TST_PASS)) flag = -6;
        } else {
            for (int e2 = tid; e2 < n * n; e2 += DT) {
                const int i = e2 % n, j = e2 / n;
                K[e2] = H[e2] + (i == j ? sh : 0.0);
            }
            __syncthreads();
            if (!(n <= 128 ? chol_2b(K, n, -1.0, tileA) : block_cholesky(K, n, sc, -1.0))) flag = -6;
        }
    }
    double stat = 0.0, feq = 0.0, fin = 0.0, csum = 0.0, gscale = 0.0, zmax = 0.0, cmax = 0.0;
    residuals(stat, feq, fin, csum, gscale, zmax, cmax);
    if (flag == 0 && !factor()) flag = -8;
    if (flag == 0) {
        solve();
        double tmin = INFINITY, tmax = -INFINITY;
        for (int j = tid; j < n; j += DT) z[j] += dz[j];
        for (int r = tid; r < me; r += DT) y[r] += dy[r];
        DQ_ROWS(i, r) { const double t = 1.0 + DTA(i, r); tmin = fmin(tmin, t); tmax = fmax(tmax, t); }
        for (int j = tid; j < n; j += DT) {
            if (up_present(j)) { const double t = 1.0 + dtB[j]; tmin = fmin(tmin, t); tmax = fmax(tmax, t); }
            if (lo_present(j)) { const double t = 1.0 + dtB[n + j]; tmin = fmin(tmin, t); tmax = fmax(tmax, t); }
        }
        tmin = red.min(tmin);
        tmax = red.max(tmax);
        const double shp = (tmin <= 0.0) ? 1.0 - tmin : 0.0;
        const double shd = (tmax >= 0.0) ? 1.0 + tmax : 0.0;
        DQ_ROWS(i, r) { const double t = 1.0 + DTA(i, r); TA(i, r) = t + shp; LA(i, r) = -t + shd; }
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
        double al_last = -1.0;            // the last step length (< 0: evaluate the residuals exactly)
        int since = 0;                    // iterations since the last exact evaluation
        const int res_every = a.res_every > 0 ? a.res_every : DQ_RES_EVERY;
        for (it = 0; it <= a.max_iter; ++it) {
            // exact residuals at the start, after a short step (the recurrence's (1 - al) hardly
            // contracts the error an inexact Newton solve leaves - pivot floor, near-singular K)
            // and every res_every iterations; scaled ones otherwise
            if (al_last < DQ_RES_SHORT || since + 1 >= res_every) {
                residuals(stat, feq, fin, csum, gscale, zmax, cmax);
                since = 0;
            } else {
                scaled_residuals(1.0 - al_last, stat, feq, fin, csum, zmax, cmax);
                ++since;
            }
            double feas = fmax(feq, fin);
            mu = csum * minv;
            auto converged = [&] {
                return stat <= a.tol_stat * (1.0 + gscale) && feas <= a.tol_feas * (1.0 + bscale) &&
                       mu <= a.tol_comp && cmax <= DQ_CMAX_K * a.tol_comp;
            };
            if (converged() && al_last >= 0.0) {   // confirm on exact residuals
                residuals(stat, feq, fin, csum, gscale, zmax, cmax);
                feas = fmax(feq, fin);
                mu = csum * minv;
            }
            if (converged()) { flag = 1; break; }
            if (!(isfinite(stat) && isfinite(feas) && isfinite(mu))) { flag = -8; break; }
            if (zmax > zbig) { flag = -3; break; }
            if (mu > DQ_MU_BLOWUP * mu_min && feas > DQ_FEAS_GUARD * (1.0 + bscale)) { flag = -2; break; }
            mu_min = fmin(mu_min, mu);
            if (it == a.max_iter) break;
            if (!factor()) { flag = -8; break; }
            DQ_ROWS(i, r) RCA(i, r) = TA(i, r) * LA(i, r);
            for (int j = tid; j < 2 * n; j += DT) rcB[j] = tB[j] * lB[j];
            __syncthreads();
            solve();
            double al = max_step();
            const double mua = comp_after(al) * minv;
            DST(4);
            double sg = mua / mu;
            sg = sg * sg * sg;
            const double smu = sg * mu;
            const double soc = (al < DQ_SOC_ALPHA && feas <= DQ_FEAS_GUARD * (1.0 + bscale)) ? 0.0 : 1.0;
            DQ_ROWS(i, r) RCA(i, r) = TA(i, r) * LA(i, r) + soc * DTA(i, r) * DLA(i, r) - smu;
            for (int j = tid; j < n; j += DT) {
                rcB[j] = up_present(j) ? tB[j] * lB[j] + soc * dtB[j] * dlB[j] - smu : 0.0;
                rcB[n + j] = lo_present(j) ? tB[n + j] * lB[n + j] + soc * dtB[n + j] * dlB[n + j] - smu : 0.0;
            }
            __syncthreads();
            solve();
            al = fmin(1.0, max_step() * a.tau);
            {   // the factor left fp64 range: keep the last finite iterate
                double bad = isfinite(al) ? 0.0 : 1.0;
                for (int j = tid; j < n; j += DT) if (!isfinite(dz[j])) bad = 1.0;
                for (int r = tid; r < me; r += DT) if (!isfinite(dy[r])) bad = 1.0;
                if (red.max(bad) != 0.0) { flag = -8; break; }
            }
            for (int j = tid; j < n; j += DT) {
                z[j] += al * dz[j];
                if (up_present(j)) { tB[j] += al * dtB[j]; lB[j] += al * dlB[j]; }
                if (lo_present(j)) { tB[n + j] += al * dtB[n + j]; lB[n + j] += al * dlB[n + j]; }
            }
            for (int r = tid; r < me; r += DT) y[r] += al * dy[r];
            DQ_ROWS(i, r) { TA(i, r) += al * DTA(i, r); LA(i, r) += al * DLA(i, r); }
            __syncthreads();
            al_last = al;
            DST(5);
        }
    }
#ifdef BQP_DSTAMPS
    if (inst == 0 && tid == 0)
        printf("DSTAMPS it %d rows %llu atw_res %llu res_rest %llu ada %llu chol %llu solve_pre %llu "
               "atw_sol %llu trsv %llu sol_post %llu step %llu upd %llu other %llu | chol: D %llu Dwait %llu "
               "P %llu Pwait %llu U %llu | trsv: pre+lc %llu chain %llu publish %llu update %llu | ada: "
               "issue %llu mfma %llu copywait %llu barrier %llu\n", it, dst_acc[0],
               dst_acc[10], dst_acc[11], dst_acc[1], dst_acc[2], dst_acc[3], dst_acc[7], dst_acc[8],
               dst_acc[9], dst_acc[4], dst_acc[5], dst_acc[6], dst_acc[12], dst_acc[13], dst_acc[14],
               dst_acc[15], dst_acc[16], dst_acc[17], dst_acc[18], dst_acc[19], dst_acc[20],
               dst_acc[21], dst_acc[22], dst_acc[23], dst_acc[24]);
#endif
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
    DQ_ROWS(i, r) {
        if (a.lam_ineqlin) a.lam_ineqlin[(int64_t)inst * m + r] = flag != -6 ? LA(i, r) : 0.0;
        if constexpr (RG) { tA[r] = TA(i, r); lA[r] = LA(i, r); }   // the repair launch's start
    }
    if constexpr (RG) {
        for (int j = tid; j < n; j += DT) W[L.z + j] = z[j];
        for (int j = tid; j < 2 * n; j += DT) { W[L.tB + j] = tB[j]; W[L.lB + j] = lB[j]; }
    }
#undef TA
#undef LA
#undef RIA
#undef RCA
#undef DTA
#undef DLA
#undef DQ_ROWS
    for (int r = tid; r < me; r += DT)
        if (a.lam_eqlin) a.lam_eqlin[(int64_t)inst * me + r] = flag != -6 ? y[r] : 0.0;
    fv = red.sum(fv);
    if (tid == 0) {
        if (a.fval) a.fval[inst] = fv;
        a.exitflag[inst] = flag;
        double* so = a.stats + (int64_t)inst * STATS_W;
        so[0] = (double)it; so[1] = stat; so[2] = fmax(feq, fin); so[3] = mu; so[4] = feq; so[5] = fin;
        so[6] = 0.0;
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
    // K, H, f, lb, ub, z, q, dz, rd, 6 x 2n bound-row vectors, 7 m-vectors, b, A (if small)
    return 2 * n * n + 8 * n + 12 * n + 8 * m + (m * n <= SW_A_LDS_MAX ? m * n : 0);
}


// A'v for the n <= 16 NT columns of A (column-major m x n): every lane accumulates its rows
// r = lane, lane + 64, ... for all columns at once, then one transposed wave sum (wsum_t) leaves
// column c's total in lane c (& 31).  No serial m-long chain on the n column lanes.
template <int NT>
__device__ __forceinline__ double atv(const double* A, const double* v, int m, int n, int lane) {
    constexpr int NM = 16 * NT;
    double acc[NM];
#pragma unroll
    for (int c = 0; c < NM; ++c) acc[c] = 0.0;
    for (int r = lane; r < m; r += 64) {
        const double vr = v[r];
#pragma unroll
        for (int c = 0; c < NM; ++c)
            if (c < n) acc[c] = fma(A[(int64_t)c * m + r], vr, acc[c]);
    }
    return wsum_t(acc, lane);
}

// small dense QPs (n <= 32, no equality rows): one wave per instance, vectors, H and K in LDS.
// K = H + A'DA on the matrix cores: v_mfma_f64_16x16x4_f64 tiles of A'(D A) over 4 rows of A per
// instruction (lane l supplies A[r0 + l/16][16 I + l%16] as the A operand and d_r times the same
// entry of column tile J as the B operand), one 16 x 16 tile for n <= 16, three for n <= 32
// (the lower block triangle).  The A'v products are transposed wave sums, the Cholesky and its
// triangular solves column-oriented with readlane broadcasts.  Same Mehrotra rules and start
// as dense_ipm_kernel; used for the LBMPC SQP sub-problems (n = N*nu + np = 11 at config C1) and
// small quadprog calls (F1 at N = 20: n = 21, m = 806).
template <int NT>
__global__ void __launch_bounds__(64) dense_wave_kernel(DenseKernelArgs a) {
    const int inst = blockIdx.x;
    if (inst >= a.batch || (a.skip && a.skip[inst])) return;
    const int n = a.n, m = a.m, lane = threadIdx.x;
    extern __shared__ double sm[];
    double* K = sm;                       // n x n column-major; lower Cholesky factor in place
    double* Hs = K + n * n;               // H (n x n column-major)
    double* fs = Hs + n * n;
    double* z = fs + n;
    double* q = z + n;
    double* dz = q + n;
    double* rd = dz + n;
    double* ubs = rd + n;
    double* lbs = ubs + n;
    double* tB = lbs + n;                 // bound rows: [upper 0..n-1, lower n..2n-1]
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
    double* bs = DA + m;
    const double* H = a.H + (int64_t)inst * a.sH;
    const double* f = a.f + (int64_t)inst * a.sf;
    const double* A = a.A ? a.A + (int64_t)inst * a.sA : nullptr;
    const double* b = a.b ? a.b + (int64_t)inst * a.sb : nullptr;
    const double* lb = a.lb ? a.lb + (int64_t)inst * a.slb : nullptr;
    const double* ub = a.ub ? a.ub + (int64_t)inst * a.sub : nullptr;
    // stage the instance's data: H, f, b, bounds (read every iteration); A when it is small
    for (int i = lane; i < n * n; i += 64) Hs[i] = H[i];
    for (int r = lane; r < m; r += 64) bs[r] = b[r];
    if (lane < n) {
        fs[lane] = f[lane];
        ubs[lane] = ub ? ub[lane] : INFINITY;
        lbs[lane] = lb ? lb[lane] : -INFINITY;
    }
    if (A && m * n <= SW_A_LDS_MAX) {
        double* As = bs + m;
        for (int i = lane; i < m * n; i += 64) As[i] = A[i];
        A = As;
    }
    wave_sync();
    // lane j < n owns variable j and both its bound rows
    const bool upj = lane < n && isfinite(ubs[lane]);
    const bool loj = lane < n && isfinite(lbs[lane]);
    const double ubj = upj ? ubs[lane] : 0.0, lbj = loj ? lbs[lane] : 0.0;
    const double minv = 1.0 / fmax(wsum((upj ? 1.0 : 0.0) + (loj ? 1.0 : 0.0)) + (double)m, 1.0);

    auto residuals = [&](double& stat, double& fin, double& csum, double& gscale, double& zmax, double& cmax) __attribute__((always_inline)) {
        double fe = 0.0, cs = 0.0, st = 0.0, gs = 0.0, zm = 0.0, cm = 0.0;
        double zc[16 * NT];
#pragma unroll
        for (int c = 0; c < 16 * NT; ++c) zc[c] = c < n ? z[c] : 0.0;
        for (int r = lane; r < m; r += 64) {
            double v = tA[r] - bs[r];
#pragma unroll
            for (int c = 0; c < 16 * NT; ++c)
                if (c < n) v = fma(A[(int64_t)c * m + r], zc[c], v);   // independent loads, one chain
            riA[r] = v;
            fe = fmax(fe, fabs(v));
            cs = fma(tA[r], lA[r], cs);
            cm = fmax(cm, tA[r] * lA[r]);
        }
        const double atl = atv<NT>(A, lA, m, n, lane);       // (A' lam)_lane
        if (lane < n) {
            const int j = lane;
            double v = fs[j];
#pragma unroll
            for (int i = 0; i < 16 * NT; ++i)
                if (i < n) v = fma(Hs[j * n + i], zc[i], v);
            gs = fabs(v);
            v += atl;
            riB[j] = 0.0; riB[n + j] = 0.0;
            if (upj) { v += lB[j]; riB[j] = z[j] + tB[j] - ubj; cs += tB[j] * lB[j]; cm = fmax(cm, tB[j] * lB[j]); }
            if (loj) { v -= lB[n + j]; riB[n + j] = -z[j] + tB[n + j] + lbj; cs += tB[n + j] * lB[n + j]; cm = fmax(cm, tB[n + j] * lB[n + j]); }
            fe = fmax(fe, fmax(fabs(riB[j]), fabs(riB[n + j])));
            rd[j] = v;
            st = fabs(v);
            zm = fabs(z[j]);
        }
        stat = wmax(st); fin = wmax(fe); csum = wsum(cs); gscale = wmax(gs); zmax = wmax(zm); cmax = wmax(cm);
        wave_sync();
    };

    // the residuals after a step of length al (as dense_ipm_kernel's scaled_residuals): (1 - al)
    // times the old ones, the complementarity and max |z| fresh, gscale from the last exact values
    auto scaled_residuals = [&](double s, double& stat, double& fin, double& csum, double& zmax,
                                double& cmax) __attribute__((always_inline)) {
        double fe = 0.0, cs = 0.0, st = 0.0, zm = 0.0, cm = 0.0;
        for (int r = lane; r < m; r += 64) {
            const double v = s * riA[r];
            riA[r] = v;
            fe = fmax(fe, fabs(v));
            cs = fma(tA[r], lA[r], cs);
            cm = fmax(cm, tA[r] * lA[r]);
        }
        if (lane < n) {
            const int j = lane;
            rd[j] *= s;
            riB[j] *= s; riB[n + j] *= s;
            if (upj) { cs += tB[j] * lB[j]; cm = fmax(cm, tB[j] * lB[j]); }
            if (loj) { cs += tB[n + j] * lB[n + j]; cm = fmax(cm, tB[n + j] * lB[n + j]); }
            fe = fmax(fe, fmax(fabs(riB[j]), fabs(riB[n + j])));
            st = fabs(rd[j]);
            zm = fabs(z[j]);
        }
        stat = wmax(st); fin = wmax(fe); csum = wsum(cs); zmax = wmax(zm); cmax = wmax(cm);
        wave_sync();
    };

    // Cholesky in registers: lane r < n holds row r of the lower factor (Lr[c], c <= r), its
    // reciprocal pivot (dinv) and, after the factorisation, column r of it (Lc[i] = L(i, r),
    // i > r, for the backward substitution).  Right-looking over the columns j: the pivot comes
    // from lane j by readlane, the scaled column entries L(c, j) from lane c - no LDS and no
    // barrier on the sequential chain.  fl >= 0: pivots floored at fl (static pivoting);
    // fl < 0: false at the first non-positive pivot (the convexity test).
    constexpr int NM = 16 * NT;
    double Lr[NM], Lc[NM], dinv = 0.0;
    auto load_rows = [&]() __attribute__((always_inline)) {                          // rows of the lower triangle of K (LDS)
#pragma unroll
        for (int c = 0; c < NM; ++c) Lr[c] = (c < n && c <= lane && lane < n) ? K[(int64_t)c * n + lane] : 0.0;
    };
    auto chol = [&](double fl) __attribute__((always_inline)) -> bool {
        bool ok = true;
#pragma unroll
        for (int jj = 0; jj < NM; ++jj) {
            if (jj < n && ok) {
                double d = rl(Lr[jj], jj);
                if (fl >= 0.0 && !(d > fl)) d = fl;
                if (!(d > 0.0)) {
                    ok = false;
                } else {
                    const double ljj = sqrt(d);
                    const double il = 1.0 / ljj;
                    if (lane > jj) Lr[jj] *= il;
                    if (lane == jj) { Lr[jj] = ljj; dinv = il; }
#pragma unroll
                    for (int c = jj + 1; c < NM; ++c) {
                        if (c < n) {
                            const double lcj = rl(Lr[jj], c);
                            if (lane >= c) Lr[c] = fma(-Lr[jj], lcj, Lr[c]);
                        }
                    }
                }
            }
        }
        if (ok) {
            // transpose through LDS (K is free now): lane c gets L(i, c) for i > c
            if (lane < n) {
#pragma unroll
                for (int c = 0; c < NM; ++c) if (c < n && c <= lane) K[(int64_t)lane * n + c] = Lr[c];
            }
            wave_sync();
#pragma unroll
            for (int ii = 0; ii < NM; ++ii) Lc[ii] = (ii < n && lane < ii) ? K[(int64_t)ii * n + lane] : 0.0;
            wave_sync();
        }
        return ok;
    };
    // K = H + A'DA + bound diagonal on the matrix cores, factored with the static pivot floor
    auto factor = [&]() __attribute__((always_inline)) -> bool {
        for (int r = lane; r < m; r += 64) DA[r] = lA[r] / tA[r];
        wave_sync();
        constexpr int NTL = NT * (NT + 1) / 2;     // lower block triangle: (0,0), (1,0), (1,1)
        dbl4 acc[NTL];
#pragma unroll
        for (int t = 0; t < NTL; ++t) acc[t] = dbl4{0.0, 0.0, 0.0, 0.0};
        const int c16 = lane & 15, k4 = lane >> 4;
        constexpr int KU = 4;                      // k-steps per trip: the loads of 4 steps in flight
        for (int r0 = 0; r0 < m; r0 += 4 * KU) {
            double av[KU][NT], dv[KU];
#pragma unroll
            for (int u = 0; u < KU; ++u) {
                const int r = r0 + 4 * u + k4;
                const bool rv = r < m;
                dv[u] = rv ? DA[r] : 0.0;
#pragma unroll
                for (int I = 0; I < NT; ++I) {
                    const int c = 16 * I + c16;
                    av[u][I] = (rv && c < n) ? A[(int64_t)c * m + r] : 0.0;
                }
            }
#pragma unroll
            for (int u = 0; u < KU; ++u) {
                int t = 0;
#pragma unroll
                for (int I = 0; I < NT; ++I)
#pragma unroll
                    for (int J = 0; J <= I; ++J, ++t)
                        acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[u][I], dv[u] * av[u][J], acc[t], 0, 0, 0);
            }
        }
        // tile (I, J), lane l, register e: K(16 I + l/16 + 4 e, 16 J + l%16)
        double dmx = 0.0;
        int t = 0;
#pragma unroll
        for (int I = 0; I < NT; ++I)
#pragma unroll
            for (int J = 0; J <= I; ++J, ++t)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int row = 16 * I + k4 + 4 * e, col = 16 * J + c16;
                    if (row < n && col < n && row >= col) {
                        double v = acc[t][e] + Hs[col * n + row];
                        if (row == col) {
                            if (isfinite(ubs[row])) v += lB[row] / tB[row];
                            if (isfinite(lbs[row])) v += lB[n + row] / tB[n + row];
                            dmx = fmax(dmx, fabs(v));
                        }
                        K[(int64_t)col * n + row] = v;        // lower: row, column col
                    }
                }
        const double kfl = DQ_PIV_FLOOR * fmax(wmax(dmx), 1e-300);
        wave_sync();
        load_rows();
        return chol(kfl);
    };

    // x = -(L L')^{-1} q with lane i holding entry i (n <= 32): column-oriented substitution on
    // the register factor, the solved entry broadcast by readlane
    auto chol_neg_solve = [&](double* x) __attribute__((always_inline)) {
        double v = (lane < n) ? -q[lane] : 0.0;
#pragma unroll
        for (int i = 0; i < NM; ++i) {                    // L y = -q
            if (i < n) {
                const double yi = rl(v, i) * rl(dinv, i);
                if (lane == i) v = yi;
                else if (lane > i) v = fma(-Lr[i], yi, v);
            }
        }
#pragma unroll
        for (int i = NM - 1; i >= 0; --i) {               // L' x = y
            if (i < n) {
                const double xi = rl(v, i) * rl(dinv, i);
                if (lane == i) v = xi;
                else if (lane < i) v = fma(-Lc[i], xi, v);
            }
        }
        if (lane < n) x[lane] = v;
        wave_sync();
    };

    auto solve = [&]() __attribute__((always_inline)) {
        for (int r = lane; r < m; r += 64) dlA[r] = (lA[r] * riA[r] - rcA[r]) / tA[r];
        wave_sync();
        const double atd = atv<NT>(A, dlA, m, n, lane);
        if (lane < n) {
            const int j = lane;
            double v = rd[j] + atd;
            if (upj) v += (lB[j] * riB[j] - rcB[j]) / tB[j];
            if (loj) v -= (lB[n + j] * riB[n + j] - rcB[n + j]) / tB[n + j];
            q[j] = v;
        }
        wave_sync();
        chol_neg_solve(dz);
        double dzc[NM];
#pragma unroll
        for (int c = 0; c < NM; ++c) dzc[c] = c < n ? dz[c] : 0.0;
        for (int r = lane; r < m; r += 64) {
            double v = 0.0;
#pragma unroll
            for (int c = 0; c < NM; ++c)
                if (c < n) v = fma(A[(int64_t)c * m + r], dzc[c], v);
            dtA[r] = -riA[r] - v;
            dlA[r] = (-rcA[r] - lA[r] * dtA[r]) / tA[r];
        }
        if (lane < n) {
            const int j = lane;
            dtB[j] = dlB[j] = dtB[n + j] = dlB[n + j] = 0.0;
            if (upj) { dtB[j] = -riB[j] - dz[j]; dlB[j] = (-rcB[j] - lB[j] * dtB[j]) / tB[j]; }
            if (loj) { dtB[n + j] = -riB[n + j] + dz[j]; dlB[n + j] = (-rcB[n + j] - lB[n + j] * dtB[n + j]) / tB[n + j]; }
        }
        wave_sync();
    };
    auto max_step = [&]() -> double {
        double al = 1.0;
#define DW_RATIO(v, dv) if ((dv) < 0.0) al = fmin(al, -(v) / (dv));
        for (int r = lane; r < m; r += 64) { DW_RATIO(tA[r], dtA[r]); DW_RATIO(lA[r], dlA[r]); }
        if (lane < n) {
            const int j = lane;
            if (upj) { DW_RATIO(tB[j], dtB[j]); DW_RATIO(lB[j], dlB[j]); }
            if (loj) { DW_RATIO(tB[n + j], dtB[n + j]); DW_RATIO(lB[n + j], dlB[n + j]); }
        }
#undef DW_RATIO
        return wmin(al);
    };
    auto comp_after = [&](double al) -> double {
        double c = 0.0;
        for (int r = lane; r < m; r += 64) c += (tA[r] + al * dtA[r]) * (lA[r] + al * dlA[r]);
        if (lane < n) {
            const int j = lane;
            if (upj) c += (tB[j] + al * dtB[j]) * (lB[j] + al * dlB[j]);
            if (loj) c += (tB[n + j] + al * dtB[n + j]) * (lB[n + j] + al * dlB[n + j]);
        }
        return wsum(c);
    };

    // initial point (as dense_ipm_kernel)
    if (lane < n) {
        const int j = lane;
        z[j] = 0.0;
        tB[j] = tB[n + j] = 1.0;
        lB[j] = upj ? 1.0 : 0.0;
        lB[n + j] = loj ? 1.0 : 0.0;
        rcB[j] = upj ? 1.0 : 0.0;
        rcB[n + j] = loj ? 1.0 : 0.0;
    }
    for (int r = lane; r < m; r += 64) { tA[r] = 1.0; lA[r] = 1.0; rcA[r] = 1.0; }
    wave_sync();
    double bsl = 0.0;
    for (int r = lane; r < m; r += 64) bsl = fmax(bsl, fabs(bs[r]));
    if (upj) bsl = fmax(bsl, fabs(ubj));
    if (loj) bsl = fmax(bsl, fabs(lbj));
    const double bscale = wmax(bsl);
    const double zbig = DQ_Z_BIG * (1.0 + bscale + wmax(lane < n ? fabs(fs[lane]) : 0.0));
    int flag = 0;
    {
        // convexity test: Cholesky of H + CONVEX_EPS max(1, max H_ii) I without pivot floor
        const double sh = DQ_CONVEX_EPS * fmax(1.0, wmax(lane < n ? fabs(Hs[lane * n + lane]) : 0.0));
        for (int e2 = lane; e2 < n * n; e2 += 64) {
            const int i = e2 % n, j = e2 / n;
            K[e2] = Hs[e2] + (i == j ? sh : 0.0);
        }
        wave_sync();
        load_rows();
        wave_sync();
        if (!chol(-1.0)) flag = -6;
    }
    const double feq = 0.0;                 // no equality rows on this path
    double stat = 0.0, fin = 0.0, csum = 0.0, gscale = 0.0, zmax = 0.0, cmax = 0.0;
    residuals(stat, fin, csum, gscale, zmax, cmax);
    if (flag == 0 && !factor()) flag = -8;
    if (flag == 0) {
        solve();
        double tmin = INFINITY, tmax = -INFINITY;
        if (lane < n) z[lane] += dz[lane];
        for (int r = lane; r < m; r += 64) { const double t = 1.0 + dtA[r]; tmin = fmin(tmin, t); tmax = fmax(tmax, t); }
        if (upj) { const double t = 1.0 + dtB[lane]; tmin = fmin(tmin, t); tmax = fmax(tmax, t); }
        if (loj) { const double t = 1.0 + dtB[n + lane]; tmin = fmin(tmin, t); tmax = fmax(tmax, t); }
        tmin = wmin(tmin);
        tmax = wmax(tmax);
        const double shp = (tmin <= 0.0) ? 1.0 - tmin : 0.0;
        const double shd = (tmax >= 0.0) ? 1.0 + tmax : 0.0;
        for (int r = lane; r < m; r += 64) { const double t = 1.0 + dtA[r]; tA[r] = t + shp; lA[r] = -t + shd; }
        if (lane < n) {
            const int j = lane;
            const double tu = 1.0 + dtB[j], tl = 1.0 + dtB[n + j];
            tB[j] = upj ? tu + shp : 1.0; lB[j] = upj ? -tu + shd : 0.0;
            tB[n + j] = loj ? tl + shp : 1.0; lB[n + j] = loj ? -tl + shd : 0.0;
        }
        wave_sync();
    }
    int it = 0;
    double mu = 0.0, mu_min = INFINITY;
    if (flag == 0) {
        double al_last = -1.0;            // the last step length (< 0: evaluate the residuals exactly)
        int since = 0;                    // iterations since the last exact evaluation
        const int res_every = a.res_every > 0 ? a.res_every : DQ_RES_EVERY;
        for (it = 0; it <= a.max_iter; ++it) {
            // exact residuals at the start, after a short step (the recurrence's (1 - al) hardly
            // contracts the error an inexact Newton solve leaves - pivot floor, near-singular K)
            // and every res_every iterations; scaled ones otherwise
            if (al_last < DQ_RES_SHORT || since + 1 >= res_every) {
                residuals(stat, fin, csum, gscale, zmax, cmax);
                since = 0;
            } else {
                scaled_residuals(1.0 - al_last, stat, fin, csum, zmax, cmax);
                ++since;
            }
            double feas = fin;
            mu = csum * minv;
            auto converged = [&] {
                return stat <= a.tol_stat * (1.0 + gscale) && feas <= a.tol_feas * (1.0 + bscale) &&
                       mu <= a.tol_comp && cmax <= DQ_CMAX_K * a.tol_comp;
            };
            if (converged() && al_last >= 0.0) {   // confirm on exact residuals
                residuals(stat, fin, csum, gscale, zmax, cmax);
                feas = fin;
                mu = csum * minv;
            }
            if (converged()) { flag = 1; break; }
            if (!(isfinite(stat) && isfinite(feas) && isfinite(mu))) { flag = -8; break; }
            if (zmax > zbig) { flag = -3; break; }
            if (mu > DQ_MU_BLOWUP * mu_min && feas > DQ_FEAS_GUARD * (1.0 + bscale)) { flag = -2; break; }
            mu_min = fmin(mu_min, mu);
            if (it == a.max_iter) break;
            if (!factor()) { flag = -8; break; }
            for (int r = lane; r < m; r += 64) rcA[r] = tA[r] * lA[r];
            if (lane < n) { rcB[lane] = tB[lane] * lB[lane]; rcB[n + lane] = tB[n + lane] * lB[n + lane]; }
            wave_sync();
            solve();
            double al = max_step();
            const double mua = comp_after(al) * minv;
            double sg = mua / mu;
            sg = sg * sg * sg;
            const double smu = sg * mu;
            const double soc = (al < DQ_SOC_ALPHA && feas <= DQ_FEAS_GUARD * (1.0 + bscale)) ? 0.0 : 1.0;
            for (int r = lane; r < m; r += 64) rcA[r] = tA[r] * lA[r] + soc * dtA[r] * dlA[r] - smu;
            if (lane < n) {
                const int j = lane;
                rcB[j] = upj ? tB[j] * lB[j] + soc * dtB[j] * dlB[j] - smu : 0.0;
                rcB[n + j] = loj ? tB[n + j] * lB[n + j] + soc * dtB[n + j] * dlB[n + j] - smu : 0.0;
            }
            wave_sync();
            solve();
            al = fmin(1.0, max_step() * a.tau);
            // the factor left fp64 range: keep the last finite iterate
            if (wmax((isfinite(al) && (lane >= n || isfinite(dz[lane]))) ? 0.0 : 1.0) != 0.0) { flag = -8; break; }
            if (lane < n) {
                const int j = lane;
                z[j] += al * dz[j];
                if (upj) { tB[j] += al * dtB[j]; lB[j] += al * dlB[j]; }
                if (loj) { tB[n + j] += al * dtB[n + j]; lB[n + j] += al * dlB[n + j]; }
            }
            for (int r = lane; r < m; r += 64) { tA[r] += al * dtA[r]; lA[r] += al * dlA[r]; }
            wave_sync();
            al_last = al;
        }
    }
    const int pm = pol_mode(a, inst);
    if (pm && (flag == 0 || flag == -8 || (pm == 2 && flag == 1)) && a.work) {
        // hand the iterate to dense_polish_kernel through the instance's workspace (DWork)
        const DWork L = DWork::make(n, m, 0);
        double* W = a.work + (int64_t)inst * a.work_stride;
        if (lane < n) {
            W[L.z + lane] = z[lane];
            W[L.tB + lane] = tB[lane]; W[L.tB + n + lane] = tB[n + lane];
            W[L.lB + lane] = lB[lane]; W[L.lB + n + lane] = lB[n + lane];
        }
        for (int r = lane; r < m; r += 64) { W[L.tA + r] = tA[r]; W[L.lA + r] = lA[r]; }
    }
    double fv = 0.0;
    if (lane < n) {
        const int j = lane;
        double hz = 0.0;
        for (int i = 0; i < n; ++i) hz += Hs[j * n + i] * z[i];
        fv = z[j] * (0.5 * hz + fs[j]);
        a.x[(int64_t)inst * n + j] = z[j];
        if (a.lam_lower) a.lam_lower[(int64_t)inst * n + j] = (loj && flag != -6) ? lB[n + j] : 0.0;
        if (a.lam_upper) a.lam_upper[(int64_t)inst * n + j] = (upj && flag != -6) ? lB[j] : 0.0;
    }
    for (int r = lane; r < m; r += 64)
        if (a.lam_ineqlin) a.lam_ineqlin[(int64_t)inst * m + r] = flag != -6 ? lA[r] : 0.0;
    fv = wsum(fv);
    if (lane == 0) {
        if (a.fval) a.fval[inst] = fv;
        a.exitflag[inst] = flag;
        double* so = a.stats + (int64_t)inst * STATS_W;
        so[0] = (double)it; so[1] = stat; so[2] = fmax(feq, fin); so[3] = mu; so[4] = feq; so[5] = fin;
        so[6] = 0.0;
    }
}

// the active-set polish of the instances that ended 0 / -8 (dense_polish), a kernel of its own;
// polish = 2 (the SQP sub-problems of bqp_lbmpc_solve_batched) polishes converged instances too,
// so that the SQP steps are the exact active-set solutions (as oracle/dense_qp.py's are)
// so that its registers do not weigh on the IPM kernels; the iterate is in the workspace (DWork
// offsets: dense_ipm_kernel keeps it there, dense_wave_kernel stores it on those exits).  On
// acceptance x, the multipliers, fval, the flag (1) and the stats are rewritten.
__global__ void __launch_bounds__(DT) dense_polish_kernel(DenseKernelArgs a) {
    const int inst = blockIdx.x;
    if (inst >= a.batch) return;
    if (a.skip && a.skip[inst]) return;
    const int flag = a.exitflag[inst];
    const int pm = pol_mode(a, inst);
    if (!pm || !(flag == 0 || flag == -8 || (pm == 2 && flag == 1))) return;
    const int n = a.n, m = a.m, me = a.me, tid = threadIdx.x;
    __shared__ double sc[16];
    __shared__ double xs[DT];
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
    double *z = W + L.z, *y = W + L.y, *tA = W + L.tA, *lA = W + L.lA, *tB = W + L.tB, *lB = W + L.lB;
    // rows present, data scale and a finite iterate (oracle/dense_ipm.py: m > 0, |Hz + f| finite)
    double cnt = 0.0, bsl = 0.0, zf = 0.0;
    for (int r = tid; r < m; r += DT) bsl = fmax(bsl, fabs(b[r]));
    for (int r = tid; r < me; r += DT) bsl = fmax(bsl, fabs(e[r]));
    for (int j = tid; j < n; j += DT) {
        if (ub && isfinite(ub[j])) { cnt += 1.0; bsl = fmax(bsl, fabs(ub[j])); }
        if (lb && isfinite(lb[j])) { cnt += 1.0; bsl = fmax(bsl, fabs(lb[j])); }
        if (!isfinite(z[j])) zf = 1.0;
    }
    const double rows = red.sum(cnt) + (double)m;
    const double bscale = red.max(bsl);
    if (rows == 0.0 || red.max(zf) != 0.0) return;
    extern __shared__ double plds[];
    double* Kl = (size_t)n * n <= DQ_POL_KLDS ? plds : nullptr;
    const DPolish pp{n, m, me, H, f, A, b, E, e, lb, ub, z, y, tA, lA, tB, lB, W, bscale, a.tol_stat, Kl};
    if (!dense_polish<DT, Red>(pp, sc, xs)) return;
    const double stat = sc[10], feas = sc[11];
    double fv = 0.0;
    for (int j = tid; j < n; j += DT) {
        double hz = 0.0;
        for (int i = 0; i < n; ++i) hz += H[(int64_t)j * n + i] * z[i];
        fv += z[j] * (0.5 * hz + f[j]);
        a.x[(int64_t)inst * n + j] = z[j];
        if (a.lam_lower) a.lam_lower[(int64_t)inst * n + j] = (lb && isfinite(lb[j])) ? lB[n + j] : 0.0;
        if (a.lam_upper) a.lam_upper[(int64_t)inst * n + j] = (ub && isfinite(ub[j])) ? lB[j] : 0.0;
    }
    for (int r = tid; r < m; r += DT)
        if (a.lam_ineqlin) a.lam_ineqlin[(int64_t)inst * m + r] = lA[r];
    for (int r = tid; r < me; r += DT)
        if (a.lam_eqlin) a.lam_eqlin[(int64_t)inst * me + r] = y[r];
    fv = red.sum(fv);
    if (tid == 0) {
        if (a.fval) a.fval[inst] = fv;
        a.exitflag[inst] = 1;
        double* so = a.stats + (int64_t)inst * STATS_W;
        so[1] = stat; so[2] = feas; so[3] = 0.0; so[4] = 0.0; so[5] = feas; so[6] = 1.0;
    }
}

// dynamic LDS above 64 KB needs the kernel attribute on the current device; set on every launch
// (a host call of about a microsecond) so that no process-wide state is kept (include/bqp.h: handles
// on several host threads and devices share nothing)
template <bool KL, bool RG>
static hipError_t dense_lds_attr(size_t lds) {
    if (lds <= 64 * 1024) return hipSuccess;
    return hipFuncSetAttribute((const void*)dense_ipm_kernel<KL, RG>, hipFuncAttributeMaxDynamicSharedMemorySize,
                               DENSE_LDS_MAX);
}

// the row state in registers (dense_ipm_kernel RG): at most DQ_RPT rows per thread, the A'DA on
// the two global_load_lds buffers (the only path that forms the tile row weights from registers)
// and A'w with the row weights staged in LDS whole.  BQP_DENSE_NO_RG=1: the workspace form (A/B).
static bool dense_rows_in_regs(int n, int m) {
    if (const char* e = getenv("BQP_DENSE_NO_RG")) if (atoi(e) != 0) return false;
    return m > 0 && m <= DQ_RPT * DT && dense_k_lds(n) && dense_glds(n) && m + n <= TILE * dense_ts(n) &&
           dense_lds_bytes(n) + sizeof(double) * DQ_NVEC * n <= DENSE_LDS_MAX;
}

// H <- (H + H')/2 in place for `count` n x n matrices `stride` doubles apart (the host entry's
// staging copy): MATLAB quadprog solves with the symmetric part of a non-symmetric H, and the
// kernels read both triangles of H (the factor the lower one, the residual H z whole rows).  A
// symmetric H is left bit for bit as it was ((h + h) / 2 = h exactly).
__global__ void dense_symmetrize_kernel(double* H, int n, int64_t stride) {
    double* Hb = H + (int64_t)blockIdx.y * stride;
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= (int64_t)n * n) return;
    const int i = (int)(e % n), j = (int)(e / n);
    if (i <= j) return;                 // one thread per pair (i > j)
    const double v = 0.5 * (Hb[(int64_t)j * n + i] + Hb[(int64_t)i * n + j]);
    Hb[(int64_t)j * n + i] = v;
    Hb[(int64_t)i * n + j] = v;
}

hipError_t launch_dense_symmetrize(double* H, int n, int count, int64_t stride, hipStream_t st) {
    if (n <= 1 || count <= 0) return hipSuccess;
    const int64_t nn = (int64_t)n * n;
    hipLaunchKernelGGL(dense_symmetrize_kernel, dim3((unsigned)((nn + 255) / 256), count), dim3(256), 0, st,
                       H, n, stride);
    return hipGetLastError();
}

hipError_t launch_dense(const DenseKernelArgs& a0, hipStream_t st) {
    DenseKernelArgs a = a0;
    // diagnostic: BQP_DENSE_RES_EVERY=k evaluates the residuals exactly every k iterations (1:
    // never by the recurrence; tests/test_gpu_quadprog_status.py compares the two)
    if (a.res_every <= 0) {
        if (const char* e = getenv("BQP_DENSE_RES_EVERY")) a.res_every = atoi(e);
    }
    if (a.n > 256 || a.me > 256) return hipErrorInvalidValue;
    if (a.me == 0 && a.n <= SW_NMAX && small_lds_doubles(a.n, a.m) <= SW_LDS_MAX) {
        const size_t lds = sizeof(double) * small_lds_doubles(a.n, a.m);
        if (a.n <= 16)
            hipLaunchKernelGGL(dense_wave_kernel<1>, dim3(a.batch), dim3(64), lds, st, a);
        else
            hipLaunchKernelGGL(dense_wave_kernel<2>, dim3(a.batch), dim3(64), lds, st, a);
    } else {
        const size_t lds = dense_lds_bytes(a.n);
        if (lds > DENSE_LDS_MAX) return hipErrorInvalidValue;
        if (dense_rows_in_regs(a.n, a.m)) {
            const size_t ldsr = lds + sizeof(double) * DQ_NVEC * a.n;
            hipError_t e = dense_lds_attr<true, true>(ldsr);
            if (e != hipSuccess) return e;
            hipLaunchKernelGGL((dense_ipm_kernel<true, true>), dim3(a.batch), dim3(DT), ldsr, st, a);
        } else if (dense_k_lds(a.n)) {
            hipError_t e = dense_lds_attr<true, false>(lds);
            if (e != hipSuccess) return e;
            hipLaunchKernelGGL((dense_ipm_kernel<true, false>), dim3(a.batch), dim3(DT), lds, st, a);
        } else {
            hipError_t e = dense_lds_attr<false, false>(lds);
            if (e != hipSuccess) return e;
            hipLaunchKernelGGL((dense_ipm_kernel<false, false>), dim3(a.batch), dim3(DT), lds, st, a);
        }
    }
    hipError_t err = hipGetLastError();
    if (err != hipSuccess || (!a.polish && !a.pol_it) || !a.work) return err;
    // K of the polish in LDS when it fits (dense_polish: DPolish::Kl)
    const size_t plds = (size_t)a.n * a.n <= DQ_POL_KLDS ? sizeof(double) * a.n * a.n : 0;
    if (plds > 64 * 1024) {
        hipError_t e = hipFuncSetAttribute((const void*)dense_polish_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                           (int)(sizeof(double) * DQ_POL_KLDS));
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(dense_polish_kernel, dim3(a.batch), dim3(DT), plds, st, a);
    return hipGetLastError();
}

}  // namespace bqp
