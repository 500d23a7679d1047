// bqp_lbmpc.hip — learning-based MPC on gfx950: the batched Nadaraya-Watson oracle and the
// device side of the Gauss-Newton SQP that solves the reference's LBMPC problems (forms F3/F4).
//
// Reference: functions/oracleL2NW.m:26-36 / examples/hybrid_LBMPC_casadi.m:331-358 (the NW
// oracle), models/learnedModel.m:25 (x+ = A x + B u + g), functions/costLBMPC.m:20-45 and
// constraintsLBMPC.m:18-45 (F3), examples/hybrid_LBMPC_casadi.m:250-311 (F4).  The algorithm
// is stated in oracle/lbmpc.py; the host loop is bqp_lbmpc_solve_batched_device (bqp_api.cpp).
//
// Kernels (one SQP iteration = rollout(GN) -> normal [-> hess] -> dense QP -> rollout(trials) -> update):
//   nw_oracle_kernel      one wave per query point: g(xi), dg/dxi; lanes over the data window
//   lbmpc_rollout_kernel  one wave per (instance, trial): the learned rollout u = K x + v,
//                         x+ = A x + B u + g(x, u) (NW sums over the window held in LDS, lanes
//                         over data points, DPP wave reductions), the nominal rollout, the
//                         weighted residuals of the quadratic cost and - GN mode - the forward
//                         sensitivities dx/dz (lanes over the columns of z) written as the rows
//                         of the residual Jacobian Jr (row-major, coalesced along z)
//   lbmpc_normal_kernel   one workgroup per instance: H = 2 Jr'Jr on the fp64 matrix cores and
//                         f = 2 Jr'er through LDS row tiles, and the QP right-hand side b_in - A_in z
//   lbmpc_hess_kernel     (exact Hessian) one workgroup per instance: H_GN + the second-order
//                         term of the learned dynamics (its row products on the matrix cores),
//                         kept if its LDS Cholesky succeeds
//   lbmpc_update_kernel   one wave per instance: convergence test (step, NLP stationarity
//                         |f + A_in' lam|), Armijo choice among the trial step lengths, z += a d
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "bqp_internal.h"
#include "bqp_wave.h"

namespace bqp {

#define LB_WAVE 64
#define LB_MAXQ 512      // NW window capacity (data points) held in LDS
#define LB_CPL 4         // z columns per lane of the update kernel's column table (n <= 256)
#define LB_RCPL 2        // z columns per lane in the rollouts' sensitivity recursion: n <= LB_MAXN = 128
                         // (lbmpc_supported); round 6 - with 4, half the recursion ran on columns past n

// a readlane broadcast kept in vector registers (round 6): as scalar registers the 50 totals of
// the Hessian rollout's NW sums outgrew the SGPR file and were spilled to and reloaded from VGPR
// lanes (~780 readlanes per stage in the stage-cost phase of the ISA)
__device__ __forceinline__ double rlv(double v, int src) {
    double r = rl(v, src);
    asm volatile("" : "+v"(r));
    return r;
}
// the lane index made opaque inside a loop: the masks derived from it (column j < n, j == k, ...)
// are formed where they are used instead of hoisted out of the stage loop and kept in scalar
// registers for its whole length
__device__ __forceinline__ int lb_opq(int v) {
    asm volatile("" : "+v"(v));
    return v;
}
// NW sums at xi over the window in LDS: point i at D[wr i .. wr i + wr - 1], wr = 7 rows
// [X; Y] (every point counts in the normaliser, oracleL2NW.m / hybrid_LBMPC_casadi.m:331-358) or
// wr = 8 rows [X; Y; v] (casadiL2NW.m:14-28: the normaliser is lambda + sum_j v_j k_j, the
// numerator is not masked - points that are not yet valid hold Y = 0).  Returns g (4) and, if
// JAC, dg (4 x 3, row-major); every lane ends with the uniform values.
// With HESS also the second derivatives d2g (4 x 6: the unique entries 00 01 02 11 12 22 of each
// symmetric 3 x 3 Hessian): with c = 2/h^2, d2k_j = k_j (c^2 d_j d_j' - c I), d_j = X_j - xi,
//   d2g_i = (d2N_i - g_i d2D - dg_i dD' - dD dg_i') / D.
template <bool JAC, bool HESS = false>
__device__ __forceinline__ void nw_eval(const double* D, int q, int wr, double hinv2, double lam,
                                        const double (&xi)[3], double (&g)[4], double (&dg)[4][3],
                                        int lane, double (*d2g)[6] = nullptr) {
    double s = 0.0, sy[4] = {0, 0, 0, 0}, ds[3] = {0, 0, 0}, dsy[4][3] = {};
    double s2[6] = {}, sy2[4][6] = {};
    for (int i = lane; i < q; i += LB_WAVE) {
        const double* p = D + wr * i;
        const double d0 = p[0] - xi[0], d1 = p[1] - xi[1], d2 = p[2] - xi[2];
        const double k = exp(-(d0 * d0 + d1 * d1 + d2 * d2) * hinv2);
        const double v = wr == 8 ? p[7] : 1.0;
        s += k * v;
#pragma unroll
        for (int r = 0; r < 4; ++r) sy[r] += p[3 + r] * k;
        if (JAC) {
            const double c = 2.0 * hinv2 * k;
            const double dk[3] = {c * d0, c * d1, c * d2};
#pragma unroll
            for (int c3 = 0; c3 < 3; ++c3) {
                ds[c3] += dk[c3] * v;
#pragma unroll
                for (int r = 0; r < 4; ++r) dsy[r][c3] += p[3 + r] * dk[c3];
            }
        }
        if (HESS) {
            const double dd[6] = {d0 * d0, d0 * d1, d0 * d2, d1 * d1, d1 * d2, d2 * d2};
#pragma unroll
            for (int e = 0; e < 6; ++e) {
                const double kd = k * dd[e];
                s2[e] += kd * v;
#pragma unroll
                for (int r = 0; r < 4; ++r) sy2[r][e] += p[3 + r] * kd;
            }
        }
    }
    // the wave sums of all accumulators together: transposed sums (wsum_t: lane k ends with the
    // total of value k), each total then broadcast by readlane - ~3x fewer DPP steps than one
    // 6-step reduction per value (50 of them in the Hessian rollout)
    {
        constexpr int KA = JAC ? 20 : 5;
        double va[KA];
        va[0] = s;
#pragma unroll
        for (int r = 0; r < 4; ++r) va[1 + r] = sy[r];
        if constexpr (JAC) {
#pragma unroll
            for (int c3 = 0; c3 < 3; ++c3) {
                va[5 + c3] = ds[c3];
#pragma unroll
                for (int r = 0; r < 4; ++r) va[8 + 3 * r + c3] = dsy[r][c3];
            }
        }
        const double ta = wsum_t(va, lane);
        s = rlv(ta, 0);
#pragma unroll
        for (int r = 0; r < 4; ++r) sy[r] = rlv(ta, 1 + r);
        if constexpr (JAC) {
#pragma unroll
            for (int c3 = 0; c3 < 3; ++c3) {
                ds[c3] = rlv(ta, 5 + c3);
#pragma unroll
                for (int r = 0; r < 4; ++r) dsy[r][c3] = rlv(ta, 8 + 3 * r + c3);
            }
        }
        if constexpr (HESS) {
            double vb[30];
#pragma unroll
            for (int e = 0; e < 6; ++e) {
                vb[e] = s2[e];
#pragma unroll
                for (int r = 0; r < 4; ++r) vb[6 + 6 * r + e] = sy2[r][e];
            }
            const double tb = wsum_t(vb, lane);
#pragma unroll
            for (int e = 0; e < 6; ++e) {
                s2[e] = rlv(tb, e);
#pragma unroll
                for (int r = 0; r < 4; ++r) sy2[r][e] = rlv(tb, 6 + 6 * r + e);
            }
        }
    }
    const double den = lam + s;
    const double iden = 1.0 / den;
#pragma unroll
    for (int r = 0; r < 4; ++r) g[r] = sy[r] * iden;
    if (JAC) {
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int c3 = 0; c3 < 3; ++c3) dg[r][c3] = (dsy[r][c3] - g[r] * ds[c3]) * iden;
    }
    if (HESS) {
        const double c = 2.0 * hinv2;
        constexpr int EA[6] = {0, 0, 0, 1, 1, 2}, EB[6] = {0, 1, 2, 1, 2, 2};
#pragma unroll
        for (int e = 0; e < 6; ++e) {
            const int ea = EA[e], eb = EB[e];
            const double id = ea == eb ? 1.0 : 0.0;
            const double d2D = c * c * s2[e] - c * s * id;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const double d2N = c * c * sy2[r][e] - c * sy[r] * id;
                d2g[r][e] = (d2N - g[r] * d2D - dg[r][ea] * ds[eb] - ds[ea] * dg[r][eb]) * iden;
            }
        }
    }
}

#ifdef BQP_RSTAMPS
// diagnostic build only: s_memtime cycles per phase of the learned rollout, printed for instance 0
#define RST_DECL unsigned long long rst_last = __builtin_amdgcn_s_memtime(), rst_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0}
#define RST(id)                                                            \
    do {                                                                   \
        __builtin_amdgcn_s_waitcnt(0);                                     \
        const unsigned long long _t = __builtin_amdgcn_s_memtime();        \
        rst_acc[id] += _t - rst_last;                                      \
        rst_last = _t;                                                     \
    } while (0)
#define RST_PRINT(tag)                                                     \
    do {                                                                   \
        if (b == 0 && t == 0 && lane == 0)                                 \
            printf("RSTAMPS %s gn %d pre %llu nw %llu post %llu term %llu costate %llu pass2 %llu\n", tag, gn, \
                   rst_acc[0], rst_acc[1], rst_acc[2], rst_acc[3], rst_acc[4], rst_acc[5]); \
    } while (0)
#else
#define RST_DECL do { } while (0)
#define RST(id) do { } while (0)
#define RST_PRINT(tag) do { } while (0)
#endif

__device__ __forceinline__ void load_window(double* D, const double* src, int len, int lane) {
    for (int i = lane; i < len; i += LB_WAVE) D[i] = src[i];
    wave_sync();
}

// ------------------------------------------------------------------------------------------
// standalone oracle: g, dg at a batch of query points (oracleL2NW.m)
// ------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(64) nw_oracle_kernel(int batch, int q, const double* data,
                                                       int64_t sdata, const double* xi_in,
                                                       double* g_out, double* dg_out,
                                                       double hinv2, double lam) {
    __shared__ double D[7 * LB_MAXQ];
    const int b = blockIdx.x;
    const int lane = threadIdx.x;
    if (b >= batch) return;
    load_window(D, data + (int64_t)b * sdata, 7 * q, lane);
    double xi[3] = {xi_in[3 * b], xi_in[3 * b + 1], xi_in[3 * b + 2]};
    double g[4], dg[4][3];
    nw_eval<true>(D, q, 7, hinv2, lam, xi, g, dg, lane);
    if (lane == 0) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            g_out[4 * b + r] = g[r];
#pragma unroll
            for (int c = 0; c < 3; ++c)
                if (dg_out) dg_out[12 * b + 3 * r + c] = dg[r][c];   // row-major 4 x 3
        }
    }
}

// ------------------------------------------------------------------------------------------
// rollout: cost (all modes), residual Jacobian (GN mode) and, with a.hess, the second-order term
// of the learned dynamics (oracle/lbmpc.py newton_model):
//   sum_k Xi_k' W_k Xi_k,  W_k = sum_i p_{k+1,i} d2g_i(xi_k),  Xi_k = dxi_k/dz (3 x n),
// with the costate p_k = dJ/dx_k of the learned rollout (backward recursion
// p_k = dphi_k/dx_k + (A + B K + G_x + g_u K)' p_{k+1}, p_N = terminal gradient).  The forward
// pass keeps dg, d2g and dphi/dx per stage in LDS (LB_SS doubles), the costate pass turns d2g
// into W_k, and a second sensitivity pass writes the rows Xi_k (Jr2) and W_k Xi_k (Tr2) that
// lbmpc_hess_kernel contracts.  LDS is dynamic: the window (wrows x q), then the stage store.
// ------------------------------------------------------------------------------------------
#define LB_SS 40         // per stage: dg 4x3 | d2g 4x6 (W_k in the first 6 after the costate pass) | dphi/dx 4
template <int NX, int NU, int NP, bool HESS>
__global__ void __launch_bounds__(64) lbmpc_rollout_kernel(LbmpcArgs a, int gn) {
    static_assert(NX == 4 && NU == 1, "NW input xi = [x_1; x_2; u] with the 4-state model, nu = 1");
    extern __shared__ double lbd[];
    double* D = lbd;
    int lane = threadIdx.x;              // re-made opaque at each stage (lb_opq)
    const int nt = gn ? 1 : a.ntrial;
    const int b = blockIdx.x / nt, t = blockIdx.x % nt;
    if (b >= a.batch || a.done[b]) return;
    const int N = a.N, n = a.n, nr = a.nr;
    constexpr bool hess = HESS;      // instantiated for the GN launch of an exact-Hessian solve
    double* SS = lbd + ((a.wrows * a.q + 1) & ~1);
    load_window(D, a.data + (int64_t)b * a.sdata, a.wrows * a.q, lane);
    const double alpha = gn ? 0.0 : ldexp(1.0, -t);
    const double* z = a.z + (int64_t)b * n;
    const double* dz = a.d + (int64_t)b * n;
    // the trial point z + alpha d in LDS (n <= 2 x 64): one global load per stage put a memory
    // round trip at the head of every stage's chain
    __shared__ double zsh[LB_WAVE * LB_RCPL];
    for (int j = lane; j < n; j += LB_WAVE) zsh[j] = gn ? z[j] : z[j] + alpha * dz[j];
    wave_sync();
    auto zv = [&](int j) __attribute__((always_inline)) -> double { return zsh[j]; };
    // column-major small matrices, copied to LDS once: read from global memory inside the stage
    // loop they were reloaded after every Jacobian-row store (the compiler cannot rule out
    // aliasing), a chain of dependent loads per stage (~60 % of the Hessian rollout's cycles in
    // its stamps)
    constexpr int OA = 0, OB = OA + NX * NX, OK = OB + NX * NU, OL = OK + NU * NX, OP = OL + NX * NP,
                  OQ = OP + NU * NP, OR = OQ + NX * NX, OEND = OR + NU * NU;
    __shared__ double cst[OEND];
    for (int i = lane; i < OEND; i += LB_WAVE) {
        double v;
        if (i < OB) v = a.A[i - OA];
        else if (i < OK) v = a.B[i - OB];
        else if (i < OL) v = a.K[i - OK];
        else if (i < OP) v = a.LAM[i - OL];
        else if (i < OQ) v = a.PSI[i - OP];
        else if (i < OR) v = a.Lq[i - OQ];
        else v = a.Lr[i - OR];
        cst[i] = v;
    }
    wave_sync();
    auto Am = [&](int i, int j) __attribute__((always_inline)) { return cst[OA + j * NX + i]; };
    auto Bm = [&](int i, int j) __attribute__((always_inline)) { return cst[OB + j * NX + i]; };
    auto Km = [&](int i, int j) __attribute__((always_inline)) { return cst[OK + j * NU + i]; };
    auto LAM = [&](int i, int j) __attribute__((always_inline)) { return cst[OL + j * NX + i]; };
    auto PSI = [&](int i, int j) __attribute__((always_inline)) { return cst[OP + j * NU + i]; };
    double th[NP];
#pragma unroll
    for (int p = 0; p < NP; ++p) th[p] = zv(N * NU + p);
    double x[NX], xn[NX];
    const double* x0 = a.x0 + (int64_t)b * a.sx0;
#pragma unroll
    for (int i = 0; i < NX; ++i) { x[i] = x0[i]; xn[i] = x0[i]; }
    // sensitivities of the learned (SL) and nominal (SN) states w.r.t. z, columns j = lane + 64 c
    double SL[LB_RCPL][NX], SN[LB_RCPL][NX];
#pragma unroll
    for (int c = 0; c < LB_RCPL; ++c)
#pragma unroll
        for (int i = 0; i < NX; ++i) { SL[c][i] = 0.0; SN[c][i] = 0.0; }
    double* Jr = gn ? a.Jr + (int64_t)b * nr * n : nullptr;
    double* er = gn ? a.er + (int64_t)b * nr : nullptr;
    double J = 0.0;
    int row = 0;
    double gx[NX];                  // dphi/dx of the current residual block (hess mode)
    // weighted residual block L (e) with L upper-triangular (row-major), e = v - M theta;
    // GN: its Jacobian rows for the lane's columns from sensitivities S (d v / d z); hess: the
    // gradient 2 L'e w.r.t. v accumulated in gv
    auto residual = [&](const double* Lw, int dim, const double* v, auto&& Mth, auto&& Scol,
                        double* gv) __attribute__((always_inline)) {
        for (int r = 0; r < dim; ++r) {
            double e = 0.0;
            for (int c2 = r; c2 < dim; ++c2) {
                double ec = v[c2];
#pragma unroll
                for (int p = 0; p < NP; ++p) ec -= Mth(c2, p) * th[p];
                e += Lw[r * dim + c2] * ec;
            }
            J += e * e;
            if (gv)
                for (int c2 = r; c2 < dim; ++c2) gv[c2] += 2.0 * e * Lw[r * dim + c2];
            if (gn) {
                if (lane == 0) er[row + r] = e;
#pragma unroll
                for (int c = 0; c < LB_RCPL; ++c) {
                    const int j = lane + LB_WAVE * c;
                    if (j < n) {
                        double acc = 0.0;
                        for (int c2 = r; c2 < dim; ++c2) {
                            double s = Scol(c, c2);
                            if (j >= N * NU) s -= Mth(c2, j - N * NU);
                            acc += Lw[r * dim + c2] * s;
                        }
                        Jr[(int64_t)(row + r) * n + j] = acc;
                    }
                }
            }
        }
        row += dim;
    };
    RST_DECL;
    for (int k = 0; k < N; ++k) {
        lane = lb_opq(lane);
        const double vk = zv(k);
        double u = vk, un = vk;
#pragma unroll
        for (int i = 0; i < NX; ++i) { u += Km(0, i) * x[i]; un += Km(0, i) * xn[i]; }
        // input sensitivities U = K S + e_k
        double UL[LB_RCPL], UN[LB_RCPL];
        if (gn) {
#pragma unroll
            for (int c = 0; c < LB_RCPL; ++c) {
                const int j = lane + LB_WAVE * c;
                double ul = (j == k) ? 1.0 : 0.0, unn = ul;
#pragma unroll
                for (int i = 0; i < NX; ++i) { ul += Km(0, i) * SL[c][i]; unn += Km(0, i) * SN[c][i]; }
                UL[c] = ul; UN[c] = unn;
            }
        }
#pragma unroll
        for (int i = 0; i < NX; ++i) gx[i] = 0.0;
        if (k < a.n_run) {
            residual(cst + OQ, NX, x, LAM, [&](int c, int i) { return SL[c][i]; }, hess ? gx : nullptr);
            double gu = 0.0;
            residual(cst + OR, NU, &u, PSI, [&](int c, int i) { return UL[c]; }, hess ? &gu : nullptr);
#pragma unroll
            for (int i = 0; i < NX; ++i) gx[i] += Km(0, i) * gu;    // u = K x + v
        }
        // learned step
        RST(0);
        const double xi[3] = {x[0], x[1], u};
        double g[4], dg[4][3], d2g[4][6];
        if constexpr (HESS) nw_eval<true, true>(D, a.q, a.wrows, a.hinv2, a.lam_nw, xi, g, dg, lane, d2g);
        else if (gn) nw_eval<true>(D, a.q, a.wrows, a.hinv2, a.lam_nw, xi, g, dg, lane);
        else nw_eval<false>(D, a.q, a.wrows, a.hinv2, a.lam_nw, xi, g, dg, lane);
        RST(1);
        if (hess && lane == 0) {
            double* st = SS + (int64_t)k * LB_SS;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
#pragma unroll
                for (int c3 = 0; c3 < 3; ++c3) st[3 * r + c3] = dg[r][c3];
#pragma unroll
                for (int e = 0; e < 6; ++e) st[12 + 6 * r + e] = d2g[r][e];
                st[36 + r] = gx[r];
            }
        }
        double x1[NX], xn1[NX];
#pragma unroll
        for (int i = 0; i < NX; ++i) {
            double v = Bm(i, 0) * u + (i < 4 ? g[i] : 0.0);
            double w = Bm(i, 0) * un;
#pragma unroll
            for (int c2 = 0; c2 < NX; ++c2) { v += Am(i, c2) * x[c2]; w += Am(i, c2) * xn[c2]; }
            x1[i] = v; xn1[i] = w;
        }
        if (gn) {
#pragma unroll
            for (int c = 0; c < LB_RCPL; ++c) {
                double sl[NX], sn[NX];
#pragma unroll
                for (int i = 0; i < NX; ++i) {
                    double gx0 = i < 4 ? dg[i][0] : 0.0, gx1 = i < 4 ? dg[i][1] : 0.0, gu = i < 4 ? dg[i][2] : 0.0;
                    double v = (Bm(i, 0) + gu) * UL[c] + gx0 * SL[c][0] + gx1 * SL[c][1];
                    double w = Bm(i, 0) * UN[c];
#pragma unroll
                    for (int c2 = 0; c2 < NX; ++c2) { v += Am(i, c2) * SL[c][c2]; w += Am(i, c2) * SN[c][c2]; }
                    sl[i] = v; sn[i] = w;
                }
#pragma unroll
                for (int i = 0; i < NX; ++i) { SL[c][i] = sl[i]; SN[c][i] = sn[i]; }
            }
        }
#pragma unroll
        for (int i = 0; i < NX; ++i) { x[i] = x1[i]; xn[i] = xn1[i]; }
        RST(2);
    }
    // terminal P on x_N (learned or nominal), T on (LAMBDA theta - xs)
#pragma unroll
    for (int i = 0; i < NX; ++i) gx[i] = 0.0;
    if (a.term_learned)
        residual(a.Lp, NX, x, LAM, [&](int c, int i) { return SL[c][i]; }, hess ? gx : nullptr);
    else
        residual(a.Lp, NX, xn, LAM, [&](int c, int i) { return SN[c][i]; }, nullptr);
    {
        // rows Lt (LAMBDA theta - xs): written as L (v - M theta) with v = -xs, M = -LAMBDA
        double mxs[NX];
#pragma unroll
        for (int i = 0; i < NX; ++i) mxs[i] = -a.xs[i];
        auto mLAM = [&](int i, int p) { return -LAM(i, p); };
        residual(a.Lt, NX, mxs, mLAM, [&](int c, int i) { return 0.0; }, nullptr);
    }
    if (lane == 0) {
        if (gn) a.cost0[b] = J;
        else a.costT[(int64_t)b * nt + t] = J;
    }
    RST(3);
    if constexpr (!HESS) { RST_PRINT("rollout"); return; }
    wave_sync();
    // ---- costate pass (uniform on every lane): W_k into the stage store ----
    double pc[NX];
#pragma unroll
    for (int i = 0; i < NX; ++i) pc[i] = gx[i];      // p_N: terminal gradient (0 for a nominal x_N)
    for (int k = N - 1; k >= 0; --k) {
        double* st = SS + (int64_t)k * LB_SS;
        double W6[6];
#pragma unroll
        for (int e = 0; e < 6; ++e) {
            double w = 0.0;
#pragma unroll
            for (int r = 0; r < 4; ++r) w += pc[r] * st[12 + 6 * r + e];
            W6[e] = w;
        }
        // p_k = dphi_k/dx_k + Jx' p_{k+1}, Jx = A + B K + [G_x0 G_x1 0 0] + g_u K
        double pn[NX];
#pragma unroll
        for (int c2 = 0; c2 < NX; ++c2) {
            double v = st[36 + c2];
#pragma unroll
            for (int i = 0; i < NX; ++i) {
                double jx = Am(i, c2) + (Bm(i, 0) + st[3 * i + 2]) * Km(0, c2);
                if (c2 < 2) jx += st[3 * i + c2];
                v += jx * pc[i];
            }
            pn[c2] = v;
        }
        wave_sync();
        if (lane == 0) {
#pragma unroll
            for (int e = 0; e < 6; ++e) st[12 + e] = W6[e];
        }
#pragma unroll
        for (int i = 0; i < NX; ++i) pc[i] = pn[i];
    }
    wave_sync();
    RST(4);
    // ---- second sensitivity pass: rows Xi_k and W_k Xi_k ----
    double* J2 = a.Jr2 + (int64_t)b * 3 * N * n;
    double* T2 = a.Tr2 + (int64_t)b * 3 * N * n;
#pragma unroll
    for (int c = 0; c < LB_RCPL; ++c)
#pragma unroll
        for (int i = 0; i < NX; ++i) SL[c][i] = 0.0;
    for (int k = 0; k < N; ++k) {
        lane = lb_opq(lane);
        const double* st = SS + (int64_t)k * LB_SS;
        const double w00 = st[12], w01 = st[13], w02 = st[14], w11 = st[15], w12 = st[16], w22 = st[17];
#pragma unroll
        for (int c = 0; c < LB_RCPL; ++c) {
            const int j = lane + LB_WAVE * c;
            double ul = (j == k) ? 1.0 : 0.0;
#pragma unroll
            for (int i = 0; i < NX; ++i) ul += Km(0, i) * SL[c][i];
            const double x0c = SL[c][0], x1c = SL[c][1];
            if (j < n) {
                const int64_t r0 = (int64_t)(3 * k) * n + j;
                J2[r0] = x0c; J2[r0 + n] = x1c; J2[r0 + 2 * n] = ul;
                T2[r0] = w00 * x0c + w01 * x1c + w02 * ul;
                T2[r0 + n] = w01 * x0c + w11 * x1c + w12 * ul;
                T2[r0 + 2 * n] = w02 * x0c + w12 * x1c + w22 * ul;
            }
            double sl[NX];
#pragma unroll
            for (int i = 0; i < NX; ++i) {
                double v = (Bm(i, 0) + st[3 * i + 2]) * ul + st[3 * i] * x0c + st[3 * i + 1] * x1c;
#pragma unroll
                for (int c2 = 0; c2 < NX; ++c2) v += Am(i, c2) * SL[c][c2];
                sl[i] = v;
            }
#pragma unroll
            for (int i = 0; i < NX; ++i) SL[c][i] = sl[i];
        }
    }
    RST(5);
    RST_PRINT("rollout");
}

// ------------------------------------------------------------------------------------------
// row-product sums on the fp64 matrix cores (round 6): sum_r X(r, :)' Y(r, :) over the rows of
// LDS row tiles (row-major, stride ld, columns zero-padded to 16 ceil(n / 16), rows past the
// data zero) into the lower block triangle of 16 x 16 tiles.  Wave w holds the tiles of lb_tile
// (diagonal tiles w, w + 4, then every fourth strictly lower tile; at most LB_TPW); per k-step of
// 4 rows lane l supplies X(4 s + l/16, 16 I + l%16) and Y(4 s + l/16, 16 J + l%16) to one
// v_mfma_f64_16x16x4f64, and tile (I, J), lane l, register e ends with entry
// (16 I + l/16 + 4 e, 16 J + l%16).  (The VALU 8 x 8 register tiles they replace ran at a few
// percent of the FP64 rate, one LDS operand pair per FMA pair.)
// ------------------------------------------------------------------------------------------
typedef double lbd4 __attribute__((ext_vector_type(4)));
#define LB_TPW 9
__device__ __forceinline__ void lb_tile(int w, int u, int nbk, int& I, int& J) {
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
// rows r0 .. r0 + rc - 1 of the row-major nrows x n matrix G into the tile T (rows 0 .. R - 1,
// stride ld, ncp = 16 ceil(n / 16) columns, zeros past rc and n) in two halves (round 6):
// lb_fetch_rows issues the loads of the next row tile into registers before the matrix cores
// consume the current one, lb_put_rows stores them after the next barrier - one memory round trip
// per tile, hidden behind the MFMAs, instead of two to four exposed ones (250k of the exact-Hessian kernel's cycles were its row-tile loads: stamps of the
// diagnostic build, gpurun_out/r06_q)
template <int R>
__device__ __forceinline__ void lb_fetch_rows(double (&v)[R / 2], const double* G, int r0, int rc, int n, int ncp,
                                              int tid) {
    const int tot = R * ncp;               // <= R * 128 = 256 * R / 2
#pragma unroll
    for (int u = 0; u < R / 2; ++u) {
        const int i = tid + 256 * u;
        const int r = i / ncp, c = i - r * ncp;
        v[u] = (i < tot && r < rc && c < n) ? G[(int64_t)(r0 + r) * n + c] : 0.0;
    }
}
template <int R>
__device__ __forceinline__ void lb_put_rows(double* T, const double (&v)[R / 2], int ncp, int ld, int tid) {
    const int tot = R * ncp;
#pragma unroll
    for (int u = 0; u < R / 2; ++u) {
        const int i = tid + 256 * u;
        const int r = i / ncp, c = i - r * ncp;
        if (i < tot) T[r * ld + c] = v[u];
    }
}
// the k-steps of one tile: acc += X'Y (and, SYM, += Y'X as well)
template <int R, bool SYM>
__device__ __forceinline__ void lb_mfma_rows(lbd4 (&acc)[LB_TPW], const int (&tI)[LB_TPW], const int (&tJ)[LB_TPW],
                                             const double* X, const double* Y, int ld, int lane) {
    const int c16 = lane & 15, k4 = lane >> 4;
#pragma unroll
    for (int s = 0; s < R / 4; ++s) {
        const double* xr = X + (4 * s + k4) * ld + c16;
        const double* yr = Y + (4 * s + k4) * ld + c16;
#pragma unroll
        for (int u = 0; u < LB_TPW; ++u) {
            if (tI[u] < 0) continue;
            acc[u] = __builtin_amdgcn_mfma_f64_16x16x4f64(xr[16 * tI[u]], yr[16 * tJ[u]], acc[u], 0, 0, 0);
            if constexpr (SYM)
                acc[u] = __builtin_amdgcn_mfma_f64_16x16x4f64(yr[16 * tI[u]], xr[16 * tJ[u]], acc[u], 0, 0, 0);
        }
    }
}

// ------------------------------------------------------------------------------------------
// exact Hessian (a.hess): Hx = H_GN + sym(Jr2' Tr2) through LDS row tiles (8 x 8 accumulators
// per thread, as the normal kernel), then a right-looking Cholesky of Hx in LDS; if every pivot
// is above 1e-10 max|Hx_ii| (oracle/lbmpc.py pd_cholesky) Hx replaces the Gauss-Newton H,
// otherwise the iteration keeps H_GN.  Dynamic LDS: 2 tiles of 16 x n, then n x n.
// ------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) lbmpc_hess_kernel(LbmpcArgs a) {
    extern __shared__ double lh[];
    const int b = blockIdx.x;
    if (b >= a.batch || a.done[b]) return;
    const int n = a.n, nr2 = 3 * a.N, tid = threadIdx.x;
    const int lane = tid & 63, wv = tid >> 6, c16 = lane & 15, k4 = lane >> 4;
    const int tx = tid & 15, ty = tid >> 4;      // the Cholesky test's 16 x 16 thread grid
    const int nbk = (n + 15) >> 4, ncp = 16 * nbk;
    double* TA = lh;
    double* TB = lh + 16 * ncp;
    double* Kx = lh + 32 * ncp;
    __shared__ double red[4];
    if (n > 128) return;
#ifdef BQP_RSTAMPS
    // diagnostic build only: cycles of the row products, the assembly and the Cholesky tests
    unsigned long long hst0 = __builtin_amdgcn_s_memtime(), hst1 = 0, hst2 = 0;
    int hatt = 0;
#define HST_ATT() (++hatt)
#else
#define HST_ATT() do { } while (0)
#endif
    const double* J2 = a.Jr2 + (int64_t)b * nr2 * n;
    const double* T2 = a.Tr2 + (int64_t)b * nr2 * n;
    // S = Jr2'Tr2 + Tr2'Jr2 on the lower block triangle (lb_mfma_rows, two MFMAs per k-step)
    int tI[LB_TPW], tJ[LB_TPW];
    lbd4 acc[LB_TPW];
#pragma unroll
    for (int u = 0; u < LB_TPW; ++u) { lb_tile(wv, u, nbk, tI[u], tJ[u]); acc[u] = lbd4{0.0, 0.0, 0.0, 0.0}; }
    double pa[8], pb[8];
    lb_fetch_rows<16>(pa, J2, 0, min(16, nr2), n, ncp, tid);
    lb_fetch_rows<16>(pb, T2, 0, min(16, nr2), n, ncp, tid);
    for (int r0 = 0; r0 < nr2; r0 += 16) {
        __syncthreads();
        lb_put_rows<16>(TA, pa, ncp, ncp, tid);
        lb_put_rows<16>(TB, pb, ncp, ncp, tid);
        __syncthreads();
        if (r0 + 16 < nr2) {                       // the next tile's loads in flight during the MFMAs
            lb_fetch_rows<16>(pa, J2, r0 + 16, min(16, nr2 - r0 - 16), n, ncp, tid);
            lb_fetch_rows<16>(pb, T2, r0 + 16, min(16, nr2 - r0 - 16), n, ncp, tid);
        }
        lb_mfma_rows<16, true>(acc, tI, tJ, TA, TB, ncp, lane);
    }
#ifdef BQP_RSTAMPS
    __builtin_amdgcn_s_waitcnt(0);
    hst1 = __builtin_amdgcn_s_memtime();
#endif
    // H_GN + the symmetric part S / 2 of Jr2'Tr2, both triangles, in LDS (column-major): each
    // entry (i >= j) belongs to one lane
    const double* H = a.H + (int64_t)b * n * n;
    double dmx = 0.0;
#pragma unroll
    for (int u = 0; u < LB_TPW; ++u) {
        if (tI[u] < 0) continue;
#pragma unroll
        for (int e2 = 0; e2 < 4; ++e2) {
            const int i = 16 * tI[u] + k4 + 4 * e2, j = 16 * tJ[u] + c16;
            if (i < n && j < n && i >= j) {
                const double v = H[(int64_t)j * n + i] + 0.5 * acc[u][e2];
                Kx[j * n + i] = v;
                Kx[i * n + j] = v;
                if (i == j) dmx = fmax(dmx, fabs(v));
            }
        }
    }
    dmx = wmax(dmx);
    if ((tid & 63) == 0) red[tid >> 6] = dmx;
    __syncthreads();
    const double tol = 1e-10 * fmax(fmax(red[0], red[1]), fmax(red[2], red[3]));
    // the Cholesky below overwrites the lower triangle and the diagonal: keep the diagonal (the
    // strict upper triangle stays the exact matrix)
    const double hd = fmax(fmax(red[0], red[1]), fmax(red[2], red[3]));
    double* dsave = TA;
    for (int j = tid; j < n; j += 256) dsave[j] = Kx[j * n + j];
    __syncthreads();
    // Cholesky test of H + sh I: lower triangle restored from the upper one, every pivot above tol
#ifdef BQP_RSTAMPS
    __builtin_amdgcn_s_waitcnt(0);
    hst2 = __builtin_amdgcn_s_memtime();
#endif
    auto attempt = [&](double sh) -> bool {
        HST_ATT();
        for (int e = tid; e < n * n; e += 256) {
            const int i = e % n, j = e / n;
            if (i > j) Kx[e] = Kx[i * n + j];
            else if (i == j) Kx[e] = dsave[i] + sh;
        }
        __syncthreads();
        // two pivots per pair of barriers (round 6): pivot j + 1 and column j + 1 after pivot j's
        // update are formed from the unscaled values (every thread the pivot, each row's thread its
        // entry), then one pass applies both rank-1 updates.  Each entry receives the same
        // operations in the same order as one pivot at a time - the scaled column, K -= L L per
        // pivot - so the outcome of the test is bitwise the one-pivot form's.
        bool pd = true;
        for (int j = 0; j < n; j += 2) {
            const double d0 = Kx[j * n + j];
            if (!(d0 > tol)) { pd = false; break; }     // uniform: every thread reads the same pivot
            if (j + 1 == n) break;
            const double sq0 = sqrt(d0);
            const double l10 = Kx[j * n + j + 1] / sq0;                  // L(j + 1, j)
            const double d1 = Kx[(j + 1) * n + j + 1] - l10 * l10;
            if (!(d1 > tol)) { pd = false; break; }
            const double sq1 = sqrt(d1);
            for (int i = j + 2 + tid; i < n; i += 256) {
                const double a0 = Kx[j * n + i] / sq0;
                Kx[j * n + i] = a0;
                Kx[(j + 1) * n + i] = (Kx[(j + 1) * n + i] - a0 * l10) / sq1;
            }
            __syncthreads();
            // trailing update over a 16 x 16 thread grid (ty: columns c, tx: rows i >= c); one
            // thread per column c ran the c loop serially (~5k cycles per pivot, round 4)
            for (int c = j + 2 + ty; c < n; c += 16) {
                const double lc0 = Kx[j * n + c], lc1 = Kx[(j + 1) * n + c];
                for (int i = c + tx; i < n; i += 16) {
                    const double v = Kx[c * n + i] - Kx[j * n + i] * lc0;
                    Kx[c * n + i] = v - Kx[(j + 1) * n + i] * lc1;
                }
            }
            __syncthreads();
        }
        __syncthreads();                                 // all have read the failing pivot
        return pd;
    };
    // regularised exact Hessian (round 5; oracle/cpu_lbmpc.c hess_shift_k, oracle/lbmpc.py
    // hess_shift): if H is not positive definite, the smallest grid shift 1e-12 hd 4^k (k = 0..20,
    // bisection: definiteness is monotone in the shift) that makes it so; H_GN (left in a.H) only
    // if none does.  (Falling back to H_GN at once converged linearly: 200 SQP iterations at one
    // step of a +-0.02 DMS instance, 7 with the shift.)
    double shift = 0.0;
    if (!attempt(0.0)) {
        int lo = -1, hi = 20;
        if (!attempt(ldexp(1e-12 * hd, 2 * hi))) return;
        while (hi - lo > 1) {
            const int mid = (lo + hi) / 2;
            if (attempt(ldexp(1e-12 * hd, 2 * mid))) hi = mid; else lo = mid;
        }
        shift = ldexp(1e-12 * hd, 2 * hi);
    }
#ifdef BQP_RSTAMPS
    if ((b & 15) == 0 && tid == 0)
        printf("HSTAMPS gemm %llu assembly %llu tests %llu attempts %d\n", hst1 - hst0, hst2 - hst1,
               __builtin_amdgcn_s_memtime() - hst2, hatt);
#endif
    double* Hw = a.H + (int64_t)b * n * n;
    for (int e = tid; e < n * n; e += 256) {
        const int i = e % n, j = e / n;
        Hw[e] = (i == j) ? dsave[i] + shift : (i < j ? Kx[e] : Kx[i * n + j]);
    }
    if (tid == 0 && a.hused) a.hused[b] += 1;
}

// ------------------------------------------------------------------------------------------
// normal equations H = 2 Jr'Jr, f = 2 Jr'er (column-major H), QP rhs b_in - A_in z
// ------------------------------------------------------------------------------------------
#define LB_RC 32         // Jr rows per LDS tile (8 k-steps of the matrix cores)
#define LB_MAXN 128      // n <= 128 for the normal kernel (16 x 16 tiles of 8 x 8 blocks)
#define LB_TS 130        // LDS row stride of the tile (the 16 ceil(n / 16) <= 128 columns + 2)
__global__ void __launch_bounds__(256) lbmpc_normal_kernel(LbmpcArgs a) {
    __shared__ double T[LB_RC * LB_TS];
    __shared__ double E[LB_RC];
    const int b = blockIdx.x;
    if (b >= a.batch || a.done[b]) return;
    const int n = a.n, nr = a.nr, tid = threadIdx.x;
    const int lane = tid & 63, wv = tid >> 6, c16 = lane & 15, k4 = lane >> 4;
    const int nbk = (n + 15) >> 4, ncp = 16 * nbk;
    const double* Jr = a.Jr + (int64_t)b * nr * n;
    const double* er = a.er + (int64_t)b * nr;
    // Jr'Jr on the lower block triangle (lb_mfma_rows); Jr'er by thread tid < n
    int tI[LB_TPW], tJ[LB_TPW];
    lbd4 acc[LB_TPW];
#pragma unroll
    for (int u = 0; u < LB_TPW; ++u) { lb_tile(wv, u, nbk, tI[u], tJ[u]); acc[u] = lbd4{0.0, 0.0, 0.0, 0.0}; }
    double fa = 0.0;
    double pj[LB_RC / 2];
    lb_fetch_rows<LB_RC>(pj, Jr, 0, min(LB_RC, nr), n, ncp, tid);
    for (int r0 = 0; r0 < nr; r0 += LB_RC) {
        const int rc = min(LB_RC, nr - r0);
        __syncthreads();
        lb_put_rows<LB_RC>(T, pj, ncp, LB_TS, tid);
        if (tid < LB_RC) E[tid] = tid < rc ? er[r0 + tid] : 0.0;
        __syncthreads();
        if (r0 + LB_RC < nr)                       // the next tile's loads in flight during the MFMAs
            lb_fetch_rows<LB_RC>(pj, Jr, r0 + LB_RC, min(LB_RC, nr - r0 - LB_RC), n, ncp, tid);
        lb_mfma_rows<LB_RC, false>(acc, tI, tJ, T, T, LB_TS, lane);
        if (tid < n)
            for (int r = 0; r < rc; ++r) fa += T[r * LB_TS + tid] * E[r];
    }
    // H = 2 Jr'Jr (column-major, both triangles from the lower one: exactly symmetric)
    double* H = a.H + (int64_t)b * n * n;
#pragma unroll
    for (int u = 0; u < LB_TPW; ++u) {
        if (tI[u] < 0) continue;
#pragma unroll
        for (int e2 = 0; e2 < 4; ++e2) {
            const int i = 16 * tI[u] + k4 + 4 * e2, j = 16 * tJ[u] + c16;
            if (i < n && j < n && i >= j) {
                const double v = 2.0 * acc[u][e2];
                H[(int64_t)j * n + i] = v;
                H[(int64_t)i * n + j] = v;
            }
        }
    }
    if (tid < n) a.f[(int64_t)b * n + tid] = 2.0 * fa;
    // b_in - A_in z (A_in column-major m x n, shared): z staged in LDS, 8 columns' loads in
    // flight and four partial sums per row (the serial column loop waited on every load)
    const double* z = a.z + (int64_t)b * n;
    const double* bin = a.bin + (int64_t)b * a.sbin;
    __syncthreads();
    double* zs = T;
    for (int j = tid; j < n; j += 256) zs[j] = z[j];
    __syncthreads();
    const int m = a.m;
    for (int r = tid; r < m; r += 256) {
        const double* ar = a.Ain + r;
        double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
        int j = 0;
        for (; j + 8 <= n; j += 8) {
            double av[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) av[u] = ar[(int64_t)(j + u) * m];
            s0 = fma(av[0], zs[j], s0); s1 = fma(av[1], zs[j + 1], s1);
            s2 = fma(av[2], zs[j + 2], s2); s3 = fma(av[3], zs[j + 3], s3);
            s0 = fma(av[4], zs[j + 4], s0); s1 = fma(av[5], zs[j + 5], s1);
            s2 = fma(av[6], zs[j + 6], s2); s3 = fma(av[7], zs[j + 7], s3);
        }
        for (; j < n; ++j) s0 = fma(ar[(int64_t)j * m], zs[j], s0);
        a.bsh[(int64_t)b * m + r] = bin[r] - ((s0 + s1) + (s2 + s3));
    }
}

// ------------------------------------------------------------------------------------------
// convergence test + Armijo line search + step (one wave per instance)
// ------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(64) lbmpc_update_kernel(LbmpcArgs a) {
    const int b = blockIdx.x;
    const int lane = threadIdx.x;
    if (b >= a.batch || a.done[b]) return;
    const int n = a.n, m = a.m;
    double* z = a.z + (int64_t)b * n;
    const double* d = a.d + (int64_t)b * n;
    const double* f = a.f + (int64_t)b * n;
    const double* lam = a.lam + (int64_t)b * m;
    const double* bsh = a.bsh + (int64_t)b * m;
    const int qflag = a.qpflag[b];
    // NLP stationarity |f + A_in' lam|, norms, slope f'd, start feasibility
    double st = 0.0, fn = 0.0, dn = 0.0, zn = 0.0, sl = 0.0, viol = 0.0;
    // A_in' lam by groups of 16 columns: lanes over the rows (coalesced loads, 16 in flight), one
    // transposed wave sum per group (round 6; one lane per column running down its m rows waited
    // on every load: ~0.2 ms per launch at m = 1024)
    __shared__ double sg[LB_WAVE * LB_CPL];
    for (int g0 = 0; g0 < n; g0 += 16) {
        double ac[16];
#pragma unroll
        for (int c = 0; c < 16; ++c) ac[c] = 0.0;
        for (int r = lane; r < m; r += LB_WAVE) {
            const double lr = lam[r];
            double av[16];
#pragma unroll
            for (int c = 0; c < 16; ++c) av[c] = a.Ain[(int64_t)min(g0 + c, n - 1) * m + r];
#pragma unroll
            for (int c = 0; c < 16; ++c) ac[c] = fma(av[c], lr, ac[c]);
        }
        const double tot = wsum_t(ac, lane);
        if (lane < 16 && g0 + lane < n) sg[g0 + lane] = tot;
    }
    wave_sync();
    for (int j = lane; j < n; j += LB_WAVE) {
        const double g = f[j] + sg[j];
        st = fmax(st, fabs(g));
        fn = fmax(fn, fabs(f[j]));
        dn = fmax(dn, fabs(d[j]));
        zn = fmax(zn, fabs(z[j]));
        sl += f[j] * d[j];
    }
    for (int r = lane; r < m; r += LB_WAVE) viol = fmax(viol, -bsh[r]);
    st = wmax(st); fn = wmax(fn); dn = wmax(dn); zn = wmax(zn); sl = wsum(sl); viol = wmax(viol);
    const bool feas0 = viol <= 1e-9;
    int it = a.iters[b];
    int flag = 0;
    bool fin = false;
    // a QP that stopped on its iteration limit or numerically (-8) still returns its last
    // interior iterate; near the SQP solution (d -> 0, multipliers of the active rows large,
    // slacks -> 0) that is the usual way the sub-problem ends, and the step is used as is
    const bool qp_ok = qflag == 1 || ((qflag == 0 || qflag == -8) && isfinite(dn) && isfinite(st));
    if (qflag == -2 || !qp_ok) {
        flag = (qflag == -2) ? -2 : -8;   // QP sub-problem infeasible / failed
        fin = true;
    } else if (feas0 && ((qflag == 1 && dn <= a.tol_step * (1.0 + zn) && st <= a.tol_stat * (1.0 + fn)) ||
                         (it > 0 && dn <= 1e-6 * (1.0 + zn) &&
                          (qflag != 1 ||
                           fabs(a.cprev[b] - a.cost0[b]) <= 1e-12 * (1.0 + fabs(a.cost0[b])))))) {
        // converged: KKT test, or the step has reached the accuracy of the interior-point QP
        // solve (|d| <= 1e-6) and the cost no longer changes (stagnation at round-off) or the
        // QP cannot resolve a smaller step
        flag = 1;
        fin = true;
    }
    if (!fin) {
        const double J0 = a.cost0[b];
        int tsel = a.ntrial - 1;
        if (feas0) {
            for (int t = 0; t < a.ntrial; ++t) {
                const double al = ldexp(1.0, -t);
                if (a.costT[(int64_t)b * a.ntrial + t] <= J0 + 1e-4 * al * sl) { tsel = t; break; }
            }
        } else {
            tsel = 0;                     // infeasible start: full step to the linearised-feasible point
        }
        const double al = ldexp(1.0, -tsel);
        for (int j = lane; j < n; j += LB_WAVE) z[j] += al * d[j];
        if (lane == 0) a.cprev[b] = J0;
        ++it;
        if (it >= a.max_iter) {
            flag = 0;
            fin = true;
            // the returned z is the stepped iterate: its cost is the trial cost of that step
            if (lane == 0) a.cost0[b] = a.costT[(int64_t)b * a.ntrial + tsel];
        }
    }
    if (lane == 0) {
        a.iters[b] = it;
        a.stat[b] = st;
        if (fin) {
            a.flag[b] = flag;
            a.done[b] = 1;
            atomicAdd(a.ndone, 1);
        }
    }
}

// ------------------------------------------------------------------------------------------
// launch helpers
// ------------------------------------------------------------------------------------------
hipError_t launch_nw_oracle(int batch, int q, const double* data, int64_t sdata, const double* xi,
                            double* g, double* dg, double bw, double lam, hipStream_t st) {
    if (q < 1 || q > LB_MAXQ) return hipErrorInvalidValue;
    hipLaunchKernelGGL(nw_oracle_kernel, dim3(batch), dim3(64), 0, st, batch, q, data, sdata, xi,
                       g, dg, 1.0 / (bw * bw), lam);
    return hipGetLastError();
}

bool lbmpc_supported(int nx, int nu, int np, int n, int q) {
    return nx == 4 && nu == 1 && np == 1 && n <= LB_MAXN && n <= LB_WAVE * LB_RCPL && q >= 1 &&
           q <= LB_MAXQ;
}

size_t lbmpc_rollout_lds(const LbmpcArgs& a, int gn) {
    size_t d = (size_t)((a.wrows * a.q + 1) & ~1);
    if (gn && a.hess) d += (size_t)LB_SS * a.N;
    return d * sizeof(double);
}

hipError_t launch_lbmpc_rollout(const LbmpcArgs& a, int gn, hipStream_t st) {
    const int grid = a.batch * (gn ? 1 : a.ntrial);
    const size_t lds = lbmpc_rollout_lds(a, gn);
    auto k = (gn && a.hess) ? lbmpc_rollout_kernel<4, 1, 1, true> : lbmpc_rollout_kernel<4, 1, 1, false>;
    // z columns: LB_RCPL per lane (the sensitivities and the LDS trial point); static LDS ~1.4 KB
    if (a.n > LB_WAVE * LB_RCPL || lds > 156 * 1024) return hipErrorInvalidValue;
    if (lds > 64 * 1024) {
        hipError_t e = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(k, dim3(grid), dim3(64), lds, st, a, gn);
    return hipGetLastError();
}

// the exact-Hessian kernel holds 16-row tiles of Jr2 and Tr2 (16 ceil(n / 16) columns) and the
// n x n sum in LDS
static size_t lbmpc_hess_lds(int n) { return sizeof(double) * ((size_t)32 * 16 * ((n + 15) / 16) + (size_t)n * n); }
bool lbmpc_hess_fits(int n) { return n <= 128 && lbmpc_hess_lds(n) <= 160 * 1024 - 64; }

hipError_t launch_lbmpc_hess(const LbmpcArgs& a, hipStream_t st) {
    const size_t lds = lbmpc_hess_lds(a.n);
    if (!lbmpc_hess_fits(a.n)) return hipErrorInvalidValue;
    if (lds > 64 * 1024) {
        hipError_t e = hipFuncSetAttribute((const void*)lbmpc_hess_kernel,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(lbmpc_hess_kernel, dim3(a.batch), dim3(256), lds, st, a);
    return hipGetLastError();
}

hipError_t launch_lbmpc_normal(const LbmpcArgs& a, hipStream_t st) {
    hipLaunchKernelGGL(lbmpc_normal_kernel, dim3(a.batch), dim3(256), 0, st, a);
    return hipGetLastError();
}

hipError_t launch_lbmpc_update(const LbmpcArgs& a, hipStream_t st) {
    hipLaunchKernelGGL(lbmpc_update_kernel, dim3(a.batch), dim3(64), 0, st, a);
    return hipGetLastError();
}

}  // namespace bqp
