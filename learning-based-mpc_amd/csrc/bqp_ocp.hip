// bqp_ocp.hip — batched structured Mehrotra predictor-corrector IPM for MPC QPs, gfx950.
//
// One wavefront (64 lanes) solves one MPC instance; a workgroup holds WPB instances that share
// the stage-cost table H_k and the polytope (terminal-set) matrix in LDS.  Inside a wave the
// lanes are re-assigned per phase:
//   * stage phases   lane k (and k+64 when SPL=2) owns stage k: s_k=[x_k;theta], u_k, pi_k,
//                    the box rows of stage k (residuals, Newton right-hand sides, recoveries);
//   * polytope rows  lane l owns rows l, l+64, ... (RPL rows): slacks/duals in registers,
//                    F_T'DF_T and F_T'e reduced with wave shuffles;
//   * Riccati factor lane (i,j) owns entry (i,j) of the (NS+NU)^2 stage matrix; P_{k+1} is
//                    broadcast from LDS each stage (sequential over k);
//   * Riccati solves every lane runs the (NS)-vector recursion redundantly (no cross-lane
//                    traffic on the sequential critical path), streaming K_k / vectors from LDS.
// The algorithm (and its operation order) is the one stated in oracle/ocp_ipm.py and restated
// in C in oracle/cpu_ipm.c; the QP is the stage-wise form of the reference's per-step OCPs
// (costLMPC.m / constraintsLMPC.m, DMS_tracking_LMPC_casadi.m:223-287, trackingMPC/costFunction.m).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "bqp_internal.h"

namespace bqp {

#define WAVE 64

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Wave-wide reductions on DPP lane moves (quad_perm xor1/xor2, row_half_mirror, row_mirror
// inside each 16-lane row, then row_bcast15/31 across rows) + one readlane of lane 63: no LDS
// traffic, result uniform (SGPR) in every lane.  EXEC must be full (all call sites are
// wave-uniform).
template <int CTRL, int ROWM>
__device__ __forceinline__ double dpp_mov(double old, double v) {
    const int2 o = __builtin_bit_cast(int2, old);
    const int2 x = __builtin_bit_cast(int2, v);
    int2 r;
    r.x = __builtin_amdgcn_update_dpp(o.x, x.x, CTRL, ROWM, 0xf, false);
    r.y = __builtin_amdgcn_update_dpp(o.y, x.y, CTRL, ROWM, 0xf, false);
    return __builtin_bit_cast(double, r);
}
__device__ __forceinline__ double lane63(double v) {
    const int2 x = __builtin_bit_cast(int2, v);
    int2 r;
    r.x = __builtin_amdgcn_readlane(x.x, 63);
    r.y = __builtin_amdgcn_readlane(x.y, 63);
    return __builtin_bit_cast(double, r);
}
__device__ __forceinline__ double wsum(double v) {
    v += dpp_mov<0xB1, 0xf>(0.0, v);
    v += dpp_mov<0x4E, 0xf>(0.0, v);
    v += dpp_mov<0x141, 0xf>(0.0, v);
    v += dpp_mov<0x140, 0xf>(0.0, v);
    v += dpp_mov<0x142, 0xa>(0.0, v);
    v += dpp_mov<0x143, 0xc>(0.0, v);
    return lane63(v);
}
__device__ __forceinline__ double wmax(double v) {
    v = fmax(v, dpp_mov<0xB1, 0xf>(-INFINITY, v));
    v = fmax(v, dpp_mov<0x4E, 0xf>(-INFINITY, v));
    v = fmax(v, dpp_mov<0x141, 0xf>(-INFINITY, v));
    v = fmax(v, dpp_mov<0x140, 0xf>(-INFINITY, v));
    v = fmax(v, dpp_mov<0x142, 0xa>(-INFINITY, v));
    v = fmax(v, dpp_mov<0x143, 0xc>(-INFINITY, v));
    return lane63(v);
}
__device__ __forceinline__ double wmin(double v) {
    v = fmin(v, dpp_mov<0xB1, 0xf>(INFINITY, v));
    v = fmin(v, dpp_mov<0x4E, 0xf>(INFINITY, v));
    v = fmin(v, dpp_mov<0x141, 0xf>(INFINITY, v));
    v = fmin(v, dpp_mov<0x140, 0xf>(INFINITY, v));
    v = fmin(v, dpp_mov<0x142, 0xa>(INFINITY, v));
    v = fmin(v, dpp_mov<0x143, 0xc>(INFINITY, v));
    return lane63(v);
}

// Per-wave LDS layout (in doubles), all sized from N at run time.
struct WaveLds {
    int P, K, Ri, xs, xpi, xu, p, wv, qt, fv, dsv, duv, qu, Dx, Du, FD, M, gp, misc, total;
    __host__ __device__ static WaveLds make(int N, int NX, int NU, int NS, int NV) {
        WaveLds o;
        int c = 0;
        o.P = c;   c += (N + 1) * NS * NS;
        o.K = c;   c += N * NU * NS;
        o.Ri = c;  c += N * NU * NU;
        o.xs = c;  c += (N + 1) * NS;
        o.xpi = c; c += (N + 1) * NS;
        o.xu = c;  c += (N + 1) * NU;
        o.p = c;   c += (N + 1) * NS;
        o.wv = c;  c += (N + 1) * NS;
        o.qt = c;  c += (N + 1) * NS;
        o.fv = c;  c += (N + 1) * NS;
        o.dsv = c; c += (N + 1) * NS;
        o.duv = c; c += (N + 1) * NU;
        o.qu = c;  c += (N + 1) * NU;
        o.Dx = c;  c += (N + 1) * NX;
        o.Du = c;  c += (N + 1) * NU;
        o.FD = c;  c += NV * NV;
        o.M = c;   c += NV * NV;
        o.gp = c;  c += NV;
        o.misc = c; c += 8;
        o.total = (c + 1) & ~1;
        return o;
    }
};

template <int NX, int NU, int NP, int SPL, int RPL>
__global__ void __launch_bounds__(256) ocp_ipm_kernel(OcpKernelArgs a) {
    constexpr int NS = NX + NP;
    constexpr int NV = NS + NU;
    extern __shared__ double lds[];
    const int N = a.N, mp = a.mp, kp = a.kp;
    const int lane = threadIdx.x & 63;
    const int wid = threadIdx.x >> 6;
    const int hstride = a.hstride;          // padded NV*NV (+1) per stage
    // ---------------- shared tables: H (N+1 stages) and Fp (column-major, mpad rows) -------
    double* Hs = lds;
    double* Fs = lds + (N + 1) * hstride;
    const int mpad = a.mpad;
    for (int i = threadIdx.x; i < (N + 1) * hstride; i += blockDim.x) Hs[i] = a.H[i];
    for (int i = threadIdx.x; i < NV * mpad; i += blockDim.x) Fs[i] = a.Fp[i];
    __syncthreads();
    const int inst = blockIdx.x * a.wpb + wid;
    if (inst >= a.batch) return;
    const WaveLds L = WaveLds::make(N, NX, NU, NS, NV);
    double* W = lds + a.shared_doubles + wid * L.total;

    // ---------------- per-instance model (wave-uniform) -------------------------------------
    double Ab[NS][NS], Bb[NS][NU], cb[NS];
    {
        const double* A = a.A + (int64_t)inst * a.sA;
        const double* B = a.B + (int64_t)inst * a.sB;
#pragma unroll
        for (int i = 0; i < NS; ++i) {
#pragma unroll
            for (int j = 0; j < NS; ++j)
                Ab[i][j] = (i < NX && j < NX) ? A[j * NX + i] : (i == j ? 1.0 : 0.0);
#pragma unroll
            for (int j = 0; j < NU; ++j) Bb[i][j] = (i < NX) ? B[j * NX + i] : 0.0;
            cb[i] = (i < NX && a.c) ? a.c[(int64_t)inst * a.sc + i] : 0.0;
        }
    }
    // Riccati-factor lane roles (columns kept in registers, constant over the stages):
    //   phase A  lane (xa, ja), xa < NU, ja < NV : input row M_{u_xa, ja} = Ht + Bbar_xa' P F_ja
    //   phase B  lane (ib, jb), ib <= jb < NS    : P_k(ib, jb) in Joseph form
    const int xa = lane / NV, ja = lane % NV;
    const bool alane = lane < NU * NV;
    const int ib = lane / NS, jb = lane % NS;
    const bool blane = lane < NS * NS && ib <= jb;
    double FjA[NS], BxA[NS], AiB[NS], AjB[NS];
#pragma unroll
    for (int a_ = 0; a_ < NS; ++a_) {
        double vf = 0, vb = 0, vi = 0, vj = 0;
#pragma unroll
        for (int c = 0; c < NV; ++c) {
            const double f = (c < NS) ? Ab[a_][c < NS ? c : 0] : Bb[a_][c >= NS ? c - NS : 0];
            vf = (c == ja) ? f : vf;
        }
#pragma unroll
        for (int c = 0; c < NU; ++c) vb = (c == xa) ? Bb[a_][c] : vb;
#pragma unroll
        for (int c = 0; c < NS; ++c) {
            vi = (c == ib) ? Ab[a_][c] : vi;
            vj = (c == jb) ? Ab[a_][c] : vj;
        }
        FjA[a_] = vf; BxA[a_] = vb; AiB[a_] = vi; AjB[a_] = vj;
    }

    // ---------------- stage-lane state ------------------------------------------------------
    double s[SPL][NS], u[SPL][NU], pi[SPL][NS], g[SPL][NV];
    double tx[SPL][NX][2], lx[SPL][NX][2], bx[SPL][NX][2];   // slack, dual, bound (ub, lb)
    double tu[SPL][NU][2], lu[SPL][NU][2], bu[SPL][NU][2];
    unsigned mx[SPL], mu_[SPL];                               // presence bits (2 per comp)
    const double* x0 = a.x0 + (int64_t)inst * a.sx0;
#pragma unroll
    for (int j = 0; j < SPL; ++j) {
        const int k = lane + WAVE * j;
        const bool act = k <= N;
        const int kk = act ? k : N;
        mx[j] = 0; mu_[j] = 0;
#pragma unroll
        for (int i = 0; i < NS; ++i) { s[j][i] = 0.0; pi[j][i] = 0.0; }
#pragma unroll
        for (int i = 0; i < NU; ++i) u[j][i] = 0.0;
        if (k == 0) {
#pragma unroll
            for (int i = 0; i < NX; ++i) s[j][i] = x0[i];
        }
        // linear term, permuted [x th u] from external [x u th]
        const double* wk = a.w ? a.w + (int64_t)inst * a.sw + (int64_t)kk * NV : nullptr;
#pragma unroll
        for (int i = 0; i < NV; ++i) {
            const int e = (i < NX) ? i : (i < NS ? NX + NU + (i - NX) : NX + (i - NS));
            g[j][i] = (wk && act && !(k == N && i >= NS)) ? wk[e] : 0.0;
        }
#pragma unroll
        for (int i = 0; i < NX; ++i) {
            double ub = INFINITY, lb = -INFINITY;
            if (act && k > 0) {
                if (a.xub) ub = a.xub[(int64_t)inst * a.sxb + (int64_t)k * NX + i];
                if (a.xlb) lb = a.xlb[(int64_t)inst * a.sxb + (int64_t)k * NX + i];
            }
            bx[j][i][0] = ub; bx[j][i][1] = lb;
            if (isfinite(ub)) mx[j] |= 1u << (2 * i);
            if (isfinite(lb)) mx[j] |= 2u << (2 * i);
        }
#pragma unroll
        for (int i = 0; i < NU; ++i) {
            double ub = INFINITY, lb = -INFINITY;
            if (act && k < N) {
                if (a.uub) ub = a.uub[(int64_t)inst * a.sub + (int64_t)k * NU + i];
                if (a.ulb) lb = a.ulb[(int64_t)inst * a.sub + (int64_t)k * NU + i];
            }
            bu[j][i][0] = ub; bu[j][i][1] = lb;
            if (isfinite(ub)) mu_[j] |= 1u << (2 * i);
            if (isfinite(lb)) mu_[j] |= 2u << (2 * i);
        }
    }
    // polytope rows
    double tp[RPL], lp[RPL], hp[RPL];
    const double* hpi = a.hp + (int64_t)inst * a.shp;
#pragma unroll
    for (int q = 0; q < RPL; ++q) {
        const int r = lane + WAVE * q;
        hp[q] = (r < mp) ? hpi[r] : 0.0;
    }
    // row count
    double mcount = 0;
#pragma unroll
    for (int j = 0; j < SPL; ++j) mcount += __builtin_popcount(mx[j]) + __builtin_popcount(mu_[j]);
#pragma unroll
    for (int q = 0; q < RPL; ++q) mcount += (lane + WAVE * q < mp) ? 1.0 : 0.0;
    mcount = wsum(mcount);
    const double minv = 1.0 / fmax(mcount, 1.0);
    // scale of the primal data for the relative feasibility test
    double bsl = 0.0;
#pragma unroll
    for (int j = 0; j < SPL; ++j) {
        const int k = lane + WAVE * j;
        if (k == 0) {
#pragma unroll
            for (int i = 0; i < NX; ++i) bsl = fmax(bsl, fabs(x0[i]));
        }
#pragma unroll
        for (int i = 0; i < NX; ++i)
#pragma unroll
            for (int h = 0; h < 2; ++h)
                if ((mx[j] >> (2 * i + h)) & 1u) bsl = fmax(bsl, fabs(bx[j][i][h]));
#pragma unroll
        for (int i = 0; i < NU; ++i)
#pragma unroll
            for (int h = 0; h < 2; ++h)
                if ((mu_[j] >> (2 * i + h)) & 1u) bsl = fmax(bsl, fabs(bu[j][i][h]));
    }
#pragma unroll
    for (int q = 0; q < RPL; ++q)
        if (lane + WAVE * q < mp) bsl = fmax(bsl, fabs(hp[q]));
    const double bscale = wmax(bsl);

    // residual registers
    double rs[SPL][NS], ru[SPL][NU], re[SPL][NS], rix[SPL][NX][2], riu[SPL][NU][2], rip[RPL];
    // step registers
    double ds[SPL][NS], du[SPL][NU], dpi[SPL][NS], dtx[SPL][NX][2], dlx[SPL][NX][2];
    double dtu[SPL][NU][2], dlu[SPL][NU][2], dtp[RPL], dlp[RPL];
    double rcx[SPL][NX][2], rcu[SPL][NU][2], rcp[RPL];   // complementarity rhs
    double kff[SPL][NU];
    double itx[SPL][NX][2], itu[SPL][NU][2], itp[RPL];   // 1/t, once per iteration

    auto xpres = [&](int j, int i, int h) -> bool { return (mx[j] >> (2 * i + h)) & 1u; };
    auto upres = [&](int j, int i, int h) -> bool { return (mu_[j] >> (2 * i + h)) & 1u; };

    // ======================= residuals (stat, feas, comp sum) ==============================
    auto residuals = [&](double& stat, double& feas, double& csum, double& gscale) {
        // publish s, u, pi for neighbour / polytope stage access
#pragma unroll
        for (int j = 0; j < SPL; ++j) {
            const int k = lane + WAVE * j;
            if (k <= N) {
#pragma unroll
                for (int i = 0; i < NS; ++i) { W[L.xs + k * NS + i] = s[j][i]; W[L.xpi + k * NS + i] = pi[j][i]; }
#pragma unroll
                for (int i = 0; i < NU; ++i) W[L.xu + k * NU + i] = u[j][i];
            }
        }
        wave_sync();
        double st = 0, fe = 0, cs = 0, gs = 0;
#pragma unroll
        for (int j = 0; j < SPL; ++j) {
            const int k = lane + WAVE * j;
            if (k > N) {
#pragma unroll
                for (int i = 0; i < NS; ++i) { rs[j][i] = 0; re[j][i] = 0; }
#pragma unroll
                for (int i = 0; i < NU; ++i) ru[j][i] = 0;
#pragma unroll
                for (int i = 0; i < NX; ++i) rix[j][i][0] = rix[j][i][1] = 0;
#pragma unroll
                for (int i = 0; i < NU; ++i) riu[j][i][0] = riu[j][i][1] = 0;
                continue;
            }
            const double* Hk = Hs + k * hstride;
            double v[NV];
#pragma unroll
            for (int i = 0; i < NS; ++i) v[i] = s[j][i];
#pragma unroll
            for (int i = 0; i < NU; ++i) v[NS + i] = (k < N) ? u[j][i] : 0.0;
            double gv[NV];
#pragma unroll
            for (int i = 0; i < NV; ++i) {
                double acc = g[j][i];
#pragma unroll
                for (int c = 0; c < NV; ++c) acc += Hk[i * NV + c] * v[c];
                gv[i] = acc;
                gs = fmax(gs, fabs(acc));
            }
            double pn[NS];
#pragma unroll
            for (int i = 0; i < NS; ++i) pn[i] = (k < N) ? W[L.xpi + (k + 1) * NS + i] : 0.0;
#pragma unroll
            for (int i = 0; i < NS; ++i) {
                double acc = gv[i];
                if (k < N) {
#pragma unroll
                    for (int c = 0; c < NS; ++c) acc += Ab[c][i] * pn[c];
                }
                if (k > 0) acc -= pi[j][i];
                rs[j][i] = acc;
            }
#pragma unroll
            for (int i = 0; i < NU; ++i) {
                double acc = gv[NS + i];
#pragma unroll
                for (int c = 0; c < NS; ++c) acc += Bb[c][i] * pn[c];
                ru[j][i] = (k < N) ? acc : 0.0;
            }
#pragma unroll
            for (int i = 0; i < NX; ++i) {
                const double xi = s[j][i];
                double r0 = 0, r1 = 0;
                if (xpres(j, i, 0)) { rs[j][i] += lx[j][i][0]; r0 = xi + tx[j][i][0] - bx[j][i][0]; cs += tx[j][i][0] * lx[j][i][0]; }
                if (xpres(j, i, 1)) { rs[j][i] -= lx[j][i][1]; r1 = -xi + tx[j][i][1] + bx[j][i][1]; cs += tx[j][i][1] * lx[j][i][1]; }
                rix[j][i][0] = r0; rix[j][i][1] = r1;
            }
#pragma unroll
            for (int i = 0; i < NU; ++i) {
                const double ui = u[j][i];
                double r0 = 0, r1 = 0;
                if (upres(j, i, 0)) { ru[j][i] += lu[j][i][0]; r0 = ui + tu[j][i][0] - bu[j][i][0]; cs += tu[j][i][0] * lu[j][i][0]; }
                if (upres(j, i, 1)) { ru[j][i] -= lu[j][i][1]; r1 = -ui + tu[j][i][1] + bu[j][i][1]; cs += tu[j][i][1] * lu[j][i][1]; }
                riu[j][i][0] = r0; riu[j][i][1] = r1;
            }
            if (k < N) {
#pragma unroll
                for (int i = 0; i < NS; ++i) {
                    double acc = cb[i] - W[L.xs + (k + 1) * NS + i];
#pragma unroll
                    for (int c = 0; c < NS; ++c) acc += Ab[i][c] * s[j][c];
#pragma unroll
                    for (int c = 0; c < NU; ++c) acc += Bb[i][c] * u[j][c];
                    re[j][i] = acc;
                }
            } else {
#pragma unroll
                for (int i = 0; i < NS; ++i) re[j][i] = 0.0;
            }
        }
        // polytope rows: ri and F'lam partials
        double vp[NV];
#pragma unroll
        for (int i = 0; i < NS; ++i) vp[i] = W[L.xs + kp * NS + i];
#pragma unroll
        for (int i = 0; i < NU; ++i) vp[NS + i] = (kp < N) ? W[L.xu + kp * NU + i] : 0.0;
        double gpp[NV];
#pragma unroll
        for (int c = 0; c < NV; ++c) gpp[c] = 0.0;
#pragma unroll
        for (int q = 0; q < RPL; ++q) {
            const int r = lane + WAVE * q;
            if (r < mp) {
                double acc = tp[q] - hp[q];
#pragma unroll
                for (int c = 0; c < NV; ++c) {
                    const double f = Fs[c * mpad + r];
                    acc += f * vp[c];
                    gpp[c] += f * lp[q];
                }
                rip[q] = acc;
                cs += tp[q] * lp[q];
            } else {
                rip[q] = 0.0;
            }
        }
#pragma unroll
        for (int c = 0; c < NV; ++c) gpp[c] = wsum(gpp[c]);
#pragma unroll
        for (int j = 0; j < SPL; ++j) {
            const int k = lane + WAVE * j;
            if (k == kp) {
#pragma unroll
                for (int i = 0; i < NS; ++i) rs[j][i] += gpp[i];
                if (kp < N) {
#pragma unroll
                    for (int i = 0; i < NU; ++i) ru[j][i] += gpp[NS + i];
                }
            }
            if (k == 0) {
#pragma unroll
                for (int i = 0; i < NX; ++i) rs[j][i] = 0.0;
            }
#pragma unroll
            for (int i = 0; i < NS; ++i) { st = fmax(st, fabs(rs[j][i])); fe = fmax(fe, fabs(re[j][i])); }
#pragma unroll
            for (int i = 0; i < NU; ++i) st = fmax(st, fabs(ru[j][i]));
#pragma unroll
            for (int i = 0; i < NX; ++i) fe = fmax(fe, fmax(fabs(rix[j][i][0]), fabs(rix[j][i][1])));
#pragma unroll
            for (int i = 0; i < NU; ++i) fe = fmax(fe, fmax(fabs(riu[j][i][0]), fabs(riu[j][i][1])));
        }
#pragma unroll
        for (int q = 0; q < RPL; ++q) fe = fmax(fe, fabs(rip[q]));
        stat = wmax(st);
        feas = wmax(fe);
        csum = wsum(cs);
        gscale = wmax(gs);
    };

    // ======================= Riccati factorisation =========================================
    double P0inv[NP][NP];
    auto factor = [&]() -> bool {
        // one reciprocal of t per row per iteration (reused by both solves and max_step)
#pragma unroll
        for (int j = 0; j < SPL; ++j) {
#pragma unroll
            for (int i = 0; i < NX; ++i) { itx[j][i][0] = 1.0 / tx[j][i][0]; itx[j][i][1] = 1.0 / tx[j][i][1]; }
#pragma unroll
            for (int i = 0; i < NU; ++i) { itu[j][i][0] = 1.0 / tu[j][i][0]; itu[j][i][1] = 1.0 / tu[j][i][1]; }
        }
#pragma unroll
        for (int q = 0; q < RPL; ++q) itp[q] = 1.0 / tp[q];
        // box diagonals -> LDS
#pragma unroll
        for (int j = 0; j < SPL; ++j) {
            const int k = lane + WAVE * j;
            if (k <= N) {
#pragma unroll
                for (int i = 0; i < NX; ++i) {
                    double d = 0;
                    if (xpres(j, i, 0)) d += lx[j][i][0] * itx[j][i][0];
                    if (xpres(j, i, 1)) d += lx[j][i][1] * itx[j][i][1];
                    W[L.Dx + k * NX + i] = d;
                }
#pragma unroll
                for (int i = 0; i < NU; ++i) {
                    double d = 0;
                    if (upres(j, i, 0)) d += lu[j][i][0] * itu[j][i][0];
                    if (upres(j, i, 1)) d += lu[j][i][1] * itu[j][i][1];
                    W[L.Du + k * NU + i] = d;
                }
            }
        }
        // polytope F'DF (upper triangle, reduced over the wave)
        double fd[NV * (NV + 1) / 2];
#pragma unroll
        for (int c = 0; c < NV * (NV + 1) / 2; ++c) fd[c] = 0.0;
#pragma unroll
        for (int q = 0; q < RPL; ++q) {
            const int r = lane + WAVE * q;
            if (r < mp) {
                const double d = lp[q] * itp[q];
                double f[NV];
#pragma unroll
                for (int c = 0; c < NV; ++c) f[c] = Fs[c * mpad + r];
                int idx = 0;
#pragma unroll
                for (int i2 = 0; i2 < NV; ++i2) {
                    const double di = d * f[i2];
#pragma unroll
                    for (int j2 = i2; j2 < NV; ++j2) fd[idx++] += di * f[j2];
                }
            }
        }
#pragma unroll
        for (int c = 0; c < NV * (NV + 1) / 2; ++c) fd[c] = wsum(fd[c]);
        if (lane == 0) {
            int idx = 0;
#pragma unroll
            for (int i2 = 0; i2 < NV; ++i2)
#pragma unroll
                for (int j2 = i2; j2 < NV; ++j2) {
                    W[L.FD + i2 * NV + j2] = fd[idx];
                    W[L.FD + j2 * NV + i2] = fd[idx];
                    ++idx;
                }
        }
        wave_sync();
        // Htilde entry (i, j) of stage k
        auto ht = [&](int k, int i, int j) -> double {
            double h = Hs[k * hstride + i * NV + j];
            if (i == j) {
                if (i < NX) h += W[L.Dx + k * NX + i];
                else if (i >= NS) h += W[L.Du + k * NU + (i - NS)];
            }
            if (k == kp) h += W[L.FD + i * NV + j];
            return h;
        };
        // P_N
        if (lane < NS * NS) W[L.P + N * NS * NS + ib * NS + jb] = ht(N, ib, jb);
        wave_sync();
        double Pr[NS][NS];
#pragma unroll
        for (int i = 0; i < NS; ++i)
#pragma unroll
            for (int c = 0; c < NS; ++c) Pr[i][c] = W[L.P + N * NS * NS + i * NS + c];
        bool ok = true;
        for (int k = N - 1; k >= 0; --k) {
            // phase A: input rows of M = Ht + F' P F
            if (alane) {
                double acc = 0.0;
#pragma unroll
                for (int a_ = 0; a_ < NS; ++a_) {
                    double pf = 0.0;
#pragma unroll
                    for (int b = 0; b < NS; ++b) pf += Pr[a_][b] * FjA[b];
                    acc += BxA[a_] * pf;
                }
                W[L.M + xa * NV + ja] = ht(k, NS + xa, ja) + acc;
            }
            wave_sync();
            double Ruu[NU][NU], Ri[NU][NU];
#pragma unroll
            for (int x = 0; x < NU; ++x)
#pragma unroll
                for (int y = 0; y < NU; ++y) Ruu[x][y] = W[L.M + x * NV + NS + y];
            if constexpr (NU == 1) {
                ok = ok && (Ruu[0][0] > 0.0);
                Ri[0][0] = 1.0 / Ruu[0][0];
            } else if constexpr (NU == 2) {
                // Cholesky-based inverse, same order as oracle/cpu_ipm.c chol_inv
                const double l00 = sqrt(Ruu[0][0]);
                const double l10 = Ruu[1][0] / l00;
                const double d1 = Ruu[1][1] - l10 * l10;
                ok = ok && (Ruu[0][0] > 0.0) && (d1 > 0.0);
                const double l11 = sqrt(d1);
                const double i00 = 1.0 / l00, i11 = 1.0 / l11;
                const double i10 = -(l10 * i00) / l11;
                Ri[0][0] = i00 * i00 + i10 * i10;
                Ri[0][1] = i10 * i11;
                Ri[1][0] = i11 * i10;
                Ri[1][1] = i11 * i11;
            }
            // phase B: K columns ib, jb; Phi = Abar + Bbar K; Joseph-form P_k(ib, jb)
            if (blane) {
                double Ki[NU], Kj[NU];
#pragma unroll
                for (int x = 0; x < NU; ++x) {
                    double vi = 0.0, vj = 0.0;
#pragma unroll
                    for (int y = 0; y < NU; ++y) {
                        vi -= Ri[x][y] * W[L.M + y * NV + ib];
                        vj -= Ri[x][y] * W[L.M + y * NV + jb];
                    }
                    Ki[x] = vi; Kj[x] = vj;
                }
                double Phi_i[NS], Phi_j[NS];
#pragma unroll
                for (int a_ = 0; a_ < NS; ++a_) {
                    double vi = AiB[a_], vj = AjB[a_];
#pragma unroll
                    for (int x = 0; x < NU; ++x) { vi += Bb[a_][x] * Ki[x]; vj += Bb[a_][x] * Kj[x]; }
                    Phi_i[a_] = vi; Phi_j[a_] = vj;
                }
                double v = ht(k, ib, jb);
#pragma unroll
                for (int x = 0; x < NU; ++x) {
                    v += Ki[x] * ht(k, NS + x, jb) + ht(k, ib, NS + x) * Kj[x];
#pragma unroll
                    for (int y = 0; y < NU; ++y) v += Ki[x] * ht(k, NS + x, NS + y) * Kj[y];
                }
                double acc = 0.0;
#pragma unroll
                for (int a_ = 0; a_ < NS; ++a_) {
                    double pf = 0.0;
#pragma unroll
                    for (int b = 0; b < NS; ++b) pf += Pr[a_][b] * Phi_j[b];
                    acc += Phi_i[a_] * pf;
                }
                v += acc;
                W[L.P + k * NS * NS + ib * NS + jb] = v;
                W[L.P + k * NS * NS + jb * NS + ib] = v;
                if (ib == 0) {
#pragma unroll
                    for (int x = 0; x < NU; ++x) W[L.K + k * NU * NS + x * NS + jb] = Kj[x];
                }
            }
            if (lane == 0) {
#pragma unroll
                for (int x = 0; x < NU; ++x)
#pragma unroll
                    for (int y = 0; y < NU; ++y) W[L.Ri + k * NU * NU + x * NU + y] = Ri[x][y];
            }
            wave_sync();
#pragma unroll
            for (int i = 0; i < NS; ++i)
#pragma unroll
                for (int c = 0; c < NS; ++c) Pr[i][c] = W[L.P + k * NS * NS + i * NS + c];
        }
        // theta block of P_0
        double Pt[NP][NP];
#pragma unroll
        for (int x = 0; x < NP; ++x)
#pragma unroll
            for (int y = 0; y < NP; ++y) Pt[x][y] = Pr[NX + x][NX + y];
        if constexpr (NP == 1) {
            ok = ok && (Pt[0][0] > 0.0);
            P0inv[0][0] = 1.0 / Pt[0][0];
        } else if constexpr (NP == 2) {
            const double l00 = sqrt(Pt[0][0]);
            const double l10 = Pt[1][0] / l00;
            const double d1 = Pt[1][1] - l10 * l10;
            ok = ok && (Pt[0][0] > 0.0) && (d1 > 0.0);
            const double l11 = sqrt(d1);
            const double i00 = 1.0 / l00, i11 = 1.0 / l11;
            const double i10 = -(l10 * i00) / l11;
            P0inv[0][0] = i00 * i00 + i10 * i10;
            P0inv[0][1] = i10 * i11;
            P0inv[1][0] = i11 * i10;
            P0inv[1][1] = i11 * i11;
        }
        return ok;
    };

    // ======================= Newton solve for a given rc ===================================
    auto solve = [&]() {
        // q = r_v + C'((lam o ri - rc)/t); stage parts -> registers, then LDS
        double qs[SPL][NS], qu[SPL][NU];
#pragma unroll
        for (int j = 0; j < SPL; ++j) {
#pragma unroll
            for (int i = 0; i < NS; ++i) qs[j][i] = rs[j][i];
#pragma unroll
            for (int i = 0; i < NX; ++i) {
                double e = 0.0;
                if (xpres(j, i, 0)) e += (lx[j][i][0] * rix[j][i][0] - rcx[j][i][0]) * itx[j][i][0];
                if (xpres(j, i, 1)) e -= (lx[j][i][1] * rix[j][i][1] - rcx[j][i][1]) * itx[j][i][1];
                qs[j][i] += e;
            }
#pragma unroll
            for (int i = 0; i < NU; ++i) {
                double e = ru[j][i];
                if (upres(j, i, 0)) e += (lu[j][i][0] * riu[j][i][0] - rcu[j][i][0]) * itu[j][i][0];
                if (upres(j, i, 1)) e -= (lu[j][i][1] * riu[j][i][1] - rcu[j][i][1]) * itu[j][i][1];
                qu[j][i] = e;
            }
        }
        {
            double gpp[NV];
#pragma unroll
            for (int c = 0; c < NV; ++c) gpp[c] = 0.0;
#pragma unroll
            for (int q = 0; q < RPL; ++q) {
                const int r = lane + WAVE * q;
                if (r < mp) {
                    const double e = (lp[q] * rip[q] - rcp[q]) * itp[q];
#pragma unroll
                    for (int c = 0; c < NV; ++c) gpp[c] += Fs[c * mpad + r] * e;
                }
            }
#pragma unroll
            for (int c = 0; c < NV; ++c) gpp[c] = wsum(gpp[c]);
#pragma unroll
            for (int j = 0; j < SPL; ++j) {
                if (lane + WAVE * j == kp) {
#pragma unroll
                    for (int i = 0; i < NS; ++i) qs[j][i] += gpp[i];
                    if (kp < N) {
#pragma unroll
                        for (int i = 0; i < NU; ++i) qu[j][i] += gpp[NS + i];
                    }
                }
            }
        }
        // pre-pass: wv_k = P_{k+1} re_k, qt_k = qs_k + K_k' qu_k ; p_N = qs_N
#pragma unroll
        for (int j = 0; j < SPL; ++j) {
            const int k = lane + WAVE * j;
            if (k < N) {
                const double* Pn = W + L.P + (k + 1) * NS * NS;
                const double* Kk = W + L.K + k * NU * NS;
#pragma unroll
                for (int i = 0; i < NS; ++i) {
                    double v = 0.0;
#pragma unroll
                    for (int c = 0; c < NS; ++c) v += Pn[i * NS + c] * re[j][c];
                    W[L.wv + k * NS + i] = v;
                    double qq = qs[j][i];
#pragma unroll
                    for (int x = 0; x < NU; ++x) qq += Kk[x * NS + i] * qu[j][x];
                    W[L.qt + k * NS + i] = qq;
                }
#pragma unroll
                for (int x = 0; x < NU; ++x) W[L.qu + k * NU + x] = qu[j][x];
            } else if (k == N) {
#pragma unroll
                for (int i = 0; i < NS; ++i) W[L.p + N * NS + i] = qs[j][i];
            }
        }
        wave_sync();
        // backward sweep (redundant in every lane)
        double pv[NS];
#pragma unroll
        for (int i = 0; i < NS; ++i) pv[i] = W[L.p + N * NS + i];
        for (int k = N - 1; k >= 0; --k) {
            const double* Kk = W + L.K + k * NU * NS;
            double y[NS], by[NU];
#pragma unroll
            for (int i = 0; i < NS; ++i) y[i] = pv[i] + W[L.wv + k * NS + i];
#pragma unroll
            for (int x = 0; x < NU; ++x) {
                double v = 0.0;
#pragma unroll
                for (int c = 0; c < NS; ++c) v += Bb[c][x] * y[c];
                by[x] = v;
            }
#pragma unroll
            for (int i = 0; i < NS; ++i) {
                double v = W[L.qt + k * NS + i];
#pragma unroll
                for (int c = 0; c < NS; ++c) v += Ab[c][i] * y[c];
#pragma unroll
                for (int x = 0; x < NU; ++x) v += Kk[x * NS + i] * by[x];
                pv[i] = v;
            }
            if (lane == 0) {
#pragma unroll
                for (int i = 0; i < NS; ++i) W[L.p + k * NS + i] = pv[i];
            }
        }
        wave_sync();
        // post-backward: kff, f
#pragma unroll
        for (int j = 0; j < SPL; ++j) {
            const int k = lane + WAVE * j;
            if (k < N) {
                double y[NS], r[NU];
#pragma unroll
                for (int i = 0; i < NS; ++i) y[i] = W[L.p + (k + 1) * NS + i] + W[L.wv + k * NS + i];
#pragma unroll
                for (int x = 0; x < NU; ++x) {
                    double v = qu[j][x];
#pragma unroll
                    for (int c = 0; c < NS; ++c) v += Bb[c][x] * y[c];
                    r[x] = v;
                }
                const double* Ri = W + L.Ri + k * NU * NU;
#pragma unroll
                for (int x = 0; x < NU; ++x) {
                    double v = 0.0;
#pragma unroll
                    for (int y2 = 0; y2 < NU; ++y2) v -= Ri[x * NU + y2] * r[y2];
                    kff[j][x] = v;
                }
#pragma unroll
                for (int i = 0; i < NS; ++i) {
                    double v = re[j][i];
#pragma unroll
                    for (int x = 0; x < NU; ++x) v += Bb[i][x] * kff[j][x];
                    W[L.fv + k * NS + i] = v;
                }
            }
        }
        wave_sync();
        // theta_0 step + forward sweep (redundant)
        double dv0[NS];
#pragma unroll
        for (int i = 0; i < NX; ++i) dv0[i] = 0.0;
#pragma unroll
        for (int x = 0; x < NP; ++x) {
            double v = 0.0;
#pragma unroll
            for (int y2 = 0; y2 < NP; ++y2) v -= P0inv[x][y2] * W[L.p + NX + y2];
            dv0[NX + x] = v;
        }
        if (lane == 0) {
#pragma unroll
            for (int i = 0; i < NS; ++i) W[L.dsv + i] = dv0[i];
        }
        for (int k = 0; k < N; ++k) {
            const double* Kk = W + L.K + k * NU * NS;
            double kd[NU];
#pragma unroll
            for (int x = 0; x < NU; ++x) {
                double v = 0.0;
#pragma unroll
                for (int c = 0; c < NS; ++c) v += Kk[x * NS + c] * dv0[c];
                kd[x] = v;
            }
            double nd[NS];
#pragma unroll
            for (int i = 0; i < NS; ++i) {
                double v = W[L.fv + k * NS + i];
#pragma unroll
                for (int c = 0; c < NS; ++c) v += Ab[i][c] * dv0[c];
#pragma unroll
                for (int x = 0; x < NU; ++x) v += Bb[i][x] * kd[x];
                nd[i] = v;
            }
#pragma unroll
            for (int i = 0; i < NS; ++i) dv0[i] = nd[i];
            if (lane == 0) {
#pragma unroll
                for (int i = 0; i < NS; ++i) W[L.dsv + (k + 1) * NS + i] = nd[i];
            }
        }
        wave_sync();
        // post-forward: ds, du, dpi, box steps; publish polytope-stage step
#pragma unroll
        for (int j = 0; j < SPL; ++j) {
            const int k = lane + WAVE * j;
            if (k > N) continue;
#pragma unroll
            for (int i = 0; i < NS; ++i) ds[j][i] = W[L.dsv + k * NS + i];
            if (k < N) {
                const double* Kk = W + L.K + k * NU * NS;
#pragma unroll
                for (int x = 0; x < NU; ++x) {
                    double v = kff[j][x];
#pragma unroll
                    for (int c = 0; c < NS; ++c) v += Kk[x * NS + c] * ds[j][c];
                    du[j][x] = v;
                }
            } else {
#pragma unroll
                for (int x = 0; x < NU; ++x) du[j][x] = 0.0;
            }
#pragma unroll
            for (int x = 0; x < NU; ++x) W[L.duv + k * NU + x] = du[j][x];
            if (k >= 1) {
                const double* Pk = W + L.P + k * NS * NS;
#pragma unroll
                for (int i = 0; i < NS; ++i) {
                    double v = W[L.p + k * NS + i];
#pragma unroll
                    for (int c = 0; c < NS; ++c) v += Pk[i * NS + c] * ds[j][c];
                    dpi[j][i] = v;
                }
            } else {
#pragma unroll
                for (int i = 0; i < NS; ++i) dpi[j][i] = 0.0;
            }
#pragma unroll
            for (int i = 0; i < NX; ++i) {
                const double dx = ds[j][i];
                dtx[j][i][0] = dtx[j][i][1] = dlx[j][i][0] = dlx[j][i][1] = 0.0;
                if (xpres(j, i, 0)) {
                    dtx[j][i][0] = -rix[j][i][0] - dx;
                    dlx[j][i][0] = (-rcx[j][i][0] - lx[j][i][0] * dtx[j][i][0]) * itx[j][i][0];
                }
                if (xpres(j, i, 1)) {
                    dtx[j][i][1] = -rix[j][i][1] + dx;
                    dlx[j][i][1] = (-rcx[j][i][1] - lx[j][i][1] * dtx[j][i][1]) * itx[j][i][1];
                }
            }
#pragma unroll
            for (int i = 0; i < NU; ++i) {
                const double dd = du[j][i];
                dtu[j][i][0] = dtu[j][i][1] = dlu[j][i][0] = dlu[j][i][1] = 0.0;
                if (upres(j, i, 0)) {
                    dtu[j][i][0] = -riu[j][i][0] - dd;
                    dlu[j][i][0] = (-rcu[j][i][0] - lu[j][i][0] * dtu[j][i][0]) * itu[j][i][0];
                }
                if (upres(j, i, 1)) {
                    dtu[j][i][1] = -riu[j][i][1] + dd;
                    dlu[j][i][1] = (-rcu[j][i][1] - lu[j][i][1] * dtu[j][i][1]) * itu[j][i][1];
                }
            }
        }
        wave_sync();
        double dvp[NV];
#pragma unroll
        for (int i = 0; i < NS; ++i) dvp[i] = W[L.dsv + kp * NS + i];
#pragma unroll
        for (int i = 0; i < NU; ++i) dvp[NS + i] = (kp < N) ? W[L.duv + kp * NU + i] : 0.0;
#pragma unroll
        for (int q = 0; q < RPL; ++q) {
            const int r = lane + WAVE * q;
            if (r < mp) {
                double acc = 0.0;
#pragma unroll
                for (int c = 0; c < NV; ++c) acc += Fs[c * mpad + r] * dvp[c];
                dtp[q] = -rip[q] - acc;
                dlp[q] = (-rcp[q] - lp[q] * dtp[q]) * itp[q];
            } else {
                dtp[q] = 0.0; dlp[q] = 0.0;
            }
        }
    };

    // alpha = min(1, 1 / max(-dt/t, -dlam/lam)) (same form as oracle/cpu_ipm.c max_step)
    auto max_step = [&]() -> double {
        double rm = 0.0;
#define BQP_RATIO(dv, iv) { const double qq = -(dv) * (iv); rm = fmax(rm, qq); }
#pragma unroll
        for (int j = 0; j < SPL; ++j) {
#pragma unroll
            for (int i = 0; i < NX; ++i)
#pragma unroll
                for (int h = 0; h < 2; ++h)
                    if (xpres(j, i, h)) { BQP_RATIO(dtx[j][i][h], itx[j][i][h]); BQP_RATIO(dlx[j][i][h], 1.0 / lx[j][i][h]); }
#pragma unroll
            for (int i = 0; i < NU; ++i)
#pragma unroll
                for (int h = 0; h < 2; ++h)
                    if (upres(j, i, h)) { BQP_RATIO(dtu[j][i][h], itu[j][i][h]); BQP_RATIO(dlu[j][i][h], 1.0 / lu[j][i][h]); }
        }
#pragma unroll
        for (int q = 0; q < RPL; ++q)
            if (lane + WAVE * q < mp) { BQP_RATIO(dtp[q], itp[q]); BQP_RATIO(dlp[q], 1.0 / lp[q]); }
#undef BQP_RATIO
        rm = wmax(rm);
        return rm > 1.0 ? 1.0 / rm : 1.0;
    };

    auto comp_after = [&](double al) -> double {
        double c = 0.0;
#pragma unroll
        for (int j = 0; j < SPL; ++j) {
#pragma unroll
            for (int i = 0; i < NX; ++i)
#pragma unroll
                for (int h = 0; h < 2; ++h)
                    if (xpres(j, i, h)) c += (tx[j][i][h] + al * dtx[j][i][h]) * (lx[j][i][h] + al * dlx[j][i][h]);
#pragma unroll
            for (int i = 0; i < NU; ++i)
#pragma unroll
                for (int h = 0; h < 2; ++h)
                    if (upres(j, i, h)) c += (tu[j][i][h] + al * dtu[j][i][h]) * (lu[j][i][h] + al * dlu[j][i][h]);
        }
#pragma unroll
        for (int q = 0; q < RPL; ++q)
            if (lane + WAVE * q < mp) c += (tp[q] + al * dtp[q]) * (lp[q] + al * dlp[q]);
        return wsum(c);
    };

    // ======================= initial point ==================================================
#pragma unroll
    for (int j = 0; j < SPL; ++j) {
#pragma unroll
        for (int i = 0; i < NX; ++i)
#pragma unroll
            for (int h = 0; h < 2; ++h) { tx[j][i][h] = 1.0; lx[j][i][h] = 1.0; rcx[j][i][h] = 1.0; }
#pragma unroll
        for (int i = 0; i < NU; ++i)
#pragma unroll
            for (int h = 0; h < 2; ++h) { tu[j][i][h] = 1.0; lu[j][i][h] = 1.0; rcu[j][i][h] = 1.0; }
    }
#pragma unroll
    for (int q = 0; q < RPL; ++q) { tp[q] = 1.0; lp[q] = 1.0; rcp[q] = 1.0; }
    double stat = 0, feas = 0, csum = 0, gscale = 0;
    residuals(stat, feas, csum, gscale);
    int flag = 0;
    bool ok = factor();
    if (!ok) flag = -8;
    solve();
    {
        double tmin = INFINITY, tmax = -INFINITY;
#pragma unroll
        for (int j = 0; j < SPL; ++j) {
#pragma unroll
            for (int i = 0; i < NS; ++i) { s[j][i] += ds[j][i]; pi[j][i] += dpi[j][i]; }
#pragma unroll
            for (int i = 0; i < NU; ++i) u[j][i] += du[j][i];
#pragma unroll
            for (int i = 0; i < NX; ++i)
#pragma unroll
                for (int h = 0; h < 2; ++h)
                    if (xpres(j, i, h)) { const double t = 1.0 + dtx[j][i][h]; tmin = fmin(tmin, t); tmax = fmax(tmax, t); }
#pragma unroll
            for (int i = 0; i < NU; ++i)
#pragma unroll
                for (int h = 0; h < 2; ++h)
                    if (upres(j, i, h)) { const double t = 1.0 + dtu[j][i][h]; tmin = fmin(tmin, t); tmax = fmax(tmax, t); }
        }
#pragma unroll
        for (int q = 0; q < RPL; ++q)
            if (lane + WAVE * q < mp) { const double t = 1.0 + dtp[q]; tmin = fmin(tmin, t); tmax = fmax(tmax, t); }
        tmin = wmin(tmin);
        tmax = wmax(tmax);
        const double shp = (tmin <= 0.0) ? 1.0 - tmin : 0.0;
        const double shd = (tmax >= 0.0) ? 1.0 + tmax : 0.0;
#pragma unroll
        for (int j = 0; j < SPL; ++j) {
#pragma unroll
            for (int i = 0; i < NX; ++i)
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const double t = 1.0 + dtx[j][i][h];
                    const bool pr = xpres(j, i, h);
                    tx[j][i][h] = pr ? t + shp : 1.0;
                    lx[j][i][h] = pr ? -t + shd : 0.0;
                }
#pragma unroll
            for (int i = 0; i < NU; ++i)
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const double t = 1.0 + dtu[j][i][h];
                    const bool pr = upres(j, i, h);
                    tu[j][i][h] = pr ? t + shp : 1.0;
                    lu[j][i][h] = pr ? -t + shd : 0.0;
                }
        }
#pragma unroll
        for (int q = 0; q < RPL; ++q) {
            const double t = 1.0 + dtp[q];
            const bool pr = lane + WAVE * q < mp;
            tp[q] = pr ? t + shp : 1.0;
            lp[q] = pr ? -t + shd : 0.0;
        }
    }

    // ======================= main loop ======================================================
    int it = 0;
    double mu = 0.0;
    const int max_iter = a.max_iter;
    if (flag == 0) {
        for (it = 0; it <= max_iter; ++it) {
            residuals(stat, feas, csum, gscale);
            mu = csum * minv;
            if (stat <= a.tol_stat * (1.0 + gscale) && feas <= a.tol_feas * (1.0 + bscale) &&
                mu <= a.tol_comp) { flag = 1; break; }
            if (!(isfinite(stat) && isfinite(feas) && isfinite(mu))) { flag = -8; break; }
            if (it == max_iter) break;
            if (!factor()) { flag = -8; break; }
            // predictor
#pragma unroll
            for (int j = 0; j < SPL; ++j) {
#pragma unroll
                for (int i = 0; i < NX; ++i)
#pragma unroll
                    for (int h = 0; h < 2; ++h) rcx[j][i][h] = tx[j][i][h] * lx[j][i][h];
#pragma unroll
                for (int i = 0; i < NU; ++i)
#pragma unroll
                    for (int h = 0; h < 2; ++h) rcu[j][i][h] = tu[j][i][h] * lu[j][i][h];
            }
#pragma unroll
            for (int q = 0; q < RPL; ++q) rcp[q] = tp[q] * lp[q];
            solve();
            double al = max_step();
            const double mua = comp_after(al) * minv;
            double sg = mua / mu;
            sg = sg * sg * sg;
            const double smu = sg * mu;
            // corrector rhs
#pragma unroll
            for (int j = 0; j < SPL; ++j) {
#pragma unroll
                for (int i = 0; i < NX; ++i)
#pragma unroll
                    for (int h = 0; h < 2; ++h) rcx[j][i][h] = tx[j][i][h] * lx[j][i][h] + dtx[j][i][h] * dlx[j][i][h] - smu;
#pragma unroll
                for (int i = 0; i < NU; ++i)
#pragma unroll
                    for (int h = 0; h < 2; ++h) rcu[j][i][h] = tu[j][i][h] * lu[j][i][h] + dtu[j][i][h] * dlu[j][i][h] - smu;
            }
#pragma unroll
            for (int q = 0; q < RPL; ++q) rcp[q] = tp[q] * lp[q] + dtp[q] * dlp[q] - smu;
            solve();
            al = max_step() * a.tau;
            if (al > 1.0) al = 1.0;
#pragma unroll
            for (int j = 0; j < SPL; ++j) {
#pragma unroll
                for (int i = 0; i < NS; ++i) { s[j][i] += al * ds[j][i]; pi[j][i] += al * dpi[j][i]; }
#pragma unroll
                for (int i = 0; i < NU; ++i) u[j][i] += al * du[j][i];
#pragma unroll
                for (int i = 0; i < NX; ++i)
#pragma unroll
                    for (int h = 0; h < 2; ++h)
                        if (xpres(j, i, h)) { tx[j][i][h] += al * dtx[j][i][h]; lx[j][i][h] += al * dlx[j][i][h]; }
#pragma unroll
                for (int i = 0; i < NU; ++i)
#pragma unroll
                    for (int h = 0; h < 2; ++h)
                        if (upres(j, i, h)) { tu[j][i][h] += al * dtu[j][i][h]; lu[j][i][h] += al * dlu[j][i][h]; }
            }
#pragma unroll
            for (int q = 0; q < RPL; ++q)
                if (lane + WAVE * q < mp) { tp[q] += al * dtp[q]; lp[q] += al * dlp[q]; }
        }
    }

    // ======================= outputs =======================================================
    double fv = 0.0;
#pragma unroll
    for (int j = 0; j < SPL; ++j) {
        const int k = lane + WAVE * j;
        if (k > N) continue;
        double* xo = a.x + ((int64_t)inst * (N + 1) + k) * NX;
#pragma unroll
        for (int i = 0; i < NX; ++i) xo[i] = s[j][i];
        if (k < N) {
            double* uo = a.u + ((int64_t)inst * N + k) * NU;
#pragma unroll
            for (int i = 0; i < NU; ++i) uo[i] = u[j][i];
        }
        if (k == 0) {
#pragma unroll
            for (int i = 0; i < NP; ++i) a.theta[(int64_t)inst * NP + i] = s[j][NX + i];
        }
        // objective 0.5 v'Hv + g'v of this stage
        const double* Hk = Hs + k * hstride;
        double v[NV];
#pragma unroll
        for (int i = 0; i < NS; ++i) v[i] = s[j][i];
#pragma unroll
        for (int i = 0; i < NU; ++i) v[NS + i] = (k < N) ? u[j][i] : 0.0;
#pragma unroll
        for (int i = 0; i < NV; ++i) {
            double hv = 0.0;
#pragma unroll
            for (int c = 0; c < NV; ++c) hv += Hk[i * NV + c] * v[c];
            fv += v[i] * (0.5 * hv + g[j][i]);
        }
        if (a.pi_out && k >= 1) {
            double* po = a.pi_out + ((int64_t)inst * N + (k - 1)) * NX;
#pragma unroll
            for (int i = 0; i < NX; ++i) po[i] = pi[j][i];
        }
        if (a.lamx_out) {
            double* lo = a.lamx_out + ((int64_t)inst * (N + 1) + k) * NX * 2;
#pragma unroll
            for (int i = 0; i < NX; ++i) {
                lo[i] = xpres(j, i, 1) ? lx[j][i][1] : 0.0;        // lower
                lo[NX + i] = xpres(j, i, 0) ? lx[j][i][0] : 0.0;   // upper
            }
        }
        if (a.lamu_out && k < N) {
            double* lo = a.lamu_out + ((int64_t)inst * N + k) * NU * 2;
#pragma unroll
            for (int i = 0; i < NU; ++i) {
                lo[i] = upres(j, i, 1) ? lu[j][i][1] : 0.0;
                lo[NU + i] = upres(j, i, 0) ? lu[j][i][0] : 0.0;
            }
        }
    }
    if (a.lamp_out) {
#pragma unroll
        for (int q = 0; q < RPL; ++q) {
            const int r = lane + WAVE * q;
            if (r < mp) a.lamp_out[(int64_t)inst * mp + r] = lp[q];
        }
    }
    fv = wsum(fv);
    if (lane == 0) {
        if (a.fval) a.fval[inst] = fv;
        a.exitflag[inst] = flag;
        if (a.stats) {
            double* so = a.stats + (int64_t)inst * 4;
            so[0] = (double)it; so[1] = stat; so[2] = feas; so[3] = mu;
        }
    }
}

// ------------------------------------------------------------------------------------------
// host-side launch helpers
// ------------------------------------------------------------------------------------------
int ocp_wave_lds_doubles(int N, int nx, int nu, int np) {
    const int ns = nx + np, nv = ns + nu;
    return WaveLds::make(N, nx, nu, ns, nv).total;
}

template <int NX, int NU, int NP, int SPL, int RPL>
static hipError_t launch_t(const OcpKernelArgs& a, int blocks, size_t lds, hipStream_t st) {
    auto k = ocp_ipm_kernel<NX, NU, NP, SPL, RPL>;
    if (lds > 64 * 1024) {
        hipError_t e = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(k, dim3(blocks), dim3(64 * a.wpb), lds, st, a);
    return hipGetLastError();
}

template <int NX, int NU, int NP, int SPL>
static hipError_t launch_rpl(const OcpKernelArgs& a, int rpl, int blocks, size_t lds, hipStream_t st) {
    switch (rpl) {
        case 1: return launch_t<NX, NU, NP, SPL, 1>(a, blocks, lds, st);
        case 4: return launch_t<NX, NU, NP, SPL, 4>(a, blocks, lds, st);
        case 10: return launch_t<NX, NU, NP, SPL, 10>(a, blocks, lds, st);
        case 16: return launch_t<NX, NU, NP, SPL, 16>(a, blocks, lds, st);
        default: return hipErrorInvalidValue;
    }
}

template <int NX, int NU, int NP>
static hipError_t launch_spl(const OcpKernelArgs& a, int spl, int rpl, int blocks, size_t lds, hipStream_t st) {
    if (spl == 1) return launch_rpl<NX, NU, NP, 1>(a, rpl, blocks, lds, st);
    if (spl == 2) return launch_rpl<NX, NU, NP, 2>(a, rpl, blocks, lds, st);
    return hipErrorInvalidValue;
}

bool ocp_supported(int nx, int nu, int np) {
    return (nx == 4 && nu == 1 && np == 1) || (nx == 2 && nu == 2 && np == 2);
}

int ocp_rpl_for(int mp) {
    if (mp <= 64) return 1;
    if (mp <= 256) return 4;
    if (mp <= 640) return 10;
    if (mp <= 1024) return 16;
    return -1;
}

hipError_t launch_ocp(const OcpKernelArgs& a, int nx, int nu, int np, hipStream_t st) {
    const int spl = (a.N + 1 <= 64) ? 1 : 2;
    const int rpl = ocp_rpl_for(a.mp);
    const int blocks = (a.batch + a.wpb - 1) / a.wpb;
    const size_t lds = sizeof(double) * ((size_t)a.shared_doubles + (size_t)a.wpb * ocp_wave_lds_doubles(a.N, nx, nu, np));
    if (nx == 4 && nu == 1 && np == 1) return launch_spl<4, 1, 1>(a, spl, rpl, blocks, lds, st);
    if (nx == 2 && nu == 2 && np == 2) return launch_spl<2, 2, 2>(a, spl, rpl, blocks, lds, st);
    return hipErrorInvalidValue;
}

}  // namespace bqp
