// bqp_ocp.hip — batched structured Mehrotra predictor-corrector IPM for MPC QPs, gfx950.
//
// One wavefront (64 lanes) solves one MPC instance; a workgroup holds WPB instances that share
// the stage-cost table H_k and the polytope (terminal-set) matrix in LDS.  Inside a wave the
// lanes are re-assigned per phase:
//   * stage phases   lane k (and k+64 when SPL=2) owns stage k: s_k=[x_k;theta], u_k, pi_k
//                    and the slacks/duals of the box rows of stage k;
//   * polytope rows  lane l owns rows l, l+64, ... (RPL rows): slack, dual, 1/slack in
//                    registers; F'DF and F'e are reduced with DPP lane moves;
//   * Riccati factor lane (i,j) owns entry (i,j) of the stage matrices (Joseph form); P_{k+1}
//                    is broadcast from LDS at each stage (sequential over k);
//   * Riccati solves every lane runs the NS-vector closed-loop recursion redundantly (no
//                    cross-lane traffic on the sequential critical path).
// Register budget (one wave per SIMD at the C2 batch): per-row residuals and steps are
// recomputed from the stage vectors when needed instead of being kept live, so the kernel
// holds ~85 fp64 values per lane.
// The algorithm (and its operation order) is stated in oracle/ocp_ipm.py and restated in C in
// oracle/cpu_ipm.c; the QP is the stage-wise form of the reference's per-step OCPs
// (costLMPC.m / constraintsLMPC.m, DMS_tracking_LMPC_casadi.m:223-287, trackingMPC/costFunction.m).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "bqp_internal.h"

namespace bqp {

#define WAVE 64
#define PIV_FLOOR 1e-14
#define MU_BLOWUP 1e6

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Wave-wide reductions on DPP lane moves (quad_perm xor1/xor2, row_half_mirror, row_mirror
// inside each 16-lane row, then row_bcast15/31 across rows) + a readlane of lane 63: no LDS
// traffic, result uniform in every lane.  EXEC must be full (all call sites are wave-uniform).
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
__device__ __forceinline__ double wmin(double v) { return -wmax(-v); }
// value of lane `src` broadcast to the wave (scalar register pair): the sequential Riccati
// sweeps pass their NS-vector from stage to stage this way instead of through LDS
__device__ __forceinline__ double rl(double v, int src) {
    const int2 x = __builtin_bit_cast(int2, v);
    int2 r;
    r.x = __builtin_amdgcn_readlane(x.x, src);
    r.y = __builtin_amdgcn_readlane(x.y, src);
    return __builtin_bit_cast(double, r);
}
template <int N>
__device__ __forceinline__ double sel(const double (&row)[N], int idx) {
    double r = row[0];
#pragma unroll
    for (int c = 1; c < N; ++c) r = (idx == c) ? row[c] : r;
    return r;
}

// Cholesky (lower, NxN with N <= 2) with static pivot floor; returns false if not PD.
template <int N>
__device__ __forceinline__ bool chol_small(const double (&M)[N][N], double (&L)[N][N]) {
    bool ok = true;
    double d0 = M[0][0];
    if (!(d0 > PIV_FLOOR * M[0][0])) d0 = PIV_FLOOR * M[0][0];
    ok = ok && (d0 > 0.0);
    L[0][0] = sqrt(d0);
    if constexpr (N == 2) {
        L[0][1] = 0.0;
        L[1][0] = M[1][0] / L[0][0];
        double d1 = M[1][1] - L[1][0] * L[1][0];
        if (!(d1 > PIV_FLOOR * M[1][1])) d1 = PIV_FLOOR * M[1][1];
        ok = ok && (d1 > 0.0);
        L[1][1] = sqrt(d1);
    }
    return ok;
}
// b <- M^{-1} b with M = L L' (substitution, same order as oracle/cpu_ipm.c spd_solve); L row-major.
// For n = 1 the factor slot holds 1/M instead (one reciprocal, no square root).
template <int N>
__device__ __forceinline__ void chol_solve_small(const double* L, double (&b)[N]) {
    if constexpr (N == 2) {
        b[0] = b[0] / L[0];
        b[1] = (b[1] - L[2] * b[0]) / L[3];
        b[1] = b[1] / L[3];
        b[0] = (b[0] - L[2] * b[1]) / L[0];
    } else {
        b[0] = b[0] * L[0];     // n = 1: L holds the reciprocal of the 1x1 matrix
    }
}

// Packed upper-triangular storage of the symmetric NS x NS Riccati matrices P_k: entry (i, j),
// i <= j, at pk_idx(i, j); each stage slot is padded to an even number of doubles so that a
// slot starts 16-byte aligned and is read back with ds_read_b128.
__host__ __device__ constexpr int pk_len(int NS) { return NS * (NS + 1) / 2; }
__host__ __device__ constexpr int pk_stride(int NS) { return (pk_len(NS) + 1) & ~1; }
__host__ __device__ constexpr int pk_idx(int NS, int i, int j) {
    return i <= j ? i * NS - i * (i - 1) / 2 + (j - i) : j * NS - j * (j - 1) / 2 + (i - j);
}

// Per-wave LDS layout (in doubles), all sized from N at run time.
struct WaveLds {
    int P, Phi, K, Lr, xs, xu, qt_xpi, rs, ru, re, pv, wv, qu, fv, dsv, duv, Dx, Du, FD, Mu, AB, L0, prp, hp, misc, total;
    __host__ __device__ static WaveLds make(int N, int NX, int NU, int NP, int mpad, bool store_phi) {
        const int NS = NX + NP, NV = NS + NU;
        WaveLds o;
        int c = 0;
        o.P = c;   c += (N + 1) * pk_stride(NS);
        o.Phi = c; c += store_phi ? N * NS * NS : 0;
        o.K = c;   c += N * NU * NS;
        o.Lr = c;  c += N * NU * NU;
        o.xs = c;  c += (N + 1) * NS;
        o.xu = c;  c += (N + 1) * NU;
        o.qt_xpi = c; c += (N + 1) * NS;   // pi exchange in residuals, qt in the solves
        o.rs = c;  c += (N + 1) * NS;
        o.ru = c;  c += (N + 1) * NU;
        o.re = c;  c += (N + 1) * NS;
        o.pv = c;  c += (N + 1) * NS;
        o.wv = c;  c += (N + 1) * NS;
        o.qu = c;  c += (N + 1) * NU;
        o.fv = c;  c += (N + 1) * NS;
        o.dsv = c; c += (N + 1) * NS;
        o.duv = c; c += (N + 1) * NU;
        o.Dx = c;  c += (N + 1) * NV;      // box diagonal of stage k in internal order (theta 0)
        o.Du = o.Dx;
        o.FD = c;  c += NV * NV;
        o.Mu = c;  c += NU * NV;
        o.AB = c;  c += NS * NS + NS * NU;
        o.L0 = c;  c += NP * NP;
        o.prp = c; c += mpad;              // predictor dt*dlam of the polytope rows
        o.hp = c;  c += mpad;              // this instance's polytope right-hand side
        o.misc = c; c += 8;
        o.total = (c + 1) & ~1;
        return o;
    }
};

template <int NX, int NU, int NP, int SPL, int RPL>
__global__ void __launch_bounds__(256) ocp_ipm_kernel(OcpKernelArgs a) {
    constexpr int NS = NX + NP;
    constexpr int NV = NS + NU;
    constexpr bool kPhi = (SPL == 1);     // store closed-loop Phi_k (LDS budget allows at N<64)
    extern __shared__ double lds[];
    const int N = a.N, mp = a.mp, kp = a.kp;
    const int lane = threadIdx.x & 63;
    const int wid = threadIdx.x >> 6;
    const int hstride = a.hstride;
    const int mpad = a.mpad;
    // ---------------- shared tables: H (N+1 stages) and Fp (column-major, mpad rows) -------
    double* Hs = lds;
    double* Fs = lds + (N + 1) * hstride;
    for (int i = threadIdx.x; i < (N + 1) * hstride; i += blockDim.x) Hs[i] = a.H[i];
    for (int i = threadIdx.x; i < NV * mpad; i += blockDim.x) Fs[i] = a.Fp[i];
    __syncthreads();
    const int inst = blockIdx.x * a.wpb + wid;
    if (inst >= a.batch) return;
    const WaveLds L = WaveLds::make(N, NX, NU, NP, mpad, kPhi);
    double* W = lds + a.shared_doubles + wid * L.total;
#ifdef BQP_STAMPS
    // diagnostic build only (see tools/stamps.py): cycles per phase, summed over the solve
    unsigned long long st_last = __builtin_amdgcn_s_memtime();
    unsigned long long st_acc[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) st_acc[i] = 0;
#define STAMP(id)                                                          \
    do {                                                                   \
        __builtin_amdgcn_s_waitcnt(0);                                     \
        const unsigned long long _t = __builtin_amdgcn_s_memtime();        \
        st_acc[id] += _t - st_last;                                        \
        st_last = _t;                                                      \
    } while (0)
#else
#define STAMP(id) do { } while (0)
#endif

    // ---------------- per-instance model -> LDS (Abar row-major, Bbar) ---------------------
    {
        const double* A = a.A + (int64_t)inst * a.sA;
        const double* B = a.B + (int64_t)inst * a.sB;
        if (lane < NS * NS) {
            const int i = lane / NS, j = lane % NS;
            W[L.AB + lane] = (i < NX && j < NX) ? A[j * NX + i] : (i == j ? 1.0 : 0.0);
        }
        if (lane < NS * NU) {
            const int i = lane / NU, j = lane % NU;
            W[L.AB + NS * NS + lane] = (i < NX) ? B[j * NX + i] : 0.0;
        }
    }
    wave_sync();
    auto Abar = [&](int i, int j) __attribute__((always_inline)) -> double { return W[L.AB + i * NS + j]; };
    auto Bbar = [&](int i, int j) __attribute__((always_inline)) -> double { return W[L.AB + NS * NS + i * NU + j]; };
    double cb[NS];
#pragma unroll
    for (int i = 0; i < NS; ++i) cb[i] = (i < NX && a.c) ? a.c[(int64_t)inst * a.sc + i] : 0.0;

    // ---------------- stage-lane state ------------------------------------------------------
    double s[SPL][NS], u[SPL][NU], pi[SPL][NS];
    double tx[SPL][NX][2], lx[SPL][NX][2], itx[SPL][NX][2], bx[SPL][NX][2];   // ub, lb
    double tu[SPL][NU][2], lu[SPL][NU][2], itu[SPL][NU][2], bu[SPL][NU][2];
    double prx[SPL][NX][2], pru[SPL][NU][2];                                    // predictor dt*dlam
    double kff[SPL][NU];
    unsigned mx[SPL], mu_[SPL];
    const double* x0 = a.x0 + (int64_t)inst * a.sx0;
#pragma unroll
    for (int j = 0; j < SPL; ++j) {
        const int k = lane + WAVE * j;
        const bool act = k <= N;
        mx[j] = 0; mu_[j] = 0;
#pragma unroll
        for (int i = 0; i < NS; ++i) { s[j][i] = 0.0; pi[j][i] = 0.0; }
#pragma unroll
        for (int i = 0; i < NU; ++i) { u[j][i] = 0.0; kff[j][i] = 0.0; }
        if (k == 0) {
#pragma unroll
            for (int i = 0; i < NX; ++i) s[j][i] = x0[i];
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
    auto xpres = [&](int j, int i, int h) __attribute__((always_inline)) -> bool { return (mx[j] >> (2 * i + h)) & 1u; };
    auto upres = [&](int j, int i, int h) __attribute__((always_inline)) -> bool { return (mu_[j] >> (2 * i + h)) & 1u; };
    // linear cost term of stage k, internal index i ([x; theta; u] from external [x; u; theta])
    const double* wb = a.w ? a.w + (int64_t)inst * a.sw : nullptr;
    auto gterm = [&](int k, int i) __attribute__((always_inline)) -> double {
        if (!wb || (k == N && i >= NS)) return 0.0;
        const int e = (i < NX) ? i : (i < NS ? NX + NU + (i - NX) : NX + (i - NS));
        return wb[(int64_t)k * NV + e];
    };
    // polytope rows
    double tp[RPL], lp[RPL], itp[RPL];
    // polytope right-hand side: one coalesced read into this wave's LDS slot
    double* hpi = W + L.hp;
    {
        const double* hg = a.hp + (int64_t)inst * a.shp;
        for (int r = lane; r < mp; r += WAVE) hpi[r] = hg[r];
        wave_sync();
    }
    auto prow = [&](int q) __attribute__((always_inline)) -> bool { return lane + WAVE * q < mp; };

    // row count and primal data scale
    double mcount = 0, bsl = 0;
#pragma unroll
    for (int j = 0; j < SPL; ++j) {
        mcount += __builtin_popcount(mx[j]) + __builtin_popcount(mu_[j]);
        if (lane + WAVE * j == 0) {
#pragma unroll
            for (int i = 0; i < NX; ++i) bsl = fmax(bsl, fabs(x0[i]));
        }
#pragma unroll
        for (int i = 0; i < NX; ++i)
#pragma unroll
            for (int h = 0; h < 2; ++h)
                if (xpres(j, i, h)) bsl = fmax(bsl, fabs(bx[j][i][h]));
#pragma unroll
        for (int i = 0; i < NU; ++i)
#pragma unroll
            for (int h = 0; h < 2; ++h)
                if (upres(j, i, h)) bsl = fmax(bsl, fabs(bu[j][i][h]));
    }
#pragma unroll
    for (int q = 0; q < RPL; ++q)
        if (prow(q)) { mcount += 1.0; bsl = fmax(bsl, fabs(hpi[lane + WAVE * q])); }
    mcount = wsum(mcount);
    const double minv = 1.0 / fmax(mcount, 1.0);
    const double bscale = wmax(bsl);

    // ----- helpers: box / polytope row residuals and steps (recomputed, never stored) -------
    auto rix = [&](int j, int i, int h) __attribute__((always_inline)) -> double {
        return h == 0 ? s[j][i] + tx[j][i][0] - bx[j][i][0] : -s[j][i] + tx[j][i][1] + bx[j][i][1];
    };
    auto riu = [&](int j, int i, int h) __attribute__((always_inline)) -> double {
        return h == 0 ? u[j][i] + tu[j][i][0] - bu[j][i][0] : -u[j][i] + tu[j][i][1] + bu[j][i][1];
    };
    auto load_vp = [&](double (&vp)[NV], int base_s, int base_u) {
#pragma unroll
        for (int c = 0; c < NS; ++c) vp[c] = W[base_s + kp * NS + c];
#pragma unroll
        for (int c = 0; c < NU; ++c) vp[NS + c] = (kp < N) ? W[base_u + kp * NU + c] : 0.0;
    };
    auto fdot = [&](int r, const double (&v)[NV]) -> double {
        double acc = 0.0;
#pragma unroll
        for (int c = 0; c < NV; ++c) acc += Fs[c * mpad + r] * v[c];
        return acc;
    };

    // ======================= residuals =====================================================
    // writes rs, ru, re (per stage) to LDS; returns stat, feas, comp sum, cost-gradient scale
    auto residuals = [&](double& stat, double& feas, double& csum, double& gscale) __attribute__((always_inline)) {
#pragma unroll
        for (int j = 0; j < SPL; ++j) {
            const int k = lane + WAVE * j;
            if (k <= N) {
#pragma unroll
                for (int i = 0; i < NS; ++i) { W[L.xs + k * NS + i] = s[j][i]; W[L.qt_xpi + k * NS + i] = pi[j][i]; }
#pragma unroll
                for (int i = 0; i < NU; ++i) W[L.xu + k * NU + i] = u[j][i];
            }
        }
        wave_sync();
        double st = 0, fe = 0, cs = 0, gs = 0;
        double rsl[SPL][NS], rul[SPL][NU];
#pragma unroll
        for (int j = 0; j < SPL; ++j) {
            const int k = lane + WAVE * j;
#pragma unroll
            for (int i = 0; i < NS; ++i) rsl[j][i] = 0.0;
#pragma unroll
            for (int i = 0; i < NU; ++i) rul[j][i] = 0.0;
            if (k > N) continue;
            const double* Hk = Hs + k * hstride;
            double v[NV];
#pragma unroll
            for (int i = 0; i < NS; ++i) v[i] = s[j][i];
#pragma unroll
            for (int i = 0; i < NU; ++i) v[NS + i] = (k < N) ? u[j][i] : 0.0;
            double gv[NV];
#pragma unroll
            for (int i = 0; i < NV; ++i) {
                double acc = gterm(k, i);
#pragma unroll
                for (int c = 0; c < NV; ++c) acc += Hk[i * NV + c] * v[c];
                gv[i] = acc;
                gs = fmax(gs, fabs(acc));
            }
            double pn[NS];
#pragma unroll
            for (int i = 0; i < NS; ++i) pn[i] = (k < N) ? W[L.qt_xpi + (k + 1) * NS + i] : 0.0;
#pragma unroll
            for (int i = 0; i < NS; ++i) {
                double acc = gv[i];
                if (k < N) {
#pragma unroll
                    for (int c = 0; c < NS; ++c) acc += Abar(c, i) * pn[c];
                }
                if (k > 0) acc -= pi[j][i];
                rsl[j][i] = acc;
            }
#pragma unroll
            for (int i = 0; i < NU; ++i) {
                double acc = gv[NS + i];
#pragma unroll
                for (int c = 0; c < NS; ++c) acc += Bbar(c, i) * pn[c];
                rul[j][i] = (k < N) ? acc : 0.0;
            }
#pragma unroll
            for (int i = 0; i < NX; ++i) {
                if (xpres(j, i, 0)) { rsl[j][i] += lx[j][i][0]; fe = fmax(fe, fabs(rix(j, i, 0))); cs += tx[j][i][0] * lx[j][i][0]; }
                if (xpres(j, i, 1)) { rsl[j][i] -= lx[j][i][1]; fe = fmax(fe, fabs(rix(j, i, 1))); cs += tx[j][i][1] * lx[j][i][1]; }
            }
#pragma unroll
            for (int i = 0; i < NU; ++i) {
                if (upres(j, i, 0)) { rul[j][i] += lu[j][i][0]; fe = fmax(fe, fabs(riu(j, i, 0))); cs += tu[j][i][0] * lu[j][i][0]; }
                if (upres(j, i, 1)) { rul[j][i] -= lu[j][i][1]; fe = fmax(fe, fabs(riu(j, i, 1))); cs += tu[j][i][1] * lu[j][i][1]; }
            }
            if (k < N) {
#pragma unroll
                for (int i = 0; i < NS; ++i) {
                    double acc = cb[i] - W[L.xs + (k + 1) * NS + i];
#pragma unroll
                    for (int c = 0; c < NS; ++c) acc += Abar(i, c) * s[j][c];
#pragma unroll
                    for (int c = 0; c < NU; ++c) acc += Bbar(i, c) * u[j][c];
                    W[L.re + k * NS + i] = acc;
                    fe = fmax(fe, fabs(acc));
                }
            }
        }
        // polytope rows: ri and F'lam partials
        double vp[NV];
        load_vp(vp, L.xs, L.xu);
        double gpp[NV];
#pragma unroll
        for (int c = 0; c < NV; ++c) gpp[c] = 0.0;
#pragma unroll
        for (int q = 0; q < RPL; ++q) {
            const int r = lane + WAVE * q;
            if (r < mp) {
                const double ri = fdot(r, vp) + tp[q] - hpi[r];
#pragma unroll
                for (int c = 0; c < NV; ++c) gpp[c] += Fs[c * mpad + r] * lp[q];
                fe = fmax(fe, fabs(ri));
                cs += tp[q] * lp[q];
            }
        }
#pragma unroll
        for (int c = 0; c < NV; ++c) gpp[c] = wsum(gpp[c]);
#pragma unroll
        for (int j = 0; j < SPL; ++j) {
            const int k = lane + WAVE * j;
            if (k > N) continue;
            if (k == kp) {
#pragma unroll
                for (int i = 0; i < NS; ++i) rsl[j][i] += gpp[i];
                if (kp < N) {
#pragma unroll
                    for (int i = 0; i < NU; ++i) rul[j][i] += gpp[NS + i];
                }
            }
            if (k == 0) {
#pragma unroll
                for (int i = 0; i < NX; ++i) rsl[j][i] = 0.0;
            }
#pragma unroll
            for (int i = 0; i < NS; ++i) { st = fmax(st, fabs(rsl[j][i])); W[L.rs + k * NS + i] = rsl[j][i]; }
#pragma unroll
            for (int i = 0; i < NU; ++i) { st = fmax(st, fabs(rul[j][i])); W[L.ru + k * NU + i] = rul[j][i]; }
        }
        stat = wmax(st);
        feas = wmax(fe);
        csum = wsum(cs);
        gscale = wmax(gs);
    };

    // ======================= Riccati factorisation =========================================
    // Riccati-factor lane roles: lane (ib, jb) = (lane / NS, lane % NS), ib <= jb < NS, owns
    // entry (ib, jb) of P_k.  Every lane forms the input-row quantities of ITS two columns
    // itself (g = P_{k+1} Bbar, M_u(:, ib), M_u(:, jb), Rhat, K_ib, K_jb), so the only
    // cross-lane traffic per stage is P_k itself, broadcast through the packed LDS table.
    const int ib = (lane < NS * NS) ? lane / NS : 0, jb = (lane < NS * NS) ? lane % NS : 0;
    const bool blane = lane < NS * NS && ib <= jb;
    auto factor = [&]() __attribute__((always_inline)) -> bool {
        // one reciprocal of t per row per iteration (reused by both solves and the steps)
#pragma unroll
        for (int j = 0; j < SPL; ++j) {
#pragma unroll
            for (int i = 0; i < NX; ++i) { itx[j][i][0] = 1.0 / tx[j][i][0]; itx[j][i][1] = 1.0 / tx[j][i][1]; }
#pragma unroll
            for (int i = 0; i < NU; ++i) { itu[j][i][0] = 1.0 / tu[j][i][0]; itu[j][i][1] = 1.0 / tu[j][i][1]; }
            const int k = lane + WAVE * j;
            if (k <= N) {
#pragma unroll
                for (int i = 0; i < NX; ++i) {
                    double d = 0;
                    if (xpres(j, i, 0)) d += lx[j][i][0] * itx[j][i][0];
                    if (xpres(j, i, 1)) d += lx[j][i][1] * itx[j][i][1];
                    W[L.Dx + k * NV + i] = d;
                }
#pragma unroll
                for (int i = 0; i < NU; ++i) {
                    double d = 0;
                    if (upres(j, i, 0)) d += lu[j][i][0] * itu[j][i][0];
                    if (upres(j, i, 1)) d += lu[j][i][1] * itu[j][i][1];
                    W[L.Dx + k * NV + NS + i] = d;
                }
#pragma unroll
                for (int i = NX; i < NS; ++i) W[L.Dx + k * NV + i] = 0.0;
            }
        }
        STAMP(1);
        // polytope F'DF (upper triangle), reduced over the wave
        double fd[NV * (NV + 1) / 2];
#pragma unroll
        for (int c = 0; c < NV * (NV + 1) / 2; ++c) fd[c] = 0.0;
#pragma unroll
        for (int q = 0; q < RPL; ++q) {
            itp[q] = 1.0 / tp[q];
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
        // per-lane columns ib, jb of Abar and the (uniform) Bbar, constant over the stages
        double Ai[NS], Aj[NS], Bl[NS][NU];
#pragma unroll
        for (int a_ = 0; a_ < NS; ++a_) {
            Ai[a_] = Abar(a_, ib);
            Aj[a_] = Abar(a_, jb);
#pragma unroll
            for (int x = 0; x < NU; ++x) Bl[a_][x] = Bbar(a_, x);
        }
        // Htilde entry (i, j) of stage k
        // (branch-free: every operand is loaded unconditionally and selected, so the loads of a
        // stage issue back to back and are waited for once)
        auto ht = [&](int k, int i, int j) __attribute__((always_inline)) -> double {
            const double h = Hs[k * hstride + i * NV + j];
            const double d = W[L.Dx + k * NV + i];
            const double f = W[L.FD + i * NV + j];
            return (h + (i == j ? d : 0.0)) + (k == kp ? f : 0.0);
        };
        // stage-k entries each lane needs, prefetched one stage ahead of the recursion as RAW
        // operands (cost entry, box diagonal): they are combined only when the stage is
        // processed, so the prefetch loads are not waited for inside the stage that issues them.
        // The polytope term F'DF enters at stage kp only (a uniform branch).
        struct StageH { double hij, dij, hui[NU], huj[NU], huu[NU][NU], duu[NU]; };
        auto load_h = [&](int k, StageH& sh) __attribute__((always_inline)) {
            const double* Hk = Hs + k * hstride;
            sh.hij = Hk[ib * NV + jb];
            sh.dij = W[L.Dx + k * NV + ib];
#pragma unroll
            for (int x = 0; x < NU; ++x) {
                sh.hui[x] = Hk[(NS + x) * NV + ib];
                sh.huj[x] = Hk[(NS + x) * NV + jb];
                sh.duu[x] = W[L.Dx + k * NV + NS + x];
#pragma unroll
                for (int y = 0; y < NU; ++y) sh.huu[x][y] = Hk[(NS + x) * NV + NS + y];
            }
        };
        // Htilde entries of the stage (same operation order as ht())
        auto combine_h = [&](int k, const StageH& sh, StageH& o) __attribute__((always_inline)) {
            o.hij = sh.hij + (ib == jb ? sh.dij : 0.0);
#pragma unroll
            for (int x = 0; x < NU; ++x) {
                o.hui[x] = sh.hui[x];
                o.huj[x] = sh.huj[x];
#pragma unroll
                for (int y = 0; y < NU; ++y) o.huu[x][y] = sh.huu[x][y] + (x == y ? sh.duu[x] : 0.0);
            }
            if (k == kp) {
                o.hij += W[L.FD + ib * NV + jb];
#pragma unroll
                for (int x = 0; x < NU; ++x) {
                    o.hui[x] += W[L.FD + (NS + x) * NV + ib];
                    o.huj[x] += W[L.FD + (NS + x) * NV + jb];
#pragma unroll
                    for (int y = 0; y < NU; ++y) o.huu[x][y] += W[L.FD + (NS + x) * NV + NS + y];
                }
            }
        };
        // P_k broadcast: the owning lanes store the packed upper triangle, every lane reads the
        // stage slot back (ds_read_b128, same address in all lanes)
        constexpr int PST = pk_stride(NS);
        double pu[PST];
        auto bcast_p = [&](int k) __attribute__((always_inline)) {
            wave_sync();
            const double2* src = reinterpret_cast<const double2*>(W + L.P + k * PST);
#pragma unroll
            for (int q = 0; q < PST / 2; ++q) {
                const double2 t2 = src[q];
                pu[2 * q] = t2.x;
                pu[2 * q + 1] = t2.y;
            }
        };
        auto Pm = [&](int a_, int b_) __attribute__((always_inline)) -> double { return pu[pk_idx(NS, a_, b_)]; };
        if (blane) W[L.P + N * PST + pk_idx(NS, ib, jb)] = ht(N, ib, jb);
        bcast_p(N);
        STAMP(2);
        bool ok = true;
        StageH raw, nxt, cur;
        load_h(N - 1, raw);
        for (int k = N - 1; k >= 0; --k) {
            combine_h(k, raw, cur);
            if (k > 0) load_h(k - 1, nxt);
            // g = P_{k+1} Bbar (uniform) and G_jb = P_{k+1} Abar(:, jb)
            double g[NS][NU], Gj[NS];
#pragma unroll
            for (int a_ = 0; a_ < NS; ++a_) {
                double gj = 0.0;
#pragma unroll
                for (int b = 0; b < NS; ++b) gj += Pm(a_, b) * Aj[b];
                Gj[a_] = gj;
#pragma unroll
                for (int x = 0; x < NU; ++x) {
                    double acc = 0.0;
#pragma unroll
                    for (int b = 0; b < NS; ++b) acc += Pm(a_, b) * Bl[b][x];
                    g[a_][x] = acc;
                }
            }
            // input rows of M = Ht + F' P F for columns ib, jb and Rhat = M_uu
            double mi[NU], mj[NU], Ruu[NU][NU];
#pragma unroll
            for (int x = 0; x < NU; ++x) {
                double vi = cur.hui[x], vj = cur.huj[x];
#pragma unroll
                for (int a_ = 0; a_ < NS; ++a_) { vi += g[a_][x] * Ai[a_]; vj += g[a_][x] * Aj[a_]; }
                mi[x] = vi;
                mj[x] = vj;
#pragma unroll
                for (int y = 0; y < NU; ++y) {
                    double r = cur.huu[x][y];
#pragma unroll
                    for (int a_ = 0; a_ < NS; ++a_) r += g[a_][x] * Bl[a_][y];
                    Ruu[x][y] = r;
                }
            }
            // K columns ib, jb:  K = -Rhat^{-1} M_us  (nu = 1: one reciprocal; else Cholesky)
            double Ki[NU], Kj[NU], Lf[NU * NU];
            if constexpr (NU == 1) {
                ok = ok && (Ruu[0][0] > 0.0);
                const double rinv = 1.0 / Ruu[0][0];
                Lf[0] = rinv;
                Ki[0] = -mi[0] * rinv;
                Kj[0] = -mj[0] * rinv;
            } else {
                double Lc[NU][NU];
                ok = chol_small<NU>(Ruu, Lc) && ok;
#pragma unroll
                for (int x = 0; x < NU; ++x)
#pragma unroll
                    for (int y = 0; y < NU; ++y) Lf[x * NU + y] = Lc[x][y];
#pragma unroll
                for (int x = 0; x < NU; ++x) { Ki[x] = -mi[x]; Kj[x] = -mj[x]; }
                chol_solve_small<NU>(Lf, Ki);
                chol_solve_small<NU>(Lf, Kj);
            }
            // Phi(:, ib) = Abar(:, ib) + Bbar K_ib ; T_jb = P Phi(:, jb) = G_jb + g K_jb
            double Phi_i[NS], Tj[NS];
#pragma unroll
            for (int a_ = 0; a_ < NS; ++a_) {
                double vi = Ai[a_], vt = Gj[a_];
#pragma unroll
                for (int x = 0; x < NU; ++x) { vi += Bl[a_][x] * Ki[x]; vt += g[a_][x] * Kj[x]; }
                Phi_i[a_] = vi;
                Tj[a_] = vt;
            }
            // Joseph form  P_k(ib, jb) = [I;K]' Ht [I;K] + Phi(:, ib)' P Phi(:, jb)
            double v = cur.hij;
#pragma unroll
            for (int x = 0; x < NU; ++x) {
                v += Ki[x] * cur.huj[x] + cur.hui[x] * Kj[x];
#pragma unroll
                for (int y = 0; y < NU; ++y) v += Ki[x] * cur.huu[x][y] * Kj[y];
            }
            double acc = 0.0;
#pragma unroll
            for (int a_ = 0; a_ < NS; ++a_) acc += Phi_i[a_] * Tj[a_];
            v += acc;
            // tables for the solves
            if (blane) W[L.P + k * PST + pk_idx(NS, ib, jb)] = v;
            if (lane < NS) {        // lane (0, jb): column jb of K
#pragma unroll
                for (int x = 0; x < NU; ++x) W[L.K + k * NU * NS + x * NS + jb] = Kj[x];
            }
            if (kPhi && blane && ib == jb) {   // diagonal lane (ib, ib): column ib of Phi
#pragma unroll
                for (int a_ = 0; a_ < NS; ++a_) W[L.Phi + k * NS * NS + a_ * NS + ib] = Phi_i[a_];
            }
            if (lane == 0) {
#pragma unroll
                for (int x = 0; x < NU * NU; ++x) W[L.Lr + k * NU * NU + x] = Lf[x];
            }
            bcast_p(k);
            raw = nxt;
        }
        STAMP(3);
        // factor of the theta block of P_0 (np = 1: its reciprocal)
        double Pt[NP][NP], L0[NP][NP];
#pragma unroll
        for (int x = 0; x < NP; ++x)
#pragma unroll
            for (int y = 0; y < NP; ++y) Pt[x][y] = Pm(NX + x, NX + y);
        if constexpr (NP == 1) {
            ok = ok && (Pt[0][0] > 0.0);
            L0[0][0] = 1.0 / Pt[0][0];
        } else {
            ok = chol_small<NP>(Pt, L0) && ok;
        }
        if (lane == 0) {
#pragma unroll
            for (int x = 0; x < NP; ++x)
#pragma unroll
                for (int y = 0; y < NP; ++y) W[L.L0 + x * NP + y] = L0[x][y];
        }
        wave_sync();
        return ok;
    };

    // complementarity right-hand side of a row: predictor t*lam, corrector + dt_a*dlam_a - sigma*mu
    auto rcv = [&](double t, double l, double pr, bool corr, double smu) __attribute__((always_inline)) -> double {
        return corr ? t * l + pr - smu : t * l;
    };

    // ======================= Newton solve ==================================================
    auto solve = [&](bool corr, double smu) __attribute__((always_inline)) {
        STAMP(15);
        // q = r_v + C'((lam o ri - rc)/t)
        double qs[SPL][NS], qu[SPL][NU];
#pragma unroll
        for (int j = 0; j < SPL; ++j) {
            const int k = lane + WAVE * j;
            const int kk = k <= N ? k : N;
#pragma unroll
            for (int i = 0; i < NS; ++i) qs[j][i] = W[L.rs + kk * NS + i];
#pragma unroll
            for (int i = 0; i < NU; ++i) qu[j][i] = W[L.ru + kk * NU + i];
#pragma unroll
            for (int i = 0; i < NX; ++i) {
                double e = 0.0;
                if (xpres(j, i, 0)) e += (lx[j][i][0] * rix(j, i, 0) - rcv(tx[j][i][0], lx[j][i][0], prx[j][i][0], corr, smu)) * itx[j][i][0];
                if (xpres(j, i, 1)) e -= (lx[j][i][1] * rix(j, i, 1) - rcv(tx[j][i][1], lx[j][i][1], prx[j][i][1], corr, smu)) * itx[j][i][1];
                qs[j][i] += e;
            }
#pragma unroll
            for (int i = 0; i < NU; ++i) {
                double e = qu[j][i];
                if (upres(j, i, 0)) e += (lu[j][i][0] * riu(j, i, 0) - rcv(tu[j][i][0], lu[j][i][0], pru[j][i][0], corr, smu)) * itu[j][i][0];
                if (upres(j, i, 1)) e -= (lu[j][i][1] * riu(j, i, 1) - rcv(tu[j][i][1], lu[j][i][1], pru[j][i][1], corr, smu)) * itu[j][i][1];
                qu[j][i] = e;
            }
        }
        {
            double vp[NV];
            load_vp(vp, L.xs, L.xu);
            double gpp[NV];
#pragma unroll
            for (int c = 0; c < NV; ++c) gpp[c] = 0.0;
#pragma unroll
            for (int q = 0; q < RPL; ++q) {
                const int r = lane + WAVE * q;
                if (r < mp) {
                    const double ri = fdot(r, vp) + tp[q] - hpi[r];
                    const double pr = corr ? W[L.prp + r] : 0.0;
                    const double e = (lp[q] * ri - rcv(tp[q], lp[q], pr, corr, smu)) * itp[q];
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
        STAMP(4);
        // pre-pass: wv_k = P_{k+1} re_k, qt_k = qs_k + K_k' qu_k, qh_k = qt_k + Phi_k' wv_k ;
        // p_N = qs_N.  qh carries everything of the backward recursion that does not depend on
        // p_{k+1}, so the sequential sweep is one NS x NS mat-vec per stage.
#pragma unroll
        for (int j = 0; j < SPL; ++j) {
            const int k = lane + WAVE * j;
            if (k < N) {
                const double* Pn = W + L.P + (k + 1) * pk_stride(NS);
                const double* Kk = W + L.K + k * NU * NS;
                double rek[NS], wk[NS], qtk[NS];
#pragma unroll
                for (int c = 0; c < NS; ++c) rek[c] = W[L.re + k * NS + c];
#pragma unroll
                for (int i = 0; i < NS; ++i) {
                    double v = 0.0;
#pragma unroll
                    for (int c = 0; c < NS; ++c) v += Pn[pk_idx(NS, i, c)] * rek[c];
                    wk[i] = v;
                    W[L.wv + k * NS + i] = v;
                    double qq = qs[j][i];
#pragma unroll
                    for (int x = 0; x < NU; ++x) qq += Kk[x * NS + i] * qu[j][x];
                    qtk[i] = qq;
                }
                if constexpr (kPhi) {
                    const double* Ph = W + L.Phi + k * NS * NS;
#pragma unroll
                    for (int i = 0; i < NS; ++i) {
                        double v = qtk[i];
#pragma unroll
                        for (int c = 0; c < NS; ++c) v += Ph[c * NS + i] * wk[c];
                        W[L.qt_xpi + k * NS + i] = v;
                    }
                } else {
                    double bw[NU];
#pragma unroll
                    for (int x = 0; x < NU; ++x) {
                        double v = 0.0;
#pragma unroll
                        for (int c = 0; c < NS; ++c) v += Bbar(c, x) * wk[c];
                        bw[x] = v;
                    }
#pragma unroll
                    for (int i = 0; i < NS; ++i) {
                        double v = qtk[i];
#pragma unroll
                        for (int c = 0; c < NS; ++c) v += Abar(c, i) * wk[c];
#pragma unroll
                        for (int x = 0; x < NU; ++x) v += Kk[x * NS + i] * bw[x];
                        W[L.qt_xpi + k * NS + i] = v;
                    }
                }
#pragma unroll
                for (int x = 0; x < NU; ++x) W[L.qu + k * NU + x] = qu[j][x];
            } else if (k == N) {
#pragma unroll
                for (int i = 0; i < NS; ++i) W[L.pv + N * NS + i] = qs[j][i];
            }
        }
        wave_sync();
        STAMP(5);
        // backward sweep: lane i < NS computes entry i of p_k = Phi_k' p_{k+1} + qh_k; the new
        // vector is broadcast with readlane (scalar registers), stage data prefetched a stage ahead
        {
            const int li = lane < NS ? lane : NS - 1;
            double p[NS];
#pragma unroll
            for (int i = 0; i < NS; ++i) p[i] = W[L.pv + N * NS + i];
            auto load_b = [&](int k, double (&col)[NS], double& q) __attribute__((always_inline)) {
                q = W[L.qt_xpi + k * NS + li];
                if constexpr (kPhi) {
#pragma unroll
                    for (int c = 0; c < NS; ++c) col[c] = W[L.Phi + k * NS * NS + c * NS + li];
                } else {
#pragma unroll
                    for (int c = 0; c < NS; ++c) {
                        double v = Abar(c, li);
#pragma unroll
                        for (int x = 0; x < NU; ++x) v += Bbar(c, x) * W[L.K + k * NU * NS + x * NS + li];
                        col[c] = v;
                    }
                }
            };
            // two register sets used alternately (stages k, k-1), each refilled two stages ahead
            double c0[NS], q0, c1[NS], q1;
            load_b(N - 1, c0, q0);
            if (N >= 2) load_b(N - 2, c1, q1);
            auto step_b = [&](int k, const double (&col)[NS], double q) __attribute__((always_inline)) {
                double acc = q;
#pragma unroll
                for (int c = 0; c < NS; ++c) acc += col[c] * p[c];
                if (lane < NS) W[L.pv + k * NS + lane] = acc;
#pragma unroll
                for (int c = 0; c < NS; ++c) p[c] = rl(acc, c);
            };
            for (int k = N - 1; k >= 0; k -= 2) {
                step_b(k, c0, q0);
                if (k >= 2) load_b(k - 2, c0, q0);
                if (k == 0) break;
                step_b(k - 1, c1, q1);
                if (k >= 3) load_b(k - 3, c1, q1);
            }
        }
        wave_sync();
        STAMP(6);
        // post-backward: kff_k = -Rhat^{-1}(qu_k + Bbar'(p_{k+1} + w_k)); f_k = Bbar kff_k + re_k
#pragma unroll
        for (int j = 0; j < SPL; ++j) {
            const int k = lane + WAVE * j;
            if (k < N) {
                double y[NS], r[NU];
#pragma unroll
                for (int i = 0; i < NS; ++i) y[i] = W[L.pv + (k + 1) * NS + i] + W[L.wv + k * NS + i];
#pragma unroll
                for (int x = 0; x < NU; ++x) {
                    double v = qu[j][x];
#pragma unroll
                    for (int c = 0; c < NS; ++c) v += Bbar(c, x) * y[c];
                    r[x] = -v;
                }
                chol_solve_small<NU>(W + L.Lr + k * NU * NU, r);
#pragma unroll
                for (int x = 0; x < NU; ++x) kff[j][x] = r[x];
#pragma unroll
                for (int i = 0; i < NS; ++i) {
                    double v = W[L.re + k * NS + i];
#pragma unroll
                    for (int x = 0; x < NU; ++x) v += Bbar(i, x) * kff[j][x];
                    W[L.fv + k * NS + i] = v;
                }
            }
        }
        wave_sync();
        STAMP(7);
        // theta_0 step + forward sweep: lane i < NS computes entry i of ds_{k+1} = Phi_k ds_k + f_k
        {
            double d[NS];
#pragma unroll
            for (int i = 0; i < NX; ++i) d[i] = 0.0;
            double r0[NP];
#pragma unroll
            for (int x = 0; x < NP; ++x) r0[x] = -W[L.pv + NX + x];
            chol_solve_small<NP>(W + L.L0, r0);
#pragma unroll
            for (int x = 0; x < NP; ++x) d[NX + x] = r0[x];
            if (lane == 0) {
#pragma unroll
                for (int i = 0; i < NS; ++i) W[L.dsv + i] = d[i];
            }
            const int li = lane < NS ? lane : NS - 1;
            auto load_f = [&](int k, double (&row)[NS], double& f) __attribute__((always_inline)) {
                f = W[L.fv + k * NS + li];
                if constexpr (kPhi) {
#pragma unroll
                    for (int c = 0; c < NS; ++c) row[c] = W[L.Phi + k * NS * NS + li * NS + c];
                } else {
#pragma unroll
                    for (int c = 0; c < NS; ++c) {
                        double v = Abar(li, c);
#pragma unroll
                        for (int x = 0; x < NU; ++x) v += Bbar(li, x) * W[L.K + k * NU * NS + x * NS + c];
                        row[c] = v;
                    }
                }
            };
            double r0_[NS], f0, r1_[NS], f1;
            load_f(0, r0_, f0);
            if (N >= 2) load_f(1, r1_, f1);
            auto step_f = [&](int k, const double (&row)[NS], double f) __attribute__((always_inline)) {
                double acc = f;
#pragma unroll
                for (int c = 0; c < NS; ++c) acc += row[c] * d[c];
                if (lane < NS) W[L.dsv + (k + 1) * NS + lane] = acc;
#pragma unroll
                for (int c = 0; c < NS; ++c) d[c] = rl(acc, c);
            };
            for (int k = 0; k < N; k += 2) {
                step_f(k, r0_, f0);
                if (k + 2 < N) load_f(k + 2, r0_, f0);
                if (k + 1 >= N) break;
                step_f(k + 1, r1_, f1);
                if (k + 3 < N) load_f(k + 3, r1_, f1);
            }
        }
        wave_sync();
        STAMP(8);
        // post-forward: du_k = K_k ds_k + kff_k
#pragma unroll
        for (int j = 0; j < SPL; ++j) {
            const int k = lane + WAVE * j;
            if (k < N) {
                const double* Kk = W + L.K + k * NU * NS;
#pragma unroll
                for (int x = 0; x < NU; ++x) {
                    double v = kff[j][x];
#pragma unroll
                    for (int c = 0; c < NS; ++c) v += Kk[x * NS + c] * W[L.dsv + k * NS + c];
                    W[L.duv + k * NU + x] = v;
                }
            } else if (k == N) {
#pragma unroll
                for (int x = 0; x < NU; ++x) W[L.duv + N * NU + x] = 0.0;
            }
        }
        wave_sync();
    };

    // ======================= row passes over the step (dt, dlam recomputed) ================
    // mode 0: max ratio (returns max of -dt/t, -dlam/lam); mode 1: comp sum after alpha and
    // store predictor products; mode 2: apply the step alpha to t, lam.
    auto row_pass = [&](int mode, bool corr, double smu, double al) __attribute__((always_inline)) -> double {
        double acc = 0.0;
#pragma unroll
        for (int j = 0; j < SPL; ++j) {
            const int k = lane + WAVE * j;
            if (k > N) continue;
            double dsk[NS], duk[NU];
#pragma unroll
            for (int i = 0; i < NS; ++i) dsk[i] = W[L.dsv + k * NS + i];
#pragma unroll
            for (int i = 0; i < NU; ++i) duk[i] = W[L.duv + k * NU + i];
#pragma unroll
            for (int i = 0; i < NX; ++i)
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    if (!xpres(j, i, h)) continue;
                    const double rc = rcv(tx[j][i][h], lx[j][i][h], prx[j][i][h], corr, smu);
                    const double dt = -rix(j, i, h) - (h == 0 ? dsk[i] : -dsk[i]);
                    const double dl = (-rc - lx[j][i][h] * dt) * itx[j][i][h];
                    if (mode == 0) {
                        acc = fmax(acc, -dt * itx[j][i][h]);
                        acc = fmax(acc, -dl / lx[j][i][h]);
                    } else if (mode == 1) {
                        acc += (tx[j][i][h] + al * dt) * (lx[j][i][h] + al * dl);
                        prx[j][i][h] = dt * dl;
                    } else {
                        tx[j][i][h] += al * dt;
                        lx[j][i][h] += al * dl;
                    }
                }
#pragma unroll
            for (int i = 0; i < NU; ++i)
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    if (!upres(j, i, h)) continue;
                    const double rc = rcv(tu[j][i][h], lu[j][i][h], pru[j][i][h], corr, smu);
                    const double dt = -riu(j, i, h) - (h == 0 ? duk[i] : -duk[i]);
                    const double dl = (-rc - lu[j][i][h] * dt) * itu[j][i][h];
                    if (mode == 0) {
                        acc = fmax(acc, -dt * itu[j][i][h]);
                        acc = fmax(acc, -dl / lu[j][i][h]);
                    } else if (mode == 1) {
                        acc += (tu[j][i][h] + al * dt) * (lu[j][i][h] + al * dl);
                        pru[j][i][h] = dt * dl;
                    } else {
                        tu[j][i][h] += al * dt;
                        lu[j][i][h] += al * dl;
                    }
                }
        }
        double vp[NV], dvp[NV];
        load_vp(vp, L.xs, L.xu);
        load_vp(dvp, L.dsv, L.duv);
#pragma unroll
        for (int q = 0; q < RPL; ++q) {
            const int r = lane + WAVE * q;
            if (r >= mp) continue;
            const double ri = fdot(r, vp) + tp[q] - hpi[r];
            const double pr = corr ? W[L.prp + r] : 0.0;
            const double rc = rcv(tp[q], lp[q], pr, corr, smu);
            const double dt = -ri - fdot(r, dvp);
            const double dl = (-rc - lp[q] * dt) * itp[q];
            if (mode == 0) {
                acc = fmax(acc, -dt * itp[q]);
                acc = fmax(acc, -dl / lp[q]);
            } else if (mode == 1) {
                acc += (tp[q] + al * dt) * (lp[q] + al * dl);
                W[L.prp + r] = dt * dl;
            } else {
                tp[q] += al * dt;
                lp[q] += al * dl;
            }
        }
        if (mode == 0) return wmax(acc);
        if (mode == 1) return wsum(acc);
        return 0.0;
    };
    auto step_len = [&](bool corr, double smu) __attribute__((always_inline)) -> double {
        const double rm = row_pass(0, corr, smu, 0.0);
        return rm > 1.0 ? 1.0 / rm : 1.0;
    };
    // primal/dual stage update by alpha (dpi_k = P_k ds_k + p_k)
    auto update_stage = [&](double al) __attribute__((always_inline)) {
#pragma unroll
        for (int j = 0; j < SPL; ++j) {
            const int k = lane + WAVE * j;
            if (k > N) continue;
            double dsk[NS];
#pragma unroll
            for (int i = 0; i < NS; ++i) dsk[i] = W[L.dsv + k * NS + i];
            if (k >= 1) {
                const double* Pk = W + L.P + k * pk_stride(NS);
#pragma unroll
                for (int i = 0; i < NS; ++i) {
                    double v = W[L.pv + k * NS + i];
#pragma unroll
                    for (int c = 0; c < NS; ++c) v += Pk[pk_idx(NS, i, c)] * dsk[c];
                    pi[j][i] += al * v;
                }
            }
#pragma unroll
            for (int i = 0; i < NS; ++i) s[j][i] += al * dsk[i];
            if (k < N) {
#pragma unroll
                for (int i = 0; i < NU; ++i) u[j][i] += al * W[L.duv + k * NU + i];
            }
        }
    };

    // ======================= initial point ==================================================
#pragma unroll
    for (int j = 0; j < SPL; ++j) {
#pragma unroll
        for (int i = 0; i < NX; ++i)
#pragma unroll
            for (int h = 0; h < 2; ++h) { tx[j][i][h] = 1.0; lx[j][i][h] = 1.0; prx[j][i][h] = 0.0; }
#pragma unroll
        for (int i = 0; i < NU; ++i)
#pragma unroll
            for (int h = 0; h < 2; ++h) { tu[j][i][h] = 1.0; lu[j][i][h] = 1.0; pru[j][i][h] = 0.0; }
    }
#pragma unroll
    for (int q = 0; q < RPL; ++q) { tp[q] = 1.0; lp[q] = 1.0; }
    double stat = 0, feas = 0, csum = 0, gscale = 0;
    residuals(stat, feas, csum, gscale);
    int flag = 0;
    if (!factor()) flag = -8;
    solve(false, 0.0);
    {
        // tt = t + dt (t = 1) at the unit-scaled least-squares point; lam~ = -tt; shift
        double tmin = INFINITY, tmax = -INFINITY;
        row_pass(2, false, 0.0, 1.0);      // t <- 1 + dt (lam is reset below)
#pragma unroll
        for (int j = 0; j < SPL; ++j) {
#pragma unroll
            for (int i = 0; i < NX; ++i)
#pragma unroll
                for (int h = 0; h < 2; ++h)
                    if (xpres(j, i, h)) { tmin = fmin(tmin, tx[j][i][h]); tmax = fmax(tmax, tx[j][i][h]); }
#pragma unroll
            for (int i = 0; i < NU; ++i)
#pragma unroll
                for (int h = 0; h < 2; ++h)
                    if (upres(j, i, h)) { tmin = fmin(tmin, tu[j][i][h]); tmax = fmax(tmax, tu[j][i][h]); }
        }
#pragma unroll
        for (int q = 0; q < RPL; ++q)
            if (prow(q)) { tmin = fmin(tmin, tp[q]); tmax = fmax(tmax, tp[q]); }
        update_stage(1.0);
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
                    const double t = tx[j][i][h];
                    const bool pr = xpres(j, i, h);
                    tx[j][i][h] = pr ? t + shp : 1.0;
                    lx[j][i][h] = pr ? -t + shd : 0.0;
                }
#pragma unroll
            for (int i = 0; i < NU; ++i)
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const double t = tu[j][i][h];
                    const bool pr = upres(j, i, h);
                    tu[j][i][h] = pr ? t + shp : 1.0;
                    lu[j][i][h] = pr ? -t + shd : 0.0;
                }
        }
#pragma unroll
        for (int q = 0; q < RPL; ++q) {
            const double t = tp[q];
            const bool pr = prow(q);
            tp[q] = pr ? t + shp : 1.0;
            lp[q] = pr ? -t + shd : 0.0;
        }
    }

    // ======================= main loop ======================================================
    int it = 0;
    double mu = 0.0, mu_min = INFINITY;
    const int max_iter = a.max_iter;
    if (flag == 0) {
        for (it = 0; it <= max_iter; ++it) {
            STAMP(14);
            residuals(stat, feas, csum, gscale);
            STAMP(0);
            mu = csum * minv;
            if (stat <= a.tol_stat * (1.0 + gscale) && feas <= a.tol_feas * (1.0 + bscale) &&
                mu <= a.tol_comp) { flag = 1; break; }
            if (!(isfinite(stat) && isfinite(feas) && isfinite(mu))) { flag = -8; break; }
            if (mu > MU_BLOWUP * mu_min && feas > 1e-6 * (1.0 + bscale)) { flag = -2; break; }
            mu_min = fmin(mu_min, mu);
            if (it == max_iter) break;
            if (!factor()) { flag = -8; break; }
            solve(false, 0.0);                                  // predictor
            STAMP(9);
            const double al_aff = step_len(false, 0.0);
            STAMP(10);
            const double mua = row_pass(1, false, 0.0, al_aff) * minv;
            STAMP(11);
            double sg = mua / mu;
            sg = sg * sg * sg;
            const double smu = sg * mu;
            solve(true, smu);                                   // corrector
            STAMP(9);
            double al = step_len(true, smu) * a.tau;
            STAMP(10);
            if (al > 1.0) al = 1.0;
            row_pass(2, true, smu, al);
            STAMP(12);
            update_stage(al);
            STAMP(13);
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
            fv += v[i] * (0.5 * hv + gterm(k, i));
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
#ifdef BQP_STAMPS
    if (lane == 0 && a.stamps) {
#pragma unroll
        for (int i = 0; i < 16; ++i) a.stamps[(int64_t)inst * 16 + i] = (double)st_acc[i];
    }
#endif
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
int ocp_wave_lds_doubles(int N, int nx, int nu, int np, int mpad) {
    return WaveLds::make(N, nx, nu, np, mpad, N + 1 <= 64).total;
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
    const size_t lds = sizeof(double) * ((size_t)a.shared_doubles +
                                         (size_t)a.wpb * ocp_wave_lds_doubles(a.N, nx, nu, np, a.mpad));
#ifdef BQP_ISA_ONLY_MG10
    // codegen inspection build (make isa): the MG N<64, 616-row instance only
    if (nx == 4 && nu == 1 && np == 1 && spl == 1 && rpl == 10) return launch_t<4, 1, 1, 1, 10>(a, blocks, lds, st);
    return hipErrorInvalidValue;
#else
    if (nx == 4 && nu == 1 && np == 1) return launch_spl<4, 1, 1>(a, spl, rpl, blocks, lds, st);
    if (nx == 2 && nu == 2 && np == 2) return launch_spl<2, 2, 2>(a, spl, rpl, blocks, lds, st);
#endif
    return hipErrorInvalidValue;
}

}  // namespace bqp
