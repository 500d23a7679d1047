// bqp_ocp.hip — batched structured Mehrotra predictor-corrector IPM for MPC QPs, gfx950.
//
// Two wavefronts solve one MPC instance; a workgroup holds QPB instances (2*QPB waves) that
// share the stage-cost table H_k and the polytope (terminal-set) matrix in LDS.
//
//   stage wave  lane k (and k+64 when SPL=2) owns stage k: s_k=[x_k;theta], u_k, pi_k.  It
//               forms the stage residuals, runs the backward Riccati factorisation (lane (i,j)
//               owns entry (i,j) of P_k, Joseph form) and the two Newton solves (closed-loop
//               sweeps, readlane broadcast), and applies the primal/dual step.
//   row wave    owns every inequality row: the box rows of stage k in lane k, and polytope rows
//               l, l+64, ... (RPL per lane).  It forms the row residuals, the diagonal weights
//               D = lam/t and F'DF, the complementarity right-hand sides, the step-length ratio
//               tests, mu_aff / sigma, and the slack/multiplier updates.
//
// The waves exchange per-stage tables and scalars through the instance's LDS slot and meet at
// six workgroup barriers per iteration (B0, B2..B6 below; I0..I3 for the starting point); both waves take the same decisions
// from the same exchanged values, so the barrier sequence is identical and an instance whose
// iteration ends leaves the loop on both waves at the same barrier (terminated waves drop out
// of s_barrier).  Each wave keeps only its own state in registers, and the row work that does
// not depend on the factorisation (F'DF, the predictor right-hand side) overlaps the stage
// wave's Riccati recursion.
//
// The algorithm (and its operation order) is stated in oracle/ocp_ipm.py and restated in C in
// oracle/cpu_ipm.c; the QP is the stage-wise form of the reference's per-step OCPs
// (costLMPC.m / constraintsLMPC.m, DMS_tracking_LMPC_casadi.m:223-287, trackingMPC/costFunction.m).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>

#include "bqp_internal.h"
#include "bqp_wave.h"

namespace bqp {

// One source, two instantiations: fp64 (this file) and fp32 (bqp_ocp_f32.hip defines BQP_F32 and
// includes this file).  The element type of the solver's LDS state and arithmetic is `real`;
// the caller's arrays in HBM stay fp64 (converted on load/store).  Each precision lives in its own
// inner namespace so the two template instantiations never merge at link time.
#ifdef BQP_F32
typedef float real;
typedef float2 real2;
#define BQP_SFX _f32
namespace sp {
#else
typedef double real;
typedef double2 real2;
#define BQP_SFX
namespace dp {
#endif
#define BQP_CAT2(a, b) a##b
#define BQP_CAT(a, b) BQP_CAT2(a, b)

#define WAVE 64
// the long-horizon LDS layout (QpLds lng) is used by the fp64 instantiation only: the fp32 one
// already fits two long-horizon instances per workgroup in the plain layout
#ifdef BQP_F32
#define BQP_LNG_OK 0
#else
#define BQP_LNG_OK 1
#endif
#ifdef BQP_F32
#define PIV_FLOOR 1e-7
#else
#define PIV_FLOOR 1e-14
#endif
#define MU_BLOWUP 1e6
// round 3 safeguards (oracle/cpu_ipm.c states the same rules):
//   -2 only while the rows are still infeasible above FEAS_GUARD (1 + |data|) (was 1e-6: nearly
//   infeasible Monte-Carlo models ended 0 after 50 iterations);
//   convergence needs every row's t lam <= CMAX_K tol_comp besides the average mu;
//   a predictor step below SOC_ALPHA on a feasible iterate drops the corrector's second-order
//   term (pure centring: the alternating stall of nearly degenerate rows);
//   the active-set polish (fp64 only) after a 0 / -8 exit (bqp_options.polish 2: also with a
//   weakly active row).
#ifdef BQP_F32
#define FEAS_GUARD 1e-6
#define BQP_POLISH 0
#else
#define FEAS_GUARD 1e-8
#define BQP_POLISH 1
#endif
#ifndef BQP_EXP_NOROW
#define BQP_EXP_NOROW 0
#endif
#ifndef BQP_EXP_NOSTAGE
#define BQP_EXP_NOSTAGE 0
#endif
#define TAU_FAST_AFF 0.99
#define TAU_FAST_MU 1e-6
#define TAU_FAST 0.99999
#define TAU_FAST_END 0.99999
#define TAU_FAST_MIN 0.995   // the fast rule applies at tau >= the default only
#define CMAX_K 100.0
#define SOC_ALPHA 0.1
#define DEG_POLISH 1e-10
#define POL_RHO 2e6
#define POL_ROUNDS 8
#define POL_PASS 3
#define POL_CG 40
#define POL_CG_SING 1e-2
#define POL_STAG 0.5

// Cholesky (lower, NxN with N <= 2) with static pivot floor; returns false if not PD.
// 1/t for the row slacks and multipliers (t > 0 inside the IPM): hardware reciprocal estimate
// refined by two Newton steps (|error| ~ 1 ulp); recomputed at every use instead of kept in
// registers (the row wave's register budget at two waves per SIMD)
__device__ __forceinline__ double frcp(double t) {
    double r = __builtin_amdgcn_rcp(t);
    double e = __builtin_fma(-t, r, 1.0);
    r = __builtin_fma(r, e, r);
    e = __builtin_fma(-t, r, 1.0);
    return __builtin_fma(r, e, r);
}
__device__ __forceinline__ float frcp(float t) {
    float r = __builtin_amdgcn_rcpf(t);
    return __builtin_fmaf(r, __builtin_fmaf(-t, r, 1.0f), r);
}

// the lane index made opaque where a phase starts: the per-lane LDS addresses of the phase are
// formed inside it instead of being hoisted to the kernel start and carried through the
// iteration loop in registers (dozens of them: the stage wave's scratch spills)
__device__ __forceinline__ int opq(int v) {
    asm volatile("" : "+v"(v));
    return v;
}
// the same for a wave-uniform value (kept in a scalar register)
__device__ __forceinline__ int opq_s(int v) {
    asm volatile("" : "+s"(v));
    return v;
}

// fused multiply-add in the instantiation's precision (no promotion of the fp32 path to fp64)
__device__ __forceinline__ double fmar(double a, double b, double c) { return __builtin_fma(a, b, c); }
__device__ __forceinline__ float fmar(float a, float b, float c) { return __builtin_fmaf(a, b, c); }

// Factor of a small SPD block for chol_solve_small (R^_k = M_uu per stage in the Riccati
// recursion, P_0[theta, theta] once per factorisation).  n = 2 (the DI model family): LDL' with
// the reciprocal pivots stored, L row-major = [1/d0, 0, l10, 1/d1] (round 6): no square root and
// two divisions on the recursion's per-stage chain instead of two square roots and five divisions
// (the DI factor was 40 % of the stage wave's cycles, profiles/stamps_C3.json); still a
// factorisation applied by substitution (oracle/cpu_ipm.c spd_fac / spd_solve, same operations),
// with the same static pivot floor on the same pivots d0 = M00, d1 = M11 - M10^2 / M00.
template <int N>
__device__ __forceinline__ bool chol_small(const real (&M)[N][N], real (&L)[N][N]) {
    bool ok = true;
    real d0 = M[0][0];
    if (!(d0 > PIV_FLOOR * M[0][0])) d0 = PIV_FLOOR * M[0][0];
    ok = ok && (d0 > 0.0);
    if constexpr (N == 2) {
        // reciprocals by frcp (estimate + two Newton steps, as the n = 1 path): the IEEE division's
        // scale / fixup sequence was twice as long on the chain
        const real r0 = frcp(d0);
        const real l10 = M[1][0] * r0;
        real d1 = M[1][1] - l10 * M[1][0];
        if (!(d1 > PIV_FLOOR * M[1][1])) d1 = PIV_FLOOR * M[1][1];
        ok = ok && (d1 > 0.0);
        L[0][0] = r0;
        L[0][1] = 0.0;
        L[1][0] = l10;
        L[1][1] = frcp(d1);
    } else {
        L[0][0] = sqrt(d0);
    }
    return ok;
}
// b <- M^{-1} b from chol_small's factor (n = 2: L z = b, D w = z, L' x = w; same order as
// oracle/cpu_ipm.c spd_solve); L row-major.  For n = 1 the factor slot holds 1/M instead (one
// reciprocal, no square root).
template <int N>
__device__ __forceinline__ void chol_solve_small(const real* L, real (&b)[N]) {
    if constexpr (N == 2) {
        const real w1 = (b[1] - L[2] * b[0]) * L[3];
        b[0] = b[0] * L[0] - L[2] * w1;
        b[1] = w1;
    } else {
        b[0] = b[0] * L[0];
    }
}

// Packed upper-triangular storage of the symmetric NS x NS Riccati matrices P_k: entry (i, j),
// i <= j, at pk_idx(i, j); each stage slot is padded to an even number of doubles so that a
// slot starts 16-byte aligned and is read back with ds_read_b128.
// The stride is also chosen against LDS bank conflicts: lane k reads stage k's slot in the
// solve pre-pass and the dual update, and ds_read_b64 banks are (a/4) mod 64 over 32-lane
// halves, so a slot of 16 doubles (32 dwords) puts every lane on two banks (16-way); an even
// stride that is 2 mod 4 doubles costs 2-way at most.
__host__ __device__ constexpr int pk_len(int NS) { return NS * (NS + 1) / 2; }
__host__ __device__ constexpr int pk_stride(int NS) {
    return (((pk_len(NS) + 1) & ~1) % 4 == 0) ? ((pk_len(NS) + 1) & ~1) + 2 : ((pk_len(NS) + 1) & ~1);
}
__host__ __device__ constexpr int pk_idx(int NS, int i, int j) {
    return i <= j ? i * NS - i * (i - 1) / 2 + (j - i) : j * NS - j * (j - 1) / 2 + (i - j);
}

// Exchange scalars between the two waves of an instance (slots of the LDS xch block).
enum : int {
    X_CNT = 0,   // number of inequality rows (row wave, once)
    X_BSR,       // max |finite bound| over the rows (row wave, once)
    X_FEASB,     // max |row residual| (row wave, per iteration)
    X_CS,        // sum t.lam over the rows (row wave, per iteration)
    X_STOP,      // 1: leave the loop at B2 (stage wave)
    X_ALPHA,     // corrector step length (row wave)
    X_CMAX,      // max t.lam over the rows (row wave, per iteration)
    X_FEASOK,    // 1: the iterate is primal feasible to FEAS_GUARD (stage wave, per iteration)
    X_FLAG,      // exit flag of the IPM (stage wave, at the stop)
    X_RHO,       // polish weight rho (stage wave, at the stop)
    X_TF,        // polish feasibility tolerance 1e-12 (1 + |data|) (stage wave)
    X_DEG,       // max over rows of min(t, lam) at the exit (row wave)
    X_PVA,       // polish: max |C v - b| over the active rows (row wave)
    X_PVIOL,     //         max (C v - b) over all rows
    X_PLNEG,     //         min multiplier over the active rows
    X_PLMX,      //         max multiplier over the active rows
    X_PCHG,      //         rows an active-set correction would move
    X_PDEC,      //         decision (stage wave): 0 pass, 1 accept, 2 correct the set, 3 give up
    X_CGD,       //         inner step (row wave): 0 CG step, 1 multiplier (AL) step, 2 pass done
    X_NXCH = 20
};
// persistent launch (ocp_queue_kernel, never the repair kernel): the slot's next instance, taken
// by the row wave (int bits; two words used alternately by successive instances of the slot) in
// two polish-only slots
constexpr int X_NEXT = X_PVA;
static_assert(X_PVIOL == X_PVA + 1, "X_NEXT + 1 must be a polish-only slot");

// Per-instance LDS layout (in doubles), sized from N at run time.
struct QpLds {
    int P, K, Lr, L0, AB, xs, xu, qt_xpi, rs, ru, re, pv, wv, bw, qu, fv, dsv, duv, dsc, duc, Dx, FD,
        blam, ebox, bnd, gpp, gpe, prp, hp, rp, xch, Fi, Hi, total;
    // fpi: the instance carries its own polytope matrix (bqp_ocp_data.sFp != 0), NV x mpad.
    // lng: long-horizon layout (N + 1 > 64, two instances per workgroup at fp64 N = 100): the
    // Riccati P_k live in global scratch (an LDS ring of two stages feeds the recursion), the
    // forward drift f_k shares the qhat_k slot, the dynamics residual re_k is recomputed from the
    // iterate where it is used, box multipliers and right-hand-side terms are stored per box
    // variable ([upper] - [lower]), and the polytope right-hand side and box bounds sit in the
    // shared tables when the batch shares them (hpsh, bndsh).  The polytope rhs is in the
    // shared tables whenever the batch shares it (hpsh, every horizon).
    // hinst: per-instance stage-cost table (bqp_ocp_data.sW != 0) in the slot (short horizons)
    __host__ __device__ __forceinline__ static QpLds make(int N, int NX, int NU, int NP, int mpad, bool fpi = false,
                                          bool lng = false, bool hpsh = false, bool bndsh = false,
                                          bool hinst = false) {
        const int NS = NX + NP, NV = NS + NU, NB = NX + NU;
        QpLds o;
        int c = 0;
        o.P = c;      c += (lng ? 2 : N + 1) * pk_stride(NS);  // Riccati P_k (packed; lng: ring)
        o.K = c;      c += N * NU * NS;              // feedback K_k (row-major NU x NS)
        o.Lr = c;     c += N * NU * NU;              // factor of Rhat_k (nu = 1: its reciprocal)
        o.L0 = c;     c += NP * NP;                  // factor of P_0[theta, theta]
        o.AB = c;     c += NS * NS + NS * NU + NS;   // Abar (row-major), Bbar, cbar
        o.xs = c;     c += (N + 1) * NS;             // s_k
        o.xu = c;     c += (N + 1) * NU;             // u_k (u_N = 0)
        o.qt_xpi = c; c += (N + 1) * NS;             // pi_k in the residuals, qhat_k in the solves
        o.rs = c;     c += (N + 1) * NS;             // stationarity residual (s part)
        o.ru = c;     c += (N + 1) * NU;             // stationarity residual (u part)
        o.re = c;     c += lng ? 0 : (N + 1) * NS;   // dynamics residual (lng: recomputed at use)
        o.pv = c;     c += (N + 1) * NS;             // p_k of the backward sweep
        o.wv = c;     c += (N + 1) * NS;             // cw_k = Phi_k' P_{k+1} re_k (prep_iter)
        o.bw = c;     c += (N + 1) * NU;             // Bbar' P_{k+1} re_k
        o.qu = c;     c += (N + 1) * NU;             // u right-hand side
        if (lng) {
            o.fv = o.qt_xpi;                         // f_k written after the backward sweep
        } else {
            o.fv = c; c += (N + 1) * NS;             // forward-sweep drift f_k
        }
        o.dsv = c;    c += (N + 1) * NS;             // predictor direction (s)
        o.duv = c;    c += (N + 1) * NU;             //                     (u)
        o.dsc = c;    c += (N + 1) * NS;             // corrector direction (s)
        o.duc = c;    c += (N + 1) * NU;             //                     (u)
        o.Dx = c;     c += (N + 1) * NV;             // box diagonal of stage k (internal order, theta 0)
        o.FD = c;     c += NV * NV;                  // polytope F'DF
        o.blam = c;   c += (N + 1) * NB * (lng ? 1 : 2);   // box multipliers [upper, lower] (0 if absent)
        o.ebox = c;   c += (N + 1) * NB * (lng ? 1 : 2);   // box right-hand-side terms [upper, lower]
        o.bnd = c;    c += bndsh ? 0 : (N + 1) * NB * 2;   // box bounds [upper, lower]
        o.gpp = c;    c += NV;                       // Fp' lam
        o.gpe = c;    c += NV;                       // Fp' e
        o.prp = c;    c += mpad;                     // predictor dt*dlam of the polytope rows
        o.hp = c;     c += hpsh ? 0 : mpad;          // polytope right-hand side (hpsh: shared)
        // polytope row residuals of the row wave (short horizons; the long-horizon kernels keep
        // them in registers: 5 KB more per instance would leave one instance per workgroup)
        o.rp = c;     c += lng ? 0 : mpad;
        o.xch = c;    c += X_NXCH;
        o.Fi = c;     c += fpi ? NV * mpad : 0;      // per-instance polytope (column-major)
        o.Hi = c;     c += (hinst && !lng) ? (N + 1) * (NV * NV + 1) : 0;   // per-instance H table
        o.total = (c + 1) & ~1;
        return o;
    }
};

// Mixed-precision handoff record of one instance (floats, OcpKernelArgs::hand_*): per stage
// k = 0..N the vectors s_k, pi_k, u_k (u_N = 0), then from a 64-aligned offset the row wave's
// box rows [t: BPL x 64 | lam: BPL x 64] and polytope rows [t: RPL x 64 | lam: RPL x 64],
// slot-major so that a wave's store of one slot is one coalesced 256-byte line
__host__ __device__ constexpr int hand_stage_w(int NS, int NU) { return 2 * NS + NU; }
__host__ __device__ constexpr int hand_rows_off(int N, int NS, int NU) {
    return ((N + 1) * hand_stage_w(NS, NU) + 63) & ~63;
}
// a warm (continued) instance of the fp64 launch: its fp32 phase ended with 1 or 0
// (fp64 instantiation only; the fp32 one only writes handoff records)
#ifdef BQP_F32
#define BQP_HAND_IN 0
#define BQP_HAND_OUT 1
#else
#define BQP_HAND_IN 1
#define BQP_HAND_OUT 0
#endif
// Only the long-horizon instantiations (two stages per lane, N + 1 > 64) carry the handoff
// code: the mixed mode pays there (the fp32 launch fits twice the instances per CU); shorter
// horizons run fp64 alone (bqp_api.cpp), and their kernels keep the register budget of the
// plain solve.
// The repair launch (POL) takes the same start as the launch whose result it repairs: an instance
// the mixed mode's cold retry launch solved again is marked pol_need = 2 there, and its repair
// starts cold too (replaying the handed-over start would overwrite the fp64 retry's result with
// the continuation's).
template <bool LONG, bool POL>
__device__ __forceinline__ bool hand_warm(const OcpKernelArgs& a, int inst) {
    return BQP_HAND_IN && LONG && a.hand_in && (a.hand_flag[inst] == 1 || a.hand_flag[inst] == 0) &&
           !(POL && a.pol_need[inst] == 2);
}

#ifdef BQP_STAMPS
// diagnostic build only (see tools/stamps.py): cycles per phase and per wave role, summed over
// the solve; slots 0..15 stage wave, 16..31 row wave
#define STAMP(id)                                                          \
    do {                                                                   \
        __builtin_amdgcn_s_waitcnt(0);                                     \
        const unsigned long long _t = __builtin_amdgcn_s_memtime();        \
        st_acc[id] += _t - st_last;                                        \
        st_last = _t;                                                      \
    } while (0)
#define STAMP_DECL                                                         \
    unsigned long long st_last = __builtin_amdgcn_s_memtime();             \
    unsigned long long st_acc[16];                                         \
    _Pragma("unroll") for (int i_ = 0; i_ < 16; ++i_) st_acc[i_] = 0
#define STAMP_STORE(base)                                                  \
    do {                                                                   \
        if (lane == 0 && a.stamps) {                                       \
            _Pragma("unroll") for (int i_ = 0; i_ < 16; ++i_)              \
                a.stamps[(int64_t)inst * 32 + (base) + i_] = (double)st_acc[i_]; \
        }                                                                  \
    } while (0)
#elif defined(BQP_ISA_ONLY_MG10) || defined(BQP_ISA_ONLY_DI) || defined(BQP_ISA_ONLY_MG_LNG)
#define STAMP(id) asm volatile(";BQP_PHASE " #id)
#define STAMP_DECL do { } while (0)
#define STAMP_STORE(base) do { } while (0)
#else
#define STAMP(id) do { } while (0)
#define STAMP_DECL do { } while (0)
#define STAMP_STORE(base) do { } while (0)
#endif

#define BARRIER() __syncthreads()
// scheduling fence between polytope rows of the row wave: keeps the scheduler from hoisting the
// Fp loads of all RPL rows to the top of a phase (register pressure at two waves per SIMD)
#define ROW_FENCE(q) do { if ((q) & 1) __builtin_amdgcn_sched_barrier(0); } while (0)

// ==========================================================================================
// stage wave
// ==========================================================================================
template <int NX, int NU, int NP, int SPL, bool POL>
__device__ __forceinline__ void stage_wave(const OcpKernelArgs& a, real* W, const QpLds& L,
                                           const real* Hs, int lane_w, int inst, int pslot) {
    const int lane = lane_w;
    // POL: the repair kernel (ocp_polish_kernel) - the same IPM, then the active-set polish
    constexpr bool PC = POL && BQP_POLISH && !BQP_EXP_NOSTAGE;
    constexpr int NS = NX + NP;
    constexpr int NV = NS + NU;
    constexpr int NB = NX + NU;
    const int N = a.N, kp = a.kp, hstride = a.hstride;
    real* X = W + L.xch;
    STAMP_DECL;
    constexpr bool LNG = BQP_LNG_OK && SPL == 2;     // long-horizon layout (QpLds lng)
    // stage cost of stage k: the shared LDS table, or (long horizons) the prepared table in
    // global memory (L2-resident, read-only); a stage pointer per use, as the address
    // arithmetic of the short-horizon kernels is register-critical
#define BQP_HK(k) const real* Hk = Hs + (k) * hstride; \
    const double* Hkg = (a.H_inst ? a.H_inst + (int64_t)inst * (N + 1) * hstride : a.H) + (int64_t)(k) * hstride
#define BQP_HV(idx) (LNG ? (real)Hkg[idx] : Hk[idx])
    // the long-horizon Riccati tables in global scratch, per instance slot: a persistent launch
    // reuses its slots' tables for every instance they take, so the tables stay in the XCD's L2
    // (512 resident slots x 12.9 KB at N = 100) instead of every instance writing its own
    // region back to HBM
    real* Pgl = LNG ? (real*)a.Pg + (int64_t)pslot * (N + 1) * pk_stride(NS) : nullptr;
    // per-instance stage costs: the instance's prepared table (global), copied into the LDS slot
    // on short horizons
    if (!LNG && a.H_inst) {
        real* Hl = W + L.Hi;
        const double* Hg = a.H_inst + (int64_t)inst * (N + 1) * hstride;
        for (int i = lane; i < (N + 1) * hstride; i += WAVE) Hl[i] = (real)Hg[i];
        wave_sync();
        Hs = Hl;
    }

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
        // the affine term c of the dynamics (theta rows 0)
        if (lane < NS) W[L.AB + NS * NS + NS * NU + lane] = (lane < NX && a.c) ? a.c[(int64_t)inst * a.sc + lane] : 0.0;
    }
    wave_sync();
    auto Abar = [&](int i, int j) __attribute__((always_inline)) -> real { return W[L.AB + i * NS + j]; };
    auto Bbar = [&](int i, int j) __attribute__((always_inline)) -> real { return W[L.AB + NS * NS + i * NU + j]; };
    // c from LDS at use (a register copy was carried through the loop: a scratch spill of the
    // DI kernel)
    auto cb = [&](int i) __attribute__((always_inline)) -> real { return W[L.AB + NS * NS + NS * NU + i]; };
    const double* wb = a.w ? a.w + (int64_t)inst * a.sw : nullptr;
    // linear cost term of stage k, internal index i ([x; theta; u] from external [x; u; theta])
    auto gterm = [&](int k, int i) __attribute__((always_inline)) -> real {
        if (!wb || (k == N && i >= NS)) return 0.0;
        const int e = (i < NX) ? i : (i < NS ? NX + NU + (i - NX) : NX + (i - NS));
        return wb[(int64_t)k * NV + e];
    };

    real s[SPL][NS], u[SPL][NU], pi[SPL][NS], kff[SPL][NU];
    const double* x0 = a.x0 + (int64_t)inst * a.sx0;
    real x0max = 0.0;
#pragma unroll
    for (int i = 0; i < NX; ++i) x0max = fmax(x0max, fabs(x0[i]));
#pragma unroll
    for (int j = 0; j < SPL; ++j) {
        const int k = lane + WAVE * j;
#pragma unroll
        for (int i = 0; i < NS; ++i) { s[j][i] = 0.0; pi[j][i] = 0.0; }
#pragma unroll
        for (int i = 0; i < NU; ++i) { u[j][i] = 0.0; kff[j][i] = 0.0; }
        if (k == 0) {
#pragma unroll
            for (int i = 0; i < NX; ++i) s[j][i] = x0[i];
        }
    }

    // ---- stage vectors to LDS (s, u, pi) ----
    auto write_state = [&]() __attribute__((always_inline)) {
        const int lane = opq(lane_w);
#pragma unroll
        for (int j = 0; j < SPL; ++j) {
            const int k = lane + WAVE * j;
            if (k <= N) {
#pragma unroll
                for (int i = 0; i < NS; ++i) { W[L.xs + k * NS + i] = s[j][i]; W[L.qt_xpi + k * NS + i] = pi[j][i]; }
#pragma unroll
                for (int i = 0; i < NU; ++i) W[L.xu + k * NU + i] = (k < N) ? u[j][i] : 0.0;
            }
        }
        wave_sync();
    };

    // ---- stage residuals without the row multipliers: rs' = g + Abar' pi_{k+1} - pi_k,
    //      ru' = g_u + Bbar' pi_{k+1}, re = Abar s + Bbar u + c - s_{k+1}; returns max|re|, max|g|
    auto stage_partials = [&](real& feasA, real& gsA) __attribute__((always_inline)) {
        const int lane = opq(lane_w);
        real fe = 0, gs = 0;
#pragma unroll
        for (int j = 0; j < SPL; ++j) {
            const int k = lane + WAVE * j;
            if (k > N) continue;
            BQP_HK(k);
            real v[NV];
#pragma unroll
            for (int i = 0; i < NS; ++i) v[i] = s[j][i];
#pragma unroll
            for (int i = 0; i < NU; ++i) v[NS + i] = (k < N) ? u[j][i] : 0.0;
            real gv[NV];
#pragma unroll
            for (int i = 0; i < NV; ++i) {
                real acc = gterm(k, i);
#pragma unroll
                for (int c = 0; c < NV; ++c) acc += BQP_HV(i * NV + c) * v[c];
                gv[i] = acc;
                gs = fmax(gs, fabs(acc));
            }
            real pn[NS];
#pragma unroll
            for (int i = 0; i < NS; ++i) pn[i] = (k < N) ? W[L.qt_xpi + (k + 1) * NS + i] : 0.0;
#pragma unroll
            for (int i = 0; i < NS; ++i) {
                real acc = gv[i];
                if (k < N) {
#pragma unroll
                    for (int c = 0; c < NS; ++c) acc += Abar(c, i) * pn[c];
                }
                if (k > 0) acc -= pi[j][i];
                W[L.rs + k * NS + i] = acc;
            }
#pragma unroll
            for (int i = 0; i < NU; ++i) {
                real acc = gv[NS + i];
#pragma unroll
                for (int c = 0; c < NS; ++c) acc += Bbar(c, i) * pn[c];
                W[L.ru + k * NU + i] = (k < N) ? acc : 0.0;
            }
            if (k < N) {
#pragma unroll
                for (int i = 0; i < NS; ++i) {
                    real acc = cb(i) - W[L.xs + (k + 1) * NS + i];
#pragma unroll
                    for (int c = 0; c < NS; ++c) acc += Abar(i, c) * s[j][c];
#pragma unroll
                    for (int c = 0; c < NU; ++c) acc += Bbar(i, c) * u[j][c];
                    if constexpr (!LNG) W[L.re + k * NS + i] = acc;
                    fe = fmax(fe, fabs(acc));
                }
            }
        }
        feasA = wmax(fe);
        gsA = wmax(gs);
    };

    // long horizons: the dynamics residual re_k of stage k = lane + 64 j, recomputed from the
    // iterate (registers) in the operation order of stage_partials instead of kept in LDS
    bool rez = false;   // polish direction solves: zero dynamics residual (PC only)
    auto re_at = [&](int j, int k, int i) __attribute__((always_inline)) -> real {
        if constexpr (PC) { if (rez) return real(0); }
        real acc = cb(i) - W[L.xs + (k + 1) * NS + i];
#pragma unroll
        for (int c = 0; c < NS; ++c) acc += Abar(i, c) * s[j][c];
#pragma unroll
        for (int c = 0; c < NU; ++c) acc += Bbar(i, c) * u[j][c];
        return acc;
    };

    // ---- add the row multipliers (box [upper, lower] in that order, polytope at kp) and
    //      return the stationarity norm ----
    auto combine = [&]() __attribute__((always_inline)) -> real {
        const int lane = opq(lane_w);
        real gpp[NV];
#pragma unroll
        for (int c = 0; c < NV; ++c) gpp[c] = W[L.gpp + c];
        real st = 0;
#pragma unroll
        for (int j = 0; j < SPL; ++j) {
            const int k = lane + WAVE * j;
            if (k > N) continue;
            real r[NS], ru[NU];
#pragma unroll
            for (int i = 0; i < NS; ++i) r[i] = W[L.rs + k * NS + i];
#pragma unroll
            for (int i = 0; i < NU; ++i) ru[i] = W[L.ru + k * NU + i];
#pragma unroll
            for (int i = 0; i < NX; ++i) {
                if constexpr (LNG) {
                    r[i] += W[L.blam + k * NB + i];
                } else {
                    r[i] += W[L.blam + (k * NB + i) * 2];
                    r[i] -= W[L.blam + (k * NB + i) * 2 + 1];
                }
            }
#pragma unroll
            for (int i = 0; i < NU; ++i) {
                if constexpr (LNG) {
                    ru[i] += W[L.blam + k * NB + NX + i];
                } else {
                    ru[i] += W[L.blam + (k * NB + NX + i) * 2];
                    ru[i] -= W[L.blam + (k * NB + NX + i) * 2 + 1];
                }
            }
            if (k == kp) {
#pragma unroll
                for (int i = 0; i < NS; ++i) r[i] += gpp[i];
                if (kp < N) {
#pragma unroll
                    for (int i = 0; i < NU; ++i) ru[i] += gpp[NS + i];
                }
            }
            if (k == 0) {
#pragma unroll
                for (int i = 0; i < NX; ++i) r[i] = 0.0;
            }
#pragma unroll
            for (int i = 0; i < NS; ++i) { st = fmax(st, fabs(r[i])); W[L.rs + k * NS + i] = r[i]; }
#pragma unroll
            for (int i = 0; i < NU; ++i) { st = fmax(st, fabs(ru[i])); W[L.ru + k * NU + i] = ru[i]; }
        }
        wave_sync();
        return wmax(st);
    };

    // ======================= Riccati factorisation =========================================
    // Standard form on the stage matrix M_k = Ht_k + F' P_{k+1} F, F = [Abar Bbar]:
    //   K_k = -M_uu^{-1} M_us,   P_k = M_ss - M_su M_uu^{-1} M_us.
    // M is linear in the packed upper triangle of P_{k+1} with CONSTANT coefficients
    //   C(r, c; a, b) = F(a,r) F(b,c) + [a != b] F(b,r) F(a,c)
    // (per instance, formed once per solve), so one entry of M is one NPK-term dot product.
    // Lane layout: quad e (lanes 4e..4e+3, e < NPK) owns packed entry e = (ie, je) of P_k.  The
    // VAL values that entry needs - M(ie,je), M(ie,u), M(je,u), M_uu - are spread over the quad
    // (lane q: values q, q+4, ...), each lane holding the coefficient rows of its values in
    // registers; lane 4e gathers them with quad DPP broadcasts, forms P_k(ie, je) (and, on the
    // diagonal, the column je of K_k) and stores it; the packed P_k is read back by every lane
    // (ds_read_b128 broadcasts).  Per stage: one dot product per lane, one LDS round trip.
    // Same association as oracle/cpu_ipm.c factor(): partial sums over m mod 4,
    // (s0 + s1) + (s2 + s3), then Ht + sum.
    constexpr int PST = pk_stride(NS);
    constexpr int NPK = pk_len(NS);
    constexpr int NUT = NU * (NU + 1) / 2;
    constexpr int VAL = 1 + 2 * NU + NUT;           // values one P_k entry needs
    constexpr int VPL = (VAL + 3) / 4;              // values per lane of the quad
    static_assert(4 * NPK <= WAVE, "one quad per packed entry of P");
    const int fq = lane >> 2, fql = lane & 3;
    const bool fquad = fq < NPK;
    int ie = 0, je = 0;                             // packed entry fq -> (ie <= je)
    {
        int e = 0;
#pragma unroll
        for (int i = 0; i < NS; ++i)
#pragma unroll
            for (int j = i; j < NS; ++j, ++e)
                if (e == fq) { ie = i; je = j; }
    }
    // (row, col) in the internal [s; u] index space of value v of entry (ie, je)
    auto vrc = [&](int v, int& r, int& c) __attribute__((always_inline)) {
        if (v == 0) { r = ie; c = je; }
        else if (v <= NU) { r = ie; c = NS + v - 1; }
        else if (v <= 2 * NU) { r = je; c = NS + v - NU - 1; }
        else {
            int t = v - 2 * NU - 1, x = 0;
#pragma unroll
            for (int xx = 0; xx < NU; ++xx) if (t >= NU - xx) { t -= NU - xx; x = xx + 1; } else break;
            r = NS + x; c = NS + x + t;
        }
    };
    auto Fab = [&](int a_, int r) __attribute__((always_inline)) -> real {
        return r < NS ? Abar(a_, r) : Bbar(a_, r - NS);
    };
    real cf[VPL][NPK];                              // coefficient rows of this lane's values
    int vr[VPL], vc[VPL];
#pragma unroll
    for (int t = 0; t < VPL; ++t) {
        const int v = fql + 4 * t;
        int r = 0, c = 0;
        if (v < VAL) vrc(v, r, c);
        vr[t] = r; vc[t] = c;
        int m = 0;
#pragma unroll
        for (int a_ = 0; a_ < NS; ++a_)
#pragma unroll
            for (int b = a_; b < NS; ++b, ++m) {
                real x = Fab(a_, r) * Fab(b, c);
                if (a_ != b) x = fmar(Fab(b, r), Fab(a_, c), x);
                cf[t][m] = (v < VAL) ? x : real(0);
            }
    }
    // Ht entry (r, c) of stage k: raw cost entry, box diagonal, polytope term at kp; the raw
    // operands are prefetched one stage ahead and combined as (H + D) + FD
    struct HRaw { real h[VPL], d[VPL]; };
    auto load_h = [&](int k, HRaw& o) __attribute__((always_inline)) {
        BQP_HK(k);
#pragma unroll
        for (int t = 0; t < VPL; ++t) {
            o.h[t] = BQP_HV(vr[t] * NV + vc[t]);
            o.d[t] = W[L.Dx + k * NV + vr[t]];
        }
    };
    auto ht = [&](int k, const HRaw& o, int t) __attribute__((always_inline)) -> real {
        real v = o.h[t] + (vr[t] == vc[t] ? o.d[t] : real(0));
        if (k == kp) v += W[L.FD + vr[t] * NV + vc[t]];
        return v;
    };
    real pu[PST];
    auto read_p = [&](int k) __attribute__((always_inline)) {
        wave_sync();
        const real2* src = reinterpret_cast<const real2*>(W + L.P + (LNG ? (k & 1) : k) * PST);
#pragma unroll
        for (int q = 0; q < PST / 2; ++q) {
            const real2 t2 = src[q];
            pu[2 * q] = t2.x;
            pu[2 * q + 1] = t2.y;
        }
    };
    auto Pm = [&](int a_, int b_) __attribute__((always_inline)) -> real { return pu[pk_idx(NS, a_, b_)]; };
    auto factor = [&]() __attribute__((always_inline)) -> bool {
        HRaw raw, nxt;
        {
            // P_N = Ht_N(s, s)
            load_h(N, raw);
            const real v0 = ht(N, raw, 0);
            if (fquad && fql == 0) {
                W[L.P + (LNG ? (N & 1) : N) * PST + fq] = v0;
                if constexpr (LNG) Pgl[N * PST + fq] = v0;
            }
        }
        read_p(N);
        bool ok = true;
        // one stage of the recursion: P_k from P_{k+1} (in pu) and the stage's raw operands
        auto fstage = [&](int k, const HRaw& raw) __attribute__((always_inline)) {
            real mv[VPL];
#pragma unroll
            for (int t = 0; t < VPL; ++t) {
                real sp0 = 0, sp1 = 0, sp2 = 0, sp3 = 0;
#pragma unroll
                for (int m = 0; m < NPK; ++m) {
                    if ((m & 3) == 0) sp0 = fmar(cf[t][m], pu[m], sp0);
                    if ((m & 3) == 1) sp1 = fmar(cf[t][m], pu[m], sp1);
                    if ((m & 3) == 2) sp2 = fmar(cf[t][m], pu[m], sp2);
                    if ((m & 3) == 3) sp3 = fmar(cf[t][m], pu[m], sp3);
                }
                mv[t] = ht(k, raw, t) + ((sp0 + sp1) + (sp2 + sp3));
            }
            // gather the VAL values in lane 4e: value v sits in lane v % 4, slot v / 4
            real g[VAL];
#pragma unroll
            for (int v = 0; v < VAL; ++v) {
                const int s = v & 3;
                const real src = mv[v >> 2];
                g[v] = (s == 0) ? dpp_mov<0x00, 0xf>(real(0), src)
                     : (s == 1) ? dpp_mov<0x55, 0xf>(real(0), src)
                     : (s == 2) ? dpp_mov<0xAA, 0xf>(real(0), src)
                                : dpp_mov<0xFF, 0xf>(real(0), src);
            }
            real pv, Kc[NU], Lf[NU * NU];
            if constexpr (NU == 1) {
                ok = ok && (g[3] > 0.0);
                const real rinv = frcp(g[3]);          // M_uu > 0 checked above
                Lf[0] = rinv;
                pv = fmar(-(g[1] * rinv), g[2], g[0]);
                Kc[0] = -(g[2] * rinv);
            } else {
                real Mu[NU][NU], Lc[NU][NU];
                {
                    int t = 2 * NU + 1;
#pragma unroll
                    for (int x = 0; x < NU; ++x)
#pragma unroll
                        for (int y = x; y < NU; ++y, ++t) { Mu[x][y] = g[t]; Mu[y][x] = g[t]; }
                }
                ok = chol_small<NU>(Mu, Lc) && ok;
#pragma unroll
                for (int x = 0; x < NU; ++x)
#pragma unroll
                    for (int y = 0; y < NU; ++y) Lf[x * NU + y] = Lc[x][y];
                real y[NU];
#pragma unroll
                for (int x = 0; x < NU; ++x) y[x] = g[1 + NU + x];   // M(je, u)
                chol_solve_small<NU>(Lf, y);
                real acc = g[1] * y[0];
#pragma unroll
                for (int x = 1; x < NU; ++x) acc = fmar(g[1 + x], y[x], acc);
                pv = g[0] - acc;
#pragma unroll
                for (int x = 0; x < NU; ++x) Kc[x] = -y[x];
            }
            if (fquad && fql == 0) {
                W[L.P + (LNG ? (k & 1) : k) * PST + fq] = pv;
                if constexpr (LNG) Pgl[k * PST + fq] = pv;   // the whole table for the solves
                if (ie == je) {
#pragma unroll
                    for (int x = 0; x < NU; ++x) W[L.K + k * NU * NS + x * NS + je] = Kc[x];
                }
                if (fq == 0) {
#pragma unroll
                    for (int x = 0; x < NU * NU; ++x) W[L.Lr + k * NU * NU + x] = Lf[x];
                }
            }
            read_p(k);
        };
        if constexpr (LNG) {
            // long horizons read H from global (L2): its operands are fetched two stages
            // ahead, three register sets in rotation
            HRaw r0, r1, r2;
            load_h(N - 1, r0);
            if (N >= 2) load_h(N - 2, r1);
            for (int k = N - 1; k >= 0; k -= 3) {
                if (k >= 2) load_h(k - 2, r2);
                fstage(k, r0);
                if (k < 1) break;
                if (k >= 3) load_h(k - 3, r0);
                fstage(k - 1, r1);
                if (k < 2) break;
                if (k >= 4) load_h(k - 4, r1);
                fstage(k - 2, r2);
            }
        } else {
            load_h(N - 1, raw);
            for (int k = N - 1; k >= 0; --k) {
                if (k > 0) load_h(k - 1, nxt);
                fstage(k, raw);
                raw = nxt;
            }
        }
        // factor of the theta block of P_0 (np = 1: its reciprocal)
        real Pt[NP][NP], L0[NP][NP];
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
        // long horizons: the global P_k stores complete before the solves read them.  Writer and
        // readers are this wave (other lanes): the stores reach this XCD's L2 once the vector
        // memory counter drains, and the reads are agent-scope (sc1, past the L1), so no L2
        // write-back is needed - the tables stay dirty in L2 and are rewritten in place by the
        // next factorisation (an agent-scope release wrote the XCD's dirty lines back to HBM
        // once per factorisation: 1.29 GB of writes per C5 launch, profiles/r02_c5pmc)
        if constexpr (LNG) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        wave_sync();
        return ok;
    };
    // packed P_k for the per-stage passes (prep_iter, update_stage): LDS or global scratch
    auto load_pk = [&](int k, real* pk) __attribute__((always_inline)) {
        if constexpr (LNG) {
            const real* src = Pgl + k * PST;
#pragma unroll
            for (int e = 0; e < NPK; ++e) pk[e] = __hip_atomic_load(src + e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
#pragma unroll
            for (int e = 0; e < NPK; ++e) pk[e] = W[L.P + k * PST + e];
        }
    };

    // ======================= once per factorisation ========================================
    // The dynamics residual re_k is the same for the predictor and the corrector solve, so the
    // part of the solves that depends on it alone is formed once: with w_k = P_{k+1} re_k,
    //   cw_k = Phi_k' w_k (Phi_k = Abar + Bbar K_k; the pre-pass adds it to qt_k),
    //   bw_k = Bbar' w_k (the post-backward pass adds it to Bbar' p_{k+1}).
    auto prep_iter = [&]() __attribute__((always_inline)) {
        const int lane = opq(lane_w);
#pragma unroll
        for (int j = 0; j < SPL; ++j) {
            const int k = lane + WAVE * j;
            if (k < N) {
                real Pn_[LNG ? PST : 1];
                const real* Pn = W + L.P + (k + 1) * PST;
                if constexpr (LNG) { load_pk(k + 1, Pn_); Pn = Pn_; }
                const real* Kk = W + L.K + k * NU * NS;
                real rek[NS], wk[NS];
#pragma unroll
                for (int c = 0; c < NS; ++c) rek[c] = LNG ? re_at(j, k, c) : W[L.re + k * NS + c];
#pragma unroll
                for (int i = 0; i < NS; ++i) {
                    real v = 0.0;
#pragma unroll
                    for (int c = 0; c < NS; ++c) v += Pn[pk_idx(NS, i, c)] * rek[c];
                    wk[i] = v;
                }
#pragma unroll
                for (int x = 0; x < NU; ++x) {
                    real v = 0.0;
#pragma unroll
                    for (int c = 0; c < NS; ++c) v += Bbar(c, x) * wk[c];
                    W[L.bw + k * NU + x] = v;
                }
#pragma unroll
                for (int i = 0; i < NS; ++i) {
                    real v = 0.0;
#pragma unroll
                    for (int c = 0; c < NS; ++c) {
                        real ph = Abar(c, i);
#pragma unroll
                        for (int x = 0; x < NU; ++x) ph += Bbar(c, x) * Kk[x * NS + i];
                        v += ph * wk[c];
                    }
                    W[L.wv + k * NS + i] = v;
                }
            }
        }
    };

    // ======================= Newton solve ==================================================
    // right-hand side q = r_v + C'((lam o ri - rc)/t): the row wave supplies the box terms
    // [upper, lower] per stage (ebox) and Fp'e (gpe); direction written to (ods, odu)
    const int li = lane < NS ? lane : NS - 1;
    auto solve = [&](int ods, int odu) __attribute__((always_inline)) {
        const int lane = opq(lane_w);
        real qs[SPL][NS], qu[SPL][NU];
        real gpe[NV];
#pragma unroll
        for (int c = 0; c < NV; ++c) gpe[c] = W[L.gpe + c];
#pragma unroll
        for (int j = 0; j < SPL; ++j) {
            const int k = lane + WAVE * j;
            const int kk = k <= N ? k : N;
#pragma unroll
            for (int i = 0; i < NS; ++i) qs[j][i] = W[L.rs + kk * NS + i];
#pragma unroll
            for (int i = 0; i < NX; ++i) {
                real e = 0.0;
                if constexpr (LNG) {
                    e += W[L.ebox + kk * NB + i];
                } else {
                    e += W[L.ebox + (kk * NB + i) * 2];
                    e -= W[L.ebox + (kk * NB + i) * 2 + 1];
                }
                qs[j][i] += e;
            }
#pragma unroll
            for (int i = 0; i < NU; ++i) {
                real e = W[L.ru + kk * NU + i];
                if constexpr (LNG) {
                    e += W[L.ebox + kk * NB + NX + i];
                } else {
                    e += W[L.ebox + (kk * NB + NX + i) * 2];
                    e -= W[L.ebox + (kk * NB + NX + i) * 2 + 1];
                }
                qu[j][i] = e;
            }
            if (k == kp) {
#pragma unroll
                for (int i = 0; i < NS; ++i) qs[j][i] += gpe[i];
                if (kp < N) {
#pragma unroll
                    for (int i = 0; i < NU; ++i) qu[j][i] += gpe[NS + i];
                }
            }
        }
        // pre-pass: qh_k = qt_k + cw_k with qt_k = qs_k + K_k' qu_k (cw_k = Phi_k' P_{k+1} re_k
        // is the right-hand-side-independent part, formed once per factorisation by
        // prep_iter); p_N = qs_N.  qh carries everything of the backward recursion that does
        // not depend on p_{k+1}, so the sequential sweep is one NS x NS mat-vec per stage.
#pragma unroll
        for (int j = 0; j < SPL; ++j) {
            const int k = lane + WAVE * j;
            if (k < N) {
                const real* Kk = W + L.K + k * NU * NS;
#pragma unroll
                for (int i = 0; i < NS; ++i) {
                    real qq = qs[j][i];
#pragma unroll
                    for (int x = 0; x < NU; ++x) qq += Kk[x * NS + i] * qu[j][x];
                    W[L.qt_xpi + k * NS + i] = qq + W[L.wv + k * NS + i];
                }
#pragma unroll
                for (int x = 0; x < NU; ++x) W[L.qu + k * NU + x] = qu[j][x];
            } else if (k == N) {
#pragma unroll
                for (int i = 0; i < NS; ++i) W[L.pv + N * NS + i] = qs[j][i];
            }
        }
        wave_sync();
        STAMP(10);
        // backward sweep: lane i < NS computes entry i of p_k = Phi_k' p_{k+1} + qh_k; the new
        // vector reaches every lane of the row by DPP row broadcasts (v_mov_b64_dpp
        // row_newbcast:c, one per entry: the value stays in vector registers - the round-3
        // readlane broadcast went through scalar registers: 9.6k -> 8.0k cycles per iteration
        // for the backward sweep, 10.9k -> 9.4k for the forward one, C2 -3.8 %); two register
        // sets used alternately (stages k, k-1), each refilled two stages ahead.  (Round 4 tried every
        // lane forming the whole vector from broadcast LDS reads, no readlane on the chain: the
        // sweeps are issue-bound at one instance per SIMD, and the 3x longer instruction
        // stream cost 9.4k -> 14.6k cycles per iteration)
        {
            real Acol[NS], Bl[NS][NU];
#pragma unroll
            for (int c = 0; c < NS; ++c) {
                Acol[c] = Abar(c, li);
#pragma unroll
                for (int x = 0; x < NU; ++x) Bl[c][x] = Bbar(c, x);
            }
            real p[NS];
#pragma unroll
            for (int i = 0; i < NS; ++i) p[i] = W[L.pv + N * NS + i];
            auto load_b = [&](int k, real (&kc)[NU], real& q) __attribute__((always_inline)) {
                q = W[L.qt_xpi + k * NS + li];
#pragma unroll
                for (int x = 0; x < NU; ++x) kc[x] = W[L.K + k * NU * NS + x * NS + li];
            };
            real k0[NU], q0, k1[NU], q1;
            load_b(N - 1, k0, q0);
            if (N >= 2) load_b(N - 2, k1, q1);
            auto step_b = [&](int k, const real (&kc)[NU], real q) __attribute__((always_inline)) {
                real acc = q;
#pragma unroll
                for (int c = 0; c < NS; ++c) {
                    real ph = Acol[c];
#pragma unroll
                    for (int x = 0; x < NU; ++x) ph += Bl[c][x] * kc[x];
                    acc += ph * p[c];
                }
                if (lane < NS) W[L.pv + k * NS + lane] = acc;
                rbc_all<0, NS>(acc, p);   // lanes c < NS of the row hold entry c
            };
            for (int k = N - 1; k >= 0; k -= 2) {
                step_b(k, k0, q0);
                if (k >= 2) load_b(k - 2, k0, q0);
                if (k == 0) break;
                step_b(k - 1, k1, q1);
                if (k >= 3) load_b(k - 3, k1, q1);
            }
        }
        wave_sync();
        STAMP(11);
        // post-backward: kff_k = -Rhat^{-1}((qu_k + bw_k) + Bbar' p_{k+1}); f_k = Bbar kff_k + re_k
#pragma unroll
        for (int j = 0; j < SPL; ++j) {
            const int k = lane + WAVE * j;
            if (k < N) {
                real y[NS], r[NU];
#pragma unroll
                for (int i = 0; i < NS; ++i) y[i] = W[L.pv + (k + 1) * NS + i];
#pragma unroll
                for (int x = 0; x < NU; ++x) {
                    real v = qu[j][x] + W[L.bw + k * NU + x];
#pragma unroll
                    for (int c = 0; c < NS; ++c) v += Bbar(c, x) * y[c];
                    r[x] = -v;
                }
                chol_solve_small<NU>(W + L.Lr + k * NU * NU, r);
#pragma unroll
                for (int x = 0; x < NU; ++x) kff[j][x] = r[x];
#pragma unroll
                for (int i = 0; i < NS; ++i) {
                    real v = LNG ? re_at(j, k, i) : W[L.re + k * NS + i];
#pragma unroll
                    for (int x = 0; x < NU; ++x) v += Bbar(i, x) * kff[j][x];
                    W[L.fv + k * NS + i] = v;
                }
            }
        }
        wave_sync();
        STAMP(12);
        // theta_0 step + forward sweep: lane i < NS computes entry i of ds_{k+1} = Phi_k ds_k + f_k
        {
            real d[NS];
#pragma unroll
            for (int i = 0; i < NX; ++i) d[i] = 0.0;
            real r0[NP];
#pragma unroll
            for (int x = 0; x < NP; ++x) r0[x] = -W[L.pv + NX + x];
            chol_solve_small<NP>(W + L.L0, r0);
#pragma unroll
            for (int x = 0; x < NP; ++x) d[NX + x] = r0[x];
            if (lane == 0) {
#pragma unroll
                for (int i = 0; i < NS; ++i) W[ods + i] = d[i];
            }
            real Arow[NS], Bli[NU];
#pragma unroll
            for (int c = 0; c < NS; ++c) Arow[c] = Abar(li, c);
#pragma unroll
            for (int x = 0; x < NU; ++x) Bli[x] = Bbar(li, x);
            auto load_f = [&](int k, real (&kr)[NU][NS], real& f) __attribute__((always_inline)) {
                f = W[L.fv + k * NS + li];
#pragma unroll
                for (int x = 0; x < NU; ++x)
#pragma unroll
                    for (int c = 0; c < NS; ++c) kr[x][c] = W[L.K + k * NU * NS + x * NS + c];
            };
            real k0[NU][NS], f0, k1[NU][NS], f1;
            load_f(0, k0, f0);
            if (N >= 2) load_f(1, k1, f1);
            auto step_f = [&](int k, const real (&kr)[NU][NS], real f) __attribute__((always_inline)) {
                real acc = f;
#pragma unroll
                for (int c = 0; c < NS; ++c) {
                    real ph = Arow[c];
#pragma unroll
                    for (int x = 0; x < NU; ++x) ph += Bli[x] * kr[x][c];
                    acc += ph * d[c];
                }
                if (lane < NS) W[ods + (k + 1) * NS + lane] = acc;
                rbc_all<0, NS>(acc, d);   // lanes c < NS of the row hold entry c
            };
            for (int k = 0; k < N; k += 2) {
                step_f(k, k0, f0);
                if (k + 2 < N) load_f(k + 2, k0, f0);
                if (k + 1 >= N) break;
                step_f(k + 1, k1, f1);
                if (k + 3 < N) load_f(k + 3, k1, f1);
            }
        }
        wave_sync();
        STAMP(13);
        // post-forward: du_k = K_k ds_k + kff_k
#pragma unroll
        for (int j = 0; j < SPL; ++j) {
            const int k = lane + WAVE * j;
            if (k < N) {
                const real* Kk = W + L.K + k * NU * NS;
#pragma unroll
                for (int x = 0; x < NU; ++x) {
                    real v = kff[j][x];
#pragma unroll
                    for (int c = 0; c < NS; ++c) v += Kk[x * NS + c] * W[ods + k * NS + c];
                    W[odu + k * NU + x] = v;
                }
            } else if (k == N) {
#pragma unroll
                for (int x = 0; x < NU; ++x) W[odu + N * NU + x] = 0.0;
            }
        }
        wave_sync();
        STAMP(14);
    };

    // primal/dual stage update by alpha along (ids, idu); dpi_k = P_k ds_k + p_k
    // the dual direction dpi_k = P_k ds_k + p_k of the corrector does not depend on the step
    // length: it is formed while the row wave runs the ratio test (before B5) and parked in the
    // cw_k slot (dead until the next factorisation); the update after B6 only scales it
    auto dual_dir = [&](int ids) __attribute__((always_inline)) {
        const int lane = opq(lane_w);
#pragma unroll
        for (int j = 0; j < SPL; ++j) {
            const int k = lane + WAVE * j;
            if (k > N || k < 1) continue;
            real dsk[NS];
#pragma unroll
            for (int i = 0; i < NS; ++i) dsk[i] = W[ids + k * NS + i];
            real Pk_[LNG ? PST : 1];
            const real* Pk = W + L.P + k * PST;
            if constexpr (LNG) { load_pk(k, Pk_); Pk = Pk_; }
#pragma unroll
            for (int i = 0; i < NS; ++i) {
                real v = W[L.pv + k * NS + i];
#pragma unroll
                for (int c = 0; c < NS; ++c) v += Pk[pk_idx(NS, i, c)] * dsk[c];
                W[L.wv + k * NS + i] = v;
            }
        }
    };
    auto update_stage_dir = [&](real al, int ids, int idu) __attribute__((always_inline)) {
        const int lane = opq(lane_w);
#pragma unroll
        for (int j = 0; j < SPL; ++j) {
            const int k = lane + WAVE * j;
            if (k > N) continue;
            if (k >= 1) {
#pragma unroll
                for (int i = 0; i < NS; ++i) pi[j][i] += al * W[L.wv + k * NS + i];
            }
#pragma unroll
            for (int i = 0; i < NS; ++i) s[j][i] += al * W[ids + k * NS + i];
            if (k < N) {
#pragma unroll
                for (int i = 0; i < NU; ++i) u[j][i] += al * W[idu + k * NU + i];
            }
        }
    };
    auto update_stage = [&](real al, int ids, int idu) __attribute__((always_inline)) {
        const int lane = opq(lane_w);
#pragma unroll
        for (int j = 0; j < SPL; ++j) {
            const int k = lane + WAVE * j;
            if (k > N) continue;
            real dsk[NS];
#pragma unroll
            for (int i = 0; i < NS; ++i) dsk[i] = W[ids + k * NS + i];
            if (k >= 1) {
                real Pk_[LNG ? PST : 1];
                const real* Pk = W + L.P + k * PST;
                if constexpr (LNG) { load_pk(k, Pk_); Pk = Pk_; }
#pragma unroll
                for (int i = 0; i < NS; ++i) {
                    real v = W[L.pv + k * NS + i];
#pragma unroll
                    for (int c = 0; c < NS; ++c) v += Pk[pk_idx(NS, i, c)] * dsk[c];
                    pi[j][i] += al * v;
                }
            }
#pragma unroll
            for (int i = 0; i < NS; ++i) s[j][i] += al * dsk[i];
            if (k < N) {
#pragma unroll
                for (int i = 0; i < NU; ++i) u[j][i] += al * W[idu + k * NU + i];
            }
        }
    };

    // ======================= initial point ==================================================
    real feasA = 0, gsA = 0;
    real minv, bscale;
    int flag = 0, it0 = 0;
    if (hand_warm<SPL == 2, POL>(a, inst)) {
        // continue the fp32 phase's iterate (mixed precision); x_0 stays the exact fp64 state
        const float* hb = a.hand_in + (int64_t)inst * a.hand_stride;
        constexpr int SW = hand_stage_w(NS, NU);
#pragma unroll
        for (int j = 0; j < SPL; ++j) {
            const int k = lane + WAVE * j;
            if (k > N) continue;
#pragma unroll
            for (int i = 0; i < NS; ++i) {
                s[j][i] = (k == 0 && i < NX) ? s[j][i] : (real)hb[k * SW + i];
                pi[j][i] = (real)hb[k * SW + NS + i];
            }
#pragma unroll
            for (int i = 0; i < NU; ++i) u[j][i] = (k < N) ? (real)hb[k * SW + 2 * NS + i] : 0.0;
        }
        write_state();
        stage_partials(feasA, gsA);
        BARRIER();                                        // W0: row wave forms residuals + tables
        minv = 1.0 / fmax(X[X_CNT], 1.0);
        bscale = fmax(x0max, X[X_BSR]);
        it0 = a.hand_it[inst];
    } else {
        write_state();
        stage_partials(feasA, gsA);
        BARRIER();                                        // I0: row-side tables of t = lam = 1
        minv = 1.0 / fmax(X[X_CNT], 1.0);
        bscale = fmax(x0max, X[X_BSR]);
        combine();
        if (!factor()) flag = -8;
        prep_iter();
        BARRIER();                                        // I1: predictor rhs of the start
        solve(L.dsv, L.duv);
        update_stage(1.0, L.dsv, L.duv);
        BARRIER();                                        // I2: row wave takes dt (old iterate), shifts
        BARRIER();                                        // I3: row wave done with the old iterate
        write_state();
        stage_partials(feasA, gsA);
    }

    // ======================= main loop ======================================================
    int it = 0;
    real mu = 0.0, mu_min = INFINITY, stat = 0.0, feas = 0.0, feq = 0.0, fin = 0.0;
    const int max_iter = a.max_iter;
    for (it = 0;; ++it) {
        BARRIER();                                        // B0: row multipliers / D / F'DF, row residual norm, comp sum ready
        STAMP(0);
        stat = combine();
        STAMP(1);
        STAMP(2);
        feq = feasA;
        fin = X[X_FEASB];
        feas = fmax(feq, fin);
        mu = X[X_CS] * minv;
        bool stop = false;
        if (flag != 0) {
            stop = true;
        } else if (stat <= a.tol_stat * (1.0 + gsA) && feas <= a.tol_feas * (1.0 + bscale) &&
                   mu <= a.tol_comp && (!BQP_POLISH || X[X_CMAX] <= CMAX_K * a.tol_comp)) {
            flag = 1; stop = true;
#ifdef BQP_F32
        } else if (mu <= a.tol_comp && feas <= a.tol_feas * (1.0 + bscale) && isfinite(stat)) {
            // fp32: complementarity and feasibility have converged; the stationarity residual
            // sums terms of |P x| ~ 1e3 and is resolved only to fp32 round-off of those terms,
            // and the next barrier factorisation (D = lam / t ~ 1/mu) would exceed fp32 range
            flag = 1; stop = true;
#endif
        } else if (!(isfinite(stat) && isfinite(feas) && isfinite(mu))) {
            flag = -8; stop = true;
        } else if (mu > MU_BLOWUP * mu_min && feas > FEAS_GUARD * (1.0 + bscale)) {
            flag = -2; stop = true;
        } else {
            mu_min = fmin(mu_min, mu);
            if (it == max_iter) stop = true;
        }
        if (!stop && !factor()) { flag = -8; stop = true; }
        if (!stop) prep_iter();
        STAMP(3);
        if (lane == 0) {
            X[X_STOP] = stop ? 1.0 : 0.0;
            X[X_FEASOK] = (feas <= FEAS_GUARD * (1.0 + bscale)) ? 1.0 : 0.0;
            X[X_FLAG] = (real)flag;
            if constexpr (PC) {
                X[X_RHO] = POL_RHO * (1.0 + gsA);
                X[X_TF] = 1e-12 * (1.0 + bscale);
            }
        }
        BARRIER();                                        // B2: predictor rhs ready; stop flag
        STAMP(4);
        if (stop) break;
        solve(L.dsv, L.duv);                              // predictor
        STAMP(5);
        BARRIER();                                        // B3: predictor direction out
        BARRIER();                                        // B4: corrector rhs ready
        STAMP(6);
        solve(L.dsc, L.duc);                              // corrector
        STAMP(7);
        BARRIER();                                        // B5: corrector direction out
        dual_dir(L.dsc);                                  // overlaps the row wave's ratio test
        BARRIER();                                        // B6: step length ready
        STAMP(8);
        const real al = X[X_ALPHA];
        update_stage_dir(al, L.dsc, L.duc);
        write_state();
        stage_partials(feasA, gsA);
        STAMP(9);
    }

    // ======================= active-set polish (fp64, repair kernel only) ====================
    // oracle/cpu_ipm.c polish(): rows with lam > t are equalities, the others are dropped; the
    // equality-constrained QP is solved on the Riccati machinery with weight rho on the active
    // rows (one factorisation per round).  A pass is one augmented-Lagrangian step (the exact
    // minimiser of the AL for the current multipliers nu) followed by conjugate gradients on nu
    // for r(nu) = C v(nu) - b = 0 (each CG step one solve with right-hand side C'p and zero
    // stage / dynamics residuals; plain multiplier steps once a direction is numerically
    // singular), then nu += rho r.  Negative multipliers leave the set and violated rows enter
    // it between rounds.  The polished point replaces the IPM iterate only if it passes the KKT
    // checks.  Barriers T0..T10 pair with the row wave's.
    real polished = 0.0;
    bool pi_kept = false;                                 // pi_out already holds the IPM's pi
    if constexpr (PC) {
        BARRIER();                                        // Q0: row wave published max min(t, lam)
        const bool dopol = a.polish > 0 && flag != -2 &&
                           (flag != 1 || (a.polish > 1 && X[X_DEG] > DEG_POLISH)) && isfinite(gsA);
        if (dopol) {
            STAMP(15);
            // the IPM iterate for the fall-back: s, u in the predictor-direction slots; pi goes
            // to its output now (overwritten below only if the polish is accepted)
#pragma unroll
            for (int j = 0; j < SPL; ++j) {
                const int k = lane + WAVE * j;
                if (a.pi_out && k >= 1 && k <= N) {
                    double* po = a.pi_out + ((int64_t)inst * N + (k - 1)) * NX;
#pragma unroll
                    for (int i = 0; i < NX; ++i) po[i] = pi[j][i];
                }
                if (k <= N) {
#pragma unroll
                    for (int i = 0; i < NS; ++i) W[L.dsv + k * NS + i] = s[j][i];
#pragma unroll
                    for (int i = 0; i < NU; ++i) W[L.duv + k * NU + i] = (k < N) ? u[j][i] : 0.0;
                }
            }
            const real tf = 1e-12 * (1.0 + bscale);
            int rd = 0, pass = 0, m = 0, dec = 0;
            real pst = 0.0;
            auto zero_stage_res = [&]() __attribute__((always_inline)) {
#pragma unroll
                for (int j = 0; j < SPL; ++j) {
                    const int k = lane + WAVE * j;
                    if (k > N) continue;
#pragma unroll
                    for (int i = 0; i < NS; ++i) {
                        W[L.rs + k * NS + i] = 0.0;
                        if constexpr (!LNG) W[L.re + k * NS + i] = 0.0;
                    }
#pragma unroll
                    for (int i = 0; i < NU; ++i) W[L.ru + k * NU + i] = 0.0;
                }
                wave_sync();
            };
            for (;;) {
                stage_partials(feasA, gsA);
                BARRIER();                                // T0: stage vectors, partial residuals
                BARRIER();                                // T1: row tables of (v, nu), mode m
                pst = combine();
                const real va = X[X_PVA];
                if (m != 1) {
                    // a new active set: one factorisation per round
                    dec = factor() ? 0 : 3;
                    pass = 0;
                } else {
                    const bool pok = isfinite(pst) && pst <= a.tol_stat * (1.0 + gsA) && va <= tf;
                    if (!pok && pass + 1 < POL_PASS) {
                        dec = 0; ++pass;
                    } else {
                        const bool ok = pok && X[X_PVIOL] <= tf &&
                                        X[X_PLNEG] >= -1e-9 * (1.0 + X[X_PLMX]) && feasA <= tf;
                        dec = ok ? 1 : ((rd + 1 < POL_ROUNDS && X[X_PCHG] > 0.0) ? 2 : 3);
                    }
                }
                if (lane == 0) X[X_PDEC] = (real)dec;
                BARRIER();                                // T2: decision out
                if (dec == 1 || dec == 3) break;
                if (dec == 2) { ++rd; m = 2; continue; }
                // AL step from the residuals of (v, nu)
                prep_iter();
                solve(L.dsc, L.duc);
                dual_dir(L.dsc);
                update_stage_dir(1.0, L.dsc, L.duc);
                write_state();
                BARRIER();                                // T3: v after the AL step
                BARRIER();                                // T4: row wave: CG start, decision
                for (;;) {
                    const int cgd = (int)X[X_CGD];
                    if (cgd == 2) break;
                    if (cgd == 0) {
                        // CG direction: right-hand side C'p (the row wave's tables)
                        zero_stage_res();
                        rez = true;
                        prep_iter();
                        solve(L.dsc, L.duc);
                        dual_dir(L.dsc);
                        rez = false;
                        BARRIER();                        // T5: direction in (dsc, duc)
                        BARRIER();                        // T6: row wave: alpha, next step
                        const real al = X[X_ALPHA];
                        if (al != 0.0) update_stage_dir(al, L.dsc, L.duc);
                    } else {
                        // multiplier step nu += rho r, then the AL step
                        write_state();
                        stage_partials(feasA, gsA);
                        BARRIER();                        // T7: v, partial residuals
                        BARRIER();                        // T8: row tables of mode 1
                        combine();
                        prep_iter();
                        solve(L.dsc, L.duc);
                        dual_dir(L.dsc);
                        update_stage_dir(1.0, L.dsc, L.duc);
                        write_state();
                        BARRIER();                        // T9: v after the AL step
                        BARRIER();                        // T10: row wave: |r|, next step
                    }
                }
                write_state();
                m = 1;
            }
            if (dec == 1) {
                polished = 1.0;
                flag = 1;
                stat = pst; feas = fmax(feasA, X[X_PVIOL]); mu = 0.0; feq = feasA; fin = X[X_PVIOL];
            } else {
                pi_kept = true;
#pragma unroll
                for (int j = 0; j < SPL; ++j) {
                    const int k = lane + WAVE * j;
                    if (k <= N) {
#pragma unroll
                        for (int i = 0; i < NS; ++i) s[j][i] = W[L.dsv + k * NS + i];
#pragma unroll
                        for (int i = 0; i < NU; ++i) u[j][i] = (k < N) ? W[L.duv + k * NU + i] : 0.0;
                    }
                }
            }
        }
    }

    // ======================= outputs =======================================================
    if (BQP_HAND_OUT && SPL == 2 && a.hand_out) {
        // fp32 phase of the mixed mode: hand the iterate to the fp64 launch
        float* hb = a.hand_out + (int64_t)inst * a.hand_stride;
        constexpr int SW = hand_stage_w(NS, NU);
#pragma unroll
        for (int j = 0; j < SPL; ++j) {
            const int k = lane + WAVE * j;
            if (k > N) continue;
#pragma unroll
            for (int i = 0; i < NS; ++i) { hb[k * SW + i] = (float)s[j][i]; hb[k * SW + NS + i] = (float)pi[j][i]; }
#pragma unroll
            for (int i = 0; i < NU; ++i) hb[k * SW + 2 * NS + i] = (k < N) ? (float)u[j][i] : 0.0f;
        }
        STAMP_STORE(0);
        if (lane == 0) {
            a.exitflag[inst] = flag;
            a.hand_it[inst] = it;
        }
        return;
    }
    real fv = 0.0;
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
        BQP_HK(k);
        real v[NV];
#pragma unroll
        for (int i = 0; i < NS; ++i) v[i] = s[j][i];
#pragma unroll
        for (int i = 0; i < NU; ++i) v[NS + i] = (k < N) ? u[j][i] : 0.0;
#pragma unroll
        for (int i = 0; i < NV; ++i) {
            real hv = 0.0;
#pragma unroll
            for (int c = 0; c < NV; ++c) hv += BQP_HV(i * NV + c) * v[c];
            fv += v[i] * (0.5 * hv + gterm(k, i));
        }
        if (a.pi_out && k >= 1 && !pi_kept) {
            double* po = a.pi_out + ((int64_t)inst * N + (k - 1)) * NX;
#pragma unroll
            for (int i = 0; i < NX; ++i) po[i] = pi[j][i];
        }
    }
    fv = wsum(fv);
    STAMP_STORE(0);
    if (lane == 0) {
        if (a.fval) a.fval[inst] = fv;
        a.exitflag[inst] = flag;
        if (a.stats) {
            double* so = a.stats + (int64_t)inst * STATS_W;
            so[0] = (double)(it + it0); so[1] = stat; so[2] = feas; so[3] = mu; so[4] = feq; so[5] = fin;
            so[6] = polished;
        }
    }
}

#undef BQP_HK
#undef BQP_HV

// ==========================================================================================
// row wave
// ==========================================================================================
template <int NX, int NU, int NP, int BPL, int RPL, bool POL>
__device__ __forceinline__ void row_wave(const OcpKernelArgs& a, real* W, const QpLds& L,
                                         const real* Fs, const real* Sh, int lane, int inst) {
    constexpr bool PC = POL && BQP_POLISH && !BQP_EXP_NOROW;
    constexpr int NS = NX + NP;
    constexpr int NV = NS + NU;
    constexpr int NB = NX + NU;          // box slots per stage: x then u, each [upper, lower]
    const int N = a.N, mp = a.mp, kp = a.kp;
    constexpr int mpad = RPL * WAVE;     // polytope table stride (host sets a.mpad to the same)
    real* X = W + L.xch;
    STAMP_DECL;
    constexpr bool LNG = BQP_LNG_OK && BPL >= 16;    // long-horizon layout (QpLds lng)
    const bool bndsh = LNG && a.sh_bnd >= 0;         // box bounds in the shared tables
    const real* bndp = bndsh ? Sh + a.sh_bnd : W + L.bnd;

    // ---------------- box rows over all stages, spread over every lane of the wave: bounds to
    //                  LDS, presence mask.  Box variable vi = k NB + sl (stage k, slot sl: x then
    //                  u) has rows r = 2 vi + h (h = 0 upper, 1 lower); lane l holds variables
    //                  vi = l + 64 p in slots b = 2 p + h, both rows of a variable in one lane ----
    constexpr int NBR2 = 2 * NB;
    const int nbr = (N + 1) * NBR2;         // r < nbr  <=>  vi < (N + 1) NB
    // per row a 16-bit code, two per register: (LDS offset of the variable in xs / xu) << 2 |
    // is_x << 1 | h
    unsigned bpk[(BPL + 1) / 2];
#pragma unroll
    for (int b = 0; b < (BPL + 1) / 2; ++b) bpk[b] = 0;
    // LDS offset of each box variable's entry of the per-stage diagonal D (L.Dx), 16 bits per
    // variable pv: the row passes read it instead of re-deriving k, sl from the lane (the derived
    // indices were hoisted and carried through the loop, the row wave's scratch spills)
    unsigned dxk[(BPL / 2 + 1) / 2];
#pragma unroll
    for (int i = 0; i < (BPL / 2 + 1) / 2; ++i) dxk[i] = 0;
#pragma unroll
    for (int pv = 0; pv < BPL / 2; ++pv) {
        const int vi = lane + WAVE * pv, k = vi / NB, sl = vi - k * NB;
        const unsigned off = (unsigned)(L.Dx + k * NV + (sl < NX ? sl : NS + (sl - NX)));
        dxk[pv >> 1] |= (off & 0xffffu) << (16 * (pv & 1));
    }
    auto dx_off = [&](int pv) __attribute__((always_inline)) -> int {
        return (int)((dxk[pv >> 1] >> (16 * (pv & 1))) & 0xffffu);
    };
    // lanes NV .. NV + NT - 1 of the transposed F'DF sum hold upper-triangle entry lane - NV =
    // (i2, j2): its two LDS offsets in L.FD, packed (one register instead of two carried indices)
    unsigned fdk = 0;
    {
        constexpr int NTF = NV * (NV + 1) / 2;
        const int idx = lane - NV;
        if (idx >= 0 && idx < NTF) {
            int i2 = 0, st = 0;
#pragma unroll
            for (int r = 1; r < NV; ++r) {
                const int sr = r * NV - r * (r - 1) / 2;
                if (idx >= sr) { i2 = r; st = sr; }
            }
            const int j2 = i2 + (idx - st);
            fdk = (unsigned)(L.FD + i2 * NV + j2) | ((unsigned)(L.FD + j2 * NV + i2) << 16);
        }
    }
    auto fd_off = [&](int h) __attribute__((always_inline)) -> int {
        unsigned k = fdk;
        asm volatile("" : "+v"(k));     // formed at the use (hoisted, the offsets were spilled)
        return (int)((k >> (16 * h)) & 0xffffu);
    };
    unsigned bmsk = 0, binr = 0;         // present rows; rows in range (r < nbr)
    real bsl = 0.0, mcount = 0.0;
#pragma unroll
    for (int b = 0; b < BPL; ++b) {
        ROW_FENCE(b);
        const int vi = lane + WAVE * (b >> 1), h = b & 1, r = 2 * vi + h;
        const int k = vi / NB, sl = vi - k * NB;
        const bool isx = sl < NX;
        const unsigned code = ((isx ? k * NS + sl : k * NU + (sl - NX)) << 2) | (isx ? 2 : 0) | h;
        bpk[b >> 1] |= (code & 0xffffu) << (16 * (b & 1));
        real bd = h ? -INFINITY : INFINITY;
        if (r < nbr) {
            binr |= 1u << b;
            if (isx) {
                const double* xb = h ? a.xlb : a.xub;
                if (k > 0 && xb) bd = xb[(int64_t)inst * a.sxb + (int64_t)k * NX + sl];
            } else {
                const double* ub_ = h ? a.ulb : a.uub;
                if (k < N && ub_) bd = ub_[(int64_t)inst * a.sub + (int64_t)k * NU + (sl - NX)];
            }
            if (isfinite(bd)) { bmsk |= 1u << b; bsl = fmax(bsl, fabs(bd)); }
            if (!bndsh) W[L.bnd + r] = bd;
        }
    }
    mcount += __builtin_popcount(bmsk);
    // theta entries of the per-stage diagonal D never change
    for (int k = lane; k <= N; k += WAVE) {
#pragma unroll
        for (int i = NX; i < NS; ++i) W[L.Dx + k * NV + i] = 0.0;
    }
    auto bpres = [&](int b) __attribute__((always_inline)) -> bool { return (bmsk >> b) & 1u; };
    auto brow = [&](int b) __attribute__((always_inline)) -> int { return 2 * (lane + WAVE * (b >> 1)) + (b & 1); };
    auto bcode = [&](int b) __attribute__((always_inline)) -> int { return (int)((bpk[b >> 1] >> (16 * (b & 1))) & 0xffffu); };
    auto binrange = [&](int b) __attribute__((always_inline)) -> bool { return (binr >> b) & 1u; };
    // polytope rows l, l+64, ...
    const bool hpsh = a.sh_hp >= 0;                  // polytope rhs in the shared tables
    real* hpi = hpsh ? const_cast<real*>(Sh) + a.sh_hp : W + L.hp;
    if (!hpsh) {
        const double* hg = a.hp + (int64_t)inst * a.shp;
        for (int r = lane; r < mp; r += WAVE) hpi[r] = hg[r];
    }
    wave_sync();
    auto prow = [&](int q) __attribute__((always_inline)) -> bool { return lane + WAVE * q < mp; };
#pragma unroll
    for (int q = 0; q < RPL; ++q)
        if (prow(q)) { mcount += 1.0; bsl = fmax(bsl, fabs(hpi[lane + WAVE * q])); }
    mcount = wsum(mcount);
    bsl = wmax(bsl);
    if (lane == 0) { X[X_CNT] = mcount; X[X_BSR] = bsl; }
    const real minv = 1.0 / fmax(mcount, 1.0);
    auto fdot = [&](int r, const real (&v)[NV]) __attribute__((always_inline)) -> real {
        real acc = 0.0;
#pragma unroll
        for (int c = 0; c < NV; ++c) acc += Fs[c * mpad + r] * v[c];
        return acc;
    };
    auto load_v = [&](real (&v)[NV], int bs, int bu) __attribute__((always_inline)) {
#pragma unroll
        for (int c = 0; c < NS; ++c) v[c] = W[bs + kp * NS + c];
#pragma unroll
        for (int c = 0; c < NU; ++c) v[NS + c] = (kp < N) ? W[bu + kp * NU + c] : 0.0;
    };

    // row state: slack t, multiplier lam, 1/t; polytope rows also their residual ri (box-row
    // residuals are re-formed from the LDS stage vector and bounds when needed)
    real tx[BPL], lx[BPL];
    real tp[RPL], lp[RPL];
    // polytope row residuals: in LDS (L.rp) for the short horizons - fewer registers carried
    // through the loop (the row wave's scratch spills of round 3); in registers for the long
    // horizons, whose LDS holds two instances per workgroup only without them (and whose
    // 512-register budget has room)
    real rpr[LNG ? RPL : 1];
    auto rp_ref = [&](int q) __attribute__((always_inline)) -> real& {
        if constexpr (LNG) return rpr[q];
        else return W[L.rp + lane + WAVE * q];
    };
#define RP(q) rp_ref(q)
    // 1: the corrector carries Mehrotra's second-order term dt_a dlam_a; 0: this iteration's
    // predictor step was short on a feasible iterate, the corrector is a pure centring step
    real socf = 1.0;
    auto prp_get = [&](int q, int r) __attribute__((always_inline)) -> real {
        (void)q;
        return socf * W[L.prp + r];
    };
#pragma unroll
    for (int b = 0; b < BPL; ++b) { tx[b] = 1.0; lx[b] = 1.0; }
#pragma unroll
    for (int q = 0; q < RPL; ++q) { tp[q] = 1.0; lp[q] = 1.0; RP(q) = 0.0; }

    // ---- multiplier-side tables (depend on t, lam only): box multipliers, Fp'lam, 1/t,
    //      D = lam/t per stage, F'DF, sum t.lam ----
    auto lam_side = [&]() __attribute__((always_inline)) {
        real cs = 0.0, cm = 0.0;
#pragma unroll
        for (int pv = 0; pv < BPL / 2; ++pv) {
            ROW_FENCE(pv);
            // D of the variable: upper then lower row (both in this lane)
            real d = 0.0, blv = 0.0;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int b = 2 * pv + h;
                if (bpres(b)) {
                    d += lx[b] * frcp(tx[b]);
                    cs += tx[b] * lx[b];
                    if constexpr (BQP_POLISH) cm = fmax(cm, tx[b] * lx[b]);
                }
                if constexpr (LNG) {
                    if (bpres(b)) blv += h ? -lx[b] : lx[b];
                } else {
                    if (binrange(b)) W[L.blam + brow(b)] = bpres(b) ? lx[b] : 0.0;
                }
            }
            if constexpr (LNG) {
                if (binrange(2 * pv)) W[L.blam + lane + WAVE * pv] = blv;   // [upper] - [lower]
            }
            if (binrange(2 * pv)) W[dx_off(pv)] = d;
        }
        real gpp[NV];
        real fd[NV * (NV + 1) / 2];
#pragma unroll
        for (int c = 0; c < NV; ++c) gpp[c] = 0.0;
#pragma unroll
        for (int c = 0; c < NV * (NV + 1) / 2; ++c) fd[c] = 0.0;
#pragma unroll
        for (int q = 0; q < RPL; ++q) {
            ROW_FENCE(q);
            const int r = lane + WAVE * q;
            if (r < mp) {
                real f[NV];
#pragma unroll
                for (int c = 0; c < NV; ++c) f[c] = Fs[c * mpad + r];
#pragma unroll
                for (int c = 0; c < NV; ++c) gpp[c] += f[c] * lp[q];
                cs += tp[q] * lp[q];
                if constexpr (BQP_POLISH) cm = fmax(cm, tp[q] * lp[q]);
                const real d = lp[q] * frcp(tp[q]);
                int idx = 0;
#pragma unroll
                for (int i2 = 0; i2 < NV; ++i2) {
                    const real di = d * f[i2];
#pragma unroll
                    for (int j2 = i2; j2 < NV; ++j2) fd[idx++] += di * f[j2];
                }
            }
        }
        // one transposed reduction of [F'lam (NV), F'DF upper triangle, sum t.lam]: lane l < 32
        // ends with the total of value l and writes it where the stage wave reads it
        constexpr int NT = NV * (NV + 1) / 2;
        real red[NV + NT + 1];
#pragma unroll
        for (int c = 0; c < NV; ++c) red[c] = gpp[c];
#pragma unroll
        for (int c = 0; c < NT; ++c) red[NV + c] = fd[c];
        red[NV + NT] = cs;
        const real tot = wsum_t(red, lane);
        if (lane < NV) {
            W[L.gpp + lane] = tot;
        } else if (lane < NV + NT) {
            // upper-triangle index -> (i2, j2), rows of length NV, NV-1, ...
            W[fd_off(0)] = tot;
            W[fd_off(1)] = tot;
        } else if (lane == NV + NT) {
            X[X_CS] = tot;
        }
        if constexpr (BQP_POLISH) {
            cm = wmax(cm);                                // per-row complementarity (stop test)
            if (lane == 0) X[X_CMAX] = cm;
        }
    };

    // box-row residual of the current iterate: v + t - ub (upper), -v + t + lb (lower); the
    // stage vector in LDS is the iterate's until the stage wave writes the next one (after B6)
    auto bvar = [&](int b, int bs, int bu) __attribute__((always_inline)) -> real {
        const int c = bcode(b);
        return W[((c & 2) ? bs : bu) + (c >> 2)];
    };
    auto box_res = [&](int b) __attribute__((always_inline)) -> real {
        const real v = bvar(b, L.xs, L.xu);
        const real bd = bndp[brow(b)];
        return (bcode(b) & 1) == 0 ? v + tx[b] - bd : -v + tx[b] + bd;
    };
    // ---- row residuals of the current iterate (box: +-v + t -+ b; polytope: Fp v + t - hp) ----
    auto row_residuals = [&]() __attribute__((always_inline)) {
        real fe = 0.0;
#pragma unroll
        for (int b = 0; b < BPL; ++b)
            if (bpres(b)) fe = fmax(fe, fabs(box_res(b)));
        real vp[NV];
        load_v(vp, L.xs, L.xu);
#pragma unroll
        for (int q = 0; q < RPL; ++q) {
            ROW_FENCE(q);
            const int r = lane + WAVE * q;
            if (r < mp) {
                const real ri = fdot(r, vp) + tp[q] - hpi[r];
                RP(q) = ri;
                fe = fmax(fe, fabs(ri));
            }
        }
        fe = wmax(fe);
        if (lane == 0) X[X_FEASB] = fe;
    };

    // complementarity right-hand side of a row: predictor t*lam, corrector + dt_a*dlam_a - sigma*mu
    auto rcv = [&](real t, real l, real pr, bool corr, real smu) __attribute__((always_inline)) -> real {
        return corr ? t * l + pr - smu : t * l;
    };
    // box-row step dt = -ri - (+-dv) along the direction (ids, idu)
    auto box_dir = [&](int b, int ids, int idu) __attribute__((always_inline)) -> real {
        const real dv = bvar(b, ids, idu);
        return -box_res(b) - ((bcode(b) & 1) == 0 ? dv : -dv);
    };
    // box-row predictor product dt_a * dlam_a (recomputed from the predictor direction)
    auto box_pred_raw = [&](int b) __attribute__((always_inline)) -> real {
        const real dt = box_dir(b, L.dsv, L.duv);
        const real dl = (-(tx[b] * lx[b]) - lx[b] * dt) * frcp(tx[b]);
        return dt * dl;
    };
    auto box_pred_prod = [&](int b) __attribute__((always_inline)) -> real {
        return socf * box_pred_raw(b);
    };

    // ---- right-hand-side terms (lam o ri - rc)/t: box [upper, lower] per stage, Fp'e ----
    auto rhs_terms = [&](bool corr, real smu) __attribute__((always_inline)) {
        real eacc = 0.0;
#pragma unroll
        for (int b = 0; b < BPL; ++b) {
            ROW_FENCE(b);
            if (!binrange(b)) continue;
            real e = 0.0;
            if (bpres(b)) {
                const real pr = corr ? box_pred_prod(b) : 0.0;
                e = (lx[b] * box_res(b) - rcv(tx[b], lx[b], pr, corr, smu)) * frcp(tx[b]);
            }
            if constexpr (LNG) {
                if ((b & 1) == 0) eacc = e;
                else W[L.ebox + lane + WAVE * (b >> 1)] = eacc - e;   // [upper] - [lower]
            } else {
                W[L.ebox + brow(b)] = e;
            }
        }
        real gpe[NV];
#pragma unroll
        for (int c = 0; c < NV; ++c) gpe[c] = 0.0;
#pragma unroll
        for (int q = 0; q < RPL; ++q) {
            ROW_FENCE(q);
            const int r = lane + WAVE * q;
            if (r < mp) {
                const real pr = corr ? prp_get(q, r) : 0.0;
                const real e = (lp[q] * RP(q) - rcv(tp[q], lp[q], pr, corr, smu)) * frcp(tp[q]);
#pragma unroll
                for (int c = 0; c < NV; ++c) gpe[c] += Fs[c * mpad + r] * e;
            }
        }
        const real tot = wsum_t(gpe, lane);           // lane c < NV: Fp'e (c)
        if (lane < NV) W[L.gpe + lane] = tot;
    };

    // ---- row passes along the direction (ids, idu): dt = -ri - C dv, dlam = (-rc - lam dt)/t.
    //      mode 0: ratio max(-dt/t, -dlam/lam); 2: apply t += al dt, lam += al dlam (the
    //      starting point; the iterations use pred_pass / box_apply / poly_apply_lam) ----
    auto row_pass = [&](int mode, bool corr, real smu, real al, int ids, int idu) __attribute__((always_inline)) -> real {
        real acc = 0.0;
#pragma unroll
        for (int b = 0; b < BPL; ++b) {
            ROW_FENCE(b);
            if (!bpres(b)) continue;
            const real pr = corr ? box_pred_prod(b) : 0.0;
            const real rc = rcv(tx[b], lx[b], pr, corr, smu);
            const real dt = box_dir(b, ids, idu);
            const real dl = (-rc - lx[b] * dt) * frcp(tx[b]);
            if (mode == 0) {
                acc = fmax(acc, -dt * frcp(tx[b]));
                acc = fmax(acc, -dl * frcp(lx[b]));
            } else {
                // residual of the stepped iterate: r + al (+-dv + dt) = (1 - al) r
                acc = fmax(acc, fabs((1.0 - al) * box_res(b)));
                tx[b] += al * dt;
                lx[b] += al * dl;
            }
        }
        real dvp[NV];
        load_v(dvp, ids, idu);
#pragma unroll
        for (int q = 0; q < RPL; ++q) {
            ROW_FENCE(q);
            const int r = lane + WAVE * q;
            if (r >= mp) continue;
            const real pr = corr ? prp_get(q, r) : 0.0;
            const real rc = rcv(tp[q], lp[q], pr, corr, smu);
            const real fd = fdot(r, dvp);
            const real dt = -RP(q) - fd;
            const real dl = (-rc - lp[q] * dt) * frcp(tp[q]);
            if (mode == 0) {
                acc = fmax(acc, -dt * frcp(tp[q]));
                acc = fmax(acc, -dl * frcp(lp[q]));
            } else {
                // the polytope residual Fp v + t - hp of the stepped iterate, by the linear
                // update r + al (Fp dv + dt): the next iteration needs no residual pass (and
                // no barrier) before its factorisation
                RP(q) += al * (fd + dt);
                acc = fmax(acc, fabs(RP(q)));
                tp[q] += al * dt;
                lp[q] += al * dl;
            }
        }
        return wmax(acc);   // mode 0: max ratio; mode 2: max |row residual| after the step
    };

    // ---- predictor pass: the ratio test, the complementarity sum and the corrector terms in ONE pass over the
    //      rows.  Along the affine direction t dlam + lam dt = -t lam, so the complementarity
    //      after any step a is  sum (t + a dt)(lam + a dlam) = S0 (1 - a) + a^2 S2  with
    //      S0 = sum t lam (X_CS) and S2 = sum dt dlam: the sum no longer needs the step length,
    //      and the pass returns the lane partials of max(-dt/t, -dlam/lam) and S2 ----
    auto pred_pass = [&](real& rmx, real (&gpe0)[NV], real (&gpi)[NV]) __attribute__((always_inline)) -> real {
        real rm = 0.0, s2 = 0.0, eacc = 0.0;
#pragma unroll
        for (int b = 0; b < BPL; ++b) {
            ROW_FENCE(b);
            if (!binrange(b)) continue;
            real e0 = 0.0;
            if (bpres(b)) {
                const real t = tx[b], l = lx[b];
                const real it = frcp(t);
                const real rc = t * l;
                const real dt = box_dir(b, L.dsv, L.duv);
                const real dl = (-rc - l * dt) * it;
                rm = fmax(rm, -dt * it);
                rm = fmax(rm, -dl * frcp(l));
                const real pr = dt * dl;
                s2 += pr;
                e0 = (l * box_res(b) - (rc + pr)) * it;
            }
            if constexpr (LNG) {
                if ((b & 1) == 0) eacc = e0;
                else W[L.ebox + lane + WAVE * (b >> 1)] = eacc - e0;
            } else {
                W[L.ebox + brow(b)] = e0;
            }
        }
#pragma unroll
        for (int c = 0; c < NV; ++c) { gpe0[c] = 0.0; gpi[c] = 0.0; }
        real dvp[NV];
        load_v(dvp, L.dsv, L.duv);
#pragma unroll
        for (int q = 0; q < RPL; ++q) {
            ROW_FENCE(q);
            const int r = lane + WAVE * q;
            if (r >= mp) continue;
            real f[NV];
#pragma unroll
            for (int c = 0; c < NV; ++c) f[c] = Fs[c * mpad + r];
            real fd = 0.0;
#pragma unroll
            for (int c = 0; c < NV; ++c) fd += f[c] * dvp[c];
            const real t = tp[q], l = lp[q];
            const real it = frcp(t);
            const real rc = t * l;
            const real dt = -RP(q) - fd;
            const real dl = (-rc - l * dt) * it;
            rm = fmax(rm, -dt * it);
            rm = fmax(rm, -dl * frcp(l));
            const real pr = dt * dl;
            s2 += pr;
            W[L.prp + r] = pr;
            const real e0 = (l * RP(q) - (rc + pr)) * it;
#pragma unroll
            for (int c = 0; c < NV; ++c) { gpe0[c] += f[c] * e0; gpi[c] += f[c] * it; }
        }
        rmx = rm;
        return s2;
    };

    // ---- corrector step, box rows (before B6, while the stage vector in LDS is still the
    //      current iterate's): t += a dt, lam += a dlam; returns max |(1 - a) r| ----
    auto box_apply = [&](real smu, real al) __attribute__((always_inline)) -> real {
        real fe = 0.0;
#pragma unroll
        for (int b = 0; b < BPL; ++b) {
            ROW_FENCE(b);
            if (!bpres(b)) continue;
            const real pr = box_pred_prod(b);
            const real rc = rcv(tx[b], lx[b], pr, true, smu);
            const real dt = box_dir(b, L.dsc, L.duc);
            const real dl = (-rc - lx[b] * dt) * frcp(tx[b]);
            fe = fmax(fe, fabs((1.0 - al) * box_res(b)));
            tx[b] += al * dt;
            lx[b] += al * dl;
        }
        return fe;
    };

    // ---- corrector step of the polytope rows fused with the multiplier-side tables of the
    //      new iterate (after B6, alongside the stage wave's update; every row reads its Fp
    //      entries once for both): residual by the linear update r + a (Fp dv + dt), t, lam,
    //      then Fp'lam, F'DF, sum t.lam exactly as lam_side; feb = the box rows' residual norm ----
    auto poly_apply_lam = [&](real smu, real al, real feb) __attribute__((always_inline)) {
        real cs = 0.0, cm = 0.0;
#pragma unroll
        for (int pv = 0; pv < BPL / 2; ++pv) {
            ROW_FENCE(pv);
            real d = 0.0, blv = 0.0;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int b = 2 * pv + h;
                if (bpres(b)) {
                    d += lx[b] * frcp(tx[b]);
                    cs += tx[b] * lx[b];
                    if constexpr (BQP_POLISH) cm = fmax(cm, tx[b] * lx[b]);
                }
                if constexpr (LNG) {
                    if (bpres(b)) blv += h ? -lx[b] : lx[b];
                } else {
                    if (binrange(b)) W[L.blam + brow(b)] = bpres(b) ? lx[b] : 0.0;
                }
            }
            if constexpr (LNG) {
                if (binrange(2 * pv)) W[L.blam + lane + WAVE * pv] = blv;   // [upper] - [lower]
            }
            if (binrange(2 * pv)) W[dx_off(pv)] = d;
        }
        real gpp[NV];
        real fdt[NV * (NV + 1) / 2];
#pragma unroll
        for (int c = 0; c < NV; ++c) gpp[c] = 0.0;
#pragma unroll
        for (int c = 0; c < NV * (NV + 1) / 2; ++c) fdt[c] = 0.0;
        real fe = feb;
        real dvp[NV];
        load_v(dvp, L.dsc, L.duc);
#pragma unroll
        for (int q = 0; q < RPL; ++q) {
            ROW_FENCE(q);
            const int r = lane + WAVE * q;
            if (r < mp) {
                real f[NV];
#pragma unroll
                for (int c = 0; c < NV; ++c) f[c] = Fs[c * mpad + r];
                real fd = 0.0;
#pragma unroll
                for (int c = 0; c < NV; ++c) fd += f[c] * dvp[c];
                const real rc = rcv(tp[q], lp[q], prp_get(q, r), true, smu);
                const real dt = -RP(q) - fd;
                const real dl = (-rc - lp[q] * dt) * frcp(tp[q]);
                RP(q) += al * (fd + dt);
                fe = fmax(fe, fabs(RP(q)));
                tp[q] += al * dt;
                lp[q] += al * dl;
#pragma unroll
                for (int c = 0; c < NV; ++c) gpp[c] += f[c] * lp[q];
                cs += tp[q] * lp[q];
                if constexpr (BQP_POLISH) cm = fmax(cm, tp[q] * lp[q]);
                const real d = lp[q] * frcp(tp[q]);
                int idx = 0;
#pragma unroll
                for (int i2 = 0; i2 < NV; ++i2) {
                    const real di = d * f[i2];
#pragma unroll
                    for (int j2 = i2; j2 < NV; ++j2) fdt[idx++] += di * f[j2];
                }
            }
        }
        fe = wmax(fe);
        if (lane == 0) X[X_FEASB] = fe;                   // row residual norm of the new iterate
        constexpr int NT = NV * (NV + 1) / 2;
        real red[NV + NT + 1];
#pragma unroll
        for (int c = 0; c < NV; ++c) red[c] = gpp[c];
#pragma unroll
        for (int c = 0; c < NT; ++c) red[NV + c] = fdt[c];
        red[NV + NT] = cs;
        const real tot = wsum_t(red, lane);
        if (lane < NV) {
            W[L.gpp + lane] = tot;
        } else if (lane < NV + NT) {
            W[fd_off(0)] = tot;
            W[fd_off(1)] = tot;
        } else if (lane == NV + NT) {
            X[X_CS] = tot;
        }
        if constexpr (BQP_POLISH) {
            cm = wmax(cm);
            if (lane == 0) X[X_CMAX] = cm;
        }
    };

    auto rhs_corr_finish = [&](real smu, real tot) __attribute__((always_inline)) {
        if constexpr (LNG) {
#pragma unroll
            for (int pv = 0; pv < BPL / 2; ++pv) {
                real add = 0.0;
                if (bpres(2 * pv)) add += smu * frcp(tx[2 * pv]);
                if (bpres(2 * pv + 1)) add -= smu * frcp(tx[2 * pv + 1]);
                if (binrange(2 * pv)) W[L.ebox + lane + WAVE * pv] += add;
            }
        } else {
#pragma unroll
            for (int b = 0; b < BPL; ++b)
                if (bpres(b)) W[L.ebox + brow(b)] += smu * frcp(tx[b]);
        }
        // tot (from the joint reduction): lane 2c = Fp'e0 (c), lane 2c+1 = Fp'(1/t) (c)
        const real other = dpp_mov<0xB1, 0xf>(real(0), tot);
        if (lane < 2 * NV && (lane & 1) == 0) W[L.gpe + lane / 2] = tot + smu * other;
    };
    // pure centring step (socf = 0): the predictor pass formed the corrector terms with
    // dt_a dlam_a; take it back out, (lam ri - rc - pr)/t + pr/t (rare: short predictor steps)
    auto rhs_drop_soc = [&]() __attribute__((always_inline)) {
        if constexpr (LNG) {
#pragma unroll
            for (int pv = 0; pv < BPL / 2; ++pv) {
                real add = 0.0;
                if (bpres(2 * pv)) add += box_pred_raw(2 * pv) * frcp(tx[2 * pv]);
                if (bpres(2 * pv + 1)) add -= box_pred_raw(2 * pv + 1) * frcp(tx[2 * pv + 1]);
                if (binrange(2 * pv)) W[L.ebox + lane + WAVE * pv] += add;
            }
        } else {
#pragma unroll
            for (int b = 0; b < BPL; ++b)
                if (bpres(b)) W[L.ebox + brow(b)] += box_pred_raw(b) * frcp(tx[b]);
        }
        real gc[NV];
#pragma unroll
        for (int c = 0; c < NV; ++c) gc[c] = 0.0;
#pragma unroll
        for (int q = 0; q < RPL; ++q) {
            const int r = lane + WAVE * q;
            if (r >= mp) continue;
            const real e = W[L.prp + r] * frcp(tp[q]);
#pragma unroll
            for (int c = 0; c < NV; ++c) gc[c] += Fs[c * mpad + r] * e;
        }
        const real tot = wsum_t(gc, lane);
        wave_sync();
        if (lane < NV) W[L.gpe + lane] += tot;
        wave_sync();
    };

    // ======================= initial point ==================================================
    constexpr int HR_T = 0, HR_L = BPL * WAVE, HP_T = 2 * BPL * WAVE, HP_L = (2 * BPL + RPL) * WAVE;
    if (hand_warm<(BPL >= 16), POL>(a, inst)) {
        // continue the fp32 phase's iterate (mixed precision): slacks and multipliers as they
        // were, the residuals and multiplier tables formed afresh in fp64
        const float* hb = a.hand_in + (int64_t)inst * a.hand_stride + hand_rows_off(N, NS, NU);
#pragma unroll
        for (int b = 0; b < BPL; ++b) {
            tx[b] = (real)hb[HR_T + b * WAVE + lane];
            lx[b] = (real)hb[HR_L + b * WAVE + lane];
        }
#pragma unroll
        for (int q = 0; q < RPL; ++q) {
            tp[q] = (real)hb[HP_T + q * WAVE + lane];
            lp[q] = (real)hb[HP_L + q * WAVE + lane];
        }
        BARRIER();                                        // W0: the stage vectors are in LDS
        row_residuals();
        lam_side();
    } else {
    lam_side();
    BARRIER();                                            // I0
    row_residuals();
    rhs_terms(false, 0.0);
    BARRIER();                                            // I1
    BARRIER();                                            // I2: start direction in (dsv, duv)
    {
        // t~ = t + dt (t = 1) at the unit-scaled least-squares point; lam~ = -t~; shift
        row_pass(2, false, 0.0, 1.0, L.dsv, L.duv);
        real tmin = INFINITY, tmax = -INFINITY;
#pragma unroll
        for (int b = 0; b < BPL; ++b)
            if (bpres(b)) { tmin = fmin(tmin, tx[b]); tmax = fmax(tmax, tx[b]); }
#pragma unroll
        for (int q = 0; q < RPL; ++q)
            if (prow(q)) { tmin = fmin(tmin, tp[q]); tmax = fmax(tmax, tp[q]); }
        tmin = wmin(tmin);
        tmax = wmax(tmax);
        const real shp = (tmin <= 0.0) ? 1.0 - tmin : 0.0;
        const real shd = (tmax >= 0.0) ? 1.0 + tmax : 0.0;
        {
            // residuals of the shifted start: the full step zeroes them (linear rows), the
            // positivity shift of t adds shp to every present row
            real fe = 0.0;
#pragma unroll
            for (int b = 0; b < BPL; ++b)
                if (bpres(b)) fe = fmax(fe, fabs(shp));
#pragma unroll
            for (int q = 0; q < RPL; ++q)
                if (prow(q)) { RP(q) += shp; fe = fmax(fe, fabs(RP(q))); }
            fe = wmax(fe);
            if (lane == 0) X[X_FEASB] = fe;
        }
#pragma unroll
        for (int b = 0; b < BPL; ++b) {
            ROW_FENCE(b);
            const real t = tx[b];
            const bool pr = bpres(b);
            tx[b] = pr ? t + shp : 1.0;
            lx[b] = pr ? -t + shd : 0.0;
        }
#pragma unroll
        for (int q = 0; q < RPL; ++q) {
            const real t = tp[q];
            const bool pr = prow(q);
            tp[q] = pr ? t + shp : 1.0;
            lp[q] = pr ? -t + shd : 0.0;
        }
    }
    lam_side();
    BARRIER();                                            // I3
    }

    // ======================= main loop ======================================================
    for (;;) {
        BARRIER();                                        // B0
        STAMP(0);
        STAMP(1);
        rhs_terms(false, 0.0);
        STAMP(2);
        BARRIER();                                        // B2
        STAMP(3);
        if (X[X_STOP] != 0.0) break;
        BARRIER();                                        // B3: predictor direction in (dsv, duv)
        STAMP(4);
        const real cs0 = X[X_CS];
        const real mu = cs0 * minv;
        real gpe0[NV], gpi[NV], rmx;
        const real s2p = pred_pass(rmx, gpe0, gpi);
        const real rm_a = wmax(rmx);
        const real al_aff = rm_a > 1.0 ? 1.0 / rm_a : 1.0;
        // joint transposed reduction: [Fp'e0, Fp'(1/t)] interleaved, then S2
        real red[2 * NV + 1];
#pragma unroll
        for (int c = 0; c < NV; ++c) { red[2 * c] = gpe0[c]; red[2 * c + 1] = gpi[c]; }
        red[2 * NV] = s2p;
        const real tot = wsum_t(red, lane);
        const real mua = (cs0 * (1.0 - al_aff) + al_aff * al_aff * rl(tot, 2 * NV)) * minv;
        real sg = mua / mu;
        sg = sg * sg * sg;
        const real smu = sg * mu;
        rhs_corr_finish(smu, tot);
        socf = (BQP_POLISH && al_aff < SOC_ALPHA && X[X_FEASOK] != 0.0) ? 0.0 : 1.0;
        if (socf == 0.0) rhs_drop_soc();
        STAMP(5);
        BARRIER();                                        // B4
        BARRIER();                                        // B5: corrector direction in (dsc, duc)
        STAMP(6);
        const real rm = row_pass(0, true, smu, 0.0, L.dsc, L.duc);
        // step rule (oracle/cpu_ipm.c TAU_FAST): a predictor step above 0.99 on an iterate with
        // mu > 1e-6, or any predictor step of at least 0.99999 (the Newton end phase), lets the
        // corrector go to 0.99999 of the boundary, else tau.  Only at the default tau or above: a
        // caller's smaller tau (bqp_options.tau, chosen for robustness) bounds every step
        const bool fast = a.tau >= TAU_FAST_MIN &&
                          ((al_aff > real(TAU_FAST_AFF) && mu > real(TAU_FAST_MU)) || al_aff >= real(TAU_FAST_END));
        const real tau = fast ? fmax(real(a.tau), real(TAU_FAST)) : real(a.tau);
        real al = (rm > 1.0 ? 1.0 / rm : 1.0) * tau;
        if (al > 1.0) al = 1.0;
        if (lane == 0) X[X_ALPHA] = al;
        const real feb = box_apply(smu, al);
        STAMP(7);
        BARRIER();                                        // B6
        poly_apply_lam(smu, al, feb);
        STAMP(8);
    }

    // ======================= outputs (multipliers) ==========================================
    if (BQP_HAND_OUT && BPL >= 16 && a.hand_out) {
        // fp32 phase of the mixed mode: slacks and multipliers to the handoff record
        float* hb = a.hand_out + (int64_t)inst * a.hand_stride + hand_rows_off(N, NS, NU);
#pragma unroll
        for (int b = 0; b < BPL; ++b) {
            hb[HR_T + b * WAVE + lane] = (float)tx[b];
            hb[HR_L + b * WAVE + lane] = (float)lx[b];
        }
#pragma unroll
        for (int q = 0; q < RPL; ++q) {
            hb[HP_T + q * WAVE + lane] = (float)tp[q];
            hb[HP_L + q * WAVE + lane] = (float)lp[q];
        }
        STAMP_STORE(16);
        return;
    }
    // multipliers of the box rows [lower; upper] per stage and of the polytope rows
    auto out_duals = [&](const real (&lb)[BPL], const real (&lq)[RPL]) __attribute__((always_inline)) {
#pragma unroll
        for (int b = 0; b < BPL; ++b) {
            ROW_FENCE(b);
            if (!binrange(b)) continue;
            int vi = lane + WAVE * (b >> 1);
            // opaque here: the output addresses are formed after the loop, not hoisted to the
            // kernel start and carried through it (they were the row wave's scratch spills)
            asm volatile("" : "+v"(vi));
            const int h = b & 1;
            const int k = vi / NB, sl = vi - k * NB;
            const real lv = bpres(b) ? lb[b] : 0.0;      // layout per stage: [lower; upper]
            if (sl < NX) {
                if (a.lamx_out) a.lamx_out[((int64_t)inst * (N + 1) + k) * NX * 2 + (h ? sl : NX + sl)] = lv;
            } else if (k < N) {
                if (a.lamu_out) a.lamu_out[((int64_t)inst * N + k) * NU * 2 + (h ? sl - NX : NU + sl - NX)] = lv;
            }
        }
        if (a.lamp_out) {
#pragma unroll
            for (int q = 0; q < RPL; ++q) {
                const int r = lane + WAVE * q;
                if (r < mp) a.lamp_out[(int64_t)inst * mp + r] = lq[q];
            }
        }
    };

    // ======================= active-set polish (fp64): row side ==============================
    // max over rows of min(t, lam): a weakly active row keeps both ~ sqrt(mu) at the exit
    real dg = 0.0;
    if (BQP_POLISH && a.polish > 1) {
#pragma unroll
        for (int b = 0; b < BPL; ++b)
            if (bpres(b)) dg = fmax(dg, fmin(tx[b], lx[b]));
#pragma unroll
        for (int q = 0; q < RPL; ++q)
            if (prow(q)) dg = fmax(dg, fmin(tp[q], lp[q]));
        dg = wmax(dg);
    }
    if constexpr (!POL) {
        // solve kernel: instances that need the polish are marked for the repair launch
        // (ocp_polish_kernel), which solves them again and polishes; the solve kernel itself
        // carries no polish state
        if (BQP_POLISH && a.pol_need && lane == 0) {
            const int flag = (int)X[X_FLAG];
            // (2: marked by the mixed mode's cold retry launch - its repair starts cold as well)
            a.pol_need[inst] = (a.polish > 0 && flag != -2 && (flag != 1 || (a.polish > 1 && dg > DEG_POLISH)))
                                   ? (a.redo_flag ? 2 : 1) : 0;
        }
    }
    if constexpr (PC) {
        if (lane == 0) X[X_DEG] = dg;
        BARRIER();                                        // Q0
        const int flag = (int)X[X_FLAG];
        const bool dopol = a.polish > 0 && flag != -2 &&
                           (flag != 1 || (a.polish > 1 && X[X_DEG] > DEG_POLISH)) && isfinite(X[X_RHO]);
        if (dopol) {
            STAMP(15);
            // the IPM's multipliers go out now (the fall-back); the row state is dead after this
            out_duals(lx, lp);
            const real rho = X[X_RHO], tf = X[X_TF];
            const real tol14 = 0.01 * tf;                 // 1e-14 (1 + |data|)
            unsigned bact = 0, pact = 0;                 // rows taken as equalities
            real nb[BPL], npq[RPL];                       // their multipliers (0 on dropped rows)
            real lmx_r = 0.0;
#pragma unroll
            for (int b = 0; b < BPL; ++b) {
                const bool ac = bpres(b) && lx[b] > tx[b];
                if (ac) bact |= 1u << b;
                nb[b] = ac ? lx[b] : real(0);
            }
#pragma unroll
            for (int q = 0; q < RPL; ++q) {
                const bool ac = prow(q) && lp[q] > tp[q];
                if (ac) pact |= 1u << q;
                npq[q] = ac ? lp[q] : real(0);
            }
            // constraint values C v - b of the current stage vectors (t = 0), multiplier update
            // (mode 1: nu += rho (C v - b)) or active-set correction (mode 2), then the tables
            // the stage wave reads: box multipliers / diagonal / rhs terms, Fp'nu, Fp'e and
            // (modes 0, 2: a new set) F'DF; the check values to the exchange block
            auto pol_tables = [&](int mode) __attribute__((always_inline)) {
                const real td = 1e-9 * (1.0 + lmx_r);
                real va = 0.0, vio = 0.0, ln = 0.0, lm = 0.0, chg = 0.0;
#pragma unroll
                for (int pv = 0; pv < BPL / 2; ++pv) {
                    ROW_FENCE(pv);
                    real d = 0.0, blv = 0.0, ev[2] = {0.0, 0.0};
#pragma unroll
                    for (int h = 0; h < 2; ++h) {
                        const int b = 2 * pv + h;
                        if (!bpres(b)) continue;
                        const real v = bvar(b, L.xs, L.xu);
                        const real bd = bndp[brow(b)];
                        const real ri = h == 0 ? v - bd : -v + bd;
                        bool ac = (bact >> b) & 1u;
                        if (mode == 1 && ac) nb[b] += rho * ri;
                        if (mode == 2) {
                            if (ac && nb[b] < -td) { bact &= ~(1u << b); nb[b] = 0.0; ac = false; }
                            else if (!ac && ri > tf) { bact |= 1u << b; ac = true; }
                        }
                        vio = fmax(vio, ri);
                        if (ac) {
                            va = fmax(va, fabs(ri)); ln = fmin(ln, nb[b]); lm = fmax(lm, nb[b]);
                            d += rho;
                            ev[h] = rho * ri;
                        } else if (ri > tf) {
                            chg += 1.0;
                        }
                        blv += h ? -nb[b] : nb[b];
                    }
                    if constexpr (LNG) {
                        if (binrange(2 * pv)) {
                            W[L.blam + lane + WAVE * pv] = blv;
                            W[L.ebox + lane + WAVE * pv] = ev[0] - ev[1];
                        }
                    } else {
#pragma unroll
                        for (int h = 0; h < 2; ++h) {
                            const int b = 2 * pv + h;
                            if (binrange(b)) {
                                W[L.blam + brow(b)] = bpres(b) ? nb[b] : 0.0;
                                W[L.ebox + brow(b)] = ev[h];
                            }
                        }
                    }
                    if (binrange(2 * pv)) W[dx_off(pv)] = d;
                }
                real vp[NV];
                load_v(vp, L.xs, L.xu);
                constexpr int NT = NV * (NV + 1) / 2;
                real red[2 * NV], rfd[NT];                // [Fp'nu, Fp'e], F'DF (wsum_t: <= 32 values)
#pragma unroll
                for (int c = 0; c < 2 * NV; ++c) red[c] = 0.0;
#pragma unroll
                for (int c = 0; c < NT; ++c) rfd[c] = 0.0;
#pragma unroll
                for (int q = 0; q < RPL; ++q) {
                    ROW_FENCE(q);
                    const int r = lane + WAVE * q;
                    if (r >= mp) continue;
                    real f[NV];
#pragma unroll
                    for (int c = 0; c < NV; ++c) f[c] = Fs[c * mpad + r];
                    real fv = 0.0;
#pragma unroll
                    for (int c = 0; c < NV; ++c) fv += f[c] * vp[c];
                    const real ri = fv - hpi[r];
                    bool ac = (pact >> q) & 1u;
                    if (mode == 1 && ac) npq[q] += rho * ri;
                    if (mode == 2) {
                        if (ac && npq[q] < -td) { pact &= ~(1u << q); npq[q] = 0.0; ac = false; }
                        else if (!ac && ri > tf) { pact |= 1u << q; ac = true; }
                    }
                    vio = fmax(vio, ri);
                    real e = 0.0;
                    if (ac) {
                        va = fmax(va, fabs(ri)); ln = fmin(ln, npq[q]); lm = fmax(lm, npq[q]);
                        e = rho * ri;
                    } else if (ri > tf) {
                        chg += 1.0;
                    }
#pragma unroll
                    for (int c = 0; c < NV; ++c) { red[c] += f[c] * npq[q]; red[NV + c] += f[c] * e; }
                    if (mode != 1 && ac) {
                        int idx = 0;
#pragma unroll
                        for (int i2 = 0; i2 < NV; ++i2) {
                            const real di = rho * f[i2];
#pragma unroll
                            for (int j2 = i2; j2 < NV; ++j2) rfd[idx++] += di * f[j2];
                        }
                    }
                }
                // Fp'nu, Fp'e (and, for a new set, F'DF) by transposed wave sums
                {
                    const real tot = wsum_t(red, lane);
                    if (lane < NV) W[L.gpp + lane] = tot;
                    else if (lane < 2 * NV) W[L.gpe + lane - NV] = tot;
                }
                if (mode != 1) {
                    const real tot = wsum_t(rfd, lane);
                    if (lane < NT) {
                        const int idx = lane;
                        int i2 = 0, st = 0;
#pragma unroll
                        for (int r = 1; r < NV; ++r) {
                            const int sr = r * NV - r * (r - 1) / 2;
                            if (idx >= sr) { i2 = r; st = sr; }
                        }
                        const int j2 = i2 + (idx - st);
                        W[L.FD + i2 * NV + j2] = tot;
                        W[L.FD + j2 * NV + i2] = tot;
                    }
                }
                va = wmax(va); vio = wmax(vio); lm = wmax(lm); ln = wmin(ln);
                // rows a correction would move: violated dropped rows (counted above) and
                // active rows whose multiplier is negative beyond this point's tolerance
                const real tdn = 1e-9 * (1.0 + lm);
#pragma unroll
                for (int b = 0; b < BPL; ++b)
                    if (((bact >> b) & 1u) && nb[b] < -tdn) chg += 1.0;
#pragma unroll
                for (int q = 0; q < RPL; ++q)
                    if (((pact >> q) & 1u) && npq[q] < -tdn) chg += 1.0;
                chg = wsum(chg);
                lmx_r = lm;
                if (lane == 0) {
                    X[X_PVA] = va; X[X_PVIOL] = vio; X[X_PLNEG] = ln; X[X_PLMX] = lm; X[X_PCHG] = chg;
                }
                wave_sync();
            };
            // conjugate gradients on the multipliers of the active rows (oracle/cpu_ipm.c
            // polish()): residual r = C v - b and direction p per active row, 0 elsewhere
            real crb[BPL], cpb[BPL], crq[RPL], cpq[RPL];
            real rr = 0.0, va_prev = INFINITY;
            // the direction solve's tables: e = p on the active rows (box rhs terms, Fp'p)
            auto dir_tables = [&]() __attribute__((always_inline)) {
#pragma unroll
                for (int pv = 0; pv < BPL / 2; ++pv) {
                    if (!binrange(2 * pv)) continue;
                    if constexpr (LNG) {
                        W[L.ebox + lane + WAVE * pv] = cpb[2 * pv] - cpb[2 * pv + 1];
                    } else {
#pragma unroll
                        for (int h = 0; h < 2; ++h) W[L.ebox + brow(2 * pv + h)] = cpb[2 * pv + h];
                    }
                }
                real red[NV];
#pragma unroll
                for (int c = 0; c < NV; ++c) red[c] = 0.0;
#pragma unroll
                for (int q = 0; q < RPL; ++q) {
                    const int r = lane + WAVE * q;
                    if (r >= mp) continue;
#pragma unroll
                    for (int c = 0; c < NV; ++c) red[c] += Fs[c * mpad + r] * cpq[q];
                }
                const real tot = wsum_t(red, lane);
                if (lane < NV) W[L.gpe + lane] = tot;
            };
            // active-row constraint values of the stage vectors in LDS: max |C v - b|
            auto act_res = [&](bool keep) __attribute__((always_inline)) -> real {
                real va = 0.0;
#pragma unroll
                for (int b = 0; b < BPL; ++b) {
                    real ri = 0.0;
                    if ((bact >> b) & 1u) {
                        const real v = bvar(b, L.xs, L.xu);
                        const real bd = bndp[brow(b)];
                        ri = (b & 1) == 0 ? v - bd : -v + bd;
                    }
                    if (keep) crb[b] = ri;
                    va = fmax(va, fabs(ri));
                }
                real vp[NV];
                load_v(vp, L.xs, L.xu);
#pragma unroll
                for (int q = 0; q < RPL; ++q) {
                    const int r = lane + WAVE * q;
                    real ri = 0.0;
                    if (((pact >> q) & 1u) && r < mp) ri = fdot(r, vp) - hpi[r];
                    if (keep) crq[q] = ri;
                    va = fmax(va, fabs(ri));
                }
                return wmax(va);
            };
            int mode = 0;
            for (;;) {
                BARRIER();                                // T0
                pol_tables(mode);
                BARRIER();                                // T1
                BARRIER();                                // T2
                const int dec = (int)X[X_PDEC];
                if (dec == 1) {
#pragma unroll
                    for (int b = 0; b < BPL; ++b) nb[b] = fmax(nb[b], real(0));
#pragma unroll
                    for (int q = 0; q < RPL; ++q) npq[q] = fmax(npq[q], real(0));
                    out_duals(nb, npq);
                    break;
                }
                if (dec == 3) break;
                if (dec == 2) { mode = 2; continue; }
                BARRIER();                                // T3: v after the AL step
                {
                    // CG start: r = p = C v - b on the active rows
                    real va = act_res(true), pr = 0.0;
#pragma unroll
                    for (int b = 0; b < BPL; ++b) { cpb[b] = crb[b]; pr += crb[b] * crb[b]; }
#pragma unroll
                    for (int q = 0; q < RPL; ++q) { cpq[q] = crq[q]; pr += crq[q] * crq[q]; }
                    rr = wsum(pr);
                    va_prev = INFINITY;
                    dir_tables();
                    if (lane == 0) X[X_CGD] = (va > tol14 && isfinite(rr) && POL_CG > 0) ? 0.0 : 2.0;
                }
                BARRIER();                                // T4
                for (int j = 0;; ++j) {
                    const int cgd = (int)X[X_CGD];
                    if (cgd == 2) break;
                    if (cgd == 0) {
                        BARRIER();                        // T5: direction in (dsc, duc)
                        // M p = -C dv on the active rows; alpha = r'r / p'Mp
                        real mpb[BPL], mpq[RPL];
                        real pq = 0.0, pp = 0.0;
#pragma unroll
                        for (int b = 0; b < BPL; ++b) {
                            real c = 0.0;
                            if ((bact >> b) & 1u) {
                                const real dv = bvar(b, L.dsc, L.duc);
                                c = (b & 1) ? dv : -dv;
                            }
                            mpb[b] = c;
                            pq += cpb[b] * c; pp += cpb[b] * cpb[b];
                        }
                        real dvp[NV];
                        load_v(dvp, L.dsc, L.duc);
#pragma unroll
                        for (int q = 0; q < RPL; ++q) {
                            const int r = lane + WAVE * q;
                            real c = 0.0;
                            if (((pact >> q) & 1u) && r < mp) c = -fdot(r, dvp);
                            mpq[q] = c;
                            pq += cpq[q] * c; pp += cpq[q] * cpq[q];
                        }
                        real red2[2] = {pq, pp};
                        const real t2 = wsum_t(red2, lane);
                        pq = rl(t2, 0); pp = rl(t2, 1);
                        real al = 0.0, va = INFINITY;
                        int nxt;
                        if (!(pq * rho > POL_CG_SING * pp)) {
                            // numerically singular direction (nearly dependent active rows):
                            // plain multiplier steps from here
                            nxt = (j + 1 < POL_CG) ? 1 : 2;
                        } else {
                            al = rr / pq;
                            real rn = 0.0;
                            va = 0.0;
#pragma unroll
                            for (int b = 0; b < BPL; ++b) {
                                nb[b] += al * cpb[b];
                                crb[b] -= al * mpb[b];
                                rn += crb[b] * crb[b]; va = fmax(va, fabs(crb[b]));
                            }
#pragma unroll
                            for (int q = 0; q < RPL; ++q) {
                                npq[q] += al * cpq[q];
                                crq[q] -= al * mpq[q];
                                rn += crq[q] * crq[q]; va = fmax(va, fabs(crq[q]));
                            }
                            rn = wsum(rn);
                            va = wmax(va);
                            const real be = rn / rr;
#pragma unroll
                            for (int b = 0; b < BPL; ++b) cpb[b] = crb[b] + be * cpb[b];
#pragma unroll
                            for (int q = 0; q < RPL; ++q) cpq[q] = crq[q] + be * cpq[q];
                            rr = rn;
                            dir_tables();
                            nxt = (j + 1 < POL_CG && va > tol14 && isfinite(rr)) ? 0 : 2;
                        }
                        if (lane == 0) { X[X_ALPHA] = al; X[X_CGD] = (real)nxt; }
                        BARRIER();                        // T6
                    } else {
                        BARRIER();                        // T7: v, partial residuals
                        pol_tables(1);
                        BARRIER();                        // T8
                        BARRIER();                        // T9: v after the AL step
                        const real va = act_res(false);
                        const int nxt = (va >= POL_STAG * va_prev) ? 2 : ((j + 1 < POL_CG && va > tol14) ? 1 : 2);
                        va_prev = va;
                        if (lane == 0) X[X_CGD] = (real)nxt;
                        BARRIER();                        // T10
                    }
                }
                mode = 1;
            }
            STAMP_STORE(16);
            return;
        }
    }
    out_duals(lx, lp);

    STAMP_STORE(16);
}
#undef RP

// ==========================================================================================
// kernel: QPB instances per workgroup, waves [0, QPB) stage waves, [QPB, 2 QPB) row waves
// ==========================================================================================
template <int NX, int NU, int NP, int SPL, int RPL, int BPL, bool POL, bool QUEUE>
__device__ __forceinline__ void ocp_body(const OcpKernelArgs& a) {
    constexpr int NS = NX + NP;
    constexpr int NV = NS + NU;
    extern __shared__ __attribute__((aligned(16))) unsigned char lds_raw[];
    real* lds = reinterpret_cast<real*>(lds_raw);
    const int N = a.N;
    const int lane_k = threadIdx.x & 63;
    const int wid = QUEUE ? __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) : (threadIdx.x >> 6);
    const int qpb = a.wpb;
    if constexpr (POL) {
        // repair launch: a workgroup none of whose instances the solve launch marked leaves
        // before staging the shared tables
        const int i0 = blockIdx.x * a.wpb + ((threadIdx.x >> 6) % a.wpb);
        const bool need = i0 < a.batch && a.pol_need[i0] != 0;
        if (!__syncthreads_or(need)) return;
    }
    // ---------------- shared tables: H (N+1 stages) and Fp (column-major, mpad rows) -------
    if constexpr (SPL == 2 && !QUEUE) {
        // mixed mode, cold retry launch: a workgroup none of whose instances needs the retry
        // leaves before staging the shared tables
        if (a.redo_flag) {
            const int i0 = blockIdx.x * a.wpb + ((threadIdx.x >> 6) % a.wpb);
            const bool need = i0 < a.batch && a.exitflag[i0] != 1 &&
                              (a.redo_flag[i0] == 1 || a.redo_flag[i0] == 0);
            if (!__syncthreads_or(need)) return;
        }
    }
    constexpr bool LNG = BQP_LNG_OK && SPL == 2;  // long-horizon layout (QpLds lng)
    const bool fpi = a.Fp_inst != nullptr;   // per-instance polytope: in the instance's LDS slot
    // shared tables: H (short horizons; long ones read it from global), Fp, and for long horizons
    // the polytope rhs and box bounds when the batch shares them
    real* Hs = lds;
    real* Fs = lds + a.sh_F;
    if (!LNG && !a.H_inst)
        for (int i = threadIdx.x; i < (N + 1) * a.hstride; i += blockDim.x) Hs[i] = a.H[i];
    if (!fpi)
        for (int i = threadIdx.x; i < NV * a.mpad; i += blockDim.x) Fs[i] = a.Fp[i];
    if (a.sh_hp >= 0)
        for (int r = threadIdx.x; r < a.mp; r += blockDim.x) lds[a.sh_hp + r] = a.hp[r];
    if (LNG && a.sh_bnd >= 0) {
        constexpr int NB = NX + NU;
        for (int r = threadIdx.x; r < (N + 1) * NB * 2; r += blockDim.x) {
            const int vi = r >> 1, h = r & 1, k = vi / NB, sl = vi - k * NB;
            double bd = h ? -INFINITY : INFINITY;
            if (sl < NX) {
                const double* xb = h ? a.xlb : a.xub;
                if (k > 0 && xb) bd = xb[(int64_t)k * NX + sl];
            } else {
                const double* ub_ = h ? a.ulb : a.uub;
                if (k < N && ub_) bd = ub_[(int64_t)k * NU + (sl - NX)];
            }
            lds[a.sh_bnd + r] = (real)bd;
        }
    }
    __syncthreads();
    const bool rowwave = wid >= qpb;
    const int slot0 = rowwave ? wid - qpb : wid;
    // one instance on this slot (both waves of the pair); a persistent launch's row wave takes the
    // ticket of the slot's next instance into the exchange word xnext first
    auto instance = [&](int inst, int slot, int lane, int xnext) __attribute__((always_inline)) {
        const QpLds L = QpLds::make(N, NX, NU, NP, a.mpad, fpi, LNG, a.sh_hp >= 0,
                                    LNG && a.sh_bnd >= 0, a.H_inst != nullptr);
        real* W = lds + a.shared_doubles + slot * L.total;
        real* Fsi = Fs;
        if (fpi && rowwave) {
            // the instance's polytope, external column-major [x; u; theta] (n_poly rows) -> internal
            // [x; theta; u] columns of mpad rows (the layout of the shared table, ocp_prep_kernel)
            Fsi = W + L.Fi;
            const double* Fg = a.Fp_inst + (int64_t)inst * a.sFp;
            for (int r = lane; r < a.mpad; r += WAVE) {
#pragma unroll
                for (int c = 0; c < NV; ++c) {
                    const int e = c < NX ? c : (c < NS ? NX + NU + (c - NX) : NX + (c - NS));
                    real v = (r < a.mp) ? (real)Fg[(int64_t)e * a.mp + r] : real(0);
                    if (a.kp == N && c >= NS) v = 0;
                    Fsi[c * a.mpad + r] = v;
                }
            }
            wave_sync();
        }
        if (rowwave && lane == 0)
            *reinterpret_cast<int*>(W + L.xch + X_NEXT + xnext) = atomicAdd(a.queue, 1) + (int)gridDim.x * qpb;
#if defined(BQP_EXP_ONLY)   // register-budget diagnostic: one wave's code alone (never run)
        if (BQP_EXP_ONLY == 1) stage_wave<NX, NU, NP, SPL, POL>(a, W, L, Hs, lane, inst, blockIdx.x * qpb + slot0);
        else row_wave<NX, NU, NP, BPL, RPL, POL>(a, W, L, Fsi, lds, lane, inst);
#else
        if (!rowwave)
            stage_wave<NX, NU, NP, SPL, POL>(a, W, L, Hs, lane, inst, blockIdx.x * qpb + slot0);
        else
            row_wave<NX, NU, NP, BPL, RPL, POL>(a, W, L, Fsi, lds, lane, inst);
#endif
        return W + L.xch;
    };
    if constexpr (!QUEUE) {
        const int inst = blockIdx.x * qpb + slot0;
        if (inst >= a.batch) return;       // both waves of an empty slot leave together
        if (POL && a.pol_need[inst] == 0) return;   // repair launch: nothing to polish here
        if (!POL && SPL == 2 && a.redo_flag &&
            !(a.exitflag[inst] != 1 && (a.redo_flag[inst] == 1 || a.redo_flag[inst] == 0)))
            return;                        // mixed mode, cold retry launch: nothing to redo here
        const int slot = slot0;
        const int lane = lane_k;
        const QpLds L = QpLds::make(N, NX, NU, NP, a.mpad, fpi, LNG, a.sh_hp >= 0,
                                    LNG && a.sh_bnd >= 0, a.H_inst != nullptr);
        real* W = lds + a.shared_doubles + slot * L.total;
        if (fpi && rowwave) {
            // the instance's polytope, external column-major [x; u; theta] (n_poly rows) -> internal
            // [x; theta; u] columns of mpad rows (the layout of the shared table, ocp_prep_kernel)
            Fs = W + L.Fi;
            const double* Fg = a.Fp_inst + (int64_t)inst * a.sFp;
            for (int r = lane; r < a.mpad; r += WAVE) {
#pragma unroll
                for (int c = 0; c < NV; ++c) {
                    const int e = c < NX ? c : (c < NS ? NX + NU + (c - NX) : NX + (c - NS));
                    real v = (r < a.mp) ? (real)Fg[(int64_t)e * a.mp + r] : real(0);
                    if (a.kp == N && c >= NS) v = 0;
                    Fs[c * a.mpad + r] = v;
                }
            }
            wave_sync();
        }
#if defined(BQP_EXP_ONLY)   // register-budget diagnostic: one wave's code alone (never run)
        if (BQP_EXP_ONLY == 1) stage_wave<NX, NU, NP, SPL, POL>(a, W, L, Hs, lane, inst, inst);
        else row_wave<NX, NU, NP, BPL, RPL, POL>(a, W, L, Fs, lds, lane, inst);
#else
        if (!rowwave)
            stage_wave<NX, NU, NP, SPL, POL>(a, W, L, Hs, lane, inst, inst);
        else
            row_wave<NX, NU, NP, BPL, RPL, POL>(a, W, L, Fs, lds, lane, inst);
#endif
    } else {
        // persistent work queue (ocp_queue_kernel; launch_t sizes the grid to the resident
        // workgroups when the batch needs more): the slot's first instance is the static one,
        // every later one comes from the counter a.queue, so a slot starts its next instance as
        // soon as its current one is done instead of idling until the workgroup's slowest instance
        // ends, and the shared tables are staged once per workgroup lifetime (SURVEY 7 "per-wave
        // early exit with a persistent-kernel work queue"; the C4 iteration counts run from 3 to
        // 42 around a mean of 8.5)
        //
        // Barrier alignment: every barrier is workgroup-wide, so the slots of a workgroup advance
        // barrier by barrier together, and a barrier interval lasts as long as the longest phase
        // any slot runs in it.  A cold-started instance passes 4 + 6 K + 2 barriers (I0..I3, K
        // full iterations B0, B2..B6, the last pass B0, B2), a multiple of 6, so an instance that
        // starts right after its predecessor's last barrier runs its iterations' phases in step
        // with the other slots' (factor beside factor, solve beside solve).  The hand-over
        // therefore takes no barrier of its own: the row wave takes the ticket of the slot's next
        // instance at the start of the current one (before I0, into one of two exchange words
        // used alternately), and both waves read it after the last barrier.  (A hand-over barrier
        // shifted every later instance of the slot by one phase: C3 2.83 -> 3.43 ms per launch,
        // gpurun_out/r06_a.)  Instances continued from the mixed mode's handoff (one barrier
        // before the loop) are not queued (launch_t).
        int inst = blockIdx.x * qpb + slot0;
        int par = 0;
        while (inst < a.batch) {
            // the lane and slot made opaque per instance: nothing lane- or slot-dependent is
            // hoisted out of the instance loop into registers carried across instances (the
            // solve phases are at the 256-VGPR budget; opq)
            real* X = instance(inst, opq_s(slot0), opq(lane_k), par);
            inst = __builtin_amdgcn_readfirstlane(*reinterpret_cast<volatile int*>(X + X_NEXT + par));
            par ^= 1;
        }
    }
}

// the solve kernel (no polish code: the main loop keeps its register budget), the repair kernel
// (same IPM, then the active-set polish) over the instances the solve kernel marked, and the
// persistent solve kernel (work queue) for batches beyond the resident workgroups
template <int NX, int NU, int NP, int SPL, int RPL, int BPL>
__global__ void __launch_bounds__(SPL == 2 ? 256 : 512) ocp_ipm_kernel(OcpKernelArgs a) {
    ocp_body<NX, NU, NP, SPL, RPL, BPL, false, false>(a);
}
template <int NX, int NU, int NP, int SPL, int RPL, int BPL>
__global__ void __launch_bounds__(SPL == 2 ? 256 : 512) ocp_polish_kernel(OcpKernelArgs a) {
    ocp_body<NX, NU, NP, SPL, RPL, BPL, true, false>(a);
}
#ifndef BQP_DI_OCC3
#define BQP_DI_OCC3 0
#endif
// A/B variant (make ab VFLAGS=-DBQP_DI_OCC3=1; host: BQP_OCP_WPB=5): the DI queue kernel with five
// instances per workgroup (145 KB of LDS) and three waves per SIMD (168 VGPRs) - VERDICT r5 item 4
template <int NX, int NU, int NP, int SPL, int RPL, int BPL>
__global__ void __launch_bounds__(SPL == 2 ? 256 : ((BQP_DI_OCC3 && NX == 2) ? 640 : 512),
                                  (BQP_DI_OCC3 && NX == 2 && SPL == 1) ? 3 : 1)
ocp_queue_kernel(OcpKernelArgs a) {
    ocp_body<NX, NU, NP, SPL, RPL, BPL, false, true>(a);
}

}  // namespace dp / sp

// ------------------------------------------------------------------------------------------
// host-side launch helpers
// ------------------------------------------------------------------------------------------
// The kernel instantiations are split over translation units by model family so that the
// build compiles them in parallel (Makefile: BQP_FAMILY=1 MG nx4/nu1/np1 with the dispatcher
// and host helpers, BQP_FAMILY=2 DI nx2/nu2/np2); without BQP_FAMILY one unit holds all.
#if !defined(BQP_FAMILY)
#define BQP_FAM_MG 1
#define BQP_FAM_DI 1
#elif BQP_FAMILY == 1
#define BQP_FAM_MG 1
#define BQP_FAM_DI 0
#else
#define BQP_FAM_MG 0
#define BQP_FAM_DI 1
#endif

// dynamic LDS of a launch: the kernel's static LDS must fit beside it (a launch past 160 KB is
// refused up front, and a failed attribute call does not leave a stale error for the next launch)
static hipError_t lds_attr(const void* k, size_t lds) {
    hipFuncAttributes fa;
    hipError_t e = hipFuncGetAttributes(&fa, k);
    if (e == hipSuccess && lds + fa.sharedSizeBytes > 160 * 1024) e = hipErrorInvalidValue;
    if (e == hipSuccess && lds > 64 * 1024)
        e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) (void)hipGetLastError();
    return e;
}

template <int NX, int NU, int NP, int SPL, int RPL, int BPL>
static hipError_t launch_t(const OcpKernelArgs& a0, int blocks, size_t lds, hipStream_t st, bool pol) {
#ifdef BQP_F32
    (void)pol;
    auto k = sp::ocp_ipm_kernel<NX, NU, NP, SPL, RPL, BPL>;
    auto kq = sp::ocp_queue_kernel<NX, NU, NP, SPL, RPL, BPL>;
#else
    auto k = pol ? dp::ocp_polish_kernel<NX, NU, NP, SPL, RPL, BPL> : dp::ocp_ipm_kernel<NX, NU, NP, SPL, RPL, BPL>;
    auto kq = dp::ocp_queue_kernel<NX, NU, NP, SPL, RPL, BPL>;
#endif
    OcpKernelArgs a = a0;
    // persistent launch (ocp_queue_kernel) when the batch needs more workgroups than fit on the
    // device at once: the grid is the resident workgroups and the slots pull the remaining
    // instances from a.queue; otherwise one instance per slot (BQP_NO_QUEUE: always, for A/B)
    const bool no_queue = getenv("BQP_NO_QUEUE") != nullptr;
    if (!pol && !a.redo_flag && !a.hand_in && a.queue && !no_queue) {
        int dev = 0, cus = 0, per_cu = 0;
        hipError_t e = hipGetDevice(&dev);
        if (e == hipSuccess) e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        if (e == hipSuccess) e = lds_attr((const void*)kq, lds);
        if (e == hipSuccess)
            e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)kq, 128 * a.wpb, lds);
        if (e != hipSuccess) return e;
        const int resident = cus * (per_cu > 0 ? per_cu : 1);
        if (blocks > resident) {
            hipLaunchKernelGGL(kq, dim3(resident), dim3(128 * a.wpb), lds, st, a);
            return hipGetLastError();
        }
    }
    a.queue = nullptr;
    if (hipError_t e = lds_attr((const void*)k, lds)) return e;
    hipLaunchKernelGGL(k, dim3(blocks), dim3(128 * a.wpb), lds, st, a);
    return hipGetLastError();
}

// box rows per lane (BPL): all (N+1) 2 (nx+nu) box rows spread over the 64 lanes; the stage
// layout per lane (SPL) is tied to it: SPL 1 (N < 64) -> 4 (<= 256 rows) or 10 (<= 640),
// SPL 2 -> 16 (<= 1024) or 20 (<= 1280)
template <int NX, int NU, int NP, int SPL, int BPL>
static hipError_t launch_rpl(const OcpKernelArgs& a, int rpl, int blocks, size_t lds, hipStream_t st, bool pol) {
    switch (rpl) {
        case 1: return launch_t<NX, NU, NP, SPL, 1, BPL>(a, blocks, lds, st, pol);
        case 4: return launch_t<NX, NU, NP, SPL, 4, BPL>(a, blocks, lds, st, pol);
        case 10: return launch_t<NX, NU, NP, SPL, 10, BPL>(a, blocks, lds, st, pol);
        case 16: return launch_t<NX, NU, NP, SPL, 16, BPL>(a, blocks, lds, st, pol);
        default: return hipErrorInvalidValue;
    }
}

template <int NX, int NU, int NP>
static hipError_t launch_spl(const OcpKernelArgs& a, int spl, int rpl, int blocks, size_t lds, hipStream_t st, bool pol) {
    const int nbr = (a.N + 1) * 2 * (NX + NU);
    if (spl == 1 && nbr <= 4 * WAVE) return launch_rpl<NX, NU, NP, 1, 4>(a, rpl, blocks, lds, st, pol);
    if (spl == 1 && nbr <= 10 * WAVE) return launch_rpl<NX, NU, NP, 1, 10>(a, rpl, blocks, lds, st, pol);
    if (spl == 2 && nbr <= 16 * WAVE) return launch_rpl<NX, NU, NP, 2, 16>(a, rpl, blocks, lds, st, pol);
    if (spl == 2 && nbr <= 20 * WAVE) return launch_rpl<NX, NU, NP, 2, 20>(a, rpl, blocks, lds, st, pol);
    return hipErrorInvalidValue;
}

hipError_t BQP_CAT(launch_ocp_mg, BQP_SFX)(const OcpKernelArgs& a, int spl, int rpl, int blocks, size_t lds, hipStream_t st, bool pol);
hipError_t BQP_CAT(launch_ocp_di, BQP_SFX)(const OcpKernelArgs& a, int spl, int rpl, int blocks, size_t lds, hipStream_t st, bool pol);

#if BQP_FAM_MG
hipError_t BQP_CAT(launch_ocp_mg, BQP_SFX)(const OcpKernelArgs& a, int spl, int rpl, int blocks, size_t lds, hipStream_t st, bool pol) {
#if defined(BQP_ISA_ONLY_MG10)
    // codegen inspection build (make isa): the MG N<64, 616-row instance only
    if (spl == 1 && rpl == 10 && a.N + 1 <= 25) return launch_t<4, 1, 1, 1, 10, 4>(a, blocks, lds, st, pol);
    return hipErrorInvalidValue;
#elif defined(BQP_ISA_ONLY_MG_LNG)
    // the MG N = 100 / 616-row long-horizon instance (config C5) only (make isa-lng)
    if (spl == 2 && rpl == 10) return launch_t<4, 1, 1, 2, 10, 16>(a, blocks, lds, st, pol);
    return hipErrorInvalidValue;
#elif defined(BQP_ISA_ONLY_DI)
    return hipErrorInvalidValue;
#else
    return launch_spl<4, 1, 1>(a, spl, rpl, blocks, lds, st, pol);
#endif
}
#endif
#if BQP_FAM_DI && !defined(BQP_ISA_ONLY_MG10) && !defined(BQP_ISA_ONLY_MG_LNG)
hipError_t BQP_CAT(launch_ocp_di, BQP_SFX)(const OcpKernelArgs& a, int spl, int rpl, int blocks, size_t lds, hipStream_t st, bool pol) {
#ifdef BQP_ISA_ONLY_DI
    // codegen inspection build (make isa-di): the DI N<64, <= 64-row instance (config C3) only
    if (spl == 1 && rpl == 1) return launch_t<2, 2, 2, 1, 1, 4>(a, blocks, lds, st, pol);
    return hipErrorInvalidValue;
#else
    return launch_spl<2, 2, 2>(a, spl, rpl, blocks, lds, st, pol);
#endif
}
#endif

#if BQP_FAM_MG
#ifndef BQP_F32
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

// box rows per lane of the instantiation launch_spl selects (-1: outside the compiled set)
int ocp_bpl_for(int N, int nx, int nu) {
    const int nbr = (N + 1) * 2 * (nx + nu);
    if (N + 1 <= WAVE) return nbr <= 4 * WAVE ? 4 : (nbr <= 10 * WAVE ? 10 : -1);
    return nbr <= 16 * WAVE ? 16 : (nbr <= 20 * WAVE ? 20 : -1);
}

int ocp_pstride(int ns) { return dp::pk_stride(ns); }

int ocp_hand_floats(int N, int nx, int nu, int np, int mp) {
    const int bpl = ocp_bpl_for(N, nx, nu), rpl = ocp_rpl_for(mp > 1 ? mp : 1);
    if (bpl < 0 || rpl < 0) return -1;
    return dp::hand_rows_off(N, nx + np, nu) + 2 * (bpl + rpl) * WAVE;
}
#endif

// LDS elements (of the instantiation's precision) per instance
int BQP_CAT(ocp_wave_lds_doubles, BQP_SFX)(int N, int nx, int nu, int np, int mpad, bool fpi,
                                          bool lng, bool hpsh, bool bndsh, bool hinst) {
#ifdef BQP_F32
    return sp::QpLds::make(N, nx, nu, np, mpad, fpi, lng, hpsh, bndsh, hinst).total;
#else
    return dp::QpLds::make(N, nx, nu, np, mpad, fpi, lng, hpsh, bndsh, hinst).total;
#endif
}

hipError_t BQP_CAT(launch_ocp, BQP_SFX)(const OcpKernelArgs& a, int nx, int nu, int np, hipStream_t st, bool pol) {
    const int spl = (a.N + 1 <= 64) ? 1 : 2;
    const int rpl = ocp_rpl_for(a.mp);
    const int blocks = (a.batch + a.wpb - 1) / a.wpb;
    const size_t lds = sizeof(real) * ((size_t)a.shared_doubles +
                                       (size_t)a.wpb * BQP_CAT(ocp_wave_lds_doubles, BQP_SFX)(a.N, nx, nu, np, a.mpad,
                                                                                      a.Fp_inst != nullptr, BQP_LNG_OK && spl == 2,
                                                                                      a.sh_hp >= 0,
                                                                                      BQP_LNG_OK && spl == 2 && a.sh_bnd >= 0,
                                                                                      a.H_inst != nullptr));
    if (nx == 4 && nu == 1 && np == 1) return BQP_CAT(launch_ocp_mg, BQP_SFX)(a, spl, rpl, blocks, lds, st, pol);
#if !defined(BQP_ISA_ONLY_MG10) && !defined(BQP_ISA_ONLY_MG_LNG)
    if (nx == 2 && nu == 2 && np == 2) return BQP_CAT(launch_ocp_di, BQP_SFX)(a, spl, rpl, blocks, lds, st, pol);
#endif
    return hipErrorInvalidValue;
}
#endif

}  // namespace bqp
