/*
 * TEST INFRASTRUCTURE ONLY (see oracle/__init__.py): C restatement of the structured Mehrotra
 * predictor-corrector IPM specified in oracle/ocp_ipm.py, written in the same restructured
 * (closed-loop) form as the HIP kernel learning-based-mpc_amd/csrc/bqp_ocp.hip so that GPU
 * iterates can be compared to it at round-off level.  It is also the timed CPU baseline of
 * bench.py (cpu_baseline.kind = "port": one instance per OpenMP thread, fp64, -O3).
 *
 * It consumes the same bqp_ocp_dims/bqp_ocp_data description as include/bqp.h.  The reference
 * itself (MATLAB fmincon-sqp / CasADi-IPOPT) cannot run here.
 *
 * Build: make -C oracle   ->  oracle/_build/libcpu_ipm.so
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>
#include <stdio.h>
#ifdef _OPENMP
#include <omp.h>
#endif
#include "../include/bqp.h"

#define MAXNS 8
#define MAXNU 4
#define MAXNV 12
#define PIV_FLOOR 1e-14
#define MU_BLOWUP 1e6     /* mu > MU_BLOWUP * min(mu) with the rows still infeasible: -2       */
#define FEAS_GUARD 1e-8   /* rows "still infeasible": residual > FEAS_GUARD (1 + |data|)         */
#define SOC_ALPHA 0.1     /* predictor step below this on a feasible iterate: corrector without  */
                          /* the second-order term (a centring step; Mehrotra's stall safeguard)  */
#ifndef CMAX_K
#define TAU_FAST_AFF 0.99   /* step rule: predictor step above this ... */
#define TAU_FAST_MU 1e-6     /* ... and mu above this: the corrector step goes to TAU_FAST */
#define TAU_FAST 0.99999
#define TAU_FAST_END 0.99999 /* predictor step at least this: the fast step at any mu */
#define TAU_FAST_MIN 0.995   /* the fast rule applies only at tau >= the default (a caller's smaller tau bounds every step) */
#define CMAX_K 100.0     /* and every row: t_i lam_i <= CMAX_K tol_comp (the average alone lets one */
#endif            /* weakly active row keep t ~ 1e-10: first moves off by 1e-7 at N = 100) */
#ifndef DEG_POLISH
#define DEG_POLISH 1e-10  /* polish = 2: also a converged iterate with max_i min(t_i, lam_i) > this */
#endif
#ifndef POL_RHO
#define POL_RHO 2e6
#endif
//       /* polish weight rho = POL_RHO (1 + |H v + g|_inf)                      */
#ifndef POL_ALM
#define POL_ALM 8
#endif
//         /* augmented-Lagrangian iterations per polish round (at most)           */
#ifndef POL_STAG
#define POL_STAG 0.5
#endif
#ifndef POL_CG_SING
#define POL_CG_SING 1e-2
#endif
#ifndef POL_PASS
#define POL_PASS 3
#endif
#ifndef POL_CG
#define POL_CG 40
#endif
#ifndef POL_ROUNDS
#define POL_ROUNDS 8
#endif
//      /* active-set corrections                                               */

typedef struct {
    int nx, nu, np, ns, nv, N, mp, kp;
    double Abar[MAXNS][MAXNS], Bbar[MAXNS][MAXNU], cbar[MAXNS];
    const double* H;   /* (N+1)*nv*nv internal order [x th u], row-major [i][j] */
    const double* Fp;  /* mp*nv internal order row-major                        */
} prob_t;

typedef struct {
    double *s, *u, *pi;                  /* (N+1)*ns, N*nu, (N+1)*ns                 */
    double *g;                           /* (N+1)*nv linear term, internal order     */
    double *xlb, *xub, *ulb, *uub, *hp;  /* bounds (inf allowed)                      */
    double *tx, *lx, *tu, *lu, *tp, *lp; /* x rows: (N+1)*nx*2 [upper,lower]; u: N*nu*2 */
    /* work */
    double *rs, *ru, *re, *rix, *riu, *rip;
    double *ds, *du, *dpi, *dtx, *dlx, *dtu, *dlu, *dtp, *dlp;
    double *Ptab, *Ktab, *Rinv, *Phit, *p, *qs, *qu, *wv, *cw, *qt, *qh, *kff, *f;
    double *Dx, *Du, *FD;
    double *itx, *ilx, *itu, *ilu, *itp, *ilp;   /* 1/t, 1/lam (once per iteration) */
    double P0inv[MAXNS * MAXNS];
    /* row residuals carried by the linear update r+ = r + a (C dv + dt) after the start, as the
     * kernel's row wave does (no residual pass before the factorisation); fe_rows is their norm */
    int rip_live;
    double fe_rows;
    /* active-set polish: weight rho on the rows taken as equalities, 0 on the dropped ones */
    int pol;
    double cmax;   /* max_i t_i lam_i of the last residuals() */
    double *wx, *wu, *wp;
    double *cgr, *cgp;   /* polish: CG residual and direction over all rows [x | u | poly] */
    double *rcb;         /* complementarity rhs over all rows [x | u | poly] (per thread, once) */
} work_t;

static int perm_of(const prob_t* P, int i) {
    /* internal index i -> external [x; u; th] index */
    if (i < P->nx) return i;
    if (i < P->ns) return P->nx + P->nu + (i - P->nx);
    return P->nx + (i - P->ns);
}

/* ---------------- small dense helpers ---------------- */
static int spd_fac(int n, const double* M, double* L) {
    /* factor of a small SPD matrix for spd_solve.  n = 1: L holds 1/M (one reciprocal, as the
     * kernel stores it); n > 1: lower Cholesky factor (row-major) with a static pivot floor,
     * applied by substitution: an explicit inverse of the ill-conditioned Rhat near convergence
     * loses the stationarity residual. */
    if (n == 1) {
        if (!(M[0] > 0)) return -1;
        L[0] = 1.0 / M[0];
        return 0;
    }
    if (n == 2) {
        /* LDL' with the reciprocal pivots stored, L = [1/d0, 0, l10, 1/d1] (the kernel's
         * chol_small, round 6: no square roots on the Riccati recursion's per-stage chain) */
        double d0 = M[0];
        if (!(d0 > PIV_FLOOR * M[0])) d0 = PIV_FLOOR * M[0];
        if (!(d0 > 0)) return -1;
        const double r0 = 1.0 / d0;
        const double l10 = M[2] * r0;
        double d1 = M[3] - l10 * M[2];
        if (!(d1 > PIV_FLOOR * M[3])) d1 = PIV_FLOOR * M[3];
        if (!(d1 > 0)) return -1;
        L[0] = r0; L[1] = 0.0; L[2] = l10; L[3] = 1.0 / d1;
        return 0;
    }
    for (int i = 0; i < n * n; ++i) L[i] = 0.0;
    for (int j = 0; j < n; ++j) {
        double d = M[j * n + j];
        for (int k = 0; k < j; ++k) d -= L[j * n + k] * L[j * n + k];
        /* static pivot floor: cancellation near convergence must not stop the iteration */
        if (!(d > PIV_FLOOR * M[j * n + j])) d = PIV_FLOOR * M[j * n + j];
        if (!(d > 0)) return -1;
        d = sqrt(d);
        L[j * n + j] = d;
        for (int i = j + 1; i < n; ++i) {
            double v = M[i * n + j];
            for (int k = 0; k < j; ++k) v -= L[i * n + k] * L[j * n + k];
            L[i * n + j] = v / d;
        }
    }
    return 0;
}

static void spd_solve(int n, const double* L, double* b) {
    /* b <- M^{-1} b from spd_fac's factor */
    if (n == 1) {
        b[0] = b[0] * L[0];
        return;
    }
    if (n == 2) {
        const double w1 = (b[1] - L[2] * b[0]) * L[3];
        b[0] = b[0] * L[0] - L[2] * w1;
        b[1] = w1;
        return;
    }
    for (int i = 0; i < n; ++i) {
        double v = b[i];
        for (int k = 0; k < i; ++k) v -= L[i * n + k] * b[k];
        b[i] = v / L[i * n + i];
    }
    for (int i = n - 1; i >= 0; --i) {
        double v = b[i];
        for (int k = i + 1; k < n; ++k) v -= L[k * n + i] * b[k];
        b[i] = v / L[i * n + i];
    }
}

/* ---------------- residuals ---------------- */
static void residuals(const prob_t* P, work_t* W, double* stat, double* feas, double* musum,
                      int* mcount, double* gscale) {
    const int N = P->N, nx = P->nx, nu = P->nu, ns = P->ns, nv = P->nv;
    double st = 0, fe = 0, cs = 0, gs = 0;
    W->cmax = 0.0;
    int mc = 0;
    for (int k = 0; k <= N; ++k) {
        const double* H = P->H + (size_t)k * nv * nv;
        double v[MAXNV];
        for (int i = 0; i < ns; ++i) v[i] = W->s[k * ns + i];
        for (int i = 0; i < nu; ++i) v[ns + i] = (k < N) ? W->u[k * nu + i] : 0.0;
        int nvk = (k < N) ? nv : ns;
        double gv[MAXNV];
        for (int i = 0; i < nvk; ++i) {
            double a = W->g[k * nv + i];
            for (int j = 0; j < nvk; ++j) a += H[i * nv + j] * v[j];
            gv[i] = a;
            gs = fmax(gs, fabs(a));
        }
        for (int i = 0; i < ns; ++i) {
            double a = gv[i];
            if (k < N)
                for (int j = 0; j < ns; ++j) a += P->Abar[j][i] * W->pi[(k + 1) * ns + j];
            if (k > 0) a -= W->pi[k * ns + i];
            W->rs[k * ns + i] = a;
        }
        if (k < N)
            for (int i = 0; i < nu; ++i) {
                double a = gv[ns + i];
                for (int j = 0; j < ns; ++j) a += P->Bbar[j][i] * W->pi[(k + 1) * ns + j];
                W->ru[k * nu + i] = a;
            }
        /* box rows */
        for (int i = 0; i < nx; ++i) {
            double xi = W->s[k * ns + i];
            int o = (k * nx + i) * 2;
            double ri_u = 0, ri_l = 0;
            if (k > 0 && isfinite(W->xub[k * nx + i])) {
                W->rs[k * ns + i] += W->lx[o];
                ri_u = xi + W->tx[o] - W->xub[k * nx + i];
                cs += W->tx[o] * W->lx[o]; ++mc; W->cmax = fmax(W->cmax, W->tx[o] * W->lx[o]);
            }
            if (k > 0 && isfinite(W->xlb[k * nx + i])) {
                W->rs[k * ns + i] -= W->lx[o + 1];
                ri_l = -xi + W->tx[o + 1] + W->xlb[k * nx + i];
                cs += W->tx[o + 1] * W->lx[o + 1]; ++mc; W->cmax = fmax(W->cmax, W->tx[o + 1] * W->lx[o + 1]);
            }
            W->rix[o] = ri_u; W->rix[o + 1] = ri_l;
        }
        if (k < N)
            for (int i = 0; i < nu; ++i) {
                double ui = W->u[k * nu + i];
                int o = (k * nu + i) * 2;
                double ri_u = 0, ri_l = 0;
                if (isfinite(W->uub[k * nu + i])) {
                    W->ru[k * nu + i] += W->lu[o];
                    ri_u = ui + W->tu[o] - W->uub[k * nu + i];
                    cs += W->tu[o] * W->lu[o]; ++mc; W->cmax = fmax(W->cmax, W->tu[o] * W->lu[o]);
                }
                if (isfinite(W->ulb[k * nu + i])) {
                    W->ru[k * nu + i] -= W->lu[o + 1];
                    ri_l = -ui + W->tu[o + 1] + W->ulb[k * nu + i];
                    cs += W->tu[o + 1] * W->lu[o + 1]; ++mc; W->cmax = fmax(W->cmax, W->tu[o + 1] * W->lu[o + 1]);
                }
                W->riu[o] = ri_u; W->riu[o + 1] = ri_l;
            }
        if (k < N)
            for (int i = 0; i < ns; ++i) {
                double a = P->cbar[i] - W->s[(k + 1) * ns + i];
                for (int j = 0; j < ns; ++j) a += P->Abar[i][j] * W->s[k * ns + j];
                for (int j = 0; j < nu; ++j) a += P->Bbar[i][j] * W->u[k * nu + j];
                W->re[k * ns + i] = a;
            }
    }
    /* polytope rows */
    {
        const int kp = P->kp;
        double v[MAXNV];
        for (int i = 0; i < ns; ++i) v[i] = W->s[kp * ns + i];
        for (int i = 0; i < nu; ++i) v[ns + i] = (kp < N) ? W->u[kp * nu + i] : 0.0;
        double gp[MAXNV];
        memset(gp, 0, sizeof(gp));
        for (int r = 0; r < P->mp; ++r) {
            const double* F = P->Fp + (size_t)r * nv;
            double a = W->tp[r] - W->hp[r];
            for (int j = 0; j < nv; ++j) {
                a += F[j] * v[j];
                gp[j] += F[j] * W->lp[r];
            }
            if (!W->rip_live) W->rip[r] = a;
            cs += W->tp[r] * W->lp[r]; ++mc; W->cmax = fmax(W->cmax, W->tp[r] * W->lp[r]);
        }
        for (int i = 0; i < ns; ++i) W->rs[kp * ns + i] += gp[i];
        if (kp < N)
            for (int i = 0; i < nu; ++i) W->ru[kp * nu + i] += gp[ns + i];
    }
    for (int i = 0; i < nx; ++i) W->rs[i] = 0.0; /* x_0 fixed */
    for (int k = 0; k <= N; ++k)
        for (int i = 0; i < ns; ++i) st = fmax(st, fabs(W->rs[k * ns + i]));
    for (int k = 0; k < N; ++k) {
        for (int i = 0; i < nu; ++i) st = fmax(st, fabs(W->ru[k * nu + i]));
        for (int i = 0; i < ns; ++i) fe = fmax(fe, fabs(W->re[k * ns + i]));
    }
    if (W->rip_live) {
        fe = fmax(fe, W->fe_rows);
    } else {
        for (int k = 0; k <= N; ++k)
            for (int i = 0; i < 2 * nx; ++i) fe = fmax(fe, fabs(W->rix[k * nx * 2 + i]));
        for (int k = 0; k < N; ++k)
            for (int i = 0; i < 2 * nu; ++i) fe = fmax(fe, fabs(W->riu[k * nu * 2 + i]));
        for (int r = 0; r < P->mp; ++r) fe = fmax(fe, fabs(W->rip[r]));
    }
    *stat = st; *feas = fe; *musum = cs; *mcount = mc; *gscale = gs;
}

/* ---------------- factorisation ---------------- */
/* column r of F = [Abar Bbar] (internal [s; u] order), row a */
static double fab(const prob_t* P, int a, int r) {
    return r < P->ns ? P->Abar[a][r] : P->Bbar[a][r - P->ns];
}

static int factor(const prob_t* P, work_t* W) {
    const int N = P->N, nx = P->nx, nu = P->nu, ns = P->ns, nv = P->nv;
    /* one reciprocal of t and lam per row per iteration; every later quotient is a product */
    for (int i = 0; i < (N + 1) * nx * 2; ++i) { W->itx[i] = 1.0 / W->tx[i]; W->ilx[i] = 1.0 / W->lx[i]; }
    for (int i = 0; i < N * nu * 2; ++i) { W->itu[i] = 1.0 / W->tu[i]; W->ilu[i] = 1.0 / W->lu[i]; }
    for (int r = 0; r < P->mp; ++r) { W->itp[r] = 1.0 / W->tp[r]; W->ilp[r] = 1.0 / W->lp[r]; }
    /* box diagonals */
    for (int k = 0; k <= N; ++k)
        for (int i = 0; i < nx; ++i) {
            int o = (k * nx + i) * 2;
            double d = 0;
            if (W->pol) {
                if (k > 0) d = W->wx[o] + W->wx[o + 1];
            } else {
                if (k > 0 && isfinite(W->xub[k * nx + i])) d += W->lx[o] * W->itx[o];
                if (k > 0 && isfinite(W->xlb[k * nx + i])) d += W->lx[o + 1] * W->itx[o + 1];
            }
            W->Dx[k * nx + i] = d;
        }
    for (int k = 0; k < N; ++k)
        for (int i = 0; i < nu; ++i) {
            int o = (k * nu + i) * 2;
            double d = 0;
            if (W->pol) {
                d = W->wu[o] + W->wu[o + 1];
            } else {
                if (isfinite(W->uub[k * nu + i])) d += W->lu[o] * W->itu[o];
                if (isfinite(W->ulb[k * nu + i])) d += W->lu[o + 1] * W->itu[o + 1];
            }
            W->Du[k * nu + i] = d;
        }
    memset(W->FD, 0, sizeof(double) * nv * nv);
    for (int r = 0; r < P->mp; ++r) {
        const double* F = P->Fp + (size_t)r * nv;
        double d = W->pol ? W->wp[r] : W->lp[r] * W->itp[r];
        for (int i = 0; i < nv; ++i) {
            double di = d * F[i];
            for (int j = i; j < nv; ++j) W->FD[i * nv + j] += di * F[j];
        }
    }
    for (int i = 0; i < nv; ++i)
        for (int j = 0; j < i; ++j) W->FD[i * nv + j] = W->FD[j * nv + i];
    /* Htilde(k)[i][j] */
#define HT(k, i, j)                                                                     \
    (P->H[((size_t)(k) * nv + (i)) * nv + (j)] +                                          \
     ((i) == (j) ? ((i) < nx ? W->Dx[(k) * nx + (i)] : ((i) >= ns ? W->Du[(k) * nu + (i) - ns] : 0.0)) : 0.0) + \
     ((k) == P->kp ? W->FD[(i) * nv + (j)] : 0.0))
    double* PN = W->Ptab + (size_t)N * ns * ns;
    for (int i = 0; i < ns; ++i)
        for (int j = 0; j < ns; ++j) PN[i * ns + j] = HT(N, i, j);
    /* Riccati recursion in standard form on the stage matrix M_k = Ht_k + F' P_{k+1} F,
     * F = [Abar Bbar]:  K_k = -M_uu^{-1} M_us,  P_k = M_ss - M_su M_uu^{-1} M_us.
     * M is linear in the packed upper triangle of P_{k+1} with constant coefficients
     * C(r, c; a, b) = F(a,r) F(b,c) + [a != b] F(b,r) F(a,c), summed as four interleaved partial
     * sums over the packed index m mod 4, combined (s0 + s1) + (s2 + s3) - the association of
     * the kernel (bqp_ocp.hip factor(), one value per lane of a quad). */
    for (int k = N - 1; k >= 0; --k) {
        const double* Pn = W->Ptab + (size_t)(k + 1) * ns * ns;
        double Mss[MAXNS][MAXNS], Msu[MAXNS][MAXNU], Muu[MAXNU * MAXNU];
        for (int r = 0; r < nv; ++r)
            for (int c = r; c < nv; ++c) {
                if (r >= ns && c < ns) continue;
                double sp[4] = {0.0, 0.0, 0.0, 0.0};
                int m = 0;
                for (int a = 0; a < ns; ++a)
                    for (int b = a; b < ns; ++b, ++m) {
                        double cf = fab(P, a, r) * fab(P, b, c);
                        if (a != b) cf = fma(fab(P, b, r), fab(P, a, c), cf);
                        sp[m & 3] = fma(cf, Pn[a * ns + b], sp[m & 3]);
                    }
                const double v = HT(k, r, c) + ((sp[0] + sp[1]) + (sp[2] + sp[3]));
                if (c < ns) Mss[r][c] = v;
                else if (r < ns) Msu[r][c - ns] = v;
                else { Muu[(r - ns) * nu + (c - ns)] = v; Muu[(c - ns) * nu + (r - ns)] = v; }
            }
        double* Lk = W->Rinv + (size_t)k * nu * nu;    /* factor of M_uu (spd_fac) */
        if (spd_fac(nu, Muu, Lk)) return -1;
        double* Kk = W->Ktab + (size_t)k * nu * ns;
        double Y[MAXNS][MAXNU];                        /* M_uu^{-1} M_u j */
        for (int j = 0; j < ns; ++j) {
            double col[MAXNU];
            for (int x = 0; x < nu; ++x) col[x] = Msu[j][x];
            spd_solve(nu, Lk, col);
            for (int x = 0; x < nu; ++x) { Y[j][x] = col[x]; Kk[x * ns + j] = -col[x]; }
        }
        double* Pk = W->Ptab + (size_t)k * ns * ns;
        for (int i = 0; i < ns; ++i)
            for (int j = i; j < ns; ++j) {
                double v;
                if (nu == 1) {
                    v = fma(-(Msu[i][0] * Lk[0]), Msu[j][0], Mss[i][j]);
                } else {
                    double acc = Msu[i][0] * Y[j][0];
                    for (int x = 1; x < nu; ++x) acc = fma(Msu[i][x], Y[j][x], acc);
                    v = Mss[i][j] - acc;
                }
                Pk[i * ns + j] = v;
                Pk[j * ns + i] = v;
            }
        /* closed loop Phi_k = Abar + Bbar K_k (row-major), used by the sweeps */
        double* Phk = W->Phit + (size_t)k * ns * ns;
        for (int a = 0; a < ns; ++a)
            for (int j = 0; j < ns; ++j) {
                double v = P->Abar[a][j];
                for (int x = 0; x < nu; ++x) v += P->Bbar[a][x] * Kk[x * ns + j];
                Phk[a * ns + j] = v;
            }
    }
#undef HT
    /* theta block of P_0 */
    {
        const int np = P->np;
        double Pt[MAXNS * MAXNS];
        const double* P0 = W->Ptab;
        for (int a = 0; a < np; ++a)
            for (int b = 0; b < np; ++b) Pt[a * np + b] = P0[(nx + a) * ns + nx + b];
        if (spd_fac(np, Pt, W->P0inv)) return -1;    /* factor of P_0[theta,theta] */
    }
    return 0;
}

/* once per factorisation: the part of both solves that depends on the dynamics residual alone
 * (the kernel's prep_iter): w_k = P_{k+1} re_k, cw_k = Phi_k' w_k, bw_k = Bbar' w_k */
static void prep_iter(const prob_t* P, work_t* W) {
    const int N = P->N, ns = P->ns, nu = P->nu;
    for (int k = 0; k < N; ++k) {
        const double* Pn = W->Ptab + (size_t)(k + 1) * ns * ns;
        const double* Phk = W->Phit + (size_t)k * ns * ns;
        double w[MAXNS];
        for (int i = 0; i < ns; ++i) {
            double v = 0;
            for (int j = 0; j < ns; ++j) v += Pn[i * ns + j] * W->re[k * ns + j];
            w[i] = v;
        }
        for (int a = 0; a < nu; ++a) {
            double v = 0;
            for (int j = 0; j < ns; ++j) v += P->Bbar[j][a] * w[j];
            W->wv[k * nu + a] = v;
        }
        for (int i = 0; i < ns; ++i) {
            double v = 0;
            for (int j = 0; j < ns; ++j) v += Phk[j * ns + i] * w[j];
            W->cw[k * ns + i] = v;
        }
    }
}

/* ---------------- solve ---------------- */
/* rcx/rcu/rcp: complementarity right-hand side per row */
static void solve_kkt(const prob_t* P, work_t* W, const double* rcx, const double* rcu,
                      const double* rcp) {
    const int N = P->N, nx = P->nx, nu = P->nu, ns = P->ns, nv = P->nv, np = P->np;
    /* q = r_v + C' e,  e = (lam o ri - rc)/t */
    for (int k = 0; k <= N; ++k) {
        for (int i = 0; i < ns; ++i) W->qs[k * ns + i] = W->rs[k * ns + i];
        for (int i = 0; i < nx; ++i) {
            int o = (k * nx + i) * 2;
            double e = 0;
            if (W->pol) {
                /* polish: the augmented-Lagrangian gradient term rho (C v - b) of active rows */
                if (k > 0) e = W->wx[o] * W->rix[o] - W->wx[o + 1] * W->rix[o + 1];
            } else {
                if (k > 0 && isfinite(W->xub[k * nx + i])) e += (W->lx[o] * W->rix[o] - rcx[o]) * W->itx[o];
                if (k > 0 && isfinite(W->xlb[k * nx + i])) e -= (W->lx[o + 1] * W->rix[o + 1] - rcx[o + 1]) * W->itx[o + 1];
            }
            W->qs[k * ns + i] += e;
        }
        if (k < N)
            for (int i = 0; i < nu; ++i) {
                int o = (k * nu + i) * 2;
                double e = W->ru[k * nu + i];
                if (W->pol) {
                    e += W->wu[o] * W->riu[o] - W->wu[o + 1] * W->riu[o + 1];
                } else {
                    if (isfinite(W->uub[k * nu + i])) e += (W->lu[o] * W->riu[o] - rcu[o]) * W->itu[o];
                    if (isfinite(W->ulb[k * nu + i])) e -= (W->lu[o + 1] * W->riu[o + 1] - rcu[o + 1]) * W->itu[o + 1];
                }
                W->qu[k * nu + i] = e;
            }
    }
    {
        double gp[MAXNV];
        memset(gp, 0, sizeof(gp));
        for (int r = 0; r < P->mp; ++r) {
            double e = W->pol ? W->wp[r] * W->rip[r] : (W->lp[r] * W->rip[r] - rcp[r]) * W->itp[r];
            const double* F = P->Fp + (size_t)r * nv;
            for (int j = 0; j < nv; ++j) gp[j] += F[j] * e;
        }
        for (int i = 0; i < ns; ++i) W->qs[P->kp * ns + i] += gp[i];
        if (P->kp < N)
            for (int i = 0; i < nu; ++i) W->qu[P->kp * nu + i] += gp[ns + i];
    }
    /* pre-pass: qt_k = qs_k + K_k' qu_k, qh_k = qt_k + cw_k (cw_k = Phi_k' P_{k+1} re_k, formed
     * once per factorisation by prep_iter), then the backward sweep
     * p_k = Phi_k' p_{k+1} + qh_k   (= Phi_k'(p_{k+1} + w_k) + qt_k) */
    for (int k = 0; k < N; ++k) {
        const double* Kk = W->Ktab + (size_t)k * nu * ns;
        for (int i = 0; i < ns; ++i) {
            double q = W->qs[k * ns + i];
            for (int a = 0; a < nu; ++a) q += Kk[a * ns + i] * W->qu[k * nu + a];
            W->qt[k * ns + i] = q;
            W->qh[k * ns + i] = q + W->cw[k * ns + i];
        }
    }
    for (int i = 0; i < ns; ++i) W->p[N * ns + i] = W->qs[N * ns + i];
    for (int k = N - 1; k >= 0; --k) {
        const double* Phk = W->Phit + (size_t)k * ns * ns;
        for (int i = 0; i < ns; ++i) {
            double v = W->qh[k * ns + i];
            for (int j = 0; j < ns; ++j) v += Phk[j * ns + i] * W->p[(k + 1) * ns + j];
            W->p[k * ns + i] = v;
        }
    }
    /* post-backward: kff_k = -Rinv_k ((qu_k + bw_k) + Bbar' p_{k+1}); f_k = Bbar kff_k + re_k
     * (wv holds bw_k = Bbar' P_{k+1} re_k, prep_iter) */
    for (int k = 0; k < N; ++k) {
        double r[MAXNU];
        for (int a = 0; a < nu; ++a) {
            double v = W->qu[k * nu + a] + W->wv[k * nu + a];
            for (int j = 0; j < ns; ++j) v += P->Bbar[j][a] * W->p[(k + 1) * ns + j];
            r[a] = v;
        }
        for (int a = 0; a < nu; ++a) r[a] = -r[a];
        spd_solve(nu, W->Rinv + (size_t)k * nu * nu, r);
        for (int a = 0; a < nu; ++a) W->kff[k * nu + a] = r[a];
        for (int i = 0; i < ns; ++i) {
            double v = W->re[k * ns + i];
            for (int a = 0; a < nu; ++a) v += P->Bbar[i][a] * W->kff[k * nu + a];
            W->f[k * ns + i] = v;
        }
    }
    /* theta_0 step and forward sweep: ds_{k+1} = Phi_k ds_k + f_k */
    for (int i = 0; i < nx; ++i) W->ds[i] = 0.0;
    {
        double r[MAXNS];
        for (int a = 0; a < np; ++a) r[a] = -W->p[nx + a];
        spd_solve(np, W->P0inv, r);
        for (int a = 0; a < np; ++a) W->ds[nx + a] = r[a];
    }
    for (int k = 0; k < N; ++k) {
        const double* Phk = W->Phit + (size_t)k * ns * ns;
        const double* d = W->ds + k * ns;
        for (int i = 0; i < ns; ++i) {
            double v = W->f[k * ns + i];
            for (int j = 0; j < ns; ++j) v += Phk[i * ns + j] * d[j];
            W->ds[(k + 1) * ns + i] = v;
        }
    }
    /* post-forward: du, dpi */
    for (int k = 0; k < N; ++k) {
        const double* Kk = W->Ktab + (size_t)k * nu * ns;
        for (int a = 0; a < nu; ++a) {
            double v = W->kff[k * nu + a];
            for (int j = 0; j < ns; ++j) v += Kk[a * ns + j] * W->ds[k * ns + j];
            W->du[k * nu + a] = v;
        }
    }
    for (int k = 1; k <= N; ++k) {
        const double* Pk = W->Ptab + (size_t)k * ns * ns;
        for (int i = 0; i < ns; ++i) {
            double v = W->p[k * ns + i];
            for (int j = 0; j < ns; ++j) v += Pk[i * ns + j] * W->ds[k * ns + j];
            W->dpi[k * ns + i] = v;
        }
    }
    /* slack / multiplier steps */
    for (int k = 0; k <= N; ++k)
        for (int i = 0; i < nx; ++i) {
            int o = (k * nx + i) * 2;
            double dx = W->ds[k * ns + i];
            W->dtx[o] = W->dtx[o + 1] = W->dlx[o] = W->dlx[o + 1] = 0;
            if (k > 0 && isfinite(W->xub[k * nx + i])) {
                W->dtx[o] = -W->rix[o] - dx;
                W->dlx[o] = (-rcx[o] - W->lx[o] * W->dtx[o]) * W->itx[o];
            }
            if (k > 0 && isfinite(W->xlb[k * nx + i])) {
                W->dtx[o + 1] = -W->rix[o + 1] + dx;
                W->dlx[o + 1] = (-rcx[o + 1] - W->lx[o + 1] * W->dtx[o + 1]) * W->itx[o + 1];
            }
        }
    for (int k = 0; k < N; ++k)
        for (int i = 0; i < nu; ++i) {
            int o = (k * nu + i) * 2;
            double du = W->du[k * nu + i];
            W->dtu[o] = W->dtu[o + 1] = W->dlu[o] = W->dlu[o + 1] = 0;
            if (isfinite(W->uub[k * nu + i])) {
                W->dtu[o] = -W->riu[o] - du;
                W->dlu[o] = (-rcu[o] - W->lu[o] * W->dtu[o]) * W->itu[o];
            }
            if (isfinite(W->ulb[k * nu + i])) {
                W->dtu[o + 1] = -W->riu[o + 1] + du;
                W->dlu[o + 1] = (-rcu[o + 1] - W->lu[o + 1] * W->dtu[o + 1]) * W->itu[o + 1];
            }
        }
    {
        const int kp = P->kp;
        double dv[MAXNV];
        for (int i = 0; i < ns; ++i) dv[i] = W->ds[kp * ns + i];
        for (int i = 0; i < nu; ++i) dv[ns + i] = (kp < N) ? W->du[kp * nu + i] : 0.0;
        for (int r = 0; r < P->mp; ++r) {
            const double* F = P->Fp + (size_t)r * nv;
            double a = 0;
            for (int j = 0; j < nv; ++j) a += F[j] * dv[j];
            W->dtp[r] = -W->rip[r] - a;
            W->dlp[r] = (-rcp[r] - W->lp[r] * W->dtp[r]) * W->itp[r];
        }
    }
}

static double max_step(const prob_t* P, work_t* W) {
    /* alpha = min(1, 1 / max(-dt/t, -dlam/lam)) over the present rows */
    const int N = P->N, nx = P->nx, nu = P->nu;
    double rm = 0.0;
#define RATIO(dv, iv) { const double q = -(dv) * (iv); if (q > rm) rm = q; }
    for (int k = 1; k <= N; ++k)
        for (int i = 0; i < nx; ++i) {
            int o = (k * nx + i) * 2;
            if (isfinite(W->xub[k * nx + i])) { RATIO(W->dtx[o], W->itx[o]); RATIO(W->dlx[o], W->ilx[o]); }
            if (isfinite(W->xlb[k * nx + i])) { RATIO(W->dtx[o + 1], W->itx[o + 1]); RATIO(W->dlx[o + 1], W->ilx[o + 1]); }
        }
    for (int k = 0; k < N; ++k)
        for (int i = 0; i < nu; ++i) {
            int o = (k * nu + i) * 2;
            if (isfinite(W->uub[k * nu + i])) { RATIO(W->dtu[o], W->itu[o]); RATIO(W->dlu[o], W->ilu[o]); }
            if (isfinite(W->ulb[k * nu + i])) { RATIO(W->dtu[o + 1], W->itu[o + 1]); RATIO(W->dlu[o + 1], W->ilu[o + 1]); }
        }
    for (int r = 0; r < P->mp; ++r) { RATIO(W->dtp[r], W->itp[r]); RATIO(W->dlp[r], W->ilp[r]); }
#undef RATIO
    return rm > 1.0 ? 1.0 / rm : 1.0;
}

static double comp_s2(const prob_t* P, work_t* W) {
    /* sum dt dlam over the present rows */
    const int N = P->N, nx = P->nx, nu = P->nu;
    double s = 0;
    for (int k = 1; k <= N; ++k)
        for (int i = 0; i < nx; ++i) {
            int o = (k * nx + i) * 2;
            if (isfinite(W->xub[k * nx + i])) s += W->dtx[o] * W->dlx[o];
            if (isfinite(W->xlb[k * nx + i])) s += W->dtx[o + 1] * W->dlx[o + 1];
        }
    for (int k = 0; k < N; ++k)
        for (int i = 0; i < nu; ++i) {
            int o = (k * nu + i) * 2;
            if (isfinite(W->uub[k * nu + i])) s += W->dtu[o] * W->dlu[o];
            if (isfinite(W->ulb[k * nu + i])) s += W->dtu[o + 1] * W->dlu[o + 1];
        }
    for (int r = 0; r < P->mp; ++r) s += W->dtp[r] * W->dlp[r];
    return s;
}

/* ---------------- active-set polish ---------------- */
/* Rows with lam > t at the end of the IPM are taken as equalities and the others are dropped; the
 * equality-constrained QP is solved by augmented-Lagrangian iterations on the same Riccati
 * factorisation (weight rho on the active rows, D = 0 elsewhere: one factorisation per round),
 * nu += rho (C v - b) after each solve.  Rows whose multiplier turns negative leave the set and
 * violated rows enter it, for up to POL_ROUNDS rounds.  The polished point replaces the IPM
 * iterate only if it is primal feasible, dual feasible and stationary; it is what makes weakly
 * active (degenerate) rows, whose slack and multiplier both stay ~sqrt(mu), and problems with
 * multipliers ~1e3-1e5 (D = lam/t beyond fp64 range near mu = 1e-14) end at
 * the exact optimum. */
#define FOR_ROWS(BX, BU, BP)                                                                    \
    for (int i = 0; i < nxr; ++i) {                                                            \
        const int k_ = i / (2 * nx), xi_ = (i / 2) % nx;                                        \
        if (!(k_ > 0 && isfinite((i & 1) ? W->xlb[k_ * nx + xi_] : W->xub[k_ * nx + xi_])))   \
            continue;                                                                           \
        BX;                                                                                     \
    }                                                                                           \
    for (int i = 0; i < nur; ++i) {                                                            \
        if (!isfinite((i & 1) ? W->ulb[i / 2] : W->uub[i / 2])) continue;                       \
        BU;                                                                                     \
    }                                                                                           \
    for (int i = 0; i < mp; ++i) { BP; }

static double poly_fdv(const prob_t* P, const work_t* W, int r);

static int polish(const prob_t* P, work_t* W, double bs, double rho, double* kkt_out) {
    const int N = P->N, nx = P->nx, ns = P->ns;
    const int nxr = (N + 1) * nx * 2, nur = N * P->nu * 2, mp = P->mp;
    const int S = (N + 1) * ns, U = N * P->nu;
    /* keep the IPM iterate for the fall-back */
    const size_t tot = 2 * (size_t)S + U + 2 * ((size_t)nxr + nur + mp);
    double* sv = (double*)malloc(sizeof(double) * tot);
    double* q = sv;
#define SAVE(a, n) do { memcpy(q, a, sizeof(double) * (n)); q += (n); } while (0)
#define LOAD(a, n) do { memcpy(a, q, sizeof(double) * (n)); q += (n); } while (0)
    SAVE(W->s, S); SAVE(W->pi, S); SAVE(W->u, U); SAVE(W->tx, nxr); SAVE(W->lx, nxr);
    SAVE(W->tu, nur); SAVE(W->lu, nur); SAVE(W->tp, mp); SAVE(W->lp, mp);
    memset(W->wx, 0, sizeof(double) * nxr); memset(W->wu, 0, sizeof(double) * nur);
    memset(W->wp, 0, sizeof(double) * mp);
    FOR_ROWS({ if (W->lx[i] > W->tx[i]) W->wx[i] = rho; else W->lx[i] = 0.0; },
             { if (W->lu[i] > W->tu[i]) W->wu[i] = rho; else W->lu[i] = 0.0; },
             { if (W->lp[i] > W->tp[i]) W->wp[i] = rho; else W->lp[i] = 0.0; })
    /* t = 0: the row residual C v + t - b is the constraint value C v - b */
    memset(W->tx, 0, sizeof(double) * nxr); memset(W->tu, 0, sizeof(double) * nur);
    memset(W->tp, 0, sizeof(double) * mp);
    W->pol = 1;
    W->rip_live = 0;
    double stat = 0, feas = 0, cs, gs = 0, viol = 0;
    int mc, ok = 0;
    for (int rd = 0; rd < POL_ROUNDS && !ok; ++rd) {
        residuals(P, W, &stat, &feas, &cs, &mc, &gs);
        if (factor(P, W)) break;
        /* one augmented-Lagrangian step: v <- argmin_v AL(v, nu) (the Newton step is exact on the
         * quadratic AL), then conjugate gradients on the multipliers of the active rows for
         * r(nu) = C v(nu) - b = 0: r is affine in nu with dr/dnu = -M, M = C (H + rho C'C)^{-1} C'
         * SPD, so CG converges in a few steps where the plain multiplier update nu += rho r
         * contracts by 1 / (1 + rho sigma) per step - slow on nearly dependent active rows
         * (a state box row held over consecutive stages: C4 instance 28 at N = 80, sigma_min of
         * the active rows 6.5e-5).  Each CG step is one solve on the same
         * factorisation with right-hand side C'p (stage residuals and dynamics residual zero). */
        /* POL_PASS passes of [AL step + CG]: the AL step from the exact residuals is an iterative
         * refinement of the stationarity, which the factorisation with rho ~ 1e9 resolves to
         * ~eps rho |C v| per solve (C4 instances 20695 / 63175 at N = 100) */
        for (int pass = 0; pass < POL_PASS; ++pass) {
            if (pass > 0) residuals(P, W, &stat, &feas, &cs, &mc, &gs);
            prep_iter(P, W);
            solve_kkt(P, W, W->dtx, W->dtu, W->dtp);
            for (int i = 0; i < S; ++i) { W->s[i] += W->ds[i]; W->pi[i] += W->dpi[i]; }
            for (int i = 0; i < U; ++i) W->u[i] += W->du[i];
            residuals(P, W, &stat, &feas, &cs, &mc, &gs);
            {
                double* cr = W->cgr;                      /* r on the active rows, 0 elsewhere */
                double* cp = W->cgp;
                double rr = 0.0, va = 0.0;
                FOR_ROWS({ cr[i] = W->wx[i] > 0 ? W->rix[i] : 0.0; },
                         { cr[nxr + i] = W->wu[i] > 0 ? W->riu[i] : 0.0; },
                         { cr[nxr + nur + i] = W->wp[i] > 0 ? W->rip[i] : 0.0; })
                for (int i = 0; i < nxr + nur + mp; ++i) { cp[i] = cr[i]; rr += cr[i] * cr[i]; va = fmax(va, fabs(cr[i])); }
                int cg = 1;
                double va_prev = INFINITY;
                for (int j = 0; j < POL_CG && va > 1e-14 * (1.0 + bs) && isfinite(rr); ++j) {
                    if (!cg) {
                        /* plain multiplier step (nearly dependent active rows: M numerically
                         * singular); the AL solve from the new nu */
                        residuals(P, W, &stat, &feas, &cs, &mc, &gs);
                        FOR_ROWS({ W->lx[i] += W->wx[i] * W->rix[i]; }, { W->lu[i] += W->wu[i] * W->riu[i]; },
                                 { W->lp[i] += W->wp[i] * W->rip[i]; })
                        residuals(P, W, &stat, &feas, &cs, &mc, &gs);
                        prep_iter(P, W);
                        solve_kkt(P, W, W->dtx, W->dtu, W->dtp);
                        for (int i = 0; i < S; ++i) { W->s[i] += W->ds[i]; W->pi[i] += W->dpi[i]; }
                        for (int i = 0; i < U; ++i) W->u[i] += W->du[i];
                        residuals(P, W, &stat, &feas, &cs, &mc, &gs);
                        va = 0.0;
                        FOR_ROWS({ if (W->wx[i] > 0) va = fmax(va, fabs(W->rix[i])); },
                                 { if (W->wu[i] > 0) va = fmax(va, fabs(W->riu[i])); },
                                 { if (W->wp[i] > 0) va = fmax(va, fabs(W->rip[i])); })
                        if (getenv("CPU_IPM_TRACE")) fprintf(stderr, "   alm %d va %.3e\n", j, va);
                        if (va >= POL_STAG * va_prev) break;
                        va_prev = va;
                        continue;
                    }
                    /* direction solve: e = p on the active rows (rix = p / rho), zero stage residuals */
                    memset(W->rs, 0, sizeof(double) * S); memset(W->ru, 0, sizeof(double) * U);
                    memset(W->re, 0, sizeof(double) * N * ns);
                    FOR_ROWS({ W->rix[i] = cp[i] / rho; }, { W->riu[i] = cp[nxr + i] / rho; },
                             { W->rip[i] = cp[nxr + nur + i] / rho; })
                    prep_iter(P, W);
                    solve_kkt(P, W, W->dtx, W->dtu, W->dtp);
                    /* M p = -C dv on the active rows; alpha = r'r / p'Mp */
                    double pq = 0.0, pp = 0.0;
                    FOR_ROWS({ const double c_ = (i & 1) ? W->ds[k_ * ns + xi_] : -W->ds[k_ * ns + xi_];
                               W->dtx[i] = W->wx[i] > 0 ? c_ : 0.0; pq += cp[i] * W->dtx[i]; },
                             { const double c_ = (i & 1) ? W->du[i / 2] : -W->du[i / 2];
                               W->dtu[i] = W->wu[i] > 0 ? c_ : 0.0; pq += cp[nxr + i] * W->dtu[i]; },
                             { W->dtp[i] = W->wp[i] > 0 ? -poly_fdv(P, W, i) : 0.0; pq += cp[nxr + nur + i] * W->dtp[i]; })
                    for (int i = 0; i < nxr + nur + mp; ++i) pp += cp[i] * cp[i];
                    /* the eigenvalues of M lie in (0, 1/rho): a Rayleigh quotient below 1e-8 / rho is a
                     * numerically singular direction (dependent rows) - plain multiplier steps from here */
                    if (!(pq * rho > POL_CG_SING * pp)) {
                        cg = 0;
                        if (getenv("CPU_IPM_TRACE")) fprintf(stderr, "   cg %d singular (rayleigh rho %.3e)\n", j, pq * rho / pp);
                        continue;
                    }
                    const double al = rr / pq;
                    for (int i = 0; i < S; ++i) { W->s[i] += al * W->ds[i]; W->pi[i] += al * W->dpi[i]; }
                    for (int i = 0; i < U; ++i) W->u[i] += al * W->du[i];
                    double rn = 0.0;
                    va = 0.0;
                    FOR_ROWS({ W->lx[i] += al * cp[i]; cr[i] -= al * W->dtx[i]; },
                             { W->lu[i] += al * cp[nxr + i]; cr[nxr + i] -= al * W->dtu[i]; },
                             { W->lp[i] += al * cp[nxr + nur + i]; cr[nxr + nur + i] -= al * W->dtp[i]; })
                    for (int i = 0; i < nxr + nur + mp; ++i) { rn += cr[i] * cr[i]; va = fmax(va, fabs(cr[i])); }
                    const double be = rn / rr;
                    for (int i = 0; i < nxr + nur + mp; ++i) cp[i] = cr[i] + be * cp[i];
                    rr = rn;
                    if (getenv("CPU_IPM_TRACE")) fprintf(stderr, "   cg %d va %.3e alpha*rho^-1 %.3e\n", j, va, al / rho);
                }
                /* the Lagrangian multipliers of v(nu): nu + rho r (exact stationarity of the AL) */
                residuals(P, W, &stat, &feas, &cs, &mc, &gs);
                FOR_ROWS({ W->lx[i] += W->wx[i] * W->rix[i]; }, { W->lu[i] += W->wu[i] * W->riu[i]; },
                         { W->lp[i] += W->wp[i] * W->rip[i]; })
            }
            residuals(P, W, &stat, &feas, &cs, &mc, &gs);
            double va2 = 0.0;
            FOR_ROWS({ if (W->wx[i] > 0) va2 = fmax(va2, fabs(W->rix[i])); },
                     { if (W->wu[i] > 0) va2 = fmax(va2, fabs(W->riu[i])); },
                     { if (W->wp[i] > 0) va2 = fmax(va2, fabs(W->rip[i])); })
            if (getenv("CPU_IPM_TRACE")) fprintf(stderr, "  pass %d stat %.3e va %.3e\n", pass, stat, va2);
            if (stat <= 1e-8 * (1.0 + gs) && va2 <= 1e-12 * (1.0 + bs)) break;
        }
        residuals(P, W, &stat, &feas, &cs, &mc, &gs);
        double va = 0.0, lneg = 0.0, lmx = 0.0;
        viol = 0.0;
        FOR_ROWS({ viol = fmax(viol, W->rix[i]); if (W->wx[i] > 0) { va = fmax(va, fabs(W->rix[i])); lneg = fmin(lneg, W->lx[i]); lmx = fmax(lmx, W->lx[i]); } },
                 { viol = fmax(viol, W->riu[i]); if (W->wu[i] > 0) { va = fmax(va, fabs(W->riu[i])); lneg = fmin(lneg, W->lu[i]); lmx = fmax(lmx, W->lu[i]); } },
                 { viol = fmax(viol, W->rip[i]); if (W->wp[i] > 0) { va = fmax(va, fabs(W->rip[i])); lneg = fmin(lneg, W->lp[i]); lmx = fmax(lmx, W->lp[i]); } })
        double fe = 0.0;
        for (int i = 0; i < N * ns; ++i) fe = fmax(fe, fabs(W->re[i]));
        const double tf = 1e-12 * (1.0 + bs), td = 1e-9 * (1.0 + lmx);
        ok = isfinite(stat) && stat <= 1e-8 * (1.0 + gs) && viol <= tf && va <= tf && lneg >= -td && fe <= tf;
        if (getenv("CPU_IPM_TRACE"))
            fprintf(stderr, "polish round %d: stat %.3e (tol %.3e) viol %.3e act %.3e lneg %.3e lmax %.3e dyn %.3e -> %d\n",
                    rd, stat, 1e-8 * (1.0 + gs), viol, va, lneg, lmx, fe, ok);
        if (ok) break;
        /* active-set correction: negative multipliers leave, violated rows enter */
        int ch = 0;
        FOR_ROWS({ if (W->wx[i] > 0 && W->lx[i] < -td) { W->wx[i] = 0; W->lx[i] = 0; ++ch; } else if (W->wx[i] == 0 && W->rix[i] > tf) { W->wx[i] = rho; ++ch; } },
                 { if (W->wu[i] > 0 && W->lu[i] < -td) { W->wu[i] = 0; W->lu[i] = 0; ++ch; } else if (W->wu[i] == 0 && W->riu[i] > tf) { W->wu[i] = rho; ++ch; } },
                 { if (W->wp[i] > 0 && W->lp[i] < -td) { W->wp[i] = 0; W->lp[i] = 0; ++ch; } else if (W->wp[i] == 0 && W->rip[i] > tf) { W->wp[i] = rho; ++ch; } })
        if (!ch) break;
    }
    W->pol = 0;
    if (ok) {
        /* slacks of the polished point t = b - C v (>= 0 up to tf), multipliers >= 0 */
        for (int i = 0; i < nxr; ++i) { W->tx[i] = fmax(-W->rix[i], 0.0); W->lx[i] = fmax(W->lx[i], 0.0); }
        for (int i = 0; i < nur; ++i) { W->tu[i] = fmax(-W->riu[i], 0.0); W->lu[i] = fmax(W->lu[i], 0.0); }
        for (int r = 0; r < mp; ++r) { W->tp[r] = fmax(-W->rip[r], 0.0); W->lp[r] = fmax(W->lp[r], 0.0); }
        kkt_out[0] = stat; kkt_out[1] = viol; kkt_out[2] = 0.0;
    } else {
        q = sv;
        LOAD(W->s, S); LOAD(W->pi, S); LOAD(W->u, U); LOAD(W->tx, nxr); LOAD(W->lx, nxr);
        LOAD(W->tu, nur); LOAD(W->lu, nur); LOAD(W->tp, mp); LOAD(W->lp, mp);
    }
#undef SAVE
#undef LOAD
    free(sv);
    return ok;
}
#undef FOR_ROWS

/* ---------------- one instance ---------------- */
typedef struct {
    int max_iter;
    double tol_stat, tol_feas, tol_comp, tau;
    int polish;
} opts_t;

/* Fp(r,:) [ds_kp; du_kp] in the kernel's order (fdot) */
static double poly_fdv(const prob_t* P, const work_t* W, int r) {
    const int ns = P->ns, nu = P->nu, nv = P->nv, kp = P->kp;
    const double* F = P->Fp + (size_t)r * nv;
    double acc = 0.0;
    for (int j = 0; j < ns; ++j) acc += F[j] * W->ds[kp * ns + j];
    for (int j = 0; j < nu; ++j) acc += F[ns + j] * ((kp < P->N) ? W->du[kp * nu + j] : 0.0);
    return acc;
}

/* diagnostic (CPU_IPM_ITER): per-iteration residuals and step lengths on stderr */
static int ipm_trace(void) {
    static int v = -1;
    if (v < 0) v = getenv("CPU_IPM_ITER") != NULL;
    return v;
}

static int solve_one(const prob_t* P, work_t* W, const opts_t* op, int* iters, double* kkt, int* polished) {
    const int N = P->N, nx = P->nx, nu = P->nu, ns = P->ns;
    W->rip_live = 0;
    W->fe_rows = 0.0;
    W->pol = 0;
    if (polished) *polished = 0;
    const int nxr = (N + 1) * nx * 2, nur = N * nu * 2;
    double stat, feas, cs, gs;
    int mc;
    double bs = 0;
    for (int i = 0; i < nx; ++i) bs = fmax(bs, fabs(W->s[i]));
    for (int k = 1; k <= N; ++k)
        for (int i = 0; i < nx; ++i) {
            if (isfinite(W->xub[k * nx + i])) bs = fmax(bs, fabs(W->xub[k * nx + i]));
            if (isfinite(W->xlb[k * nx + i])) bs = fmax(bs, fabs(W->xlb[k * nx + i]));
        }
    for (int k = 0; k < N * nu; ++k) {
        if (isfinite(W->uub[k])) bs = fmax(bs, fabs(W->uub[k]));
        if (isfinite(W->ulb[k])) bs = fmax(bs, fabs(W->ulb[k]));
    }
    for (int r = 0; r < P->mp; ++r) bs = fmax(bs, fabs(W->hp[r]));
    /* init: t = lam = 1 on every row, unit-scaled least-squares Newton solve (rc = t o lam) */
    for (int i = 0; i < nxr; ++i) { W->tx[i] = 1.0; W->lx[i] = 1.0; }
    for (int i = 0; i < nur; ++i) { W->tu[i] = 1.0; W->lu[i] = 1.0; }
    for (int r = 0; r < P->mp; ++r) { W->tp[r] = 1.0; W->lp[r] = 1.0; }
    double *rcx = W->rcb;
    double *rcu = rcx + nxr, *rcp = rcu + nur;
    for (int i = 0; i < nxr + nur + P->mp; ++i) rcx[i] = 1.0;
    residuals(P, W, &stat, &feas, &cs, &mc, &gs);
    if (factor(P, W)) return -8;
    prep_iter(P, W);
    solve_kkt(P, W, rcx, rcu, rcp);
    for (int i = 0; i < (N + 1) * ns; ++i) { W->s[i] += W->ds[i]; W->pi[i] += W->dpi[i]; }
    for (int i = 0; i < N * nu; ++i) W->u[i] += W->du[i];
    /* tt = b - C v = t_old + dt = 1 + dt ; lam~ = -tt ; shift */
    double tmin = INFINITY, tmax = -INFINITY;
#define PRESENT_X(k, i, o) ((k) > 0 && isfinite(((o) & 1) ? W->xlb[(k) * nx + (i)] : W->xub[(k) * nx + (i)]))
#define PRESENT_U(k, i, o) (isfinite(((o) & 1) ? W->ulb[(k) * nu + (i)] : W->uub[(k) * nu + (i)]))
    for (int k = 0; k <= N; ++k)
        for (int i = 0; i < nx; ++i)
            for (int h = 0; h < 2; ++h)
                if (PRESENT_X(k, i, h)) {
                    double t = 1.0 + W->dtx[(k * nx + i) * 2 + h];
                    tmin = fmin(tmin, t); tmax = fmax(tmax, t);
                }
    for (int k = 0; k < N; ++k)
        for (int i = 0; i < nu; ++i)
            for (int h = 0; h < 2; ++h)
                if (PRESENT_U(k, i, h)) {
                    double t = 1.0 + W->dtu[(k * nu + i) * 2 + h];
                    tmin = fmin(tmin, t); tmax = fmax(tmax, t);
                }
    for (int r = 0; r < P->mp; ++r) {
        double t = 1.0 + W->dtp[r];
        tmin = fmin(tmin, t); tmax = fmax(tmax, t);
    }
    double shp = (tmin <= 0) ? 1.0 - tmin : 0.0;
    double shd = (tmax >= 0) ? 1.0 + tmax : 0.0;
    for (int k = 0; k <= N; ++k)
        for (int i = 0; i < nx; ++i)
            for (int h = 0; h < 2; ++h) {
                int o = (k * nx + i) * 2 + h;
                if (PRESENT_X(k, i, h)) {
                    double t = 1.0 + W->dtx[o];
                    W->tx[o] = t + shp; W->lx[o] = -t + shd;
                } else { W->tx[o] = 1.0; W->lx[o] = 0.0; }
            }
    for (int k = 0; k < N; ++k)
        for (int i = 0; i < nu; ++i)
            for (int h = 0; h < 2; ++h) {
                int o = (k * nu + i) * 2 + h;
                if (PRESENT_U(k, i, h)) {
                    double t = 1.0 + W->dtu[o];
                    W->tu[o] = t + shp; W->lu[o] = -t + shd;
                } else { W->tu[o] = 1.0; W->lu[o] = 0.0; }
            }
    {
        /* residuals of the shifted start (the kernel's update): full step, then + shp */
        double fe = 0.0;
        for (int k = 0; k <= N; ++k)
            for (int i = 0; i < nx; ++i)
                for (int h = 0; h < 2; ++h)
                    if (PRESENT_X(k, i, h)) fe = fmax(fe, fabs(shp));
        for (int k = 0; k < N; ++k)
            for (int i = 0; i < nu; ++i)
                for (int h = 0; h < 2; ++h)
                    if (PRESENT_U(k, i, h)) fe = fmax(fe, fabs(shp));
        for (int r = 0; r < P->mp; ++r) {
            const double fd = poly_fdv(P, W, r);
            W->rip[r] += 1.0 * (fd + W->dtp[r]);
            W->rip[r] += shp;
            fe = fmax(fe, fabs(W->rip[r]));
        }
        W->fe_rows = fe;
        W->rip_live = 1;
    }
    for (int r = 0; r < P->mp; ++r) {
        double t = 1.0 + W->dtp[r];
        W->tp[r] = t + shp; W->lp[r] = -t + shd;
    }
    /* main loop */
    int flag = 0, it;
    double mu = 0, mu_min = INFINITY;
    for (it = 0; it <= op->max_iter; ++it) {
        residuals(P, W, &stat, &feas, &cs, &mc, &gs);
        mu = cs / (mc > 0 ? mc : 1);
        if (stat <= op->tol_stat * (1.0 + gs) && feas <= op->tol_feas * (1.0 + bs) && mu <= op->tol_comp && W->cmax <= CMAX_K * op->tol_comp) { flag = 1; break; }
        if (ipm_trace())
            fprintf(stderr, "it %2d stat %.3e (tol %.3e) feas %.3e mu %.3e cmax %.3e gs %.3e\n", it, stat,
                    op->tol_stat * (1.0 + gs), feas, mu, W->cmax, gs);
        if (!(isfinite(stat) && isfinite(feas) && isfinite(mu))) { flag = -8; break; }
        if (mu > MU_BLOWUP * mu_min && feas > FEAS_GUARD * (1.0 + bs)) { flag = -2; break; }
        if (mu < mu_min) mu_min = mu;
        if (it == op->max_iter) break;
        if (factor(P, W)) { flag = -8; break; }
        prep_iter(P, W);
        for (int i = 0; i < nxr; ++i) rcx[i] = W->tx[i] * W->lx[i];
        for (int i = 0; i < nur; ++i) rcu[i] = W->tu[i] * W->lu[i];
        for (int r = 0; r < P->mp; ++r) rcp[r] = W->tp[r] * W->lp[r];
        solve_kkt(P, W, rcx, rcu, rcp);
        double a = max_step(P, W);
        const double a_pred_keep = a;
        /* along the affine direction t dlam + lam dt = -t lam: the complementarity after the
         * step is cs (1 - a) + a^2 sum dt dlam (the kernel's pred_pass) */
        double mua = (cs * (1.0 - a) + a * a * comp_s2(P, W)) / (mc > 0 ? mc : 1);
        double sg = mua / mu;
        sg = sg * sg * sg;
        /* a short predictor step on a feasible iterate: the second-order term dt_a dlam_a is
         * dropped (pure centring, Mehrotra's safeguard against the alternating stall of
         * nearly-degenerate rows; C4 instance 6264) */
        const double soc = (a < SOC_ALPHA && feas <= FEAS_GUARD * (1.0 + bs)) ? 0.0 : 1.0;
        for (int i = 0; i < nxr; ++i) rcx[i] = W->tx[i] * W->lx[i] + soc * (W->dtx[i] * W->dlx[i]) - sg * mu;
        for (int i = 0; i < nur; ++i) rcu[i] = W->tu[i] * W->lu[i] + soc * (W->dtu[i] * W->dlu[i]) - sg * mu;
        for (int r = 0; r < P->mp; ++r) rcp[r] = W->tp[r] * W->lp[r] + soc * (W->dtp[r] * W->dlp[r]) - sg * mu;
        solve_kkt(P, W, rcx, rcu, rcp);
        {
            /* step rule (round 5): a predictor step >= TAU_FAST_AFF marks a well-centred iterate
             * whose affine direction is nearly feasible - the corrector then goes to TAU_FAST of
             * the boundary while mu > TAU_FAST_MU, else tau.  Below ~1e-7 such steps overshoot
             * mu (DI instances of F5 went from 7e-8 to 1e-10 in one step and then stalled at
             * mu ~ 1e-17 with the stationarity residual stuck at 1.3x its tolerance: the barrier
             * Hessian ~ 1/mu resolves it no further).  At any mu, a predictor step >= TAU_FAST_END
             * (the affine direction is all but feasible: the Newton end phase, sigma ~ 0) takes the
             * fast corrector step too.  Iterations on the C port: C2 9.13 -> 7.20 (stored states;
             * max 16 -> 15), C3 12.60 -> 11.49, C5 9.54 -> 7.87, C4 10.29 -> 8.53 (the exact
             * classification unchanged). */
            const double tau = op->tau >= TAU_FAST_MIN &&
                                       ((a_pred_keep > TAU_FAST_AFF && mu > TAU_FAST_MU) || a_pred_keep >= TAU_FAST_END)
                                   ? fmax(op->tau, TAU_FAST) : op->tau;
            a = max_step(P, W) * tau;
        }
        if (a > 1.0) a = 1.0;
        if (ipm_trace()) fprintf(stderr, "   a_aff %.3e sigma %.3e soc %g a %.3e\n", a_pred_keep, sg, soc, a);
        {
            /* row residuals of the stepped iterate (the kernel's linear update) */
            double fe = 0.0;
            for (int k = 0; k <= N; ++k)
                for (int i = 0; i < nx; ++i)
                    for (int h = 0; h < 2; ++h)
                        if (PRESENT_X(k, i, h)) fe = fmax(fe, fabs((1.0 - a) * W->rix[(k * nx + i) * 2 + h]));
            for (int k = 0; k < N; ++k)
                for (int i = 0; i < nu; ++i)
                    for (int h = 0; h < 2; ++h)
                        if (PRESENT_U(k, i, h)) fe = fmax(fe, fabs((1.0 - a) * W->riu[(k * nu + i) * 2 + h]));
            for (int r = 0; r < P->mp; ++r) {
                const double fd = poly_fdv(P, W, r);
                W->rip[r] += a * (fd + W->dtp[r]);
                fe = fmax(fe, fabs(W->rip[r]));
            }
            W->fe_rows = fe;
        }
        for (int i = 0; i < (N + 1) * ns; ++i) { W->s[i] += a * W->ds[i]; W->pi[i] += a * W->dpi[i]; }
        for (int i = 0; i < N * nu; ++i) W->u[i] += a * W->du[i];
        for (int k = 0; k <= N; ++k)
            for (int i = 0; i < nx; ++i)
                for (int h = 0; h < 2; ++h)
                    if (PRESENT_X(k, i, h)) {
                        int o = (k * nx + i) * 2 + h;
                        W->tx[o] += a * W->dtx[o]; W->lx[o] += a * W->dlx[o];
                    }
        for (int k = 0; k < N; ++k)
            for (int i = 0; i < nu; ++i)
                for (int h = 0; h < 2; ++h)
                    if (PRESENT_U(k, i, h)) {
                        int o = (k * nu + i) * 2 + h;
                        W->tu[o] += a * W->dtu[o]; W->lu[o] += a * W->dlu[o];
                    }
        for (int r = 0; r < P->mp; ++r) { W->tp[r] += a * W->dtp[r]; W->lp[r] += a * W->dlp[r]; }
    }
    if (flag != -2 && op->polish > 0) {
        /* polish when the IPM did not converge (0 / -8: the factorisation left fp64 range) and,
         * with polish = 2, when it converged with a weakly active row
         * (max_i min(t_i, lam_i) > DEG_POLISH) */
        double degm = 0.0;
        for (int k = 0; k <= N; ++k)
            for (int i = 0; i < nx; ++i)
                for (int h = 0; h < 2; ++h)
                    if (PRESENT_X(k, i, h)) { const int o = (k * nx + i) * 2 + h; degm = fmax(degm, fmin(W->tx[o], W->lx[o])); }
        for (int k = 0; k < N; ++k)
            for (int i = 0; i < nu; ++i)
                for (int h = 0; h < 2; ++h)
                    if (PRESENT_U(k, i, h)) { const int o = (k * nu + i) * 2 + h; degm = fmax(degm, fmin(W->tu[o], W->lu[o])); }
        for (int r = 0; r < P->mp; ++r) degm = fmax(degm, fmin(W->tp[r], W->lp[r]));
        if (flag != 1 || (op->polish > 1 && degm > DEG_POLISH)) {
            double k3p[3];
            if (isfinite(gs) && polish(P, W, bs, POL_RHO * (1.0 + gs), k3p)) {
                flag = 1; stat = k3p[0]; feas = k3p[1]; mu = k3p[2];
                if (polished) *polished = 1;
            }
        }
    }
#undef PRESENT_X
#undef PRESENT_U
    *iters = it;
    kkt[0] = stat; kkt[1] = feas; kkt[2] = mu;
    return flag;
}

/* ---------------- batched entry ---------------- */
static double* alloc0(size_t n) { return (double*)calloc(n ? n : 1, sizeof(double)); }

int cpu_ocp_solve(const bqp_ocp_dims* d, int batch, const bqp_ocp_data* D, int max_iter,
                  double tol_stat, double tol_feas, double tol_comp, double tau, int nthreads,
                  double* x, double* u, double* theta, int* exitflag, int* iters, double* kkt3,
                  int polish, int* polished) {
    const int nx = d->nx, nu = d->nu, np = d->np, N = d->N;
    const int ns = nx + np, nv = ns + nu, mp = d->n_poly;
    if (ns > MAXNS || nu > MAXNU || nv > MAXNV || N < 1) return BQP_E_ARG;
    opts_t op = {max_iter, tol_stat, tol_feas, tol_comp, tau, polish};
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#endif
    int err = 0;
#pragma omp parallel
    {
        /* per-thread workspace */
        double* H = alloc0((size_t)(N + 1) * nv * nv);
        double* Fp = alloc0((size_t)mp * nv);
        work_t W;
        memset(&W, 0, sizeof(W));
        W.s = alloc0((N + 1) * ns); W.u = alloc0(N * nu); W.pi = alloc0((N + 1) * ns);
        W.g = alloc0((N + 1) * nv);
        W.xlb = alloc0((N + 1) * nx); W.xub = alloc0((N + 1) * nx);
        W.ulb = alloc0(N * nu); W.uub = alloc0(N * nu); W.hp = alloc0(mp);
        W.tx = alloc0((N + 1) * nx * 2); W.lx = alloc0((N + 1) * nx * 2);
        W.tu = alloc0(N * nu * 2); W.lu = alloc0(N * nu * 2);
        W.tp = alloc0(mp); W.lp = alloc0(mp);
        W.rs = alloc0((N + 1) * ns); W.ru = alloc0(N * nu); W.re = alloc0(N * ns);
        W.rix = alloc0((N + 1) * nx * 2); W.riu = alloc0(N * nu * 2); W.rip = alloc0(mp);
        W.ds = alloc0((N + 1) * ns); W.du = alloc0(N * nu); W.dpi = alloc0((N + 1) * ns);
        W.dtx = alloc0((N + 1) * nx * 2); W.dlx = alloc0((N + 1) * nx * 2);
        W.dtu = alloc0(N * nu * 2); W.dlu = alloc0(N * nu * 2);
        W.dtp = alloc0(mp); W.dlp = alloc0(mp);
        W.Ptab = alloc0((size_t)(N + 1) * ns * ns); W.Ktab = alloc0((size_t)N * nu * ns);
        W.Phit = alloc0((size_t)N * ns * ns);
        W.Rinv = alloc0((size_t)N * nu * nu); W.p = alloc0((N + 1) * ns);
        W.qs = alloc0((N + 1) * ns); W.qu = alloc0(N * nu); W.wv = alloc0(N * ns); W.cw = alloc0(N * ns);
        W.qt = alloc0(N * ns); W.qh = alloc0(N * ns); W.kff = alloc0(N * nu); W.f = alloc0(N * ns);
        W.Dx = alloc0((N + 1) * nx); W.Du = alloc0(N * nu); W.FD = alloc0(nv * nv);
        W.itx = alloc0((N + 1) * nx * 2); W.ilx = alloc0((N + 1) * nx * 2);
        W.itu = alloc0(N * nu * 2); W.ilu = alloc0(N * nu * 2); W.itp = alloc0(mp); W.ilp = alloc0(mp);
        W.wx = alloc0((N + 1) * nx * 2); W.wu = alloc0(N * nu * 2); W.wp = alloc0(mp);
        W.cgr = alloc0((N + 1) * nx * 2 + N * nu * 2 + mp); W.cgp = alloc0((N + 1) * nx * 2 + N * nu * 2 + mp);
        W.rcb = alloc0((N + 1) * nx * 2 + N * nu * 2 + mp + 1);
        prob_t P;
        memset(&P, 0, sizeof(P));
        P.nx = nx; P.nu = nu; P.np = np; P.ns = ns; P.nv = nv; P.N = N; P.mp = mp;
        P.kp = d->poly_stage;
        P.H = H; P.Fp = Fp;
#pragma omp for schedule(dynamic, 4)
        for (int b = 0; b < batch; ++b) {
            const double* A = D->A + b * D->sA;
            const double* B = D->B + b * D->sB;
            for (int i = 0; i < ns; ++i)
                for (int j = 0; j < ns; ++j)
                    P.Abar[i][j] = (i < nx && j < nx) ? A[j * nx + i] : (i == j ? 1.0 : 0.0);
            for (int i = 0; i < ns; ++i)
                for (int j = 0; j < nu; ++j) P.Bbar[i][j] = (i < nx) ? B[j * nx + i] : 0.0;
            for (int i = 0; i < ns; ++i) P.cbar[i] = (i < nx && D->c) ? D->c[b * D->sc + i] : 0.0;
            /* permuted H (internal [x th u]) from W (external [x u th], column-major) */
            const double* Wb = D->W + b * D->sW;
            for (int k = 0; k <= N; ++k)
                for (int i = 0; i < nv; ++i)
                    for (int j = 0; j < nv; ++j) {
                        int ei = perm_of(&P, i), ej = perm_of(&P, j);
                        double v = Wb[(size_t)k * nv * nv + (size_t)ej * nv + ei];
                        if (k == N && (i >= ns || j >= ns)) v = 0.0;
                        H[((size_t)k * nv + i) * nv + j] = v;
                    }
            for (int k = 0; k <= N; ++k)
                for (int i = 0; i < nv; ++i) {
                    double v = D->w ? D->w[b * D->sw + (size_t)k * nv + perm_of(&P, i)] : 0.0;
                    W.g[k * nv + i] = (k == N && i >= ns) ? 0.0 : v;
                }
            const double* Fb = D->Fp ? D->Fp + b * D->sFp : NULL;
            for (int r = 0; r < mp; ++r)
                for (int i = 0; i < nv; ++i) {
                    double v = Fb[(size_t)perm_of(&P, i) * mp + r];
                    Fp[(size_t)r * nv + i] = (P.kp == N && i >= ns) ? 0.0 : v;
                }
            for (int r = 0; r < mp; ++r) W.hp[r] = D->hp[b * D->shp + r];
            for (int i = 0; i < (N + 1) * nx; ++i) {
                W.xlb[i] = D->xlb ? D->xlb[b * D->sxb + i] : -INFINITY;
                W.xub[i] = D->xub ? D->xub[b * D->sxb + i] : INFINITY;
            }
            for (int i = 0; i < N * nu; ++i) {
                W.ulb[i] = D->ulb ? D->ulb[b * D->sub + i] : -INFINITY;
                W.uub[i] = D->uub ? D->uub[b * D->sub + i] : INFINITY;
            }
            memset(W.s, 0, sizeof(double) * (N + 1) * ns);
            memset(W.u, 0, sizeof(double) * N * nu);
            memset(W.pi, 0, sizeof(double) * (N + 1) * ns);
            for (int i = 0; i < nx; ++i) W.s[i] = D->x0[b * D->sx0 + i];
            int it = 0;
            double k3[3] = {0, 0, 0};
            int pz = 0;
            int fl = solve_one(&P, &W, &op, &it, k3, &pz);
            if (polished) polished[b] = pz;
            if (fl == -8) { /* keep going; report */ }
            for (int k = 0; k <= N; ++k)
                for (int i = 0; i < nx; ++i) x[((size_t)b * (N + 1) + k) * nx + i] = W.s[k * ns + i];
            for (int k = 0; k < N; ++k)
                for (int i = 0; i < nu; ++i) u[((size_t)b * N + k) * nu + i] = W.u[k * nu + i];
            for (int i = 0; i < np; ++i) theta[(size_t)b * np + i] = W.s[nx + i];
            exitflag[b] = fl;
            if (iters) iters[b] = it;
            if (kkt3) for (int i = 0; i < 3; ++i) kkt3[(size_t)b * 3 + i] = k3[i];
        }
        free(H); free(Fp);
        free(W.s); free(W.u); free(W.pi); free(W.g); free(W.xlb); free(W.xub); free(W.ulb);
        free(W.uub); free(W.hp); free(W.tx); free(W.lx); free(W.tu); free(W.lu); free(W.tp);
        free(W.lp); free(W.rs); free(W.ru); free(W.re); free(W.rix); free(W.riu); free(W.rip);
        free(W.ds); free(W.du); free(W.dpi); free(W.dtx); free(W.dlx); free(W.dtu); free(W.dlu);
        free(W.dtp); free(W.dlp); free(W.Ptab); free(W.Phit); free(W.Ktab); free(W.Rinv); free(W.p);
        free(W.qs); free(W.qu); free(W.wv); free(W.cw); free(W.qt); free(W.qh); free(W.kff); free(W.f); free(W.Dx);
        free(W.Du); free(W.FD); free(W.itx); free(W.ilx); free(W.itu); free(W.ilu); free(W.itp);
        free(W.ilp); free(W.wx); free(W.wu); free(W.wp); free(W.cgr); free(W.cgp); free(W.rcb);
    }
    return err;
}
