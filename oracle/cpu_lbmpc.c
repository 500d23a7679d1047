/* TEST INFRASTRUCTURE ONLY (see oracle/__init__.py): the CPU baseline of bench.py's CLL line
 * and a checker of the GPU learned-model closed loop (tests/test_cpu_lbmpc_host.py).
 *
 * C restatement of the product algorithm of bqp_closed_loop_sqp (csrc/bqp_api.cpp, kernels in
 * csrc/bqp_lbmpc.hip and csrc/bqp_dense.hip) for the DMS LBMPC closed loop of
 * DMS_LBMPC_casadi.m:157-218, one instance per OpenMP thread:
 *   per time step, at the measured state x (deviation dx = x - x_eq),
 *     SQP on z = [du_0..du_{N-1}; theta] (oracle/lbmpc.py sqp / dms_problem):
 *       learned rollout x+ = A x + B u + g(xi), g the Nadaraya-Watson estimate over the 8 x q
 *       window [X; Y; v] (casadiL2NW.m:14-28), forward sensitivities, Gauss-Newton model
 *       (oracle/lbmpc.py gn_model) plus the second-order term of the learned dynamics
 *       (newton_model, costate recursion) whenever that Hessian passes pd_cholesky (pivots above
 *       1e-10 max H_ii) - bqp_lbmpc.hip lbmpc_hess_kernel;
 *       QP min 0.5 d'Hd + f'd s.t. Ain d <= bin - Ain z by the dense Mehrotra IPM of
 *       oracle/dense_ipm.py (the algorithm of bqp_dense.hip) with its active-set polish after
 *       0 / -8 exits and, from SQP iteration 6 on, after every sub-problem (LB_POLISH_STALL);
 *       the update of lbmpc_update_kernel: KKT / stagnation test, Armijo on 2^-j, j = 0..7;
 *     u = u_eq + z[0] to the RK4 plant (DMS_LBMPC_casadi.m:297-304), the sample
 *     [dx1; dx2; du; Y; 1] into the window (utilities/get_data.m), the shifted warm start
 *     (:209-213).
 * Constraints (nominal model, constraintsLBMPC.m / DMS_LBMPC_casadi.m:262-276): F_x_d x_1 <=
 * h_x_d, F_T [x_1; theta] <= h_T, F_x x_k <= h_x and F_u u_{k-1} <= h_u for k = 1..N; affine
 * in z, built once (rows keep their nonzero column range, which the normal-equation products
 * use).  Only the DMS form (K = 0, nu = np = 1, nx = 4, running cost delta-weighted for k < N,
 * terminal cost on the learned x_N) - the CLL workload. */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

typedef struct {
    int N, q, max_iter;
    int nd, nT, nFx, nFu;
    double A[16], B[4], Q[16], R, P[16], T[16], LAM[4], PSI, xeq[4], ueq;
    double w_run, dt_plant, bw, lam_nw, tol;
    int hessian;                         /* 1: exact Hessian where positive definite */
    const double *Fxd, *hxd, *FT, *hT, *Fx, *hx, *Fu, *hu;   /* row-major */
} cll_prob;

#define NTRIAL 8
#define POL_STALL 6
#define PIV_FLOOR 1e-14
#define CONVEX_EPS 1e-10
#define MU_BLOWUP 1e6
#define Z_BIG 1e12
#define FEAS_GUARD 1e-8
#define CMAX_K 100.0
#define SOC_ALPHA 0.1
#define POL_ROUNDS 4

typedef struct {
    int n, m, N, q;
    double *Ain, *b0;                    /* m x n, constant part of the right-hand side */
    int *lo, *hi;                        /* nonzero column range of each row */
    double *bin, *bsh, *z, *d, *lam, *ztr;
    double *xL, *uL, *S, *dg, *d2g, *H, *Hg, *f;
    double *data;                        /* 8 x q, point i at data[8 i] */
    /* dense IPM */
    double *K, *t, *l, *dz, *dtt, *dl, *rd, *ri, *rc, *qv, *tmp, *zq;
    /* polish */
    int *idx;
    double *Y, *Sp, *w, *mult, *ra, *zn, *nu, *rin;
} cll_work;

static void *xcalloc(size_t n, size_t s) { return calloc(n ? n : 1, s); }

/* ---------------------------------------------------------------- Nadaraya-Watson -------- */
/* g (4), dg (4 x 3), d2g (4 x 3 x 3) at xi over the 8-row window (oracle/lbmpc.py nw_hess) */
static void nw_eval(const cll_prob *P, const double *data, const double xi[3], double g[4],
                    double *dg, double *d2g) {
    const double hinv2 = 1.0 / (P->bw * P->bw), c = 2.0 * hinv2;
    double s = 0, sy[4] = {0}, ds[3] = {0}, dsy[12] = {0}, s2[9] = {0}, sy2[36] = {0};
    for (int i = 0; i < P->q; ++i) {
        const double *p = data + 8 * i;
        const double d[3] = {p[0] - xi[0], p[1] - xi[1], p[2] - xi[2]};
        const double k = exp(-(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]) * hinv2);
        const double v = p[7];
        s += k * v;
        for (int r = 0; r < 4; ++r) sy[r] += p[3 + r] * k;
        if (!dg) continue;
        for (int a = 0; a < 3; ++a) {
            const double dk = c * k * d[a];
            ds[a] += dk * v;
            for (int r = 0; r < 4; ++r) dsy[3 * r + a] += p[3 + r] * dk;
        }
        if (!d2g) continue;
        for (int a = 0; a < 3; ++a)
            for (int b = 0; b < 3; ++b) {
                const double kd = k * d[a] * d[b];
                s2[3 * a + b] += kd * v;
                for (int r = 0; r < 4; ++r) sy2[9 * r + 3 * a + b] += p[3 + r] * kd;
            }
    }
    const double den = P->lam_nw + s;
    for (int r = 0; r < 4; ++r) g[r] = sy[r] / den;
    if (!dg) return;
    for (int r = 0; r < 4; ++r)
        for (int a = 0; a < 3; ++a) dg[3 * r + a] = (dsy[3 * r + a] - g[r] * ds[a]) / den;
    if (!d2g) return;
    /* d2k_j = k_j (c^2 d_j d_j' - c I): d2N_r = c^2 sy2_r - c sy_r I, d2D = c^2 s2 - c s I */
    for (int r = 0; r < 4; ++r)
        for (int a = 0; a < 3; ++a)
            for (int b = 0; b < 3; ++b) {
                const double id = a == b ? 1.0 : 0.0;
                const double d2N = c * c * sy2[9 * r + 3 * a + b] - c * sy[r] * id;
                const double d2D = c * c * s2[3 * a + b] - c * s * id;
                d2g[9 * r + 3 * a + b] = (d2N - g[r] * d2D - dg[3 * r + a] * ds[b] -
                                          ds[a] * dg[3 * r + b]) / den;
            }
}

/* ---------------------------------------------------------------- learned rollout -------- */
/* x_L, u_L of z from dx0; with sens the sensitivities S_k (4 x n, row-major, columns < k nonzero)
 * and the per-stage dg / d2g (oracle/lbmpc.py rollout).  Returns the cost (lbmpc.py cost). */
static double rollout(const cll_prob *P, cll_work *W, const double *dx0, const double *z,
                      int sens, int hess) {
    const int N = W->N, n = W->n;
    double *x = W->xL, *u = W->uL;
    const double th = z[n - 1];
    memcpy(x, dx0, 4 * sizeof(double));
    if (sens) memset(W->S, 0, sizeof(double) * 4 * n);
    double J = 0.0;
    for (int k = 0; k < N; ++k) {
        const double *xk = x + 4 * k;
        u[k] = z[k];
        const double xi[3] = {xk[0], xk[1], u[k]};
        double g[4], *dg = sens ? W->dg + 12 * k : NULL, *d2 = (sens && hess) ? W->d2g + 36 * k : NULL;
        nw_eval(P, W->data, xi, g, dg, d2);
        for (int r = 0; r < 4; ++r) {
            double v = P->B[r] * u[k] + g[r];
            for (int c = 0; c < 4; ++c) v += P->A[4 * r + c] * xk[c];
            x[4 * (k + 1) + r] = v;
        }
        /* running cost (DMS_LBMPC_casadi.m:229-233) */
        double ex[4], Je = 0.0;
        for (int r = 0; r < 4; ++r) ex[r] = xk[r] - P->LAM[r] * th;
        for (int r = 0; r < 4; ++r)
            for (int c = 0; c < 4; ++c) Je += ex[r] * P->Q[4 * r + c] * ex[c];
        const double eu = u[k] - P->PSI * th;
        J += P->w_run * (Je + P->R * eu * eu);
        if (sens) {
            const double *Sk = W->S + (size_t)4 * n * k;
            double *Sn = W->S + (size_t)4 * n * (k + 1);
            double Ak[16], Bk[4];
            for (int r = 0; r < 4; ++r) {
                for (int c = 0; c < 4; ++c) Ak[4 * r + c] = P->A[4 * r + c] + (c < 2 ? dg[3 * r + c] : 0.0);
                Bk[r] = P->B[r] + dg[3 * r + 2];
            }
            for (int r = 0; r < 4; ++r) {
                double *row = Sn + (size_t)r * n;
                for (int j = 0; j < k; ++j)
                    row[j] = Ak[4 * r] * Sk[j] + Ak[4 * r + 1] * Sk[n + j] + Ak[4 * r + 2] * Sk[2 * n + j] +
                             Ak[4 * r + 3] * Sk[3 * n + j];
                row[k] = Bk[r];
                for (int j = k + 1; j < n; ++j) row[j] = 0.0;
            }
        }
    }
    double eT[4], es[4], JT = 0.0;
    for (int r = 0; r < 4; ++r) { eT[r] = x[4 * N + r] - P->LAM[r] * th; es[r] = P->LAM[r] * th; }
    for (int r = 0; r < 4; ++r)
        for (int c = 0; c < 4; ++c) JT += eT[r] * P->P[4 * r + c] * eT[c] + es[r] * P->T[4 * r + c] * es[c];
    return J + JT;
}

/* H += s Jx' M Jx, f += s Jx' M e for Jx = [S_k (cols < kc) | theta column tc] (4 x n) */
static void add_quad(int n, double *H, double *f, const double *Sk, int kc, const double tc[4],
                     const double *M, const double e[4], double s) {
    const int th = n - 1;
    double Me[4];
    for (int r = 0; r < 4; ++r) {
        Me[r] = 0.0;
        for (int c = 0; c < 4; ++c) Me[r] += M[4 * r + c] * e[c];
    }
    /* MJ = M Jx on the active columns, column-major per active column */
    for (int a = 0; a <= kc; ++a) {
        const int ja = a < kc ? a : th;
        double ca[4], Mca[4];
        for (int r = 0; r < 4; ++r) ca[r] = a < kc ? (Sk ? Sk[(size_t)r * n + a] : 0.0) : tc[r];
        for (int r = 0; r < 4; ++r) {
            Mca[r] = 0.0;
            for (int c = 0; c < 4; ++c) Mca[r] += M[4 * r + c] * ca[c];
        }
        f[ja] += s * (ca[0] * Me[0] + ca[1] * Me[1] + ca[2] * Me[2] + ca[3] * Me[3]);
        for (int b = 0; b <= a; ++b) {
            const int jb = b < kc ? b : th;
            double cb[4];
            for (int r = 0; r < 4; ++r) cb[r] = b < kc ? (Sk ? Sk[(size_t)r * n + b] : 0.0) : tc[r];
            const double v = s * (Mca[0] * cb[0] + Mca[1] * cb[1] + Mca[2] * cb[2] + Mca[3] * cb[3]);
            H[(size_t)ja * n + jb] += v;
            if (ja != jb) H[(size_t)jb * n + ja] += v;
        }
    }
}

/* Gauss-Newton model (oracle/lbmpc.py gn_model) at the rollout in W (sens done) */
static void gn_model(const cll_prob *P, cll_work *W, const double *z) {
    const int N = W->N, n = W->n, th = n - 1;
    double *H = W->H, *f = W->f;
    memset(H, 0, sizeof(double) * n * n);
    memset(f, 0, sizeof(double) * n);
    const double tht = z[th], w2 = 2.0 * P->w_run;
    double mL[4];
    for (int r = 0; r < 4; ++r) mL[r] = -P->LAM[r];
    for (int k = 0; k < N; ++k) {
        double ex[4];
        for (int r = 0; r < 4; ++r) ex[r] = W->xL[4 * k + r] - P->LAM[r] * tht;
        add_quad(n, H, f, W->S + (size_t)4 * n * k, k, mL, P->Q, ex, w2);
        const double eu = W->uL[k] - P->PSI * tht;
        /* Ju = e_k - PSI e_theta */
        H[(size_t)k * n + k] += w2 * P->R;
        H[(size_t)k * n + th] -= w2 * P->R * P->PSI;
        H[(size_t)th * n + k] -= w2 * P->R * P->PSI;
        H[(size_t)th * n + th] += w2 * P->R * P->PSI * P->PSI;
        f[k] += w2 * P->R * eu;
        f[th] -= w2 * P->PSI * P->R * eu;
    }
    double eT[4], es[4];
    for (int r = 0; r < 4; ++r) { eT[r] = W->xL[4 * N + r] - P->LAM[r] * tht; es[r] = P->LAM[r] * tht; }
    add_quad(n, H, f, W->S + (size_t)4 * n * N, N, mL, P->P, eT, 2.0);
    add_quad(n, H, f, NULL, 0, P->LAM, P->T, es, 2.0);
}

/* H += sum_k Xi_k' W_k Xi_k with W_k = sum_i p_{k+1,i} d2g_i (oracle/lbmpc.py newton_model) */
static void newton_term(const cll_prob *P, cll_work *W, const double *z) {
    const int N = W->N, n = W->n;
    const double tht = z[n - 1];
    double pk[4];
    for (int r = 0; r < 4; ++r) {
        pk[r] = 0.0;
        for (int c = 0; c < 4; ++c) pk[r] += 2.0 * P->P[4 * r + c] * (W->xL[4 * N + c] - P->LAM[c] * tht);
    }
    for (int k = N - 1; k >= 0; --k) {
        const double *d2 = W->d2g + 36 * k, *dg = W->dg + 12 * k;
        double Wk[9];
        for (int e = 0; e < 9; ++e) Wk[e] = pk[0] * d2[e] + pk[1] * d2[9 + e] + pk[2] * d2[18 + e] + pk[3] * d2[27 + e];
        for (int a = 0; a < 3; ++a)
            for (int b = 0; b < a; ++b) Wk[3 * a + b] = Wk[3 * b + a] = 0.5 * (Wk[3 * a + b] + Wk[3 * b + a]);
        const double *S0 = W->S + (size_t)4 * n * k, *S1 = S0 + n;
        /* Xi columns: (S0[a], S1[a], 0) for a < k, (0, 0, 1) for a = k */
        for (int a = 0; a <= k; ++a) {
            const double xa[3] = {a < k ? S0[a] : 0.0, a < k ? S1[a] : 0.0, a < k ? 0.0 : 1.0};
            double wa[3];
            for (int r = 0; r < 3; ++r) wa[r] = Wk[3 * r] * xa[0] + Wk[3 * r + 1] * xa[1] + Wk[3 * r + 2] * xa[2];
            for (int b = 0; b <= a; ++b) {
                const double v = b < k ? wa[0] * S0[b] + wa[1] * S1[b] : wa[2];
                W->H[(size_t)a * n + b] += v;
                if (a != b) W->H[(size_t)b * n + a] += v;
            }
        }
        /* p_k = (A + [dg_:2 0])' p_{k+1} + 2 w Q e_k */
        double pn[4], ex[4];
        for (int r = 0; r < 4; ++r) ex[r] = W->xL[4 * k + r] - P->LAM[r] * tht;
        for (int c = 0; c < 4; ++c) {
            double v = 0.0;
            for (int r = 0; r < 4; ++r) v += (P->A[4 * r + c] + (c < 2 ? dg[3 * r + c] : 0.0)) * pk[r];
            for (int r = 0; r < 4; ++r) v += 2.0 * P->w_run * P->Q[4 * c + r] * ex[r];
            pn[c] = v;
        }
        memcpy(pk, pn, sizeof pk);
    }
}

/* ---------------------------------------------------------------- dense algebra ---------- */
/* in-place lower Cholesky of the row-major K (lower triangle read).  mode 0: every pivot floored
 * at thr (never fails); mode 1: returns 0 as soon as a pivot is not above thr */
static int chol(double *K, int n, double thr, int mode) {
    for (int j = 0; j < n; ++j) {
        double *Kj = K + (size_t)j * n;
        double d = Kj[j];
        for (int k = 0; k < j; ++k) d -= Kj[k] * Kj[k];
        if (!(d > thr)) {
            if (mode) return 0;
            d = thr;
        }
        d = sqrt(d);
        Kj[j] = d;
        const double id = 1.0 / d;
        for (int i = j + 1; i < n; ++i) {
            double *Ki = K + (size_t)i * n;
            double s = Ki[j];
            for (int k = 0; k < j; ++k) s -= Ki[k] * Kj[k];
            Ki[j] = s * id;
        }
    }
    return 1;
}

/* regularised exact Hessian (round 5): smallest grid shift delta_k = 1e-12 hd 4^k, k = 0..20,
 * with H + delta_k I positive definite (chol pivots above 1e-10 hd), by bisection over k; -1 if
 * none.  Same grid, test and search in oracle/lbmpc.py (hess_shift) and bqp_lbmpc.hip. */
#define HSHIFT(hd, k) ldexp(1e-12 * (hd), 2 * (k))
static int hess_try(cll_work *W, int n, double hd, double sh) {
    for (int i = 0; i < n; ++i) memcpy(W->K + (size_t)i * n, W->H + (size_t)i * n, sizeof(double) * (i + 1));
    for (int i = 0; i < n; ++i) W->K[(size_t)i * n + i] += sh;
    return chol(W->K, n, 1e-10 * hd, 1);
}
static int hess_shift_k(cll_work *W, int n, double hd) {
    int lo = -1, hi = 20;
    if (!hess_try(W, n, hd, HSHIFT(hd, hi))) return -1;
    while (hi - lo > 1) {
        const int mid = (lo + hi) / 2;
        if (hess_try(W, n, hd, HSHIFT(hd, mid))) hi = mid; else lo = mid;
    }
    return hi;
}

static void chol_solve(const double *L, int n, double *x) {
    for (int i = 0; i < n; ++i) {
        const double *Li = L + (size_t)i * n;
        double s = x[i];
        for (int k = 0; k < i; ++k) s -= Li[k] * x[k];
        x[i] = s / Li[i];
    }
    for (int i = n - 1; i >= 0; --i) {
        double s = x[i];
        for (int k = i + 1; k < n; ++k) s -= L[(size_t)k * n + i] * x[k];
        x[i] = s / L[(size_t)i * n + i];
    }
}

static double amax(const double *v, int n) {
    double a = 0.0;
    for (int i = 0; i < n; ++i) a = fmax(a, fabs(v[i]));
    return a;
}

static double rdot(const cll_work *W, int r, const double *v) {
    const double *g = W->Ain + (size_t)r * W->n;
    double s = 0.0;
    for (int j = W->lo[r]; j < W->hi[r]; ++j) s += g[j] * v[j];
    return s;
}

static void raxpy(const cll_work *W, int r, double a, double *v) {
    const double *g = W->Ain + (size_t)r * W->n;
    for (int j = W->lo[r]; j < W->hi[r]; ++j) v[j] += a * g[j];
}

/* K (lower) = H + sum_r D_r g_r g_r' */
static void normal_matrix(const cll_work *W, const double *D, const int *act, double rho) {
    const int n = W->n, m = W->m;
    for (int i = 0; i < n; ++i) memcpy(W->K + (size_t)i * n, W->H + (size_t)i * n, sizeof(double) * (i + 1));
    for (int r = 0; r < m; ++r) {
        const double dr = act ? (act[r] ? rho : 0.0) : D[r];
        if (dr == 0.0) continue;
        const double *g = W->Ain + (size_t)r * n;
        for (int a = W->lo[r]; a < W->hi[r]; ++a) {
            const double ga = dr * g[a];
            if (ga == 0.0) continue;
            double *Ka = W->K + (size_t)a * n;
            for (int b = W->lo[r]; b <= a; ++b) Ka[b] += ga * g[b];
        }
    }
}

static double kdiag_max(const cll_work *W) {
    double mx = 0.0;
    for (int i = 0; i < W->n; ++i) mx = fmax(mx, fabs(W->K[(size_t)i * W->n + i]));
    return mx;
}

/* CLL_TRACE=1: per sub-problem exit diagnostics on stderr (read once) */
static int cll_trace(void) {
    static int v = -1;
    if (v < 0) { const char *e = getenv("CLL_TRACE"); v = e ? (atoi(e) > 1 ? atoi(e) : 1) : 0; }
    return v;
}

/* ---------------------------------------------------------------- active-set polish ------ */
/* oracle/dense_ipm.py _polish (bqp_dense.hip dense_polish) without equality rows / bounds */
static int polish(cll_work *W, double bscale, double tol_stat) {
    const int n = W->n, m = W->m;
    const double *H = W->H, *f = W->f, *h = W->bsh, *z = W->zq;
    int *act = W->idx + m;              /* act flags after the index list */
    for (int r = 0; r < m; ++r) act[r] = W->l[r] > W->t[r];
    double hd = 0.0;
    for (int j = 0; j < n; ++j) hd = fmax(hd, fabs(H[(size_t)j * n + j]));
    const double rho = fmax(1.0, hd), tf = 1e-12 * (1.0 + bscale);
    for (int round = 0; round < POL_ROUNDS; ++round) {
        int na = 0;
        for (int r = 0; r < m; ++r)
            if (act[r]) {
                if (na == n) return 0;  /* more active rows than variables */
                W->idx[na++] = r;
            }
        normal_matrix(W, NULL, act, rho);
        chol(W->K, n, PIV_FLOOR * fmax(kdiag_max(W), 1e-300), 0);
        for (int k = 0; k < na; ++k) {
            const int r = W->idx[k];
            double *y = W->Y + (size_t)k * n;
            memset(y, 0, sizeof(double) * n);
            raxpy(W, r, 1.0, y);
            chol_solve(W->K, n, y);
            W->ra[k] = rdot(W, r, z) - h[r];
        }
        double smx = 0.0;
        for (int a = 0; a < na; ++a) {
            for (int b = 0; b <= a; ++b) W->Sp[(size_t)a * na + b] = rdot(W, W->idx[a], W->Y + (size_t)b * n);
            smx = fmax(smx, fabs(W->Sp[(size_t)a * na + a]));
        }
        for (int j = 0; j < n; ++j) {
            double v = f[j];
            for (int i = 0; i < n; ++i) v += H[(size_t)j * n + i] * z[i];
            W->w[j] = v;
        }
        for (int k = 0; k < na; ++k) raxpy(W, W->idx[k], rho * W->ra[k], W->w);
        for (int j = 0; j < n; ++j) W->w[j] = -W->w[j];
        chol_solve(W->K, n, W->w);
        if (na) chol(W->Sp, na, PIV_FLOOR * fmax(smx, 1e-300), 0);
        for (int k = 0; k < na; ++k) W->mult[k] = rdot(W, W->idx[k], W->w) + W->ra[k];
        if (na) chol_solve(W->Sp, na, W->mult);
        for (int j = 0; j < n; ++j) {
            double v = z[j] + W->w[j];
            for (int k = 0; k < na; ++k) v -= W->Y[(size_t)k * n + j] * W->mult[k];
            W->zn[j] = v;
        }
        memset(W->nu, 0, sizeof(double) * m);
        for (int k = 0; k < na; ++k) W->nu[W->idx[k]] = W->mult[k];
        double viol = 0.0, va = 0.0, lmx = 0.0, lneg = 0.0;
        for (int r = 0; r < m; ++r) {
            const double v = rdot(W, r, W->zn) - h[r];
            W->rin[r] = v;
            viol = fmax(viol, v);
            if (act[r]) { va = fmax(va, fabs(v)); lmx = fmax(lmx, W->nu[r]); lneg = fmin(lneg, W->nu[r]); }
        }
        for (int j = 0; j < n; ++j) {
            double v = f[j];
            for (int i = 0; i < n; ++i) v += H[(size_t)j * n + i] * W->zn[i];
            W->tmp[j] = v;
        }
        const double gs = amax(W->tmp, n);
        for (int r = 0; r < m; ++r) if (W->nu[r] != 0.0) raxpy(W, r, W->nu[r], W->tmp);
        const double st = amax(W->tmp, n), td = 1e-9 * (1.0 + lmx);
        if (isfinite(st) && st <= tol_stat * (1.0 + gs) && viol <= tf && va <= tf && lneg >= -td) {
            memcpy(W->zq, W->zn, sizeof(double) * n);
            for (int r = 0; r < m; ++r) { W->l[r] = fmax(W->nu[r], 0.0); W->t[r] = fmax(-W->rin[r], 0.0); }
            return 1;
        }
        int change = 0;
        for (int r = 0; r < m; ++r) {
            if (act[r] && W->nu[r] < -td) { act[r] = 0; change = 1; }
            else if (!act[r] && W->rin[r] > tf) { act[r] = 1; change = 1; }
        }
        if (!change) return 0;
    }
    return 0;
}

/* ---------------------------------------------------------------- dense IPM -------------- */
/* oracle/dense_ipm.py solve (bqp_dense.hip): min 0.5 d'Hd + f'd s.t. G d <= h, G = Ain,
 * h = bsh.  Solution in W->zq, multipliers in W->l.  Returns the quadprog exit flag. */
static void ipm_resid(cll_work *W, double *gs) {
    const int n = W->n, m = W->m;
    for (int j = 0; j < n; ++j) {
        double v = W->f[j];
        for (int i = 0; i < n; ++i) v += W->H[(size_t)j * n + i] * W->zq[i];
        W->rd[j] = v;
    }
    *gs = amax(W->rd, n);
    for (int r = 0; r < m; ++r) {
        raxpy(W, r, W->l[r], W->rd);
        W->ri[r] = rdot(W, r, W->zq) + W->t[r] - W->bsh[r];
    }
}

static void ipm_factor(cll_work *W) {
    for (int r = 0; r < W->m; ++r) W->tmp[W->n + r] = W->l[r] / W->t[r];
    normal_matrix(W, W->tmp + W->n, NULL, 0.0);
    chol(W->K, W->n, PIV_FLOOR * fmax(kdiag_max(W), 1e-300), 0);
}

static void ipm_newton(cll_work *W) {
    const int n = W->n, m = W->m;
    memcpy(W->dz, W->rd, sizeof(double) * n);
    for (int r = 0; r < m; ++r) raxpy(W, r, (W->l[r] * W->ri[r] - W->rc[r]) / W->t[r], W->dz);
    for (int j = 0; j < n; ++j) W->dz[j] = -W->dz[j];
    chol_solve(W->K, n, W->dz);
    for (int r = 0; r < m; ++r) {
        W->dtt[r] = -W->ri[r] - rdot(W, r, W->dz);
        W->dl[r] = (-W->rc[r] - W->l[r] * W->dtt[r]) / W->t[r];
    }
}

static double ipm_step(const cll_work *W) {
    double a = 1.0;
    for (int r = 0; r < W->m; ++r) {
        if (W->dtt[r] < 0) a = fmin(a, -W->t[r] / W->dtt[r]);
        if (W->dl[r] < 0) a = fmin(a, -W->l[r] / W->dl[r]);
    }
    return a;
}

static int dense_ipm(cll_work *W, int polish_mode, int max_iter) {
    const int n = W->n, m = W->m;
    const double tol_stat = 1e-8, tol_feas = 1e-10, tol_comp = 1e-14, tau = 0.995;
    const double minv = 1.0 / (m > 0 ? m : 1);
    const double bscale = amax(W->bsh, m);
    const double zscale = Z_BIG * (1.0 + bscale + amax(W->f, n));
    /* convexity (-6) */
    double hd = 1.0;
    for (int j = 0; j < n; ++j) hd = fmax(hd, fabs(W->H[(size_t)j * n + j]));
    for (int i = 0; i < n; ++i) memcpy(W->K + (size_t)i * n, W->H + (size_t)i * n, sizeof(double) * (i + 1));
    for (int i = 0; i < n; ++i) W->K[(size_t)i * n + i] += CONVEX_EPS * hd;
    if (!chol(W->K, n, 0.0, 1)) {
        memset(W->zq, 0, sizeof(double) * n);
        memset(W->l, 0, sizeof(double) * m);
        return -6;
    }
    memset(W->zq, 0, sizeof(double) * n);
    for (int r = 0; r < m; ++r) { W->t[r] = 1.0; W->l[r] = 1.0; W->rc[r] = 1.0; }
    double gs, stat = 0.0;
    ipm_resid(W, &gs);
    ipm_factor(W);
    ipm_newton(W);
    double tmn = INFINITY, tmx = -INFINITY;
    for (int j = 0; j < n; ++j) W->zq[j] += W->dz[j];
    for (int r = 0; r < m; ++r) {
        const double tt = 1.0 + W->dtt[r];
        tmn = fmin(tmn, tt); tmx = fmax(tmx, tt);
    }
    const double shp = (m && tmn <= 0) ? 1.0 - tmn : 0.0, shd = (m && tmx >= 0) ? 1.0 + tmx : 0.0;
    for (int r = 0; r < m; ++r) {
        const double tt = 1.0 + W->dtt[r];
        W->t[r] = tt + shp;
        W->l[r] = -tt + shd;
    }
    double mu_min = INFINITY;
    int flag = 0;
    for (int it = 0; it <= max_iter; ++it) {
        ipm_resid(W, &gs);
        stat = amax(W->rd, n);
        const double feas = amax(W->ri, m);
        double mu = 0.0, cmax = 0.0;
        for (int r = 0; r < m; ++r) { const double c = W->t[r] * W->l[r]; mu += c; cmax = fmax(cmax, c); }
        mu *= minv;
        if (stat <= tol_stat * (1 + gs) && feas <= tol_feas * (1 + bscale) && mu <= tol_comp &&
            cmax <= CMAX_K * tol_comp) { flag = 1; break; }
        if (!(isfinite(stat) && isfinite(feas) && isfinite(mu))) {
            if (cll_trace()) fprintf(stderr, "ipm -8 residual at it %d stat %g feas %g mu %g\n", it, stat, feas, mu);
            flag = -8; break; }
        if (amax(W->zq, n) > zscale) { flag = -3; break; }
        if (mu > MU_BLOWUP * mu_min && feas > FEAS_GUARD * (1 + bscale)) { flag = -2; break; }
        mu_min = fmin(mu_min, mu);
        if (it == max_iter) break;
        ipm_factor(W);
        for (int r = 0; r < m; ++r) W->rc[r] = W->t[r] * W->l[r];
        ipm_newton(W);
        const double a0 = ipm_step(W);
        double mua = 0.0;
        for (int r = 0; r < m; ++r) mua += (W->t[r] + a0 * W->dtt[r]) * (W->l[r] + a0 * W->dl[r]);
        mua *= minv;
        const double sg = pow(mua / mu, 3.0);
        const double soc = (a0 < SOC_ALPHA && feas <= FEAS_GUARD * (1 + bscale)) ? 0.0 : 1.0;
        for (int r = 0; r < m; ++r) W->rc[r] = W->t[r] * W->l[r] + soc * W->dtt[r] * W->dl[r] - sg * mu;
        ipm_newton(W);
        const double a = fmin(1.0, tau * ipm_step(W));
        int fin = isfinite(a);
        for (int j = 0; j < n && fin; ++j) fin = isfinite(W->dz[j]);
        if (!fin) {
            if (cll_trace()) fprintf(stderr, "ipm -8 step at it %d mu %g a %g\n", it, mu, a);
            flag = -8; break; }
        for (int j = 0; j < n; ++j) W->zq[j] += a * W->dz[j];
        for (int r = 0; r < m; ++r) { W->t[r] += a * W->dtt[r]; W->l[r] += a * W->dl[r]; }
    }
    if (cll_trace()) fprintf(stderr, "ipm flag %d\n", flag);
    if (polish_mode && (flag == 0 || flag == -8 || (polish_mode == 2 && flag == 1)) && m && isfinite(gs))
        if (polish(W, bscale, tol_stat)) flag = 1;
    return flag;
}

/* ---------------------------------------------------------------- SQP -------------------- */
/* one NLP at dx0 from the guess in W->z; returns the exit flag (lbmpc_update_kernel rules) */
static int sqp(const cll_prob *P, cll_work *W, const double *dx0, int *iters) {
    const int N = W->N, n = W->n, m = W->m;
    /* bin = b0 - (F x_k of the free nominal response); x_k = A^k dx0 */
    double xk[4], xn[4];
    memcpy(xk, dx0, sizeof xk);
    int r = 0;
    for (int k = 1; k <= N; ++k) {
        for (int i = 0; i < 4; ++i) {
            xn[i] = 0.0;
            for (int c = 0; c < 4; ++c) xn[i] += P->A[4 * i + c] * xk[c];
        }
        memcpy(xk, xn, sizeof xk);
        if (k == 1) {
            for (int i = 0; i < P->nd; ++i, ++r) {
                double v = P->hxd[i];
                for (int c = 0; c < 4; ++c) v -= P->Fxd[4 * i + c] * xk[c];
                W->bin[r] = v;
            }
            for (int i = 0; i < P->nT; ++i, ++r) {
                double v = P->hT[i];
                for (int c = 0; c < 4; ++c) v -= P->FT[5 * i + c] * xk[c];
                W->bin[r] = v;
            }
        }
        for (int i = 0; i < P->nFx; ++i, ++r) {
            double v = P->hx[i];
            for (int c = 0; c < 4; ++c) v -= P->Fx[4 * i + c] * xk[c];
            W->bin[r] = v;
        }
        for (int i = 0; i < P->nFu; ++i, ++r) W->bin[r] = P->hu[i];
    }
    const double tol_step = P->tol, tol_stat = 10.0 * P->tol;
    double cprev = 0.0;
    int it = 0, flag = 0;
    for (int outer = 0; outer < P->max_iter; ++outer) {
        const double J0 = rollout(P, W, dx0, W->z, 1, P->hessian);
        gn_model(P, W, W->z);
        if (P->hessian) {
            memcpy(W->Hg, W->H, sizeof(double) * n * n);
            newton_term(P, W, W->z);
            /* pd_cholesky (oracle/lbmpc.py): pivots above 1e-10 max |H_ii| */
            double hd = 0.0;
            for (int j = 0; j < n; ++j) hd = fmax(hd, fabs(W->H[(size_t)j * n + j]));
            for (int i = 0; i < n; ++i) memcpy(W->K + (size_t)i * n, W->H + (size_t)i * n, sizeof(double) * (i + 1));
            if (!chol(W->K, n, 1e-10 * hd, 1)) {
                /* indefinite: the smallest shift delta_k = 1e-12 hd 4^k (k = 0 .. 20, found by
                 * bisection - positive definiteness is monotone in the shift) for which H + delta
                 * I passes the same test; Gauss-Newton only when even k = 20 fails (VERDICT r4
                 * item 6: falling back to H_GN at once converged linearly - 200 SQP iterations on
                 * a +-0.02 DMS instance whose exact Hessian is indefinite; 7 with the shift) */
                const int k = hess_shift_k(W, n, hd);
                if (k < 0) memcpy(W->H, W->Hg, sizeof(double) * n * n);
                else for (int i = 0; i < n; ++i) W->H[(size_t)i * n + i] += HSHIFT(hd, k);
            }
        }
        for (int i = 0; i < m; ++i) W->bsh[i] = W->bin[i] - rdot(W, i, W->z);
        const int qflag = dense_ipm(W, it >= POL_STALL ? 2 : 0, 100);
        if (cll_trace()) fprintf(stderr, "sqp it %d qflag %d\n", it, qflag);
        memcpy(W->d, W->zq, sizeof(double) * n);
        memcpy(W->lam, W->l, sizeof(double) * m);
        /* lbmpc_update_kernel */
        memcpy(W->tmp, W->f, sizeof(double) * n);
        for (int i = 0; i < m; ++i) if (W->lam[i] != 0.0) raxpy(W, i, W->lam[i], W->tmp);
        const double st = amax(W->tmp, n), fn = amax(W->f, n), dn = amax(W->d, n), zn = amax(W->z, n);
        double sl = 0.0, viol = 0.0;
        for (int j = 0; j < n; ++j) sl += W->f[j] * W->d[j];
        for (int i = 0; i < m; ++i) viol = fmax(viol, -W->bsh[i]);
        const int feas0 = viol <= 1e-9;
        if (cll_trace() >= 2) fprintf(stderr, "sqp it %d qflag %d |d| %.3e stat %.3e (tol %.3e) J %.15e\n", it, qflag, dn,
                                      st, tol_stat * (1.0 + fn), J0);
        const int qp_ok = qflag == 1 || ((qflag == 0 || qflag == -8) && isfinite(dn) && isfinite(st));
        if (qflag == -2 || !qp_ok) { flag = qflag == -2 ? -2 : -8; break; }
        if (feas0 && ((qflag == 1 && dn <= tol_step * (1.0 + zn) && st <= tol_stat * (1.0 + fn)) ||
                      (it > 0 && dn <= 1e-6 * (1.0 + zn) &&
                       (qflag != 1 || fabs(cprev - J0) <= 1e-12 * (1.0 + fabs(J0)))))) {
            flag = 1;
            break;
        }
        double al = ldexp(1.0, -(NTRIAL - 1));
        if (feas0) {
            for (int t = 0; t < NTRIAL; ++t) {
                const double a = ldexp(1.0, -t);
                for (int j = 0; j < n; ++j) W->ztr[j] = W->z[j] + a * W->d[j];
                if (rollout(P, W, dx0, W->ztr, 0, 0) <= J0 + 1e-4 * a * sl) { al = a; break; }
            }
        } else {
            al = 1.0;
        }
        for (int j = 0; j < n; ++j) W->z[j] += al * W->d[j];
        cprev = J0;
        if (++it >= P->max_iter) { flag = 0; break; }
    }
    *iters = it;
    return flag;
}

/* ---------------------------------------------------------------- closed loop ------------ */
static void mg_rhs(const double x[4], double u, double dx[4]) {
    dx[0] = -x[1] + 1.0 + 3.0 * (x[0] / 2.0) - (x[0] * x[0] * x[0] / 2.0);
    dx[1] = x[0] + 1.0 - x[2] * sqrt(x[1]);
    dx[2] = x[3];
    dx[3] = -1000.0 * x[2] - 2.0 * sqrt(500.0) * x[3] + 1000.0 * u;
}

static void mg_rk4(double dt, const double x[4], double u, double xn[4]) {
    double k1[4], k2[4], k3[4], k4[4], y[4];
    mg_rhs(x, u, k1);
    for (int i = 0; i < 4; ++i) y[i] = x[i] + dt / 2 * k1[i];
    mg_rhs(y, u, k2);
    for (int i = 0; i < 4; ++i) y[i] = x[i] + dt / 2 * k2[i];
    mg_rhs(y, u, k3);
    for (int i = 0; i < 4; ++i) y[i] = x[i] + dt * k3[i];
    mg_rhs(y, u, k4);
    for (int i = 0; i < 4; ++i) xn[i] = x[i] + dt / 6 * (k1[i] + 2 * k2[i] + 2 * k3[i] + k4[i]);
}

/* the condensed nominal constraint rows (shared by every instance) */
static void build_rows(const cll_prob *P, int n, double *Ain, int *lo, int *hi) {
    const int N = P->N;
    double *Sn = xcalloc((size_t)4 * n, sizeof(double)), *Sx = xcalloc((size_t)4 * n, sizeof(double));
    int r = 0;
    for (int k = 1; k <= N; ++k) {
        /* S_k = A S_{k-1} + B e_{k-1} */
        for (int i = 0; i < 4; ++i)
            for (int j = 0; j < n; ++j) {
                double v = 0.0;
                for (int c = 0; c < 4; ++c) v += P->A[4 * i + c] * Sn[(size_t)c * n + j];
                Sx[(size_t)i * n + j] = v + (j == k - 1 ? P->B[i] : 0.0);
            }
        memcpy(Sn, Sx, sizeof(double) * 4 * n);
        if (k == 1) {
            for (int i = 0; i < P->nd; ++i, ++r) {
                for (int j = 0; j < n; ++j) {
                    double v = 0.0;
                    for (int c = 0; c < 4; ++c) v += P->Fxd[4 * i + c] * Sn[(size_t)c * n + j];
                    Ain[(size_t)r * n + j] = v;
                }
                lo[r] = 0; hi[r] = 1;
            }
            for (int i = 0; i < P->nT; ++i, ++r) {
                for (int j = 0; j < n; ++j) {
                    double v = 0.0;
                    for (int c = 0; c < 4; ++c) v += P->FT[5 * i + c] * Sn[(size_t)c * n + j];
                    Ain[(size_t)r * n + j] = v;
                }
                Ain[(size_t)r * n + n - 1] += P->FT[5 * i + 4];
                lo[r] = 0; hi[r] = n;
            }
        }
        for (int i = 0; i < P->nFx; ++i, ++r) {
            for (int j = 0; j < n; ++j) {
                double v = 0.0;
                for (int c = 0; c < 4; ++c) v += P->Fx[4 * i + c] * Sn[(size_t)c * n + j];
                Ain[(size_t)r * n + j] = v;
            }
            lo[r] = 0; hi[r] = k;
        }
        for (int i = 0; i < P->nFu; ++i, ++r) {
            Ain[(size_t)r * n + k - 1] = P->Fu[i];
            lo[r] = k - 1; hi[r] = k;
        }
    }
    free(Sn); free(Sx);
}

int cll_rows(const cll_prob *P) { return P->nd + P->nT + P->N * (P->nFx + P->nFu); }

/* nb closed loops of `steps` steps from x_init (nb x 4, absolute): X (nb x (steps+1) x 4),
 * U (nb x steps), iterations and exit flags (nb x steps).  mask: the 8 x q window starts with
 * only its first (zero) point valid (DMS_LBMPC_casadi.m:158-161); else every point counts.
 * Returns 0, or -1 on bad arguments / allocation failure. */
int cll_loop(const cll_prob *P, int mask, int nb, const double *x_init, int steps, double *X,
             double *U, int *iters, int *flags, int threads) {
    if (!P || P->N < 1 || P->q < 1 || nb < 0 || steps < 0) return -1;
    (void)cll_trace();                    /* read before the worker threads start */
    const int N = P->N, n = N + 1, m = cll_rows(P), q = P->q;
    double *Ain = xcalloc((size_t)m * n, sizeof(double));
    int *lo = xcalloc(m, sizeof(int)), *hi = xcalloc(m, sizeof(int));
    if (!Ain || !lo || !hi) return -1;
    build_rows(P, n, Ain, lo, hi);
    int bad = 0;
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#pragma omp parallel for schedule(dynamic, 1) reduction(| : bad)
#endif
    for (int b = 0; b < nb; ++b) {
        cll_work W;
        memset(&W, 0, sizeof W);
        W.n = n; W.m = m; W.N = N; W.q = q;
        W.Ain = Ain; W.lo = lo; W.hi = hi;
        const size_t mn = (size_t)(m > n ? m : n);
        double *pool = xcalloc((size_t)(N + 1) * 4 * n + 4 * (size_t)n * n + (size_t)n * n + 24 * mn +
                               (size_t)N * 60 + 8 * (size_t)q + 16, sizeof(double));
        W.idx = xcalloc(2 * mn, sizeof(int));
        if (!pool || !W.idx) { bad |= 1; free(pool); free(W.idx); continue; }
        double *p = pool;
        W.S = p; p += (size_t)(N + 1) * 4 * n;
        W.H = p; p += (size_t)n * n; W.Hg = p; p += (size_t)n * n; W.K = p; p += (size_t)n * n;
        W.Y = p; p += (size_t)n * n; W.Sp = p; p += (size_t)n * n;
        W.xL = p; p += 4 * (size_t)(N + 1); W.uL = p; p += N; W.dg = p; p += 12 * (size_t)N;
        W.d2g = p; p += 36 * (size_t)N; W.data = p; p += 8 * (size_t)q;
        double **vec[] = {&W.bin, &W.bsh, &W.z, &W.d, &W.lam, &W.ztr, &W.f, &W.t, &W.l, &W.dz, &W.dtt,
                          &W.dl, &W.rd, &W.ri, &W.rc, &W.qv, &W.zq, &W.w, &W.mult, &W.ra, &W.zn, &W.nu,
                          &W.rin};
        for (size_t i = 0; i < sizeof vec / sizeof vec[0]; ++i) { *vec[i] = p; p += mn; }
        W.tmp = p;                        /* n + m doubles (the IPM's D = lam / t after n) */
        p += 2 * mn;
        for (int i = 0; i < q; ++i) W.data[8 * i + 7] = mask ? 0.0 : 1.0;
        W.data[7] = 1.0;
        double x[4];
        memcpy(x, x_init + 4 * (size_t)b, sizeof x);
        memcpy(X + (size_t)b * (steps + 1) * 4, x, sizeof x);
        for (int s = 0; s < steps; ++s) {
            double dx[4], xn[4];
            for (int i = 0; i < 4; ++i) dx[i] = x[i] - P->xeq[i];
            int itn = 0;
            const int fl = sqp(P, &W, dx, &itn);
            iters[(size_t)b * steps + s] = itn;
            flags[(size_t)b * steps + s] = fl;
            const double du = W.z[0];
            mg_rk4(P->dt_plant, x, du + P->ueq, xn);
            /* get_data.m: [dx1; dx2; du; (x+ - x_eq) - (A dx + B du); 1] */
            double col[8] = {dx[0], dx[1], du, 0, 0, 0, 0, 1.0};
            for (int i = 0; i < 4; ++i) {
                double nom = P->B[i] * du;
                for (int c = 0; c < 4; ++c) nom += P->A[4 * i + c] * dx[c];
                col[3 + i] = (xn[i] - P->xeq[i]) - nom;
            }
            const int it1 = s + 1;
            if (it1 < q) {
                memcpy(W.data + 8 * (size_t)it1, col, sizeof col);
            } else {
                memmove(W.data, W.data + 8, sizeof(double) * 8 * (size_t)(q - 1));
                memcpy(W.data + 8 * (size_t)(q - 1), col, sizeof col);
            }
            U[(size_t)b * steps + s] = du + P->ueq;
            /* shifted warm start: moves one stage on, zero last move, theta kept */
            memmove(W.z, W.z + 1, sizeof(double) * (N - 1));
            W.z[N - 1] = 0.0;
            memcpy(x, xn, sizeof x);
            memcpy(X + ((size_t)b * (steps + 1) + s + 1) * 4, x, sizeof x);
        }
        free(pool);
        free(W.idx);
    }
    free(Ain); free(lo); free(hi);
    return bad ? -1 : 0;
}
