/*
 * bqp.h — C ABI of the MI355X batched MPC QP solver (libbqp.so).
 *
 * Drop-in boundary for the per-step optimal-control solve of bevanda/Learning-Based-MPC.
 * The reference issues that solve through two MATLAB call surfaces; each entry point below
 * names the one it replaces:
 *
 *   fmincon(COSTFUN, opt_var, [],[],[],[],[],[], CONSFUN, options)
 *       matlab/LBMPC/functions/ocpLMPC.m:20-24      (LMPC, form F1)
 *       matlab/LBMPC/functions/ocpLBMPC.m:27-31      (LBMPC, form F3: Gauss-Newton SQP whose
 *                                                     QP sub-problems run in the dense kernel)
 *       matlab/trackingMPC/RunExample.m:134-136      (tracking MPC, form F5)
 *   solver('x0',..,'lbx',..,'ubx',..,'lbg',..,'ubg',..)  (CasADi nlpsol/IPOPT)
 *       matlab/LBMPC/examples/DMS_tracking_LMPC_casadi.m:163-167  (form F2)
 *       matlab/LBMPC/examples/DSS_tracking_LMPC_casadi.m:155-160
 *
 * Two solver entry points:
 *   bqp_solve_ocp_batched   structured stage-wise OCP (the fast path; Riccati KKT on GPU)
 *   bqp_quadprog_batched    MATLAB quadprog semantics on dense per-instance (H,f,A,b,Aeq,beq,lb,ub)
 * and *_device variants taking device pointers + a hipStream_t (passed as void*).
 *
 * Conventions
 *   - all matrices are column-major (MATLAB layout), fp64;
 *   - every input array carries an element stride between instances; stride 0 = one copy shared
 *     by the whole batch (broadcast);
 *   - return code: BQP_OK (0) or a negative BQP_E_* (API error: bad dims, HIP failure, missing
 *     GPU); per-instance status is exitflag[] with quadprog meanings:
 *       1 converged, 0 iteration limit, -2 primal infeasible, -3 dual infeasible/unbounded,
 *       -6 non-convex, -8 numerical failure;
 *   - thread safety: one bqp_handle per host thread / stream; no global mutable state.
 */
#ifndef BQP_H
#define BQP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BQP_OK 0
#define BQP_E_ARG (-1)       /* invalid dimensions / NULL required pointer */
#define BQP_E_HIP (-2)       /* HIP runtime error (allocation, launch, copy) */
#define BQP_E_NODEV (-3)     /* no usable gfx950 device */
#define BQP_E_UNSUPPORTED (-4) /* dimensions outside the compiled kernel set */

typedef struct bqp_handle_s* bqp_handle;

typedef struct {
    int max_iter;      /* default 50 */
    double tol_stat;   /* stationarity inf-norm / (1 + |cost gradient|_inf), default 1e-8 */
    double tol_feas;   /* primal residual inf-norm / (1 + |bounds, rhs|_inf), default 1e-10 */
    double tol_comp;   /* average complementarity mu (absolute), default 1e-14 */
    double tau;        /* fraction-to-boundary, default 0.995.  At tau >= 0.995 the structured
                          solver's step rule lets the corrector step go to 0.99999 of the boundary
                          on a well-centred iterate; a smaller tau bounds every
                          step */
    int precision;     /* structured API: 0 = fp64 (default); 1 = fp32 solver arithmetic/LDS state
                          (inputs and outputs stay fp64; tolerances floored at 1e-5 / 1e-6 / 1e-9);
                          2 = mixed: an fp32 launch to those floored tolerances, then an fp64 launch
                          that continues every instance from its fp32 iterate to the fp64
                          tolerances (fp64 results; instances the fp32 phase ends with -2/-8,
                          or whose continuation does not converge, restart in fp64); applies to
                          long horizons (N >= 64), shorter ones are solved in fp64.  In mixed
                          mode max_iter applies per phase, and bqp_output.iterations counts the
                          fp32 + fp64 iterations of a continued instance, or only the fp64
                          restart's iterations for an instance that restarts */
    int want_duals;    /* reserved (set 0): the structured API writes the multiplier outputs
                          whenever its `duals` argument is non-NULL */
    int polish;        /* structured API, fp64 active-set polish: the rows with lam > t are solved
                          as equalities (augmented-Lagrangian steps and conjugate gradients on
                          their multipliers, on the Riccati factorisation with weight rho on
                          the active rows, with active-set corrections) and the result replaces
                          the interior-point iterate if it passes the KKT checks
                          (bqp_output.polished).  It runs in a separate repair launch over the
                          instances the solve launch marks, so the solve kernel carries no
                          polish state.
                          0 (default) or 1: after an iteration-limit or numerical-failure exit
                          (e.g. multipliers ~1e3-1e5 drive D = lam/t out of fp64 range);
                          2: also when a row is left weakly active (slack and multiplier both
                          above 1e-10); 3 (SQP routines bqp_lbmpc_* / bqp_closed_loop_sqp;
                          the closed loop's default): the sub-problems are polished only once
                          the SQP has stalled at a step; -1: off (interior-point iterate only) */
} bqp_options;

typedef struct {
    int iterations;
    double constrviolation;  /* max(primal eq, primal ineq) at exit */
    double firstorderopt;    /* stationarity inf-norm at exit */
    double mu;               /* average complementarity at exit */
    double kkt[4];           /* stationarity, primal eq, primal ineq (inf-norms of the solver's
                                residuals at exit), complementarity (average t.lam = mu) */
    int polished;            /* 1: the answer is the active-set polish (bqp_options.polish) */
} bqp_output;

/* ------------------------------------------------------------------------------------------
 * Structured OCP (form F1/F2/F4/F5 after the host shim's change of variables):
 *
 *   x_{k+1} = A x_k + B u_k + c              k = 0..N-1,   x_0 = x0 (fixed)
 *   theta  in R^np  (global steady-state parameter, free)
 *   min  sum_{k=0}^{N} 0.5 v_k' W_k v_k + w_k' v_k,  v_k = [x_k; u_k; theta]  (nv = nx+nu+np;
 *        for k = N the u block of W_N / w_N is ignored)
 *   s.t. xlb_k <= x_k <= xub_k (k = 1..N),  ulb_k <= u_k <= uub_k (k = 0..N-1)  (+-INFINITY ok)
 *        Fp [x_kp; u_kp; theta] <= hp     (n_poly rows, polytope at stage kp = poly_stage)
 *
 * Reference mapping: costLMPC.m:20-45 / constraintsLMPC.m:15-41 (F1),
 * DMS_tracking_LMPC_casadi.m:223-287 (F2), trackingMPC/costFunction.m:20-39 /
 * constraintsFunction.m:20-38 (F5); the terminal polytope is term_set.mat's F_w_N (616x5).
 * ---------------------------------------------------------------------------------------- */
typedef struct {
    int nx, nu, np, N;
    int n_poly;      /* rows of the polytope block (>= 0) */
    int poly_stage;  /* stage the polytope acts on, 0..N */
} bqp_ocp_dims;

typedef struct {
    const double* A;    /* nx*nx                                  stride sA  */
    const double* B;    /* nx*nu                                  stride sB  */
    const double* c;    /* nx, NULL = 0                           stride sc  */
    const double* W;    /* (N+1) blocks nv*nv                     stride sW  */
    const double* w;    /* (N+1)*nv, NULL = 0                     stride sw  */
    const double* xlb;  /* (N+1)*nx, NULL = -inf (stage 0 unused) stride sxb */
    const double* xub;  /* (N+1)*nx, NULL = +inf                  stride sxb */
    const double* ulb;  /* N*nu, NULL = -inf                      stride sub */
    const double* uub;  /* N*nu, NULL = +inf                      stride sub */
    const double* Fp;   /* n_poly*nv (column-major, n_poly rows)  stride sFp */
    const double* hp;   /* n_poly                                 stride shp */
    const double* x0;   /* nx                                     stride sx0 */
    int64_t sA, sB, sc, sW, sw, sxb, sub, sFp, shp, sx0;
} bqp_ocp_data;

/* Optional multiplier outputs of the structured solve (NULL members are skipped).  Sign
 * convention: the Lagrangian is  cost + sum_k pi_k'(A x_k + B u_k + c - x_{k+1})
 * + sum lam_upper (v - ub) + sum lam_lower (lb - v) + lam_p'(Fp v - hp), all lam >= 0. */
typedef struct {
    double* pi;     /* batch*N*nx: dynamics multipliers for x_{k+1} = A x_k + B u_k + c   */
    double* lam_x;  /* batch*(N+1)*nx*2: [lower, upper] per stage (0 for absent bounds) */
    double* lam_u;  /* batch*N*nu*2                                                    */
    double* lam_p;  /* batch*n_poly                                                    */
} bqp_ocp_duals;

/* Lifecycle.  device < 0 selects the current HIP device. */
int bqp_create(bqp_handle* h, int device);
int bqp_destroy(bqp_handle h);
void bqp_default_options(bqp_options* opt);
const char* bqp_version(void);
/* SHA-1 of the sources the library was built from (csrc files in name order, then include/bqp.h) */
const char* bqp_build_source_sha1(void);

/* Host-pointer structured solve.  Outputs (host): x batch*(N+1)*nx, u batch*N*nu,
 * theta batch*np, fval batch, exitflag batch, out batch (out/fval/duals may be NULL). */
int bqp_solve_ocp_batched(bqp_handle h, const bqp_ocp_dims* dims, int batch,
                          const bqp_ocp_data* data, const bqp_options* opt,
                          double* x, double* u, double* theta, double* fval, int* exitflag,
                          bqp_output* out, const bqp_ocp_duals* duals);

/* Device-pointer structured solve (all data/output pointers are device memory owned by the
 * caller; stream is a hipStream_t, NULL = default stream).  Asynchronous: returns after the
 * launch; synchronise the stream before reading outputs. */
int bqp_solve_ocp_batched_device(bqp_handle h, const bqp_ocp_dims* dims, int batch,
                                 const bqp_ocp_data* data, const bqp_options* opt,
                                 double* x, double* u, double* theta, double* fval,
                                 int* exitflag, bqp_output* out, const bqp_ocp_duals* duals,
                                 void* stream);

/* ------------------------------------------------------------------------------------------
 * quadprog-compatible dense batched solve:
 *   [x,fval,exitflag,output,lambda] = quadprog(H,f,A,b,Aeq,beq,lb,ub,x0,options)
 *   min 0.5 x'Hx + f'x  s.t.  A x <= b, Aeq x = beq, lb <= x <= ub.
 * H n*n, f n, A m*n, b m, Aeq me*n, beq me, lb/ub n (NULL = unbounded), x0 ignored (IPM).
 * lambda outputs follow quadprog: H x + f + A'l_ineqlin + Aeq'l_eqlin - l_lower + l_upper = 0.
 * H: as quadprog, the host entry solves with the symmetric part (H + H')/2 (a symmetric H is
 * used bit for bit); the _device entry takes H as given and requires it symmetric (the kernels
 * read both triangles).
 * ---------------------------------------------------------------------------------------- */
typedef struct {
    int n;   /* variables */
    int m;   /* inequality rows */
    int me;  /* equality rows */
} bqp_dims;

typedef struct {
    int64_t sH, sf, sA, sb, sAeq, sbeq, slb, sub;  /* element strides, 0 = shared */
} bqp_strides;

int bqp_quadprog_batched(bqp_handle h, const bqp_dims* d, int batch, const bqp_strides* st,
                         const double* H, const double* f, const double* A, const double* b,
                         const double* Aeq, const double* beq, const double* lb,
                         const double* ub, const double* x0, const bqp_options* opt,
                         double* x, double* fval, int* exitflag, double* lam_ineqlin,
                         double* lam_eqlin, double* lam_lower, double* lam_upper,
                         bqp_output* out);

int bqp_quadprog_batched_device(bqp_handle h, const bqp_dims* d, int batch,
                                const bqp_strides* st, const double* H, const double* f,
                                const double* A, const double* b, const double* Aeq,
                                const double* beq, const double* lb, const double* ub,
                                const bqp_options* opt, double* x, double* fval, int* exitflag,
                                double* lam_ineqlin, double* lam_eqlin, double* lam_lower,
                                double* lam_upper, bqp_output* out, void* stream);

/* ------------------------------------------------------------------------------------------
 * Learning-based MPC (forms F3/F4): the learned prediction model
 *   x+ = A x + B u + g(x, u),  g = Nadaraya-Watson oracle over a data window (oracleL2NW.m)
 * makes the per-step problem an NLP; it is solved by a Gauss-Newton SQP whose QP sub-problems
 * run in the dense kernel.  Replaces
 *   fmincon(costLBMPC, constraintsLBMPC)   matlab/LBMPC/functions/ocpLBMPC.m:27-31   (F3)
 *   solver(..., 'p', data)                 matlab/LBMPC/examples/hybrid_LBMPC_casadi.m:173-178 (F4)
 *   oracleL2NW(x, u, data)                 matlab/LBMPC/functions/oracleL2NW.m:1-36
 *
 * Decision z = [v_0..v_{N-1}; theta] (n = N*nu + np) with the rollout input u_k = K x_k + v_k
 * (F3: v = c, K = Kstabil; F4: v = u - u_eq, K = 0), deviation coordinates.  Cost:
 *   sum_{k < n_run} |Lq (x^L_k - LAMBDA th)|^2 + |Lr (u^L_k - PSI th)|^2
 *     + |Lp (x^T_N - LAMBDA th)|^2 + |Lt (LAMBDA th - xs)|^2
 * on the LEARNED rollout x^L (terminal x^T = learned or nominal x_N), subject to the condensed
 * NOMINAL-model constraints Ain z <= bin (the host shim builds them from constraintsLBMPC.m /
 * hybrid_LBMPC_casadi.m:283-310).  The NW window is 7 x q column-major per instance: rows 1-3
 * X = [dx1; dx2; du], rows 4-7 Y (hybrid_LBMPC_casadi.m:128 layout; no validity mask), or with
 * mask = 1 the 8 x q window of DMS_LBMPC_casadi.m:158-161 whose row 8 is the validity v of
 * casadiL2NW.m:14-28 (normaliser lambda + sum_j v_j k_j).
 * ---------------------------------------------------------------------------------------- */
typedef struct {
    int nx, nu, np, N;
    int n_run;          /* running-cost stages k = 0..n_run-1 (F3: N-2, costLBMPC.m:30; F4: N) */
    int term_learned;   /* terminal P cost on the learned (1, F3) or nominal (0, F4) x_N */
    int q;              /* points in the NW window (<= 512) */
    int m;              /* rows of Ain */
    int mask;           /* 0: 7 x q window, every point counts; 1: 8 x q window with validity row */
    int hessian;        /* 0: Gauss-Newton; 1: + the second-order term of the learned dynamics
                           (costate-weighted NW Hessians) whenever the sum is positive definite
                           (Cholesky pivots > 1e-10 max|H_ii|), Gauss-Newton otherwise.  GN
                           converges linearly (rate ~0.5) on DMS_LBMPC_casadi.m's learned-state
                           costs: 60-200 SQP iterations against 4-6 with 1.  The exact
                           term needs n = N nu + np <= 127 (its n x n sum lives in LDS);
                           longer horizons run Gauss-Newton */
} bqp_lbmpc_dims;

typedef struct {
    const double *A, *B, *K;          /* nx*nx, nx*nu, nu*nx (column-major), shared */
    const double *Lq, *Lr, *Lp, *Lt;  /* upper-triangular ROW-major weight factors:
                                         Lq'Lq = w Q, Lr'Lr = w R (w = running weight), Lp'Lp = P, Lt'Lt = T */
    const double *LAMBDA, *PSI, *xs;  /* nx*np, nu*np (column-major), nx */
    const double* data; int64_t sdata;  /* NW window (7 or 8)*q per instance (stride; 0 = shared) */
    const double* x0;   int64_t sx0;    /* nx per instance */
    const double* Ain;                  /* m*n column-major, shared */
    const double* bin;  int64_t sbin;   /* m per instance */
    double bandwidth, lambda;           /* NW kernel; <= 0 selects the reference's 0.5, 1e-3 */
} bqp_lbmpc_data;

/* Batched NW oracle: g (batch*4) and optionally dg/dxi (batch*4*3, row-major per instance) at
 * the query points xi (batch*3). */
int bqp_nw_oracle(bqp_handle h, int batch, int q, const double* data, int64_t sdata,
                  const double* xi, double* g, double* dg, double bandwidth, double lambda);
int bqp_nw_oracle_device(bqp_handle h, int batch, int q, const double* data, int64_t sdata,
                         const double* xi, double* g, double* dg, double bandwidth,
                         double lambda, void* stream);

/* SQP solve.  z (batch*n): in = start (fmincon's opt_var warm start), out = solution; lam
 * (batch*m, may be NULL): multipliers of Ain z <= bin; cost (batch, may be NULL); exitflag:
 * 1 converged, 0 iteration limit (opt->max_iter SQP iterations), -2 QP sub-problem infeasible,
 * -8 numerical failure.  The _device variant synchronises its stream every 4 SQP iterations
 * (early exit when the whole batch has converged). */
int bqp_lbmpc_solve_batched(bqp_handle h, const bqp_lbmpc_dims* d, int batch,
                            const bqp_lbmpc_data* data, const bqp_options* opt, double* z,
                            double* lam, double* cost, int* exitflag, int* iterations);
int bqp_lbmpc_solve_batched_device(bqp_handle h, const bqp_lbmpc_dims* d, int batch,
                                   const bqp_lbmpc_data* data, const bqp_options* opt, double* z,
                                   double* lam, double* cost, int* exitflag, int* iterations,
                                   void* stream);

/* ------------------------------------------------------------------------------------------
 * Closed-loop simulation: per time step, the batched structured solve at
 * the measured states, then one step of the true plant with the first input - the loop of
 * DMS_tracking_LMPC_casadi.m:153-189 / DSS_tracking_LMPC_casadi.m (solver(...), then
 * xmeasure = dynamic(delta, xmeasure, u_OL(1:m))) for a whole batch of initial states.
 * The OCP is posed in deviation coordinates around (x_eq, u_eq); data->x0 is ignored (the
 * measured states are fed back).  x_init (batch*nx), X (batch*(steps+1)*nx) and
 * U (batch*steps*nu) are absolute; exitflag (batch*steps, may be NULL) per solve.
 * Plant BQP_PLANT_MG_RK4: Moore-Greitzer `system` (:215-221) under one RK4 step of length
 * delta (`dynamic`, :297-304); nx = 4, nu = 1.  BQP_PLANT_MG_ODE23: the same model integrated
 * over delta by MATLAB's ode23 at its default options (RelTol 1e-3, AbsTol 1e-6, MaxStep
 * delta/10) - models/trueModel.m:14/48 behind functions/transitionTrue.m, the plant of the
 * fmincon loops (functions/ocpLMPC.m:11-40, ocpLBMPC.m); with bqp.LMPC's problem this runs
 * examples/LMPC_RunExample.m's loop.
 * ---------------------------------------------------------------------------------------- */
#define BQP_PLANT_MG_RK4 1
#define BQP_PLANT_MG_ODE23 2
typedef struct {
    int plant;           /* BQP_PLANT_MG_RK4 or BQP_PLANT_MG_ODE23 */
    int steps;           /* closed-loop steps (mpciterations) */
    double delta;        /* plant step (s) */
    const double* x_eq;  /* nx working point (device memory in the _device variant) */
    const double* u_eq;  /* nu */
} bqp_closed_loop;

int bqp_closed_loop_ocp(bqp_handle h, const bqp_ocp_dims* d, int batch, const bqp_ocp_data* data,
                        const bqp_options* opt, const bqp_closed_loop* cl, const double* x_init,
                        double* X, double* U, int* exitflag);
int bqp_closed_loop_ocp_device(bqp_handle h, const bqp_ocp_dims* d, int batch,
                               const bqp_ocp_data* data, const bqp_options* opt,
                               const bqp_closed_loop* cl, const double* x_init, double* X,
                               double* U, int* exitflag, void* stream);

/* ------------------------------------------------------------------------------------------
 * LBMPC closed loop with the learned model's data window: the data
 * acquisition of matlab/LBMPC/examples/DMS_LBMPC_casadi.m:198-207 around a structured QP
 * solve (LBMPC_casadi.m:163-218).  Per step: the structured solve at the
 * measured state, the plant step, then the data acquisition of the reference -
 *   X = [dx1; dx2; du], Y = (x+ - x_eq) - (A dx + B du)          (:202-206, deviation coords)
 *   window <- get_data(X, Y, q, it, window)                     (utilities/get_data.m)
 * and the logged learned prediction xl = x_eq + A dx + B du + g(X, Y, v) with the window before
 * the update (:199, casadiL2NW.m).  The per-step OCP is the QP the caller poses in `data`: the
 * loop of matlab/LBMPC/examples/LBMPC_casadi.m (its learned dynamics are commented out of the
 * constraints, :292, so the per-step problem is the tracking QP with F_x_d and the terminal set
 * on x_1, polytope at stage 1; the window drives xl).  The learned-model NLP loop of
 * DMS_LBMPC_casadi.m, whose cost reads the learned states, is bqp_closed_loop_sqp below.  A, B of
 * the window update are data->A / data->B.  Same loop and outputs as bqp_closed_loop_ocp, plus: */
typedef struct {
    int q;               /* points in the data window (get_data.m's q) */
    int mask;            /* 1: 8 x q window with validity row v, only the first (zero) point valid
                            at the start (DMS_LBMPC_casadi.m:160-161); 0: every point counts (the
                            7-row window of hybrid_LBMPC_casadi.m:160) */
    double bandwidth, lambda;  /* NW kernel; <= 0 selects the reference's 0.5, 1e-3 */
    double* XL;          /* out: batch*(steps+1)*nx learned predictions xl (XL[:,0] = x_init) */
    double* window;      /* out, may be NULL: batch*q*8 final windows, [X; Y; v] per point, ring
                            order (iteration it's sample in point it mod q) */
} bqp_learning;

int bqp_closed_loop_lbmpc(bqp_handle h, const bqp_ocp_dims* d, int batch, const bqp_ocp_data* data,
                          const bqp_options* opt, const bqp_closed_loop* cl,
                          const bqp_learning* lw, const double* x_init, double* X, double* U,
                          int* exitflag);
int bqp_closed_loop_lbmpc_device(bqp_handle h, const bqp_ocp_dims* d, int batch,
                                 const bqp_ocp_data* data, const bqp_options* opt,
                                 const bqp_closed_loop* cl, const bqp_learning* lw,
                                 const double* x_init, double* X, double* U, int* exitflag,
                                 void* stream);

/* ------------------------------------------------------------------------------------------
 * Learned-model NLP closed loop: per time step the batched SQP of
 * bqp_lbmpc_solve_batched at the measured states, one plant step with the first input, and the
 * data acquisition of the reference into each instance's window - the loops of
 *   matlab/LBMPC/examples/DMS_LBMPC_casadi.m:163-218   (d->mask = 1, lw->mask = 1: 8 x q window,
 *       learned states in the cost incl. the terminal term: term_learned = 1, K = 0, n_run = N)
 *   matlab/LBMPC/examples/hybrid_LBMPC_casadi.m:163-204 (F4: term_learned = 0, K = 0, n_run = N;
 *       7-row window: lw->mask = 0 keeps every point valid)
 *   matlab/LBMPC/examples/LBMPC_RunExample.m / functions/ocpLBMPC.m (F3: K = Kstabil)
 * The solver's window is the loop's own ring buffer (8 doubles per point, data->data, data->sdata,
 * data->x0 and data->bin are ignored): get_data.m's window with its columns in ring order (the NW
 * sums do not depend on the column order).  The condensed nominal constraints of each step are
 *   Ain z <= bin0 + Bx dx0   (dx0 = measured state - x_eq; bin0: m, Bx: m*nx column-major),
 * the first input applied is u_0 = u_eq + K dx0 + z_0.  Warm start (warm = 1): the previous
 * solution shifted one stage with a zero last move and the same theta (the scripts' guess
 * u0 = [u_OL(2:end); u_eq + Kstabil x_N], DMS_LBMPC_casadi.m:209-213, with the tail move of the
 * scripts' Kstabil = 0 case); warm = 0: z = 0 every step (u = u_eq, theta = 0).  opt->max_iter
 * bounds the SQP iterations per step.  The NW kernel parameters are lw->bandwidth / lw->lambda
 * when > 0, else data->bandwidth / data->lambda, else the reference's 0.5 / 1e-3.  X, U, exitflag
 * and lw->XL / lw->window as in bqp_closed_loop_lbmpc; Z (batch*steps*n, may be NULL): every step's SQP solution z;
 * iterations (batch*steps, may be NULL): SQP iterations per step.
 * ---------------------------------------------------------------------------------------- */
typedef struct {
    const double* bin0;  /* m */
    const double* Bx;    /* m * nx, column-major */
    int warm;
    double* Z;           /* out, may be NULL */
    int* iterations;     /* out, may be NULL */
} bqp_sqp_loop;

int bqp_closed_loop_sqp(bqp_handle h, const bqp_lbmpc_dims* d, int batch,
                        const bqp_lbmpc_data* data, const bqp_sqp_loop* sl,
                        const bqp_options* opt, const bqp_closed_loop* cl, const bqp_learning* lw,
                        const double* x_init, double* X, double* U, int* exitflag);
int bqp_closed_loop_sqp_device(bqp_handle h, const bqp_lbmpc_dims* d, int batch,
                               const bqp_lbmpc_data* data, const bqp_sqp_loop* sl,
                               const bqp_options* opt, const bqp_closed_loop* cl,
                               const bqp_learning* lw, const double* x_init, double* X, double* U,
                               int* exitflag, void* stream);

/* Timing of the most recent solve on this handle: kernel time measured with hipEvents on the
 * launch stream (ms), and the number of kernel launches it covered. */
int bqp_last_kernel_ms(bqp_handle h, double* ms, int* launches);

/* Diagnostic: per instance of the most recent mixed-precision structured solve on this handle
 * (bqp_options.precision = 2, N + 1 > 64), the fp32 phase's exit flag (1 / 0: continued in fp64
 * from its iterate; -2 / -8: solved from the fp64 initial point), or 2 where the continuation did
 * not converge and the retry launch solved the instance again from the fp64 initial point
 * (tests/test_gpu_mixed.py).  batch must equal that solve's. */
int bqp_debug_mixed_flags(bqp_handle h, int batch, int* flags);

#ifdef __cplusplus
}
#endif
#endif /* BQP_H */
