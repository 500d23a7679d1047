// bqp_internal.h — kernel argument blocks and launch helpers shared by the HIP kernels and the
// C-ABI implementation (bqp_api.cpp).  Not part of the public ABI (include/bqp.h is).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace bqp {

// per-instance exit statistics written by every solve kernel and turned into bqp_output by
// finalize_kernel: iterations, stationarity, max(primal eq, primal ineq), mu, primal eq,
// primal ineq (inf-norms at exit), 1 if the answer is the structured solver's active-set polish
constexpr int STATS_W = 7;

// Structured OCP kernel arguments (device pointers).  H and Fp are the prepared shared tables:
//   H  : (N+1) stages x hstride doubles, stage cost in internal order [x; theta; u], row-major
//   Fp : column-major [NV][mpad] polytope matrix in internal order
// All other arrays are in the public (external) layout with per-instance element strides.
constexpr int OCP_QUEUES = 4;   // work-queue counters per structured solve (one per launch)
struct OcpKernelArgs {
    int N, mp, kp, batch, wpb, hstride, mpad, shared_doubles, max_iter;
    // persistent work queue: when the batch needs more workgroups than the
    // device holds at once, the launch is sized to the resident workgroups and every instance
    // slot (stage / row wave pair) takes its next instance from this counter (zeroed by the prep
    // kernel) as soon as its current one is done; nullptr: one instance per slot, grid = batch
    int* queue;
    double tol_stat, tol_feas, tol_comp, tau;
    const double* H;
    const double* Fp;
    const double *A, *B, *c, *w, *xlb, *xub, *ulb, *uub, *hp, *x0;
    int64_t sA, sB, sc, sw, sxb, sub, shp, sx0;
    double *x, *u, *theta, *fval;
    int* exitflag;
    double* stats;  // batch x STATS_W (see STATS_W)
    double *pi_out, *lamx_out, *lamu_out, *lamp_out;
    double* stamps;  // diagnostic build (BQP_STAMPS): batch x 16 phase cycle counts
    // mixed precision (bqp_options.precision = 2): the fp32 launch ends each instance at its
    // (floored) tolerances and writes its iterate (s, pi, u, row slacks and multipliers) to
    // hand_out; the fp64 launch continues from hand_in the instances whose fp32 exit flag
    // (hand_flag) is 1 or 0, and starts the others (-2, -8) from its own initial point
    float* hand_out;
    const float* hand_in;
    const int* hand_flag;
    int* hand_it;           // fp32-phase iterations (written by the fp32 launch, added by the fp64 one)
    int64_t hand_stride;    // floats per instance (ocp_hand_floats)
    // third launch of the mixed mode (cold fp64): only the instances whose warm continuation
    // did not converge (exitflag != 1 with a warm hand_flag) are solved again from the fp64
    // initial point; every other instance leaves at once
    const int* redo_flag;
    // per-instance polytope (bqp_ocp_data.sFp != 0): the caller's column-major n_poly x nv
    // blocks, stride sFp; the shared Fp table is then unused
    const double* Fp_inst;
    int64_t sFp;
    // long-horizon layout (two stages per lane, N + 1 > 64; QpLds lng): Riccati tables in global
    // scratch (batch x (N+1) x ocp_pstride elements of the instantiation's precision) and the
    // shared-LDS offsets of the polytope matrix, polytope rhs and box bounds (-1: not shared).
    // The stage-cost table H is then read from global (L2) instead of LDS.
    void* Pg;
    int sh_F, sh_hp, sh_bnd;
    // per-instance stage costs (bqp_ocp_data.sW != 0): prepared tables batch x (N+1) x hstride;
    // short horizons copy the instance's table into its LDS slot, long ones read it from L2
    const double* H_inst;
    // active-set polish (fp64 instantiation, bqp_options.polish): 0 off, 1 after a 0 / -8 exit,
    // 2 also with a weakly active row.  The solve kernel marks the instances that need it in
    // pol_need (batch ints); the repair launch (launch_ocp(..., pol = true)) solves those again
    // and polishes them
    int polish;
    int* pol_need;
};

bool ocp_supported(int nx, int nu, int np);
int ocp_rpl_for(int mp);
int ocp_bpl_for(int N, int nx, int nu);
int ocp_hand_floats(int N, int nx, int nu, int np, int mp);
int ocp_wave_lds_doubles(int N, int nx, int nu, int np, int mpad, bool fpi, bool lng, bool hpsh,
                         bool bndsh, bool hinst);
int ocp_pstride(int ns);
hipError_t launch_ocp(const OcpKernelArgs& a, int nx, int nu, int np, hipStream_t st, bool pol = false);
// fp32 instantiation (bqp_ocp_f32.hip): LDS element count per instance (floats) and launch
int ocp_wave_lds_doubles_f32(int N, int nx, int nu, int np, int mpad, bool fpi, bool lng,
                             bool hpsh, bool bndsh, bool hinst);
hipError_t launch_ocp_f32(const OcpKernelArgs& a, int nx, int nu, int np, hipStream_t st, bool pol = false);
hipError_t launch_ocp_prep(const double* W, const double* Fp, int nx, int nu, int np, int N,
                           int mp, int kp, int hstride, int mpad, double* Hout, double* Fout,
                           int* qzero, hipStream_t st);
hipError_t launch_ocp_prep_h(const double* W, int64_t sW, int batch, int nx, int nu, int np,
                             int N, int hstride, double* Hout, hipStream_t st);
hipError_t launch_ocp_finalize(const double* stats, int batch, void* out, hipStream_t st);

// Dense quadprog kernel arguments.
struct DenseKernelArgs {
    int n, m, me, batch, max_iter, mrows;  // mrows = m + finite bound rows (set per instance)
    double tol_stat, tol_feas, tol_comp, tau;
    const double *H, *f, *A, *b, *Aeq, *beq, *lb, *ub;
    int64_t sH, sf, sA, sb, sAeq, sbeq, slb, sub;
    double *x, *fval, *lam_ineqlin, *lam_eqlin, *lam_lower, *lam_upper;
    int* exitflag;
    double* stats;
    double* work;      // per-instance scratch (global), work_stride doubles each
    int64_t work_stride;
    int polish;        // 1: active-set polish after a 0 / -8 exit (bqp_dense.hip::dense_polish);
                       // 2: also after a converged exit (exact active-set steps for the SQP)
    const int* pol_it; // optional: per-instance SQP iteration counts; mode 2 where >= pol_stall
    int pol_stall;     // (the learned-model loop, whose instances run at their own SQP iteration)
    const int* skip;   // optional: instances with skip[i] != 0 are not solved (finished SQPs)
    int res_every;     // exact residual evaluation at least every res_every iterations (0: 8;
                       // 1: every iteration, the diagnostic BQP_DENSE_RES_EVERY)
};

int dense_work_doubles(int n, int m, int me);
hipError_t launch_dense(const DenseKernelArgs& a, hipStream_t st);
hipError_t launch_dense_symmetrize(double* H, int n, int count, int64_t stride, hipStream_t st);

// Learning-based MPC (Gauss-Newton SQP on the NW-learned model), bqp_lbmpc.hip.  Small
// matrices column-major (A nx*nx, B nx*nu, K nu*nx, LAMBDA nx*np, PSI nu*np); weight factors
// upper-triangular row-major (Lq nx*nx, Lr nu*nu, Lp, Lt nx*nx); NW window wrows x q
// column-major (7: [X; Y], 8: [X; Y; v] with the validity row of casadiL2NW.m).
struct LbmpcArgs {
    int N, n, nr, m, q, n_run, term_learned, batch, ntrial, max_iter, wrows;
    double hinv2, lam_nw, tol_step, tol_stat;
    const double *A, *B, *K, *Lq, *Lr, *Lp, *Lt, *LAM, *PSI, *xs;
    const double* data; int64_t sdata;
    const double* x0; int64_t sx0;
    const double* Ain;                  // m x n column-major, shared
    const double* bin; int64_t sbin;    // m per instance
    double* z;                          // batch x n iterate (in: start, out: solution)
    double* d;                          // batch x n QP step
    double* lam;                        // batch x m QP multipliers
    double *Jr, *er;                    // batch x nr x n (row-major), batch x nr
    double *H, *f, *bsh;                // batch x n x n (column-major), batch x n, batch x m
    double *cost0, *costT, *stat, *cprev;  // batch, batch x ntrial, batch, batch
    int *qpflag, *flag, *done, *iters, *ndone;
    // exact Hessian (hess = 1): rows Xi_k (Jr2) and W_k Xi_k (Tr2), batch x 3N x n row-major;
    // hused (may be null): per instance, the iterations that used the exact Hessian
    int hess;
    double *Jr2, *Tr2;
    int* hused;
};

hipError_t launch_nw_oracle(int batch, int q, const double* data, int64_t sdata, const double* xi,
                            double* g, double* dg, double bw, double lam, hipStream_t st);
bool lbmpc_hess_fits(int n);   // exact-Hessian LDS fits (n <= 127); else Gauss-Newton
bool lbmpc_supported(int nx, int nu, int np, int n, int q);
hipError_t launch_lbmpc_rollout(const LbmpcArgs& a, int gn, hipStream_t st);
hipError_t launch_lbmpc_normal(const LbmpcArgs& a, hipStream_t st);
hipError_t launch_lbmpc_update(const LbmpcArgs& a, hipStream_t st);
hipError_t launch_lbmpc_hess(const LbmpcArgs& a, hipStream_t st);

// closed-loop simulation (bqp_plant.hip): Moore-Greitzer plant (RK4 step or MATLAB ode23,
// BQP_PLANT_*) between batched solves
hipError_t launch_closed_loop_init(int batch, int nx, int steps, const double* xinit,
                                   const double* xeq, double* s, double* X, hipStream_t st);
hipError_t launch_mg_plant(int plant, int batch, int N, int steps, int t, double delta,
                           const double* uo, const int* fl, const double* xeq, const double* ueq,
                           double* s, double* X, double* U, int* flags, hipStream_t st);
// learned-model NLP closed loop glue (bqp_closed_loop_sqp): per instance bin = bin0 + Bx s and
// the warm start (z shifted one stage, zero last move, theta kept) before the SQP; u_0 = K s + z_0
// for the plant, and the step's z / iteration count into the caller's logs after it
// asynchronous learned-model loop: one instance's advance to its next closed-loop step
struct SqpAdvanceArgs {
    int batch, nx, nu, n, m, nv, warm, steps, q, plant;
    double delta, hinv2, lam;
    const double *K, *bin0, *Bx, *xeq, *ueq, *A, *Bm;
    double *s, *z, *bin, *X, *U, *win, *XL, *Zlog;
    int *done, *iters, *flag, *hused, *ts, *nfin, *flags, *itlog;
};
hipError_t launch_sqp_loop_advance(const SqpAdvanceArgs& a, hipStream_t st);
hipError_t launch_sqp_loop_prep(int batch, int nx, int n, int m, int nv, int shift, const double* s,
                                const double* bin0, const double* Bx, double* bin, double* z,
                                hipStream_t st);
hipError_t launch_sqp_loop_u0(int batch, int nx, int n, const double* K, const double* s,
                              const double* z, double* uo, const int* it, int steps, int t,
                              double* Zlog, int* itlog, hipStream_t st);
hipError_t launch_lbmpc_window_init(int batch, int steps, int q, int mask, const double* xinit,
                                    double* win, double* XL, hipStream_t st);
hipError_t launch_lbmpc_window(int batch, int steps, int t, int q, double bw, double lam,
                               const double* A, int64_t sA, const double* B, int64_t sB,
                               const double* xeq, const double* ueq, const double* X,
                               const double* U, double* win, double* XL, hipStream_t st);

}  // namespace bqp
