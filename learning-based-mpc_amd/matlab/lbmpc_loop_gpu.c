/*
 * lbmpc_loop_gpu.c — MATLAB MEX gateway of the learned-model NLP closed loop on the GPU
 * (bqp_closed_loop_sqp).  Source for a MATLAB user (mex -R2018a lbmpc_loop_gpu.c
 * -I<repo>/include -L<repo>/learning-based-mpc_amd/bqp -lbqp); exercised here by
 * tests/test_mex_gateway.py against the stub mex.h of tests/mex_stub/.
 *
 *   [X, U, exitflag, XL, iterations, window, Z] = lbmpc_loop_gpu(P, L, x_init, options)
 *
 * It replaces the whole closed loop of matlab/LBMPC/examples/DMS_LBMPC_casadi.m:163-218 (per
 * step: solver(...) at :174, the RK4 plant `dynamic`, get_data.m's window update) for a batch
 * of initial states, through dms_lbmpc_loop_gpu.m.
 *
 * P (struct, bqp_lbmpc_dims / bqp_lbmpc_data of include/bqp.h, as for lbmpc_gpu):
 *   N, n_run, term_learned, hessian (optional, default 1), bandwidth, lambda (optional)
 *   A, B, K, Lq, Lr, Lp, Lt, LAMBDA, PSI, xs, Ain (m x n)
 *   bin0 m, Bx m x nx   the condensed constraints of each step: Ain z <= bin0 + Bx dx0
 * L (struct, bqp_closed_loop / bqp_sqp_loop / bqp_learning):
 *   steps, delta (plant step), x_eq nx, u_eq nu, q (window points), mask (1: 8 x q window with
 *   the validity row, DMS_LBMPC_casadi.m:158-161; 0: every point counts), warm (1: the
 *   scripts' shifted warm start), bandwidth, lambda (optional, the NW kernel of the window's
 *   predictions; default the model's)
 * x_init nx x batch   absolute initial states
 * options (optional struct): max_iter (SQP iterations per step), tol.
 * Outputs: X nx*(steps+1) x batch, U nu*steps x batch (absolute), exitflag steps x batch,
 * XL nx*(steps+1) x batch (learned one-step predictions, casadiL2NW.m), iterations steps x
 * batch (SQP iterations per step), window 8*q x batch (final windows, ring order), Z n*steps x
 * batch (every step's SQP solution, only computed when requested).
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "mex.h"
#include "bqp.h"

static bqp_handle g_handle = NULL;

static void cleanup(void) {
    if (g_handle) bqp_destroy(g_handle);
    g_handle = NULL;
}

static const mxArray* field(const mxArray* S, const char* sname, const char* name, int required) {
    const mxArray* f = mxGetField(S, 0, name);
    if (f && mxIsEmpty(f)) f = NULL;
    if (!f && required) mexErrMsgIdAndTxt("bqp:args", "%s.%s is required", sname, name);
    if (f && (!mxIsDouble(f) || mxIsComplex(f)))
        mexErrMsgIdAndTxt("bqp:args", "%s.%s must be a real double array", sname, name);
    return f;
}

static double scalar_or(const mxArray* S, const char* sname, const char* name, double dflt) {
    const mxArray* f = field(S, sname, name, 0);
    if (!f) return dflt;
    if (mxGetNumberOfElements(f) != 1) mexErrMsgIdAndTxt("bqp:args", "%s.%s must be a scalar", sname, name);
    return mxGetScalar(f);
}

static int scalar_int(const mxArray* S, const char* sname, const char* name, int required, int dflt) {
    const mxArray* f = field(S, sname, name, required);
    if (!f) return dflt;
    if (mxGetNumberOfElements(f) != 1) mexErrMsgIdAndTxt("bqp:args", "%s.%s must be a scalar", sname, name);
    const double v = mxGetScalar(f);
    if (v != floor(v)) mexErrMsgIdAndTxt("bqp:args", "%s.%s must be an integer", sname, name);
    return (int)v;
}

static const double* sized(const mxArray* S, const char* sname, const char* name, size_t m, size_t n) {
    const mxArray* f = field(S, sname, name, 1);
    if (mxGetM(f) * mxGetN(f) != m * n || (n > 1 && mxGetM(f) != m))
        mexErrMsgIdAndTxt("bqp:dims", "%s.%s must be %zu x %zu", sname, name, m, n);
    return mxGetDoubles(f);
}

static double* row_major(const mxArray* P, const char* name, size_t n) {
    const double* a = sized(P, "P", name, n, n);
    double* o = (double*)mxCalloc(n * n, sizeof(double));
    for (size_t i = 0; i < n; ++i)
        for (size_t j = 0; j < n; ++j) o[i * n + j] = a[j * n + i];
    return o;
}

void mexFunction(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
    if (nrhs < 3 || !mxIsStruct(prhs[0]) || !mxIsStruct(prhs[1]))
        mexErrMsgIdAndTxt("bqp:args", "[X,U,exitflag,XL,iterations,window,Z] = lbmpc_loop_gpu(P, L, x_init, options)");
    const mxArray *P = prhs[0], *Ls = prhs[1], *XI = prhs[2];
    if (!mxIsDouble(XI) || mxIsComplex(XI)) mexErrMsgIdAndTxt("bqp:args", "x_init must be a real double array");
    const mxArray* A = field(P, "P", "A", 1);
    const mxArray* Bm = field(P, "P", "B", 1);
    const mxArray* LA = field(P, "P", "LAMBDA", 1);
    const mxArray* Ain = field(P, "P", "Ain", 1);
    bqp_lbmpc_dims d;
    memset(&d, 0, sizeof(d));
    d.nx = (int)mxGetM(A);
    d.nu = (int)mxGetN(Bm);
    d.np = (int)mxGetN(LA);
    d.N = scalar_int(P, "P", "N", 1, 0);
    d.n_run = scalar_int(P, "P", "n_run", 0, d.N);
    d.term_learned = scalar_int(P, "P", "term_learned", 0, 1);
    d.hessian = scalar_int(P, "P", "hessian", 0, 1);
    const int nx = d.nx, nu = d.nu, np = d.np, N = d.N;
    if (nx < 1 || nu < 1 || np < 1 || N < 1) mexErrMsgIdAndTxt("bqp:dims", "need nx, nu, np, N >= 1");
    const int n = N * nu + np;
    d.m = (int)mxGetM(Ain);
    if (mxGetN(Ain) != (size_t)n) mexErrMsgIdAndTxt("bqp:dims", "P.Ain must have n = N*nu + np = %d columns", n);
    if (mxGetM(XI) != (size_t)nx) mexErrMsgIdAndTxt("bqp:dims", "x_init must have nx = %d rows", nx);
    const int batch = (int)mxGetN(XI);
    if (batch < 1) mexErrMsgIdAndTxt("bqp:dims", "x_init is empty");
    const int steps = scalar_int(Ls, "L", "steps", 1, 0);
    if (steps < 1) mexErrMsgIdAndTxt("bqp:args", "L.steps must be >= 1");
    d.q = scalar_int(Ls, "L", "q", 1, 0);
    d.mask = 1;
    if (d.q < 1) mexErrMsgIdAndTxt("bqp:args", "L.q must be >= 1");

    bqp_lbmpc_data D;
    memset(&D, 0, sizeof(D));
    D.A = sized(P, "P", "A", nx, nx);
    D.B = sized(P, "P", "B", nx, nu);
    D.K = sized(P, "P", "K", nu, nx);
    D.Lq = row_major(P, "Lq", nx);
    D.Lr = row_major(P, "Lr", nu);
    D.Lp = row_major(P, "Lp", nx);
    D.Lt = row_major(P, "Lt", nx);
    D.LAMBDA = sized(P, "P", "LAMBDA", nx, np);
    D.PSI = sized(P, "P", "PSI", nu, np);
    D.xs = sized(P, "P", "xs", nx, 1);
    D.Ain = mxGetDoubles(Ain);
    D.bandwidth = scalar_or(P, "P", "bandwidth", 0.0);
    D.lambda = scalar_or(P, "P", "lambda", 0.0);
    /* data, x0 and bin are the loop's own (bqp_closed_loop_sqp ignores them) */
    bqp_sqp_loop sl;
    memset(&sl, 0, sizeof(sl));
    sl.bin0 = sized(P, "P", "bin0", d.m, 1);
    sl.Bx = sized(P, "P", "Bx", d.m, nx);
    sl.warm = scalar_int(Ls, "L", "warm", 0, 1);
    bqp_closed_loop cl;
    memset(&cl, 0, sizeof(cl));
    cl.plant = BQP_PLANT_MG_RK4;
    cl.steps = steps;
    cl.delta = scalar_or(Ls, "L", "delta", 0.01);
    cl.x_eq = sized(Ls, "L", "x_eq", nx, 1);
    cl.u_eq = sized(Ls, "L", "u_eq", nu, 1);
    bqp_learning lw;
    memset(&lw, 0, sizeof(lw));
    lw.q = d.q;
    lw.mask = scalar_int(Ls, "L", "mask", 0, 1);
    if (lw.mask != 0 && lw.mask != 1) mexErrMsgIdAndTxt("bqp:args", "L.mask must be 0 or 1");
    lw.bandwidth = scalar_or(Ls, "L", "bandwidth", 0.0);
    lw.lambda = scalar_or(Ls, "L", "lambda", 0.0);
    bqp_options opt;
    bqp_default_options(&opt);
    if (nrhs > 3 && !mxIsEmpty(prhs[3])) {
        if (!mxIsStruct(prhs[3])) mexErrMsgIdAndTxt("bqp:args", "options must be a struct");
        const mxArray* f;
        if ((f = mxGetField(prhs[3], 0, "max_iter"))) opt.max_iter = (int)mxGetScalar(f);
        if ((f = mxGetField(prhs[3], 0, "tol"))) opt.tol_stat = mxGetScalar(f);
    }
    if (!g_handle) {
        if (bqp_create(&g_handle, -1) != BQP_OK) mexErrMsgIdAndTxt("bqp:gpu", "no gfx950 device");
        mexAtExit(cleanup);
    }
    mxArray* Xo = mxCreateDoubleMatrix((size_t)nx * (steps + 1), batch, mxREAL);
    mxArray* Uo = mxCreateDoubleMatrix((size_t)nu * steps, batch, mxREAL);
    mxArray* XLo = mxCreateDoubleMatrix((size_t)nx * (steps + 1), batch, mxREAL);
    mxArray* Wo = mxCreateDoubleMatrix((size_t)8 * d.q, batch, mxREAL);
    mxArray* Zo = nlhs > 6 ? mxCreateDoubleMatrix((size_t)n * steps, batch, mxREAL) : NULL;
    int* flag = (int*)mxCalloc((size_t)batch * steps, sizeof(int));
    int* iters = (int*)mxCalloc((size_t)batch * steps, sizeof(int));
    lw.XL = mxGetDoubles(XLo);
    lw.window = mxGetDoubles(Wo);
    sl.Z = Zo ? mxGetDoubles(Zo) : NULL;
    sl.iterations = iters;
    const int rc = bqp_closed_loop_sqp(g_handle, &d, batch, &D, &sl, &opt, &cl, &lw,
                                       mxGetDoubles(XI), mxGetDoubles(Xo), mxGetDoubles(Uo), flag);
    if (rc == BQP_E_UNSUPPORTED) mexErrMsgIdAndTxt("bqp:unsupported", "dimensions outside the compiled set (nx 4, nu 1, np 1, q <= 512)");
    if (rc != BQP_OK) mexErrMsgIdAndTxt("bqp:solve", "bqp_closed_loop_sqp failed (%d)", rc);
    mxArray* Eo = mxCreateDoubleMatrix(steps, batch, mxREAL);
    mxArray* Io = mxCreateDoubleMatrix(steps, batch, mxREAL);
    for (size_t i = 0; i < (size_t)batch * steps; ++i) {
        mxGetDoubles(Eo)[i] = flag[i];
        mxGetDoubles(Io)[i] = iters[i];
    }
    mxFree(flag); mxFree(iters);
    mxArray* outs[7] = {Xo, Uo, Eo, XLo, Io, Wo, Zo};
    for (int i = 0; i < 7; ++i) {
        if (!outs[i]) continue;
        if (i < (nlhs > 0 ? nlhs : 1)) plhs[i] = outs[i];
        else mxDestroyArray(outs[i]);
    }
}
