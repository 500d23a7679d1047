/*
 * ocp_gpu.c — MATLAB MEX gateway of the structured fast path (bqp_solve_ocp_batched).  Source
 * for a MATLAB user (mex -R2018a ocp_gpu.c -I<repo>/include -L<repo>/learning-based-mpc_amd/bqp
 * -lbqp); exercised here by tests/test_mex_gateway.py against the stub mex.h of tests/mex_stub/.
 *
 *   [X, U, theta, fval, exitflag, output, lambda] = ocp_gpu(P, x0, options)
 *
 * It replaces the per-step OCP solve of the reference through the .m shims next to it:
 *   lmpc_solve_gpu.m       for fmincon(COSTFUN, opt_var, ..., CONSFUN) at ocpLMPC.m:20-24 (F1)
 *   dms_tracking_solve_gpu.m  for solver('x0',..,'lbx',..) at DMS_tracking_LMPC_casadi.m:163-167 (F2)
 *
 * P (struct, the stage-wise problem of include/bqp.h; all fp64, column-major):
 *   N, nu, np          scalars; nx = rows of A; nv = nx + nu + np, v_k = [x_k; u_k; theta]
 *   A  nx x nx,  B  nx x nu,  c  nx (optional)            one copy, or a copy per instance
 *   W  nv x nv x (N+1)  stage Hessians (shared by the batch)
 *   w  nv x (N+1)       linear terms (optional; shared or per instance)
 *   xlb, xub  nx x (N+1),  ulb, uub  nu x N  (optional, +-Inf allowed; shared or per instance)
 *   Fp  n_poly x nv (shared),  hp  n_poly (shared or per instance),  poly_stage  0..N (0-based)
 * x0: nx x batch (one column per instance).  An array "per instance" has batch times the
 * elements of one copy (a trailing batch dimension in MATLAB).
 * options (optional struct): max_iter, tol_stat, tol_feas, tol_comp, tau, precision (0 fp64,
 * 1 fp32, 2 mixed).
 * Outputs: X nx*(N+1) x batch, U nu*N x batch, theta np x batch, fval / exitflag 1 x batch,
 * output (1 x batch struct: iterations, constrviolation, firstorderopt, mu), lambda (1 x batch
 * struct: pi nx*N, lam_x 2*nx*(N+1) [lower; upper] per stage, lam_u 2*nu*N, lam_p n_poly).
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

static const mxArray* field(const mxArray* P, const char* name, int required) {
    const mxArray* f = mxGetField(P, 0, name);
    if (f && mxIsEmpty(f)) f = NULL;
    if (!f && required) mexErrMsgIdAndTxt("bqp:args", "P.%s is required", name);
    /* mxGetDoubles returns NULL for single / integer / complex arrays: reject them rather than
       read an optional field as absent */
    if (f && (!mxIsDouble(f) || mxIsComplex(f)))
        mexErrMsgIdAndTxt("bqp:args", "P.%s must be a real double array", name);
    return f;
}

static int scalar_int(const mxArray* P, const char* name) {
    const mxArray* f = field(P, name, 1);
    if (mxGetNumberOfElements(f) != 1) mexErrMsgIdAndTxt("bqp:args", "P.%s must be a scalar", name);
    const double v = mxGetScalar(f);
    if (v != floor(v)) mexErrMsgIdAndTxt("bqp:args", "P.%s must be an integer", name);
    return (int)v;
}

/* element stride between instances: 0 = one copy for the batch, per = a copy per instance */
static int64_t stride_of(const mxArray* a, const char* name, size_t per, int batch, int shared_only) {
    if (!a) return 0;
    const size_t n = mxGetNumberOfElements(a);
    if (n == per) return 0;
    if (!shared_only && n == per * (size_t)batch) return (int64_t)per;
    mexErrMsgIdAndTxt("bqp:dims", "P.%s has %zu elements, expected %zu%s", name, n, per,
                      shared_only ? " (shared by the batch)" : " or one copy per instance");
    return 0;
}

static const double* data_of(const mxArray* a) { return a ? mxGetDoubles(a) : NULL; }

static void read_options(const mxArray* o, bqp_options* opt) {
    bqp_default_options(opt);
    if (!o || mxIsEmpty(o)) return;
    if (!mxIsStruct(o)) mexErrMsgIdAndTxt("bqp:args", "options must be a struct");
    const mxArray* f;
    if ((f = mxGetField(o, 0, "max_iter"))) opt->max_iter = (int)mxGetScalar(f);
    if ((f = mxGetField(o, 0, "tol_stat"))) opt->tol_stat = mxGetScalar(f);
    if ((f = mxGetField(o, 0, "tol_feas"))) opt->tol_feas = mxGetScalar(f);
    if ((f = mxGetField(o, 0, "tol_comp"))) opt->tol_comp = mxGetScalar(f);
    if ((f = mxGetField(o, 0, "tau"))) opt->tau = mxGetScalar(f);
    if ((f = mxGetField(o, 0, "precision"))) opt->precision = (int)mxGetScalar(f);
}

void mexFunction(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
    if (nrhs < 2 || !mxIsStruct(prhs[0]))
        mexErrMsgIdAndTxt("bqp:args", "[X,U,theta,fval,exitflag,output,lambda] = ocp_gpu(P, x0, options)");
    const mxArray* P = prhs[0];
    const mxArray* X0 = prhs[1];
    if (!mxIsDouble(X0) || mxIsComplex(X0)) mexErrMsgIdAndTxt("bqp:args", "x0 must be a real double array");
    const mxArray* A = field(P, "A", 1);
    bqp_ocp_dims d;
    d.nx = (int)mxGetM(A);
    d.N = scalar_int(P, "N");
    d.nu = scalar_int(P, "nu");
    d.np = scalar_int(P, "np");
    const int nx = d.nx, nu = d.nu, np = d.np, N = d.N;
    if (nx < 1 || nu < 1 || np < 1 || N < 1) mexErrMsgIdAndTxt("bqp:dims", "need nx, nu, np, N >= 1");
    if (mxGetM(X0) != (size_t)nx) mexErrMsgIdAndTxt("bqp:dims", "x0 must have nx = %d rows", nx);
    const int batch = (int)mxGetN(X0);
    if (batch < 1) mexErrMsgIdAndTxt("bqp:dims", "x0 is empty");
    const int nv = nx + nu + np;
    const mxArray* Fp = field(P, "Fp", 0);
    d.n_poly = Fp ? (int)mxGetM(Fp) : 0;
    d.poly_stage = Fp ? scalar_int(P, "poly_stage") : N;
    if (Fp && mxGetN(Fp) != (size_t)nv) mexErrMsgIdAndTxt("bqp:dims", "P.Fp must have nv = %d columns", nv);
    if (d.poly_stage < 0 || d.poly_stage > N) mexErrMsgIdAndTxt("bqp:dims", "P.poly_stage must be in 0..N");

    bqp_ocp_data D;
    memset(&D, 0, sizeof(D));
    const mxArray *B = field(P, "B", 1), *c = field(P, "c", 0), *W = field(P, "W", 1),
                  *w = field(P, "w", 0), *xlb = field(P, "xlb", 0), *xub = field(P, "xub", 0),
                  *ulb = field(P, "ulb", 0), *uub = field(P, "uub", 0), *hp = field(P, "hp", 0);
    if (d.n_poly > 0 && !hp) mexErrMsgIdAndTxt("bqp:args", "P.hp is required with P.Fp");
    D.A = data_of(A);     D.sA = stride_of(A, "A", (size_t)nx * nx, batch, 0);
    D.B = data_of(B);     D.sB = stride_of(B, "B", (size_t)nx * nu, batch, 0);
    D.c = data_of(c);     D.sc = stride_of(c, "c", nx, batch, 0);
    D.W = data_of(W);     D.sW = stride_of(W, "W", (size_t)(N + 1) * nv * nv, batch, 1);
    D.w = data_of(w);     D.sw = stride_of(w, "w", (size_t)(N + 1) * nv, batch, 0);
    D.xlb = data_of(xlb); D.sxb = stride_of(xlb, "xlb", (size_t)(N + 1) * nx, batch, 0);
    D.xub = data_of(xub);
    if (xub && stride_of(xub, "xub", (size_t)(N + 1) * nx, batch, 0) != D.sxb && xlb)
        mexErrMsgIdAndTxt("bqp:dims", "P.xlb and P.xub must both be shared or both per instance");
    if (!xlb) D.sxb = stride_of(xub, "xub", (size_t)(N + 1) * nx, batch, 0);
    D.ulb = data_of(ulb); D.sub = stride_of(ulb, "ulb", (size_t)N * nu, batch, 0);
    D.uub = data_of(uub);
    if (uub && stride_of(uub, "uub", (size_t)N * nu, batch, 0) != D.sub && ulb)
        mexErrMsgIdAndTxt("bqp:dims", "P.ulb and P.uub must both be shared or both per instance");
    if (!ulb) D.sub = stride_of(uub, "uub", (size_t)N * nu, batch, 0);
    D.Fp = data_of(Fp);   D.sFp = 0;
    if (Fp) stride_of(Fp, "Fp", (size_t)d.n_poly * nv, batch, 1);
    D.hp = data_of(hp);   D.shp = hp ? stride_of(hp, "hp", (size_t)d.n_poly, batch, 0) : 0;
    D.x0 = mxGetDoubles(X0); D.sx0 = nx;
    bqp_options opt;
    read_options(nrhs > 2 ? prhs[2] : NULL, &opt);

    if (!g_handle) {
        if (bqp_create(&g_handle, -1) != BQP_OK) mexErrMsgIdAndTxt("bqp:gpu", "no gfx950 device");
        mexAtExit(cleanup);
    }
    mxArray* Xo = mxCreateDoubleMatrix((size_t)nx * (N + 1), batch, mxREAL);
    mxArray* Uo = mxCreateDoubleMatrix((size_t)nu * N, batch, mxREAL);
    mxArray* To = mxCreateDoubleMatrix(np, batch, mxREAL);
    mxArray* Fo = mxCreateDoubleMatrix(1, batch, mxREAL);
    mxArray* Eo = mxCreateDoubleMatrix(1, batch, mxREAL);
    int* flag = (int*)mxCalloc(batch, sizeof(int));
    bqp_output* out = (bqp_output*)mxCalloc(batch, sizeof(bqp_output));
    bqp_ocp_duals du;
    memset(&du, 0, sizeof(du));
    const int mp = d.n_poly;
    if (nlhs > 6) {
        du.pi = (double*)mxCalloc((size_t)batch * N * nx, sizeof(double));
        du.lam_x = (double*)mxCalloc((size_t)batch * (N + 1) * nx * 2, sizeof(double));
        du.lam_u = (double*)mxCalloc((size_t)batch * N * nu * 2, sizeof(double));
        du.lam_p = (double*)mxCalloc((size_t)batch * (mp ? mp : 1), sizeof(double));
    }
    const int rc = bqp_solve_ocp_batched(g_handle, &d, batch, &D, &opt, mxGetDoubles(Xo),
                                         mxGetDoubles(Uo), mxGetDoubles(To), mxGetDoubles(Fo),
                                         flag, out, nlhs > 6 ? &du : NULL);
    if (rc != BQP_OK) mexErrMsgIdAndTxt("bqp:solve", "bqp_solve_ocp_batched failed (%d)", rc);
    for (int i = 0; i < batch; ++i) mxGetDoubles(Eo)[i] = flag[i];
    mxArray* outs[5] = {Xo, Uo, To, Fo, Eo};
    for (int i = 0; i < 5; ++i) {
        if (i == 0 || nlhs > i) plhs[i] = outs[i];
        else mxDestroyArray(outs[i]);
    }
    if (nlhs > 5) {
        const char* fields[] = {"iterations", "constrviolation", "firstorderopt", "mu"};
        plhs[5] = mxCreateStructMatrix(1, batch, 4, fields);
        for (int i = 0; i < batch; ++i) {
            mxSetField(plhs[5], i, "iterations", mxCreateDoubleScalar(out[i].iterations));
            mxSetField(plhs[5], i, "constrviolation", mxCreateDoubleScalar(out[i].constrviolation));
            mxSetField(plhs[5], i, "firstorderopt", mxCreateDoubleScalar(out[i].firstorderopt));
            mxSetField(plhs[5], i, "mu", mxCreateDoubleScalar(out[i].mu));
        }
    }
    if (nlhs > 6) {
        const char* fields[] = {"pi", "lam_x", "lam_u", "lam_p"};
        const size_t len[4] = {(size_t)N * nx, (size_t)(N + 1) * nx * 2, (size_t)N * nu * 2, (size_t)mp};
        const double* src[4] = {du.pi, du.lam_x, du.lam_u, du.lam_p};
        plhs[6] = mxCreateStructMatrix(1, batch, 4, fields);
        for (int i = 0; i < batch; ++i)
            for (int f = 0; f < 4; ++f) {
                mxArray* a = mxCreateDoubleMatrix(len[f], 1, mxREAL);
                if (len[f]) memcpy(mxGetDoubles(a), src[f] + (size_t)i * len[f], sizeof(double) * len[f]);
                mxSetField(plhs[6], i, fields[f], a);
            }
    }
}
