/*
 * quadprog_gpu.c — MATLAB MEX gateway for libbqp (source only: MATLAB's mex.h is not available in
 * the build image, so this file is compiled by a MATLAB user with
 *     mex -R2018a quadprog_gpu.c -I<repo>/include -L<repo>/learning-based-mpc_amd/bqp -lbqp
 * and exercised here by tests/test_mex_gateway.py, which compiles it against a stub mex.h
 * (tests/mex_stub/) and drives the gateway from C).
 *
 * Drop-in for the per-step QP solve of the reference:
 *     [x,fval,exitflag,output,lambda] = quadprog_gpu(H,f,A,b,Aeq,beq,lb,ub,x0,options)
 * with MATLAB quadprog's argument meaning (x0 ignored: interior-point method).  A batch is
 * passed by giving f/b/beq/lb/ub (and optionally H/A/Aeq) a trailing batch dimension:
 *     f: n x B, b: m x B, beq: me x B, lb/ub: n x B, H: n x n (x B), A: m x n (x B) ...
 * A 2-D f (n x 1) is a single instance, exactly like quadprog.  Fixed variables (lb == ub) are
 * turned into equality rows here, as the kernel requires.
 *
 * The structured fast path (bqp_solve_ocp_batched) is reached from MATLAB through
 * ocp_gpu.m-style wrappers built on the same pattern; see INTEGRATION.md.
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

static int64_t stride_of(const mxArray* a, size_t per, int batch) {
    if (!a || mxIsEmpty(a)) return 0;
    size_t n = mxGetNumberOfElements(a);
    if (n == per) return 0;                     /* shared by the batch */
    if (n == per * (size_t)batch) return (int64_t)per;
    mexErrMsgIdAndTxt("bqp:dims", "argument has %zu elements, expected %zu or %zu", n, per,
                      per * (size_t)batch);
    return 0;
}

void mexFunction(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
    if (nrhs < 2) mexErrMsgIdAndTxt("bqp:args", "quadprog_gpu(H,f,A,b,Aeq,beq,lb,ub,x0,options)");
    const mxArray* H = prhs[0];
    const mxArray* f = prhs[1];
    const mxArray* A = nrhs > 2 ? prhs[2] : NULL;
    const mxArray* b = nrhs > 3 ? prhs[3] : NULL;
    const mxArray* Aeq = nrhs > 4 ? prhs[4] : NULL;
    const mxArray* beq = nrhs > 5 ? prhs[5] : NULL;
    const mxArray* lb = nrhs > 6 ? prhs[6] : NULL;
    const mxArray* ub = nrhs > 7 ? prhs[7] : NULL;
    /* every numeric argument must be real double: mxGetDoubles returns NULL for other classes,
       which would otherwise read as an absent argument */
    for (int i = 0; i < nrhs && i < 9; ++i)
        if (prhs[i] && !mxIsEmpty(prhs[i]) && (!mxIsDouble(prhs[i]) || mxIsComplex(prhs[i])))
            mexErrMsgIdAndTxt("bqp:args", "argument %d must be a real double array", i + 1);
    const int n = (int)mxGetM(f);
    const int batch = (int)mxGetN(f);
    const int m = (A && !mxIsEmpty(A)) ? (int)mxGetM(A) : 0;
    int me0 = (Aeq && !mxIsEmpty(Aeq)) ? (int)mxGetM(Aeq) : 0;

    if (!mxIsEmpty(H) && mxGetNumberOfElements(H) % ((size_t)n * n) != 0)
        mexErrMsgIdAndTxt("bqp:dims", "H must be n x n (x batch) with n = rows of f = %d", n);
    if (m && mxGetN(A) % (size_t)n != 0)
        mexErrMsgIdAndTxt("bqp:dims", "A must have n = %d columns (x batch)", n);
    const int64_t sH = stride_of(H, (size_t)n * n, batch), sA = stride_of(A, (size_t)m * n, batch),
                  sb = stride_of(b, m, batch);
    /* fixed variables (lb == ub) -> equality rows (same pattern for every instance) */
    const double* lbp = (lb && !mxIsEmpty(lb)) ? mxGetDoubles(lb) : NULL;
    const double* ubp = (ub && !mxIsEmpty(ub)) ? mxGetDoubles(ub) : NULL;
    const int64_t slb = stride_of(lb, n, batch), sub = stride_of(ub, n, batch);
    int nfix = 0;
    int* fix = (int*)mxCalloc(n, sizeof(int));
    if (lbp && ubp) {
        for (int j = 0; j < n; ++j)
            if (isfinite(lbp[j]) && lbp[j] == ubp[j]) fix[nfix++] = j;
        /* the kernel takes one equality-row pattern for the batch: every instance must fix the
           same variables (bqp/quadprog.py raises the same error) */
        for (int i = 1; i < batch; ++i)
            for (int j = 0, r = 0; j < n; ++j) {
                const int fx = isfinite(lbp[i * slb + j]) && lbp[i * slb + j] == ubp[i * sub + j];
                const int f0 = r < nfix && fix[r] == j;
                if (f0) ++r;
                if (fx != f0)
                    mexErrMsgIdAndTxt("bqp:fixed", "fixed variables (lb == ub) must be the same "
                                      "for every instance (instance %d, variable %d)", i + 1, j + 1);
            }
    }
    const int me = me0 + nfix;
    double* E = (double*)mxCalloc((size_t)me * n * batch + 1, sizeof(double));
    double* e = (double*)mxCalloc((size_t)me * batch + 1, sizeof(double));
    double* L2 = (double*)mxCalloc((size_t)n * batch + 1, sizeof(double));
    double* U2 = (double*)mxCalloc((size_t)n * batch + 1, sizeof(double));
    const int64_t sAeq0 = stride_of(Aeq, (size_t)me0 * n, batch), sbeq0 = stride_of(beq, me0, batch);
    for (int i = 0; i < batch; ++i) {
        for (int c = 0; c < n; ++c)
            for (int r = 0; r < me0; ++r)
                E[(size_t)i * me * n + (size_t)c * me + r] = mxGetDoubles(Aeq)[i * sAeq0 + (size_t)c * me0 + r];
        for (int r = 0; r < nfix; ++r) {
            E[(size_t)i * me * n + (size_t)fix[r] * me + me0 + r] = 1.0;
            e[(size_t)i * me + me0 + r] = lbp[i * slb + fix[r]];
        }
        for (int r = 0; r < me0; ++r) e[(size_t)i * me + r] = mxGetDoubles(beq)[i * sbeq0 + r];
        for (int j = 0; j < n; ++j) {
            L2[(size_t)i * n + j] = lbp ? lbp[i * slb + j] : -INFINITY;
            U2[(size_t)i * n + j] = ubp ? ubp[i * sub + j] : INFINITY;
        }
        for (int r = 0; r < nfix; ++r) {
            L2[(size_t)i * n + fix[r]] = -INFINITY;
            U2[(size_t)i * n + fix[r]] = INFINITY;
        }
    }
    /* arguments are validated above: only now take the device (first call) */
    if (!g_handle) {
        if (bqp_create(&g_handle, -1) != BQP_OK) mexErrMsgIdAndTxt("bqp:gpu", "no gfx950 device");
        mexAtExit(cleanup);
    }
    bqp_dims d = {n, m, me};
    bqp_strides st;
    st.sH = sH;
    st.sf = n;
    st.sA = sA;
    st.sb = sb;
    st.sAeq = (int64_t)me * n;
    st.sbeq = me;
    st.slb = n;
    st.sub = n;
    plhs[0] = mxCreateDoubleMatrix(n, batch, mxREAL);
    mxArray* fv = mxCreateDoubleMatrix(1, batch, mxREAL);
    mxArray* ef = mxCreateDoubleMatrix(1, batch, mxREAL);
    int* flag = (int*)mxCalloc(batch, sizeof(int));
    double* lin = (double*)mxCalloc((size_t)(m ? m : 1) * batch, sizeof(double));
    double* leq = (double*)mxCalloc((size_t)(me ? me : 1) * batch, sizeof(double));
    double* llo = (double*)mxCalloc((size_t)n * batch, sizeof(double));
    double* lup = (double*)mxCalloc((size_t)n * batch, sizeof(double));
    bqp_output* out = (bqp_output*)mxCalloc(batch, sizeof(bqp_output));
    int rc = bqp_quadprog_batched(g_handle, &d, batch, &st, mxGetDoubles(H), mxGetDoubles(f),
                                  m ? mxGetDoubles(A) : NULL, m ? mxGetDoubles(b) : NULL,
                                  me ? E : NULL, me ? e : NULL, L2, U2, NULL, NULL,
                                  mxGetDoubles(plhs[0]), mxGetDoubles(fv), flag, lin, leq, llo,
                                  lup, out);
    if (rc != BQP_OK) mexErrMsgIdAndTxt("bqp:solve", "bqp_quadprog_batched failed (%d)", rc);
    for (int i = 0; i < batch; ++i) mxGetDoubles(ef)[i] = flag[i];
    if (nlhs > 1) plhs[1] = fv; else mxDestroyArray(fv);
    if (nlhs > 2) plhs[2] = ef; else mxDestroyArray(ef);
    if (nlhs > 3) {
        const char* fields[] = {"iterations", "constrviolation", "firstorderopt", "algorithm"};
        plhs[3] = mxCreateStructMatrix(1, batch, 4, fields);
        for (int i = 0; i < batch; ++i) {
            mxSetField(plhs[3], i, "iterations", mxCreateDoubleScalar(out[i].iterations));
            mxSetField(plhs[3], i, "constrviolation", mxCreateDoubleScalar(out[i].constrviolation));
            mxSetField(plhs[3], i, "firstorderopt", mxCreateDoubleScalar(out[i].firstorderopt));
            mxSetField(plhs[3], i, "algorithm", mxCreateString("bqp-mehrotra-gfx950"));
        }
    }
    if (nlhs > 4) {
        const char* fields[] = {"ineqlin", "eqlin", "lower", "upper"};
        plhs[4] = mxCreateStructMatrix(1, batch, 4, fields);
        for (int i = 0; i < batch; ++i) {
            mxArray* a1 = mxCreateDoubleMatrix(m, 1, mxREAL);
            mxArray* a2 = mxCreateDoubleMatrix(me0, 1, mxREAL);
            mxArray* a3 = mxCreateDoubleMatrix(n, 1, mxREAL);
            mxArray* a4 = mxCreateDoubleMatrix(n, 1, mxREAL);
            if (m) memcpy(mxGetDoubles(a1), lin + (size_t)i * m, sizeof(double) * m);
            if (me0) memcpy(mxGetDoubles(a2), leq + (size_t)i * me, sizeof(double) * me0);
            memcpy(mxGetDoubles(a3), llo + (size_t)i * n, sizeof(double) * n);
            memcpy(mxGetDoubles(a4), lup + (size_t)i * n, sizeof(double) * n);
            for (int r = 0; r < nfix; ++r) {   /* fixed variables: multiplier by sign */
                const double y = leq[(size_t)i * me + me0 + r];
                mxGetDoubles(a4)[fix[r]] = y > 0 ? y : 0.0;
                mxGetDoubles(a3)[fix[r]] = y < 0 ? -y : 0.0;
            }
            mxSetField(plhs[4], i, "ineqlin", a1);
            mxSetField(plhs[4], i, "eqlin", a2);
            mxSetField(plhs[4], i, "lower", a3);
            mxSetField(plhs[4], i, "upper", a4);
        }
    }
}
