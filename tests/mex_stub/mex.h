/*
 * mex.h — stand-in for MATLAB's MEX API, for the C emulation test of the gateways in
 * learning-based-mpc_amd/matlab/ (tests/test_mex_gateway.py).  Test infrastructure only: it
 * declares the subset of the documented mx / mex interface (R2018a interleaved-complex API) that
 * the gateways use, implemented in mex_stub.c with plain heap arrays; errors raised through
 * mexErrMsgIdAndTxt unwind to mexemu_call (setjmp/longjmp), as MATLAB unwinds to the prompt.
 */
#ifndef BQP_MEX_STUB_H
#define BQP_MEX_STUB_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct mxArray_tag mxArray;
typedef enum { mxREAL = 0 } mxComplexity;

size_t mxGetM(const mxArray* a);
size_t mxGetN(const mxArray* a);
size_t mxGetNumberOfElements(const mxArray* a);
int mxIsEmpty(const mxArray* a);
int mxIsStruct(const mxArray* a);
int mxIsDouble(const mxArray* a);
int mxIsComplex(const mxArray* a);
double* mxGetDoubles(const mxArray* a);
double* mxGetPr(const mxArray* a);
double mxGetScalar(const mxArray* a);
mxArray* mxCreateDoubleMatrix(size_t m, size_t n, mxComplexity c);
mxArray* mxCreateDoubleScalar(double v);
mxArray* mxCreateString(const char* s);
mxArray* mxCreateStructMatrix(size_t m, size_t n, int nfields, const char** names);
void mxSetField(mxArray* s, size_t i, const char* name, mxArray* v);
mxArray* mxGetField(const mxArray* s, size_t i, const char* name);
void mxDestroyArray(mxArray* a);
void* mxCalloc(size_t n, size_t size);
void mxFree(void* p);
void mexErrMsgIdAndTxt(const char* id, const char* fmt, ...) __attribute__((noreturn));
int mexAtExit(void (*f)(void));

void mexFunction(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]);

#ifdef __cplusplus
}
#endif
#endif
