/*
 * mex_stub.c — heap-array implementation of the mx / mex subset declared in mex.h, linked with
 * one MEX gateway into a test library (libmexemu_<name>.so).  Python drives it through ctypes:
 * build mxArrays with mxCreateDoubleMatrix / mxCreateStructMatrix / mxSetField, call
 * mexemu_call (which runs mexFunction under setjmp and reports an error's id and message), read
 * the outputs with mxGetDoubles / mxGetField, release with mxDestroyArray.  mxCalloc blocks live
 * until the call returns, as in MATLAB.  Test infrastructure only.
 */
#define _POSIX_C_SOURCE 200809L
#include <setjmp.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "mex.h"

struct mxArray_tag {
    int kind;             /* 0 double, 1 struct, 2 char */
    size_t m, n;
    double* pr;           /* double data (m*n) */
    int nf;               /* struct: fields, m*n elements of nf slots each */
    char** names;
    mxArray** slots;
    char* str;
};

static jmp_buf g_jmp;
static int g_in_call = 0;
static char g_errid[128], g_errmsg[512];
static void** g_blocks = NULL;
static size_t g_nblocks = 0, g_capblocks = 0;
static void (*g_atexit)(void) = NULL;

size_t mxGetM(const mxArray* a) { return a ? a->m : 0; }
size_t mxGetN(const mxArray* a) { return a ? a->n : 0; }
size_t mxGetNumberOfElements(const mxArray* a) { return a ? a->m * a->n : 0; }
int mxIsEmpty(const mxArray* a) { return !a || a->m * a->n == 0; }
int mxIsStruct(const mxArray* a) { return a && a->kind == 1; }
int mxIsDouble(const mxArray* a) { return a && a->kind == 0; }
int mxIsComplex(const mxArray* a) { (void)a; return 0; }
double* mxGetDoubles(const mxArray* a) { return (a && a->kind == 0) ? a->pr : NULL; }
double* mxGetPr(const mxArray* a) { return mxGetDoubles(a); }
double mxGetScalar(const mxArray* a) { return (a && a->kind == 0 && a->m * a->n > 0) ? a->pr[0] : 0.0; }

mxArray* mxCreateDoubleMatrix(size_t m, size_t n, mxComplexity c) {
    (void)c;
    mxArray* a = (mxArray*)calloc(1, sizeof(mxArray));
    a->kind = 0; a->m = m; a->n = n;
    a->pr = (double*)calloc(m * n + 1, sizeof(double));
    return a;
}

mxArray* mxCreateDoubleScalar(double v) {
    mxArray* a = mxCreateDoubleMatrix(1, 1, mxREAL);
    a->pr[0] = v;
    return a;
}

mxArray* mxCreateString(const char* s) {
    mxArray* a = (mxArray*)calloc(1, sizeof(mxArray));
    a->kind = 2; a->m = 1; a->n = strlen(s);
    a->str = strdup(s);
    return a;
}

mxArray* mxCreateStructMatrix(size_t m, size_t n, int nfields, const char** names) {
    mxArray* a = (mxArray*)calloc(1, sizeof(mxArray));
    a->kind = 1; a->m = m; a->n = n; a->nf = nfields;
    a->names = (char**)calloc(nfields, sizeof(char*));
    for (int i = 0; i < nfields; ++i) a->names[i] = strdup(names[i]);
    a->slots = (mxArray**)calloc(m * n * nfields + 1, sizeof(mxArray*));
    return a;
}

static int field_index(const mxArray* s, const char* name) {
    if (!s || s->kind != 1) return -1;
    for (int i = 0; i < s->nf; ++i)
        if (strcmp(s->names[i], name) == 0) return i;
    return -1;
}

void mxSetField(mxArray* s, size_t i, const char* name, mxArray* v) {
    const int f = field_index(s, name);
    if (f < 0 || i >= s->m * s->n) return;
    mxArray** slot = &s->slots[i * s->nf + f];
    if (*slot) mxDestroyArray(*slot);
    *slot = v;
}

mxArray* mxGetField(const mxArray* s, size_t i, const char* name) {
    const int f = field_index(s, name);
    if (f < 0 || i >= s->m * s->n) return NULL;
    return s->slots[i * s->nf + f];
}

void mxDestroyArray(mxArray* a) {
    if (!a) return;
    if (a->kind == 1) {
        for (size_t i = 0; i < a->m * a->n * (size_t)a->nf; ++i) mxDestroyArray(a->slots[i]);
        for (int i = 0; i < a->nf; ++i) free(a->names[i]);
        free(a->names);
        free(a->slots);
    }
    free(a->pr);
    free(a->str);
    free(a);
}

void* mxCalloc(size_t n, size_t size) {
    void* p = calloc(n ? n : 1, size ? size : 1);
    if (g_nblocks == g_capblocks) {
        g_capblocks = g_capblocks ? 2 * g_capblocks : 64;
        g_blocks = (void**)realloc(g_blocks, g_capblocks * sizeof(void*));
    }
    g_blocks[g_nblocks++] = p;
    return p;
}

void mxFree(void* p) {
    for (size_t i = 0; i < g_nblocks; ++i)
        if (g_blocks[i] == p) { g_blocks[i] = NULL; break; }
    free(p);
}

void mexErrMsgIdAndTxt(const char* id, const char* fmt, ...) {
    snprintf(g_errid, sizeof(g_errid), "%s", id);
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_errmsg, sizeof(g_errmsg), fmt, ap);
    va_end(ap);
    if (g_in_call) longjmp(g_jmp, 1);
    fprintf(stderr, "%s: %s\n", g_errid, g_errmsg);
    abort();
}

int mexAtExit(void (*f)(void)) {
    g_atexit = f;
    return 0;
}

/* ---- driver entry points (ctypes) ---- */

/* runs mexFunction; returns 0, or 1 with the error id / message copied out */
int mexemu_call(int nlhs, mxArray** plhs, int nrhs, const mxArray** prhs, char* errid,
                char* errmsg) {
    for (int i = 0; i < nlhs; ++i) plhs[i] = NULL;
    int rc = 0;
    g_in_call = 1;
    if (setjmp(g_jmp) == 0) {
        mexFunction(nlhs, plhs, nrhs, prhs);
    } else {
        rc = 1;
        if (errid) strcpy(errid, g_errid);
        if (errmsg) strcpy(errmsg, g_errmsg);
    }
    g_in_call = 0;
    for (size_t i = 0; i < g_nblocks; ++i) free(g_blocks[i]);
    g_nblocks = 0;
    return rc;
}

/* what `clear mex` does: run the gateway's mexAtExit hook */
void mexemu_clear(void) {
    if (g_atexit) g_atexit();
    g_atexit = NULL;
}

/* struct inspection for the driver (MATLAB's mxGetNumberOfFields / mxGetFieldNameByNumber) */
int mexemu_nfields(const mxArray* s) { return (s && s->kind == 1) ? s->nf : 0; }
const char* mexemu_field_name(const mxArray* s, int i) {
    return (s && s->kind == 1 && i >= 0 && i < s->nf) ? s->names[i] : NULL;
}
int mexemu_is_char(const mxArray* a) { return a && a->kind == 2; }
