/* mx_shim.c — the mx-API subset of mex.h over plain heap arrays (test infrastructure only).
 * Arrays are column-major like MATLAB's.  mexErrMsgIdAndTxt longjmps back into shim_call, which
 * frees every mxMalloc block and output array of the failed call (MATLAB does the same). */
#include "mex.h"
#include <setjmp.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

struct mxArray_tag { mxClassID cls; size_t m, n; void* data; };

static size_t elem_size(mxClassID c)
{
    switch (c) {
    case mxDOUBLE_CLASS: case mxINT64_CLASS: case mxUINT64_CLASS: return 8;
    case mxSINGLE_CLASS: case mxINT32_CLASS: case mxUINT32_CLASS: return 4;
    case mxINT16_CLASS: case mxUINT16_CLASS: case mxCHAR_CLASS: return 2;
    default: return 1;
    }
}

/* allocations of the call in progress (released on error): mxMalloc blocks and arrays */
#define MAXBLK 4096
static void* g_blk[MAXBLK];
static int g_kind[MAXBLK];                  /* 0 = mxMalloc block, 1 = mxArray */
static int g_nblk = 0;
static jmp_buf g_jmp;
static int g_in_call = 0;
static char g_err_id[128], g_err_msg[512];
static void (*g_atexit)(void) = NULL;

static void track(void* p, int kind)
{
    if (g_in_call && p && g_nblk < MAXBLK) { g_kind[g_nblk] = kind; g_blk[g_nblk++] = p; }
}
static void untrack(void* p)
{
    for (int i = 0; i < g_nblk; ++i)
        if (g_blk[i] == p) { --g_nblk; g_blk[i] = g_blk[g_nblk]; g_kind[i] = g_kind[g_nblk]; return; }
}

size_t mxGetM(const mxArray* a) { return a->m; }
size_t mxGetN(const mxArray* a) { return a->n; }
size_t mxGetNumberOfDimensions(const mxArray* a) { (void)a; return 2; }
mxClassID mxGetClassID(const mxArray* a) { return a->cls; }
bool mxIsComplex(const mxArray* a) { (void)a; return false; }
bool mxIsChar(const mxArray* a) { return a->cls == mxCHAR_CLASS; }
bool mxIsSingle(const mxArray* a) { return a->cls == mxSINGLE_CLASS; }
bool mxIsDouble(const mxArray* a) { return a->cls == mxDOUBLE_CLASS; }

int mxGetString(const mxArray* a, char* buf, size_t buflen)
{
    if (a->cls != mxCHAR_CLASS || buflen == 0) return 1;
    const size_t len = a->m * a->n;
    const uint16_t* s = (const uint16_t*)a->data;       /* mxChar is 16-bit */
    size_t k = 0;
    for (; k < len && k + 1 < buflen; ++k) buf[k] = (char)s[k];
    buf[k] = 0;
    return k < len ? 1 : 0;
}

static mxArray* create(size_t m, size_t n, mxClassID cls)
{
    mxArray* a = (mxArray*)calloc(1, sizeof(mxArray));
    a->cls = cls; a->m = m; a->n = n;
    a->data = calloc(m * n + 1, elem_size(cls));
    return a;
}
mxArray* mxCreateNumericMatrix(size_t m, size_t n, mxClassID cls, mxComplexity flag) { (void)flag; mxArray* a = create(m, n, cls); track(a, 1); return a; }
mxArray* mxCreateDoubleMatrix(size_t m, size_t n, mxComplexity flag) { return mxCreateNumericMatrix(m, n, mxDOUBLE_CLASS, flag); }
mxArray* mxCreateLogicalMatrix(size_t m, size_t n) { return mxCreateNumericMatrix(m, n, mxLOGICAL_CLASS, mxREAL); }
mxArray* mxCreateDoubleScalar(double v) { mxArray* a = mxCreateDoubleMatrix(1, 1, mxREAL); ((double*)a->data)[0] = v; return a; }
void mxDestroyArray(mxArray* a) { if (a) { free(a->data); free(a); } }

#define GETTER(name, type, CL) type* name(const mxArray* a) { return a->cls == (CL) ? (type*)a->data : NULL; }
GETTER(mxGetDoubles, double, mxDOUBLE_CLASS)
GETTER(mxGetSingles, float, mxSINGLE_CLASS)
GETTER(mxGetUint8s, uint8_t, mxUINT8_CLASS)
GETTER(mxGetInt32s, int32_t, mxINT32_CLASS)
GETTER(mxGetUint32s, uint32_t, mxUINT32_CLASS)
GETTER(mxGetLogicals, mxLogical, mxLOGICAL_CLASS)

void* mxMalloc(size_t n) { void* p = malloc(n ? n : 1); track(p, 0); return p; }
void mxFree(void* p) { untrack(p); free(p); }

void mexErrMsgIdAndTxt(const char* id, const char* fmt, ...)
{
    va_list ap;
    va_start(ap, fmt);
    snprintf(g_err_id, sizeof g_err_id, "%s", id);
    vsnprintf(g_err_msg, sizeof g_err_msg, fmt, ap);
    va_end(ap);
    if (g_in_call) longjmp(g_jmp, 1);
    fprintf(stderr, "mexErrMsgIdAndTxt outside a call: %s: %s\n", g_err_id, g_err_msg);
    abort();
}

int mexAtExit(void (*fn)(void)) { g_atexit = fn; return 0; }

/* ---- test-only entry points ---- */
mxArray* shim_create(int cls, size_t m, size_t n, const void* data)
{
    mxArray* a = create(m, n, (mxClassID)cls);
    if (data) memcpy(a->data, data, m * n * elem_size((mxClassID)cls));
    return a;
}
mxArray* shim_string(const char* s)
{
    const size_t len = strlen(s);
    mxArray* a = create(1, len, mxCHAR_CLASS);
    for (size_t k = 0; k < len; ++k) ((uint16_t*)a->data)[k] = (uint8_t)s[k];
    return a;
}
int shim_class(const mxArray* a) { return (int)a->cls; }
size_t shim_m(const mxArray* a) { return a->m; }
size_t shim_n(const mxArray* a) { return a->n; }
void* shim_data(const mxArray* a) { return a->data; }
void shim_destroy(mxArray* a) { mxDestroyArray(a); }
const char* shim_err_id(void) { return g_err_id; }
const char* shim_err_msg(void) { return g_err_msg; }

/* Call the gateway like MATLAB does: 0 = ok, 1 = mexErrMsgIdAndTxt was raised (outputs and
 * mxMalloc blocks of the call freed, plhs cleared).  Blocks still allocated after a
 * successful call are a gateway leak: the count is returned through *leaked. */
int shim_call(int nlhs, mxArray** plhs, int nrhs, const mxArray** prhs, int* leaked)
{
    g_nblk = 0;
    g_err_id[0] = g_err_msg[0] = 0;
    for (int k = 0; k < nlhs; ++k) plhs[k] = NULL;
    g_in_call = 1;
    if (setjmp(g_jmp)) {
        g_in_call = 0;
        for (int k = 0; k < nlhs; ++k) plhs[k] = NULL;
        for (int i = 0; i < g_nblk; ++i) {
            if (g_kind[i]) mxDestroyArray((mxArray*)g_blk[i]);
            else free(g_blk[i]);
        }
        g_nblk = 0;
        return 1;
    }
    mexFunction(nlhs, plhs, nrhs, prhs);
    g_in_call = 0;
    for (int k = 0; k < nlhs; ++k) untrack(plhs[k]);
    if (leaked) *leaked = g_nblk;
    g_nblk = 0;
    return 0;
}

void shim_at_exit(void) { if (g_atexit) { g_atexit(); g_atexit = NULL; } }
