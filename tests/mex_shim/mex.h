/*
 * mex.h — minimal stand-in for MATLAB's MEX / mx-API (test infrastructure only).
 *
 * MATLAB is not installed in this pipeline, so the gateway matlab/vo_mex.c is compiled against
 * this header and mx_shim.c: the subset of the interleaved-complex (-R2018a) C Matrix API the
 * gateway uses, with the same names, class IDs, column-major storage and error behaviour
 * (mexErrMsgIdAndTxt does not return).  The test-only entry points (shim_*) let the Python
 * tests build mxArrays, call mexFunction and read the outputs through ctypes.
 */
#ifndef VO_TEST_MEX_H
#define VO_TEST_MEX_H
#include <stddef.h>
#include <stdbool.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum {
    mxUNKNOWN_CLASS = 0, mxCELL_CLASS, mxSTRUCT_CLASS, mxLOGICAL_CLASS, mxCHAR_CLASS, mxVOID_CLASS,
    mxDOUBLE_CLASS, mxSINGLE_CLASS, mxINT8_CLASS, mxUINT8_CLASS, mxINT16_CLASS, mxUINT16_CLASS,
    mxINT32_CLASS, mxUINT32_CLASS, mxINT64_CLASS, mxUINT64_CLASS, mxFUNCTION_CLASS
} mxClassID;
typedef enum { mxREAL = 0, mxCOMPLEX } mxComplexity;
typedef bool mxLogical;
typedef struct mxArray_tag mxArray;

size_t mxGetM(const mxArray* a);
size_t mxGetN(const mxArray* a);
size_t mxGetNumberOfDimensions(const mxArray* a);
mxClassID mxGetClassID(const mxArray* a);
bool mxIsComplex(const mxArray* a);
bool mxIsChar(const mxArray* a);
bool mxIsSingle(const mxArray* a);
bool mxIsDouble(const mxArray* a);
int mxGetString(const mxArray* a, char* buf, size_t buflen);
mxArray* mxCreateNumericMatrix(size_t m, size_t n, mxClassID cls, mxComplexity flag);
mxArray* mxCreateDoubleMatrix(size_t m, size_t n, mxComplexity flag);
mxArray* mxCreateLogicalMatrix(size_t m, size_t n);
mxArray* mxCreateDoubleScalar(double v);
void mxDestroyArray(mxArray* a);
double* mxGetDoubles(const mxArray* a);
float* mxGetSingles(const mxArray* a);
uint8_t* mxGetUint8s(const mxArray* a);
int32_t* mxGetInt32s(const mxArray* a);
uint32_t* mxGetUint32s(const mxArray* a);
mxLogical* mxGetLogicals(const mxArray* a);
void* mxMalloc(size_t n);
void mxFree(void* p);
void mexErrMsgIdAndTxt(const char* id, const char* fmt, ...);
int mexAtExit(void (*fn)(void));

void mexFunction(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]);

#ifdef __cplusplus
}
#endif
#endif
