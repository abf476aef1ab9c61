/* mex.h — the subset of MATLAB's MEX / MX C API (R2018a interleaved-complex
 * flavour) that matlab/swrt_mex.cpp uses, declared for a TEST build of the
 * gateway outside MATLAB (the image has no MATLAB).  mex_shim.cpp implements
 * it over a minimal in-memory mxArray and exposes a ctypes entry point, so
 * tests/test_mex_gateway.py drives the real gateway source against libswrt.
 * Semantics follow MathWorks' documentation: column-major arrays, dims[0] =
 * rows, complex data interleaved (re, im), mexErrMsgIdAndTxt does not return. */
#pragma once
#include <stddef.h>
#include <stdbool.h>

typedef size_t mwSize;
typedef size_t mwIndex;
typedef struct mxArray_tag mxArray;
typedef double mxDouble;
typedef struct { double real, imag; } mxComplexDouble;
typedef enum { mxUNKNOWN_CLASS = 0, mxDOUBLE_CLASS = 6 } mxClassID;
typedef enum { mxREAL = 0, mxCOMPLEX = 1 } mxComplexity;

#ifdef __cplusplus
extern "C" {
#endif
double mxGetScalar(const mxArray* a);
bool mxIsDouble(const mxArray* a);
bool mxIsComplex(const mxArray* a);
bool mxIsChar(const mxArray* a);
int mxGetString(const mxArray* a, char* buf, mwSize buflen);
size_t mxGetM(const mxArray* a);
size_t mxGetN(const mxArray* a);
size_t mxGetNumberOfElements(const mxArray* a);
mwSize mxGetNumberOfDimensions(const mxArray* a);
const mwSize* mxGetDimensions(const mxArray* a);
mxDouble* mxGetDoubles(const mxArray* a);
mxComplexDouble* mxGetComplexDoubles(const mxArray* a);
mxArray* mxCreateDoubleMatrix(mwSize m, mwSize n, mxComplexity c);
mxArray* mxCreateNumericArray(mwSize ndim, const mwSize* dims, mxClassID cls, mxComplexity c);
mxArray* mxCreateDoubleScalar(double v);
mxArray* mxDuplicateArray(const mxArray* a);
void mxDestroyArray(mxArray* a);
mxArray* mxGetField(const mxArray* s, mwIndex i, const char* name);
void mexErrMsgIdAndTxt(const char* id, const char* fmt, ...) __attribute__((noreturn));
int mexAtExit(void (*fn)(void));
void mexLock(void);
void mexUnlock(void);
bool mexIsLocked(void);
/* the gateway's entry point: C linkage, found by name when MATLAB loads the MEX file */
void mexFunction(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]);
#ifdef __cplusplus
}
#endif
