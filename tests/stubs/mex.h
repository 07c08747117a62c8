/* Minimal declarations of the MATLAB MEX C API used by integration/matlab/qsp_nmpc_mex.c,
 * for a syntax/type check of the gateway only (MATLAB is not in this image).  Not a MEX
 * implementation; nothing is linked against it. */
#ifndef QSP_TEST_MEX_STUB_H
#define QSP_TEST_MEX_STUB_H
#include <stddef.h>
#include <stdbool.h>
typedef struct mxArray_tag mxArray;
typedef enum { mxUNKNOWN_CLASS, mxDOUBLE_CLASS = 6, mxINT32_CLASS = 12, mxUINT64_CLASS = 15 } mxClassID;
typedef enum { mxREAL, mxCOMPLEX } mxComplexity;
void mexErrMsgIdAndTxt(const char* id, const char* fmt, ...);
int mxGetString(const mxArray* a, char* buf, size_t n);
double mxGetScalar(const mxArray* a);
double* mxGetPr(const mxArray* a);
void* mxGetData(const mxArray* a);
size_t mxGetM(const mxArray* a);
size_t mxGetN(const mxArray* a);
size_t mxGetNumberOfElements(const mxArray* a);
bool mxIsDouble(const mxArray* a);
bool mxIsComplex(const mxArray* a);
bool mxIsUint64(const mxArray* a);
mxArray* mxGetCell(const mxArray* a, size_t i);
mxArray* mxCreateDoubleMatrix(size_t m, size_t n, mxComplexity c);
mxArray* mxCreateNumericMatrix(size_t m, size_t n, mxClassID id, mxComplexity c);
void* mxCalloc(size_t n, size_t sz);
void* mxMalloc(size_t n);
void mxFree(void* p);
void mexFunction(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]);
#endif
