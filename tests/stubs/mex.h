/* The subset of the MATLAB MEX C API that integration/matlab/qsp_nmpc_mex.c uses, with a
 * functional implementation in mex_stub.c (MATLAB is not in this image): the gateway is
 * compiled as is and driven by mex_driver.c (tests/test_gpu_mex.py). */
#ifndef QSP_TEST_MEX_STUB_H
#define QSP_TEST_MEX_STUB_H
#include <stddef.h>
#include <stdbool.h>
typedef struct mxArray_tag mxArray;
typedef enum { mxUNKNOWN_CLASS, mxCELL_CLASS = 1, mxSTRUCT_CLASS = 2, mxCHAR_CLASS = 4, mxDOUBLE_CLASS = 6,
               mxINT32_CLASS = 12, mxUINT64_CLASS = 15 } mxClassID;
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
bool mxIsStruct(const mxArray* a);
bool mxIsCell(const mxArray* a);
mxArray* mxGetCell(const mxArray* a, size_t i);
mxArray* mxGetField(const mxArray* a, size_t i, const char* name);
mxArray* mxCreateDoubleMatrix(size_t m, size_t n, mxComplexity c);
mxArray* mxCreateNumericMatrix(size_t m, size_t n, mxClassID id, mxComplexity c);
mxArray* mxCreateNumericArray(size_t ndim, const size_t* dims, mxClassID id, mxComplexity c);
void mxDestroyArray(mxArray* a);
void* mxCalloc(size_t n, size_t sz);
void* mxMalloc(size_t n);
void mxFree(void* p);
void mexFunction(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]);
/* test-side constructors (not MATLAB API) */
mxArray* stub_string(const char* s);
mxArray* stub_scalar(double v);
mxArray* stub_cell(size_t m, size_t n);            /* then stub_cell_set */
void stub_cell_set(mxArray* c, size_t i, mxArray* v);
mxArray* stub_struct(void);                         /* then stub_struct_set */
void stub_struct_set(mxArray* s, const char* name, mxArray* v);
#endif
