/* Functional stand-in for the MEX API subset in mex.h, so that integration/matlab/qsp_nmpc_mex.c
 * runs unmodified outside MATLAB (test infrastructure).  Errors longjmp to the driver's handler. */
#include "mex.h"

#include <setjmp.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

struct mxArray_tag {
    mxClassID cls;
    size_t ndim, dims[3];
    void* data;                  /* numeric / char payload */
    size_t nfields;              /* struct: names + values */
    char** names;
    mxArray** values;
};

jmp_buf stub_err_jmp;
char stub_err_msg[512];

void mexErrMsgIdAndTxt(const char* id, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    int k = snprintf(stub_err_msg, sizeof stub_err_msg, "%s: ", id);
    vsnprintf(stub_err_msg + k, sizeof stub_err_msg - k, fmt, ap);
    va_end(ap);
    longjmp(stub_err_jmp, 1);
}

static size_t numel(const mxArray* a) {
    size_t n = 1;
    for (size_t i = 0; i < a->ndim; ++i) n *= a->dims[i];
    return n;
}
static size_t elsize(mxClassID c) {
    return c == mxDOUBLE_CLASS || c == mxUINT64_CLASS ? 8 : (c == mxINT32_CLASS ? 4 : (c == mxCHAR_CLASS ? 1 : sizeof(mxArray*)));
}
static mxArray* alloc(mxClassID c, size_t ndim, const size_t* dims) {
    mxArray* a = (mxArray*)calloc(1, sizeof(mxArray));
    a->cls = c;
    a->ndim = ndim;
    for (size_t i = 0; i < ndim; ++i) a->dims[i] = dims[i];
    a->data = calloc(numel(a) ? numel(a) : 1, elsize(c));
    return a;
}

int mxGetString(const mxArray* a, char* buf, size_t n) {
    if (!a || a->cls != mxCHAR_CLASS) return 1;
    const size_t len = numel(a);
    if (len + 1 > n) return 1;
    memcpy(buf, a->data, len);
    buf[len] = 0;
    return 0;
}
double mxGetScalar(const mxArray* a) {
    if (a->cls == mxDOUBLE_CLASS) return ((double*)a->data)[0];
    if (a->cls == mxINT32_CLASS) return ((int32_t*)a->data)[0];
    if (a->cls == mxUINT64_CLASS) return (double)((uint64_t*)a->data)[0];
    return 0.0;
}
double* mxGetPr(const mxArray* a) { return (double*)a->data; }
void* mxGetData(const mxArray* a) { return a->data; }
size_t mxGetM(const mxArray* a) { return a->dims[0]; }
size_t mxGetN(const mxArray* a) {
    size_t n = 1;
    for (size_t i = 1; i < a->ndim; ++i) n *= a->dims[i];
    return n;
}
size_t mxGetNumberOfElements(const mxArray* a) { return numel(a); }
bool mxIsDouble(const mxArray* a) { return a->cls == mxDOUBLE_CLASS; }
bool mxIsComplex(const mxArray* a) { (void)a; return false; }
bool mxIsUint64(const mxArray* a) { return a->cls == mxUINT64_CLASS; }
bool mxIsStruct(const mxArray* a) { return a->cls == mxSTRUCT_CLASS; }
bool mxIsCell(const mxArray* a) { return a->cls == mxCELL_CLASS; }
mxArray* mxGetCell(const mxArray* a, size_t i) { return ((mxArray**)a->data)[i]; }
mxArray* mxGetField(const mxArray* a, size_t i, const char* name) {
    (void)i;
    for (size_t k = 0; k < a->nfields; ++k)
        if (!strcmp(a->names[k], name)) return a->values[k];
    return NULL;
}
mxArray* mxCreateDoubleMatrix(size_t m, size_t n, mxComplexity c) {
    (void)c;
    const size_t d[2] = {m, n};
    return alloc(mxDOUBLE_CLASS, 2, d);
}
mxArray* mxCreateNumericMatrix(size_t m, size_t n, mxClassID id, mxComplexity c) {
    (void)c;
    const size_t d[2] = {m, n};
    return alloc(id, 2, d);
}
mxArray* mxCreateNumericArray(size_t ndim, const size_t* dims, mxClassID id, mxComplexity c) {
    (void)c;
    return alloc(id, ndim, dims);
}
void mxDestroyArray(mxArray* a) {
    if (!a) return;
    if (a->cls == mxCELL_CLASS)
        for (size_t i = 0; i < numel(a); ++i) mxDestroyArray(((mxArray**)a->data)[i]);
    for (size_t k = 0; k < a->nfields; ++k) { free(a->names[k]); mxDestroyArray(a->values[k]); }
    free(a->names);
    free(a->values);
    free(a->data);
    free(a);
}
void* mxCalloc(size_t n, size_t sz) { return calloc(n, sz); }
void* mxMalloc(size_t n) { return malloc(n); }
void mxFree(void* p) { free(p); }

mxArray* stub_string(const char* s) {
    const size_t d[2] = {1, strlen(s)};
    mxArray* a = alloc(mxCHAR_CLASS, 2, d);
    memcpy(a->data, s, strlen(s));
    return a;
}
mxArray* stub_scalar(double v) {
    mxArray* a = mxCreateDoubleMatrix(1, 1, mxREAL);
    ((double*)a->data)[0] = v;
    return a;
}
mxArray* stub_cell(size_t m, size_t n) {
    const size_t d[2] = {m, n};
    return alloc(mxCELL_CLASS, 2, d);
}
void stub_cell_set(mxArray* c, size_t i, mxArray* v) { ((mxArray**)c->data)[i] = v; }
mxArray* stub_struct(void) {
    const size_t d[2] = {1, 1};
    return alloc(mxSTRUCT_CLASS, 2, d);
}
void stub_struct_set(mxArray* s, const char* name, mxArray* v) {
    s->names = (char**)realloc(s->names, (s->nfields + 1) * sizeof(char*));
    s->values = (mxArray**)realloc(s->values, (s->nfields + 1) * sizeof(mxArray*));
    s->names[s->nfields] = strdup(name);
    s->values[s->nfields] = v;
    s->nfields++;
}
