// mex_shim.cpp — in-memory implementation of tests/mex_shim/mex.h plus a
// ctypes-callable entry point (shim_call) around the gateway's mexFunction.
// TEST INFRASTRUCTURE ONLY: lets tests/test_mex_gateway.py compile and drive
// matlab/swrt_mex.cpp without MATLAB.  Errors raised by the gateway
// (mexErrMsgIdAndTxt) are C++ exceptions caught in shim_call.
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <map>
#include <stdexcept>
#include <string>
#include <vector>

#include "mex.h"

struct mxArray_tag {
  std::vector<mwSize> dims{0, 0};
  bool is_char = false, is_complex = false, is_struct = false;
  std::vector<double> data;  // n reals, or 2n interleaved (re, im)
  std::string str;
  std::map<std::string, mxArray*> fields;
};

namespace {
struct MexError : std::runtime_error {
  std::string id;
  MexError(const char* i, const std::string& m) : std::runtime_error(m), id(i) {}
};
void (*g_atexit)(void) = nullptr;
bool g_locked = false;
size_t numel(const mxArray* a) {
  size_t n = 1;
  for (mwSize d : a->dims) n *= d;
  return n;
}
mxArray* make(mwSize ndim, const mwSize* dims, bool cplx) {
  auto* a = new mxArray;
  a->dims.assign(dims, dims + ndim);
  while (a->dims.size() < 2) a->dims.push_back(1);
  while (a->dims.size() > 2 && a->dims.back() == 1) a->dims.pop_back();  // MATLAB drops trailing singletons
  a->is_complex = cplx;
  a->data.assign(numel(a) * (cplx ? 2 : 1), 0.0);
  return a;
}
}  // namespace

extern "C" {
double mxGetScalar(const mxArray* a) { return a->data.empty() ? 0.0 : a->data[0]; }
bool mxIsDouble(const mxArray* a) { return !a->is_char && !a->is_struct; }
bool mxIsComplex(const mxArray* a) { return a->is_complex; }
bool mxIsChar(const mxArray* a) { return a->is_char; }
int mxGetString(const mxArray* a, char* buf, mwSize n) {
  if (!a->is_char || n == 0) return 1;
  std::snprintf(buf, n, "%s", a->str.c_str());
  return a->str.size() + 1 > n ? 1 : 0;
}
size_t mxGetM(const mxArray* a) { return a->dims[0]; }
size_t mxGetN(const mxArray* a) { return a->dims[0] ? numel(a) / a->dims[0] : 0; }
size_t mxGetNumberOfElements(const mxArray* a) { return numel(a); }
mwSize mxGetNumberOfDimensions(const mxArray* a) { return a->dims.size(); }
const mwSize* mxGetDimensions(const mxArray* a) { return a->dims.data(); }
mxDouble* mxGetDoubles(const mxArray* a) {
  return (a->is_complex || a->is_char || a->is_struct) ? nullptr : const_cast<double*>(a->data.data());
}
mxComplexDouble* mxGetComplexDoubles(const mxArray* a) {
  return a->is_complex ? reinterpret_cast<mxComplexDouble*>(const_cast<double*>(a->data.data())) : nullptr;
}
mxArray* mxCreateDoubleMatrix(mwSize m, mwSize n, mxComplexity c) {
  const mwSize d[2] = {m, n};
  return make(2, d, c == mxCOMPLEX);
}
mxArray* mxCreateNumericArray(mwSize ndim, const mwSize* dims, mxClassID, mxComplexity c) {
  return make(ndim, dims, c == mxCOMPLEX);
}
mxArray* mxCreateDoubleScalar(double v) {
  mxArray* a = mxCreateDoubleMatrix(1, 1, mxREAL);
  a->data[0] = v;
  return a;
}
mxArray* mxDuplicateArray(const mxArray* a) { return new mxArray(*a); }
void mxDestroyArray(mxArray* a) { delete a; }
mxArray* mxGetField(const mxArray* s, mwIndex, const char* name) {
  auto it = s->fields.find(name);
  return it == s->fields.end() ? nullptr : it->second;
}
void mexErrMsgIdAndTxt(const char* id, const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  std::vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  throw MexError(id, buf);
}
int mexAtExit(void (*fn)(void)) {
  g_atexit = fn;
  return 0;
}
void mexLock(void) { g_locked = true; }
void mexUnlock(void) { g_locked = false; }
bool mexIsLocked(void) { return g_locked; }

// ---- ctypes side -----------------------------------------------------------
void* shim_array(const double* data, int ndim, const size_t* dims, int cplx) {
  mxArray* a = make((mwSize)ndim, dims, cplx != 0);
  if (data) std::memcpy(a->data.data(), data, a->data.size() * sizeof(double));
  return a;
}
void* shim_string(const char* s) {
  auto* a = new mxArray;
  a->is_char = true;
  a->str = s;
  a->dims = {1, a->str.size()};
  return a;
}
void* shim_struct(int nf, const char** names, void** values) {
  auto* a = new mxArray;
  a->is_struct = true;
  a->dims = {1, 1};
  for (int i = 0; i < nf; ++i) a->fields[names[i]] = static_cast<mxArray*>(values[i]);
  return a;
}
void shim_free(void* p) {
  auto* a = static_cast<mxArray*>(p);
  if (!a) return;
  for (auto& kv : a->fields) delete kv.second;
  delete a;
}
int shim_ndim(void* p) { return (int)static_cast<mxArray*>(p)->dims.size(); }
void shim_dims(void* p, size_t* out) {
  const auto& d = static_cast<mxArray*>(p)->dims;
  std::copy(d.begin(), d.end(), out);
}
int shim_is_complex(void* p) { return static_cast<mxArray*>(p)->is_complex ? 1 : 0; }
size_t shim_ndata(void* p) { return static_cast<mxArray*>(p)->data.size(); }
const double* shim_data(void* p) { return static_cast<mxArray*>(p)->data.data(); }
// mexFunction(nlhs, plhs, nrhs, prhs); 0 = ok, 1 = mexErrMsgIdAndTxt (id: msg in err)
int shim_call(int nlhs, void** plhs, int nrhs, void** prhs, char* err, int errlen) {
  for (int i = 0; i < nlhs; ++i) plhs[i] = nullptr;
  try {
    mexFunction(nlhs, reinterpret_cast<mxArray**>(plhs), nrhs, const_cast<const mxArray**>(
                                                                    reinterpret_cast<mxArray**>(prhs)));
  } catch (const MexError& e) {
    std::snprintf(err, (size_t)errlen, "%s: %s", e.id.c_str(), e.what());
    return 1;
  }
  return 0;
}
void shim_at_exit(void) {
  if (g_atexit) g_atexit();
  g_atexit = nullptr;
}
}
