// flexflow_amd C API: an embedded CPython runtime forwarding every call to flexflow_amd.capi_impl
// (reference src/c/flexflow_c.cc wraps the C++ FFModel; here the FFModel is the Python package,
// whose compute path is the HIP kernel library and RCCL, so C callers get the same runtime).
//
// Handles own one reference to the wrapped Python object; *_destroy drops it. All entry points
// take the GIL (PyGILState_Ensure), so the API may be called from any host thread.
#include "flexflow_c.h"

#include <Python.h>

#include <cstdarg>
#include <cstdio>
#include <mutex>
#include <string>

namespace {

std::once_flag g_init;
PyObject* g_impl = nullptr;
thread_local std::string g_err;

struct Gil {
  PyGILState_STATE s;
  Gil() : s(PyGILState_Ensure()) {}
  ~Gil() { PyGILState_Release(s); }
};

void record_error() {
  PyObject *t, *v, *tb;
  PyErr_Fetch(&t, &v, &tb);
  PyErr_NormalizeException(&t, &v, &tb);
  g_err = "unknown error";
  if (v) {
    PyObject* s = PyObject_Str(v);
    if (s) {
      const char* u = PyUnicode_AsUTF8(s);  // NULL when the message cannot be encoded
      if (u) g_err = u;
      else PyErr_Clear();
      Py_DECREF(s);
    } else {
      PyErr_Clear();
    }
  }
  std::fprintf(stderr, "[flexflow_c] %s\n", g_err.c_str());
  Py_XDECREF(t);
  Py_XDECREF(v);
  Py_XDECREF(tb);
}

void init_once() {
  std::call_once(g_init, [] {
    if (!Py_IsInitialized()) {
      Py_InitializeEx(0);
      PyEval_SaveThread();  // release the GIL taken by initialisation; entry points re-acquire it
    }
    Gil gil;
    g_impl = PyImport_ImportModule("flexflow_amd.capi_impl");
    if (!g_impl) record_error();
  });
}

// call flexflow_amd.capi_impl.<fn>(*args) with a Py_BuildValue format; returns a new reference
PyObject* callv(const char* fn, const char* fmt, va_list ap) {
  if (!g_impl) return nullptr;
  PyObject* f = PyObject_GetAttrString(g_impl, fn);
  if (!f) {
    record_error();
    return nullptr;
  }
  PyObject* args = Py_VaBuildValue(fmt, ap);
  if (args && !PyTuple_Check(args)) {
    PyObject* t = PyTuple_Pack(1, args);
    Py_DECREF(args);
    args = t;
  }
  PyObject* r = args ? PyObject_CallObject(f, args) : nullptr;
  Py_XDECREF(args);
  Py_DECREF(f);
  if (!r) record_error();
  return r;
}

PyObject* call(const char* fn, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  PyObject* r = callv(fn, fmt, ap);
  va_end(ap);
  return r;
}

template <typename H>
H wrap(PyObject* o) {
  H h;
  h.impl = o;  // owns the reference
  return h;
}

PyObject* obj(const void* impl) { return impl ? (PyObject*)impl : Py_None; }

PyObject* int_list(const int* v, int n) {
  PyObject* l = PyList_New(n);
  for (int i = 0; i < n; ++i) PyList_SET_ITEM(l, i, PyLong_FromLong(v[i]));
  return l;
}

void drop(void* impl) {
  if (!impl) return;
  init_once();
  Gil gil;
  Py_DECREF((PyObject*)impl);
}

bool as_bool_ok(PyObject* r) {
  if (!r) return false;
  Py_DECREF(r);
  return true;
}

flexflow_tensor_t unary(flexflow_model_t m, const char* op, flexflow_tensor_t x, const char* name) {
  init_once();
  Gil gil;
  return wrap<flexflow_tensor_t>(call("add_unary", "(OsOz)", obj(m.impl), op, obj(x.impl), name));
}

flexflow_tensor_t binary(flexflow_model_t m, const char* op, flexflow_tensor_t a, flexflow_tensor_t b,
                         const char* name) {
  init_once();
  Gil gil;
  return wrap<flexflow_tensor_t>(call("add_binary", "(OsOOz)", obj(m.impl), op, obj(a.impl), obj(b.impl), name));
}

flexflow_tensor_t scalar(flexflow_model_t m, const char* op, flexflow_tensor_t x, float s, const char* name) {
  init_once();
  Gil gil;
  return wrap<flexflow_tensor_t>(call("add_scalar", "(OsOdz)", obj(m.impl), op, obj(x.impl), (double)s, name));
}

int config_int(flexflow_config_t h, const char* key) {
  init_once();
  Gil gil;
  PyObject* r = call("config_get", "(Os)", obj(h.impl), key);
  if (!r) return -1;
  const int v = (int)PyLong_AsLong(r);
  Py_DECREF(r);
  return v;
}

void model_call(flexflow_model_t h, const char* method) {
  init_once();
  Gil gil;
  as_bool_ok(call("model_call", "(Os)", obj(h.impl), method));
}

}  // namespace

extern "C" {

int flexflow_initialize(void) {
  init_once();
  return g_impl ? 0 : -1;
}
const char* flexflow_last_error(void) { return g_err.c_str(); }

// ------------------------------------------------------------------------------------ config
flexflow_config_t flexflow_config_create(void) {
  init_once();
  Gil gil;
  return wrap<flexflow_config_t>(call("config_create", "()"));
}
void flexflow_config_destroy(flexflow_config_t h) { drop(h.impl); }
void flexflow_config_parse_args(flexflow_config_t h, char** argv, int argc) {
  init_once();
  Gil gil;
  PyObject* l = PyList_New(argc);
  for (int i = 0; i < argc; ++i) PyList_SET_ITEM(l, i, PyUnicode_FromString(argv[i]));
  as_bool_ok(call("config_parse_args", "(ON)", obj(h.impl), l));
}
int flexflow_config_get_batch_size(flexflow_config_t h) { return config_int(h, "batch_size"); }
void flexflow_config_set_batch_size(flexflow_config_t h, int b) {
  init_once();
  Gil gil;
  as_bool_ok(call("config_set_batch_size", "(Oi)", obj(h.impl), b));
}
int flexflow_config_get_workers_per_node(flexflow_config_t h) { return config_int(h, "workers_per_node"); }
int flexflow_config_get_num_nodes(flexflow_config_t h) { return config_int(h, "num_nodes"); }
int flexflow_config_get_epochs(flexflow_config_t h) { return config_int(h, "epochs"); }

// ------------------------------------------------------------------------------------- model
flexflow_model_t flexflow_model_create(flexflow_config_t config) {
  init_once();
  Gil gil;
  return wrap<flexflow_model_t>(call("model_create", "(O)", obj(config.impl)));
}
void flexflow_model_destroy(flexflow_model_t h) { drop(h.impl); }
void flexflow_model_compile(flexflow_model_t h, int loss_type, const int* metrics, int nb_metrics, int comp_mode) {
  init_once();
  Gil gil;
  as_bool_ok(call("model_compile", "(OiNi)", obj(h.impl), loss_type, int_list(metrics, nb_metrics), comp_mode));
}
void flexflow_model_forward(flexflow_model_t h, int) { model_call(h, "forward"); }
void flexflow_model_backward(flexflow_model_t h, int) { model_call(h, "backward"); }
void flexflow_model_update(flexflow_model_t h) { model_call(h, "update"); }
void flexflow_model_zero_gradients(flexflow_model_t h) { model_call(h, "zero_gradients"); }
void flexflow_model_reset_metrics(flexflow_model_t h) { model_call(h, "reset_metrics"); }
void flexflow_model_compute_metrics(flexflow_model_t h) { model_call(h, "compute_metrics"); }
void flexflow_model_init_layers(flexflow_model_t h) { model_call(h, "init_layers"); }
void flexflow_model_train_step(flexflow_model_t h) { model_call(h, "train_step"); }
flexflow_tensor_t flexflow_model_get_label_tensor(flexflow_model_t h) {
  init_once();
  Gil gil;
  return wrap<flexflow_tensor_t>(call("model_label_tensor", "(O)", obj(h.impl)));
}
static float perf(flexflow_model_t h, int what) {
  init_once();
  Gil gil;
  PyObject* r = call("model_perf", "(Oi)", obj(h.impl), what);
  if (!r) return -1.f;
  const float v = (float)PyFloat_AsDouble(r);
  Py_DECREF(r);
  return v;
}
float flexflow_model_get_accuracy(flexflow_model_t h) { return perf(h, 0); }
float flexflow_model_get_loss(flexflow_model_t h) { return perf(h, 1); }

// -------------------------------------------------------------------------------- optimizers
flexflow_optimizer_t flexflow_sgd_optimizer_create(flexflow_model_t m, double lr, double momentum, bool nesterov,
                                                   double wd) {
  init_once();
  Gil gil;
  return wrap<flexflow_optimizer_t>(call("sgd_create", "(Oddid)", obj(m.impl), lr, momentum, (int)nesterov, wd));
}
flexflow_optimizer_t flexflow_adam_optimizer_create(flexflow_model_t m, double alpha, double b1, double b2, double wd,
                                                    double eps) {
  init_once();
  Gil gil;
  return wrap<flexflow_optimizer_t>(call("adam_create", "(Oddddd)", obj(m.impl), alpha, b1, b2, wd, eps));
}
void flexflow_optimizer_destroy(flexflow_optimizer_t h) { drop(h.impl); }
void flexflow_model_set_optimizer(flexflow_model_t m, flexflow_optimizer_t o) {
  init_once();
  Gil gil;
  as_bool_ok(call("model_set_optimizer", "(OO)", obj(m.impl), obj(o.impl)));
}
void flexflow_optimizer_set_lr(flexflow_optimizer_t h, double lr) {
  init_once();
  Gil gil;
  as_bool_ok(call("optimizer_set_lr", "(Od)", obj(h.impl), lr));
}

// ----------------------------------------------------------------------------------- tensors
flexflow_tensor_t flexflow_tensor_create(flexflow_model_t m, int num_dims, const int* dims, int data_type,
                                         bool create_grad) {
  init_once();
  Gil gil;
  return wrap<flexflow_tensor_t>(
      call("tensor_create", "(ONii)", obj(m.impl), int_list(dims, num_dims), data_type, (int)create_grad));
}
void flexflow_tensor_destroy(flexflow_tensor_t h) { drop(h.impl); }
int flexflow_tensor_get_num_dims(flexflow_tensor_t h) {
  init_once();
  Gil gil;
  PyObject* r = call("tensor_dims", "(O)", obj(h.impl));
  if (!r) return -1;
  const int n = (int)PyList_Size(r);
  Py_DECREF(r);
  return n;
}
int flexflow_tensor_get_dims(flexflow_tensor_t h, int* dims) {
  init_once();
  Gil gil;
  PyObject* r = call("tensor_dims", "(O)", obj(h.impl));
  if (!r) return -1;
  const int n = (int)PyList_Size(r);
  for (int i = 0; i < n; ++i) dims[i] = (int)PyLong_AsLong(PyList_GetItem(r, i));
  Py_DECREF(r);
  return n;
}
static bool set_data(flexflow_tensor_t h, flexflow_model_t m, const void* p, int64_t n, int dtype) {
  init_once();
  Gil gil;
  return as_bool_ok(call("tensor_set_data", "(OOKLi)", obj(m.impl), obj(h.impl), (unsigned long long)(uintptr_t)p,
                         (long long)n, dtype));
}
bool flexflow_tensor_set_data_float(flexflow_tensor_t h, flexflow_model_t m, const float* d, int64_t n) {
  return set_data(h, m, d, n, 44 /* DT_FLOAT */);
}
bool flexflow_tensor_set_data_int(flexflow_tensor_t h, flexflow_model_t m, const int32_t* d, int64_t n) {
  return set_data(h, m, d, n, 41 /* DT_INT32 */);
}
bool flexflow_tensor_get_data_float(flexflow_tensor_t h, flexflow_model_t m, float* d, int64_t n) {
  init_once();
  Gil gil;
  return as_bool_ok(call("tensor_get_data", "(OOKL)", obj(m.impl), obj(h.impl), (unsigned long long)(uintptr_t)d,
                         (long long)n));
}

// ------------------------------------------------------------------------------------ layers
flexflow_tensor_t flexflow_model_add_dense(flexflow_model_t m, flexflow_tensor_t x, int out_dim, int act,
                                           bool use_bias, const char* name) {
  init_once();
  Gil gil;
  return wrap<flexflow_tensor_t>(
      call("add_dense", "(OOiiiz)", obj(m.impl), obj(x.impl), out_dim, act, (int)use_bias, name));
}
flexflow_tensor_t flexflow_model_add_conv2d(flexflow_model_t m, flexflow_tensor_t x, int oc, int kh, int kw, int sh,
                                            int sw, int ph, int pw, int act, int groups, bool use_bias,
                                            const char* name) {
  init_once();
  Gil gil;
  return wrap<flexflow_tensor_t>(call("add_conv2d", "(OOiiiiiiiiiiz)", obj(m.impl), obj(x.impl), oc, kh, kw, sh, sw,
                                      ph, pw, act, groups, (int)use_bias, name));
}
flexflow_tensor_t flexflow_model_add_pool2d(flexflow_model_t m, flexflow_tensor_t x, int kh, int kw, int sh, int sw,
                                            int ph, int pw, int pool_type, int act, const char* name) {
  init_once();
  Gil gil;
  return wrap<flexflow_tensor_t>(call("add_pool2d", "(OOiiiiiiiiz)", obj(m.impl), obj(x.impl), kh, kw, sh, sw, ph,
                                      pw, pool_type, act, name));
}
flexflow_tensor_t flexflow_model_add_batch_norm(flexflow_model_t m, flexflow_tensor_t x, bool relu, const char* name) {
  init_once();
  Gil gil;
  return wrap<flexflow_tensor_t>(call("add_batch_norm", "(OOiz)", obj(m.impl), obj(x.impl), (int)relu, name));
}
flexflow_tensor_t flexflow_model_add_layer_norm(flexflow_model_t m, flexflow_tensor_t x, int n_axes, const int* axes,
                                                bool affine, float eps, const char* name) {
  init_once();
  Gil gil;
  return wrap<flexflow_tensor_t>(call("add_layer_norm", "(OONidz)", obj(m.impl), obj(x.impl),
                                      int_list(axes, n_axes), (int)affine, (double)eps, name));
}
flexflow_tensor_t flexflow_model_add_embedding(flexflow_model_t m, flexflow_tensor_t x, int num, int dim, int aggr,
                                               const char* name) {
  init_once();
  Gil gil;
  return wrap<flexflow_tensor_t>(call("add_embedding", "(OOiiiz)", obj(m.impl), obj(x.impl), num, dim, aggr, name));
}
flexflow_tensor_t flexflow_model_add_multihead_attention(flexflow_model_t m, flexflow_tensor_t q, flexflow_tensor_t k,
                                                         flexflow_tensor_t v, int embed, int heads, int kdim, int vdim,
                                                         float dropout, bool bias, const char* name) {
  init_once();
  Gil gil;
  return wrap<flexflow_tensor_t>(call("add_mha", "(OOOOiiiidiz)", obj(m.impl), obj(q.impl), obj(k.impl),
                                      obj(v.impl), embed, heads, kdim, vdim, (double)dropout, (int)bias, name));
}
flexflow_tensor_t flexflow_model_add_flat(flexflow_model_t m, flexflow_tensor_t x, const char* n) {
  return unary(m, "flat", x, n);
}
flexflow_tensor_t flexflow_model_add_softmax(flexflow_model_t m, flexflow_tensor_t x, int axis, const char* name) {
  init_once();
  Gil gil;
  return wrap<flexflow_tensor_t>(call("add_softmax", "(OOiz)", obj(m.impl), obj(x.impl), axis, name));
}
flexflow_tensor_t flexflow_model_add_relu(flexflow_model_t m, flexflow_tensor_t x, const char* n) { return unary(m, "relu", x, n); }
flexflow_tensor_t flexflow_model_add_gelu(flexflow_model_t m, flexflow_tensor_t x, const char* n) { return unary(m, "gelu", x, n); }
flexflow_tensor_t flexflow_model_add_sigmoid(flexflow_model_t m, flexflow_tensor_t x, const char* n) { return unary(m, "sigmoid", x, n); }
flexflow_tensor_t flexflow_model_add_tanh(flexflow_model_t m, flexflow_tensor_t x, const char* n) { return unary(m, "tanh", x, n); }
flexflow_tensor_t flexflow_model_add_elu(flexflow_model_t m, flexflow_tensor_t x, const char* n) { return unary(m, "elu", x, n); }
flexflow_tensor_t flexflow_model_add_identity(flexflow_model_t m, flexflow_tensor_t x, const char* n) { return unary(m, "identity", x, n); }
flexflow_tensor_t flexflow_model_add_exp(flexflow_model_t m, flexflow_tensor_t x, const char* n) { return unary(m, "exp", x, n); }
flexflow_tensor_t flexflow_model_add_sin(flexflow_model_t m, flexflow_tensor_t x, const char* n) { return unary(m, "sin", x, n); }
flexflow_tensor_t flexflow_model_add_cos(flexflow_model_t m, flexflow_tensor_t x, const char* n) { return unary(m, "cos", x, n); }
flexflow_tensor_t flexflow_model_add_rsqrt(flexflow_model_t m, flexflow_tensor_t x, const char* n) { return unary(m, "rsqrt", x, n); }
flexflow_tensor_t flexflow_model_add_scalar_multiply(flexflow_model_t m, flexflow_tensor_t x, float s, const char* n) {
  return scalar(m, "scalar_multiply", x, s, n);
}
flexflow_tensor_t flexflow_model_add_scalar_add(flexflow_model_t m, flexflow_tensor_t x, float s, const char* n) {
  return scalar(m, "scalar_add", x, s, n);
}
flexflow_tensor_t flexflow_model_add_pow(flexflow_model_t m, flexflow_tensor_t x, float e, const char* n) {
  return scalar(m, "pow", x, e, n);
}
flexflow_tensor_t flexflow_model_add_add(flexflow_model_t m, flexflow_tensor_t a, flexflow_tensor_t b, const char* n) {
  return binary(m, "add", a, b, n);
}
flexflow_tensor_t flexflow_model_add_subtract(flexflow_model_t m, flexflow_tensor_t a, flexflow_tensor_t b, const char* n) {
  return binary(m, "subtract", a, b, n);
}
flexflow_tensor_t flexflow_model_add_multiply(flexflow_model_t m, flexflow_tensor_t a, flexflow_tensor_t b, const char* n) {
  return binary(m, "multiply", a, b, n);
}
flexflow_tensor_t flexflow_model_add_divide(flexflow_model_t m, flexflow_tensor_t a, flexflow_tensor_t b, const char* n) {
  return binary(m, "divide", a, b, n);
}
flexflow_tensor_t flexflow_model_add_batch_matmul(flexflow_model_t m, flexflow_tensor_t a, flexflow_tensor_t b,
                                                  const char* n) {
  return binary(m, "batch_matmul", a, b, n);
}
flexflow_tensor_t flexflow_model_add_concat(flexflow_model_t m, int n, const flexflow_tensor_t* xs, int axis,
                                            const char* name) {
  init_once();
  Gil gil;
  PyObject* l = PyList_New(n);
  for (int i = 0; i < n; ++i) {
    PyObject* o = obj(xs[i].impl);
    Py_INCREF(o);
    PyList_SET_ITEM(l, i, o);
  }
  return wrap<flexflow_tensor_t>(call("add_concat", "(ONiz)", obj(m.impl), l, axis, name));
}
flexflow_tensor_t flexflow_model_add_dropout(flexflow_model_t m, flexflow_tensor_t x, float rate,
                                             unsigned long long seed, const char* name) {
  init_once();
  Gil gil;
  return wrap<flexflow_tensor_t>(call("add_dropout", "(OOdKz)", obj(m.impl), obj(x.impl), (double)rate, seed, name));
}
flexflow_tensor_t flexflow_model_add_reshape(flexflow_model_t m, flexflow_tensor_t x, int nd, const int* shape,
                                             const char* name) {
  init_once();
  Gil gil;
  return wrap<flexflow_tensor_t>(call("add_reshape", "(OONz)", obj(m.impl), obj(x.impl), int_list(shape, nd), name));
}
flexflow_tensor_t flexflow_model_add_transpose(flexflow_model_t m, flexflow_tensor_t x, int nd, const int* perm,
                                               const char* name) {
  init_once();
  Gil gil;
  return wrap<flexflow_tensor_t>(call("add_transpose", "(OONz)", obj(m.impl), obj(x.impl), int_list(perm, nd), name));
}

flexflow_tensor_t flexflow_model_add_embedding_typed(flexflow_model_t m, flexflow_tensor_t x, int num, int dim,
                                                     int aggr, int dtype, const char* name) {
  init_once();
  Gil gil;
  return wrap<flexflow_tensor_t>(
      call("add_embedding_typed", "(OOiiiiz)", obj(m.impl), obj(x.impl), num, dim, aggr, dtype, name));
}
flexflow_tensor_t flexflow_model_add_max(flexflow_model_t m, flexflow_tensor_t a, flexflow_tensor_t b, const char* n) {
  return binary(m, "max", a, b, n);
}
flexflow_tensor_t flexflow_model_add_min(flexflow_model_t m, flexflow_tensor_t a, flexflow_tensor_t b, const char* n) {
  return binary(m, "min", a, b, n);
}
static flexflow_tensor_t reduce(flexflow_model_t m, const char* op, flexflow_tensor_t x, int nd, const int* dims,
                                bool keep, const char* name) {
  init_once();
  Gil gil;
  return wrap<flexflow_tensor_t>(
      call("add_reduce", "(OsONiz)", obj(m.impl), op, obj(x.impl), int_list(dims, nd), (int)keep, name));
}
flexflow_tensor_t flexflow_model_add_mean(flexflow_model_t m, flexflow_tensor_t x, int nd, const int* dims, bool keep,
                                          const char* name) {
  return reduce(m, "mean", x, nd, dims, keep, name);
}
flexflow_tensor_t flexflow_model_add_reduce_sum(flexflow_model_t m, flexflow_tensor_t x, int nd, const int* axes,
                                                bool keep, const char* name) {
  return reduce(m, "reduce_sum", x, nd, axes, keep, name);
}
flexflow_tensor_t flexflow_model_add_gather(flexflow_model_t m, flexflow_tensor_t x, flexflow_tensor_t idx, int dim,
                                            const char* name) {
  init_once();
  Gil gil;
  return wrap<flexflow_tensor_t>(call("add_gather", "(OOOiz)", obj(m.impl), obj(x.impl), obj(idx.impl), dim, name));
}
flexflow_tensor_t flexflow_model_add_cast(flexflow_model_t m, flexflow_tensor_t x, int dtype, const char* name) {
  init_once();
  Gil gil;
  return wrap<flexflow_tensor_t>(call("add_cast", "(OOiz)", obj(m.impl), obj(x.impl), dtype, name));
}
flexflow_tensor_t flexflow_model_add_rms_norm(flexflow_model_t m, flexflow_tensor_t x, float eps, const char* name) {
  init_once();
  Gil gil;
  return wrap<flexflow_tensor_t>(call("add_rms_norm", "(OOdz)", obj(m.impl), obj(x.impl), (double)eps, name));
}
flexflow_tensor_t flexflow_model_add_reverse(flexflow_model_t m, flexflow_tensor_t x, int axis, const char* name) {
  init_once();
  Gil gil;
  return wrap<flexflow_tensor_t>(call("add_reverse", "(OOiz)", obj(m.impl), obj(x.impl), axis, name));
}

// a Python list of tensors -> outputs[0..n) (each a new reference); returns n, or -1 on error
// or when the list holds more than `cap` tensors (the caller's array size)
static int unpack(PyObject* r, flexflow_tensor_t* outputs, int cap) {
  if (!r) return -1;
  if (!PyList_Check(r)) {
    Py_DECREF(r);
    g_err = "expected a list of tensors";
    return -1;
  }
  const int n = (int)PyList_Size(r);
  if (n > cap || !outputs) {
    Py_DECREF(r);
    g_err = "output array too small for the op's outputs";
    return -1;
  }
  for (int i = 0; i < n; ++i) {
    PyObject* o = PyList_GetItem(r, i);
    Py_INCREF(o);
    outputs[i] = wrap<flexflow_tensor_t>(o);
  }
  Py_DECREF(r);
  return n;
}
static PyObject* tensor_list(int n, const flexflow_tensor_t* xs) {
  PyObject* l = PyList_New(n);
  for (int i = 0; i < n; ++i) {
    PyObject* o = obj(xs[i].impl);
    Py_INCREF(o);
    PyList_SET_ITEM(l, i, o);
  }
  return l;
}
int flexflow_model_add_split(flexflow_model_t m, flexflow_tensor_t x, int n, const int* sizes, int axis,
                             flexflow_tensor_t* outputs, const char* name) {
  init_once();
  Gil gil;
  return unpack(call("add_split", "(OONiz)", obj(m.impl), obj(x.impl), int_list(sizes, n), axis, name), outputs, n);
}
int flexflow_model_add_top_k(flexflow_model_t m, flexflow_tensor_t x, int k, bool sorted, flexflow_tensor_t* outputs,
                             const char* name) {
  init_once();
  Gil gil;
  return unpack(call("add_top_k", "(OOiiz)", obj(m.impl), obj(x.impl), k, (int)sorted, name), outputs, 2);
}
int flexflow_model_add_group_by(flexflow_model_t m, flexflow_tensor_t data, flexflow_tensor_t assign, int n,
                                float alpha, flexflow_tensor_t* outputs, const char* name) {
  init_once();
  Gil gil;
  return unpack(call("add_group_by", "(OOOidz)", obj(m.impl), obj(data.impl), obj(assign.impl), n, (double)alpha,
                     name),
                outputs, n);
}
static flexflow_tensor_t aggregate(flexflow_model_t m, int ni, const flexflow_tensor_t* xs, int n, float lam, int spec,
                                   const char* name) {
  init_once();
  Gil gil;
  return wrap<flexflow_tensor_t>(
      call("add_aggregate", "(ONidiz)", obj(m.impl), tensor_list(ni, xs), n, (double)lam, spec, name));
}
flexflow_tensor_t flexflow_model_add_aggregate(flexflow_model_t m, int ni, const flexflow_tensor_t* xs, int n,
                                               float lam, const char* name) {
  return aggregate(m, ni, xs, n, lam, 0, name);
}
flexflow_tensor_t flexflow_model_add_aggregate_spec(flexflow_model_t m, int ni, const flexflow_tensor_t* xs, int n,
                                                    float lam, const char* name) {
  return aggregate(m, ni, xs, n, lam, 1, name);
}
flexflow_tensor_t flexflow_model_add_moe(flexflow_model_t m, flexflow_tensor_t x, int num_exp, int num_select,
                                         int hidden, float alpha, float lam) {
  init_once();
  Gil gil;
  return wrap<flexflow_tensor_t>(call("add_moe", "(OOiiidd)", obj(m.impl), obj(x.impl), num_exp, num_select, hidden,
                                      (double)alpha, (double)lam));
}
bool flexflow_tensor_set_data_int64(flexflow_tensor_t h, flexflow_model_t m, const int64_t* d, int64_t n) {
  return set_data(h, m, d, n, 42 /* DT_INT64 */);
}
void flexflow_model_print_layers(flexflow_model_t m, int id) {
  init_once();
  Gil gil;
  as_bool_ok(call("model_print_layers", "(Oi)", obj(m.impl), id));
}
int flexflow_model_get_num_layers(flexflow_model_t m) {
  init_once();
  Gil gil;
  PyObject* r = call("model_num_layers", "(O)", obj(m.impl));
  if (!r) return -1;
  const int n = (int)PyLong_AsLong(r);
  Py_DECREF(r);
  return n;
}
const char* flexflow_model_get_strategy_name(flexflow_model_t m) {
  static thread_local std::string s;
  init_once();
  Gil gil;
  PyObject* r = call("model_search_algo", "(O)", obj(m.impl));
  s = r ? PyUnicode_AsUTF8(r) : "";
  Py_XDECREF(r);
  return s.c_str();
}

}  // extern "C"
