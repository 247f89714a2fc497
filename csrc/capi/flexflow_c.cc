// flexflow_amd C API: an embedded CPython runtime forwarding every call to flexflow_amd.capi_impl
// (reference src/c/flexflow_c.cc wraps the C++ FFModel; here the FFModel is the Python package,
// whose compute path is the HIP kernel library and RCCL, so C callers get the same runtime).
// All 144 reference entry points (include/flexflow/flexflow_c.h) plus extensions; see flexflow_c.h
// for the few deliberate semantic differences.
//
// Handles own one reference to the wrapped Python object; *_destroy drops it. All entry points
// take the GIL (PyGILState_Ensure), so the API may be called from any host thread.
#include "flexflow_c.h"

#include <Python.h>

#include <cstdarg>
#include <cstdio>
#include <map>
#include <mutex>
#include <string>
#include <vector>

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


int to_int(PyObject* r, int dflt = -1) {
  if (!r) return dflt;
  const long v = PyLong_AsLong(r);
  Py_DECREF(r);
  if (PyErr_Occurred()) {
    record_error();
    return dflt;
  }
  return (int)v;
}

double to_double(PyObject* r, double dflt) {
  if (!r) return dflt;
  const double v = PyFloat_AsDouble(r);
  Py_DECREF(r);
  if (PyErr_Occurred()) {
    record_error();
    return dflt;
  }
  return v;
}

void* to_ptr(PyObject* r) {
  if (!r) return nullptr;
  void* p = PyLong_AsVoidPtr(r);
  Py_DECREF(r);
  if (PyErr_Occurred()) {
    record_error();
    return nullptr;
  }
  return p;
}

// storage behind pointer / string results, keyed by the handle they describe (freed on destroy)
std::mutex g_cache_mu;
std::map<std::pair<const void*, std::string>, std::vector<int>> g_int_cache;
std::map<std::pair<const void*, std::string>, std::string> g_str_cache;

int* cached_ints(const void* key, const char* field, PyObject* r, bool with_count) {
  if (!r) return nullptr;
  std::vector<int> v;
  if (with_count) v.push_back(0);
  const Py_ssize_t n = PyList_Check(r) ? PyList_Size(r) : 0;
  for (Py_ssize_t i = 0; i < n; ++i) v.push_back((int)PyLong_AsLong(PyList_GetItem(r, i)));
  Py_DECREF(r);
  if (with_count) v[0] = (int)n;
  std::lock_guard<std::mutex> lk(g_cache_mu);
  auto& slot = g_int_cache[{key, field}];
  slot.swap(v);
  return slot.data();
}

const char* cached_str(const void* key, const char* field, PyObject* r) {
  if (!r) return nullptr;
  const char* u = PyUnicode_Check(r) ? PyUnicode_AsUTF8(r) : nullptr;
  std::string s = u ? u : "";
  if (!u) PyErr_Clear();
  Py_DECREF(r);
  std::lock_guard<std::mutex> lk(g_cache_mu);
  auto& slot = g_str_cache[{key, field}];
  slot = s;
  return slot.c_str();
}

void forget(const void* key) {
  std::lock_guard<std::mutex> lk(g_cache_mu);
  for (auto it = g_int_cache.begin(); it != g_int_cache.end();) it = it->first.first == key ? g_int_cache.erase(it) : std::next(it);
  for (auto it = g_str_cache.begin(); it != g_str_cache.end();) it = it->first.first == key ? g_str_cache.erase(it) : std::next(it);
}

PyObject* tensor_list(int n, const flexflow_tensor_t* xs) {
  PyObject* l = PyList_New(n);
  for (int i = 0; i < n; ++i) {
    PyObject* o = obj(xs[i].impl);
    Py_INCREF(o);
    PyList_SET_ITEM(l, i, o);
  }
  return l;
}

// a Python list of tensors -> outputs[0..n) (each a new reference); returns n, or -1 on error or
// when the list holds more than `cap` tensors (the caller's array size)
int unpack(PyObject* r, flexflow_tensor_t* outputs, int cap) {
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
    outputs[i].impl = o;
  }
  Py_DECREF(r);
  return n;
}

}  // namespace

// every entry point: initialise the embedded runtime once, hold the GIL for the call
#define FF_ENTRY \
  init_once();   \
  Gil gil_
#define FF_HANDLE(T, ...) \
  FF_ENTRY;               \
  return wrap<T>(call(__VA_ARGS__))
#define FF_VOID(...) \
  FF_ENTRY;          \
  as_bool_ok(call(__VA_ARGS__))
#define FF_BOOL(...) \
  FF_ENTRY;          \
  return as_bool_ok(call(__VA_ARGS__))
#define FF_INT(...) \
  FF_ENTRY;         \
  return to_int(call(__VA_ARGS__))

extern "C" {

int flexflow_initialize(void) {
  init_once();
  return g_impl ? 0 : -1;
}
const char* flexflow_last_error(void) { return g_err.c_str(); }

// ------------------------------------------------------------------------------------ config
flexflow_config_t flexflow_config_create(void) { FF_HANDLE(flexflow_config_t, "config_create", "()"); }
void flexflow_config_destroy(flexflow_config_t h) {
  forget(h.impl);
  drop(h.impl);
}
void flexflow_config_parse_args(flexflow_config_t h, char** argv, int argc) {
  FF_ENTRY;
  PyObject* l = PyList_New(argc);
  for (int i = 0; i < argc; ++i) PyList_SET_ITEM(l, i, PyUnicode_FromString(argv[i]));
  as_bool_ok(call("config_parse_args", "(ON)", obj(h.impl), l));
}
void flexflow_config_parse_args_default(flexflow_config_t h) { FF_VOID("config_parse_default", "(O)", obj(h.impl)); }
int flexflow_config_get_batch_size(flexflow_config_t h) { return config_int(h, "batch_size"); }
int flexflow_config_get_workers_per_node(flexflow_config_t h) { return config_int(h, "workers_per_node"); }
int flexflow_config_get_num_nodes(flexflow_config_t h) { return config_int(h, "num_nodes"); }
int flexflow_config_get_epochs(flexflow_config_t h) { return config_int(h, "epochs"); }
bool flexflow_config_get_enable_control_replication(flexflow_config_t h) {
  FF_ENTRY;
  return to_int(call("config_attr", "(Osi)", obj(h.impl), "enable_control_replication", 0), 0) != 0;
}
int flexflow_config_get_python_data_loader_type(flexflow_config_t h) {
  FF_INT("config_attr", "(Osi)", obj(h.impl), "python_data_loader_type", 2);
}
void flexflow_config_set_batch_size(flexflow_config_t h, int b) {
  FF_VOID("config_set_batch_size", "(Oi)", obj(h.impl), b);
}

// ------------------------------------------------------------------------------------- model
flexflow_model_t flexflow_model_create(flexflow_config_t config) {
  FF_HANDLE(flexflow_model_t, "model_create", "(O)", obj(config.impl));
}
void flexflow_model_destroy(flexflow_model_t h) {
  forget(h.impl);
  drop(h.impl);
}
void flexflow_model_reset_metrics(flexflow_model_t h) { model_call(h, "reset_metrics"); }
void flexflow_model_init_layers(flexflow_model_t h) { model_call(h, "init_layers"); }
void flexflow_model_prefetch(flexflow_model_t h) { model_call(h, "prefetch"); }
void flexflow_model_forward(flexflow_model_t h, int) { model_call(h, "forward"); }
void flexflow_model_backward(flexflow_model_t h, int) { model_call(h, "backward"); }
void flexflow_model_compute_metrics(flexflow_model_t h) { model_call(h, "compute_metrics"); }
void flexflow_model_update(flexflow_model_t h) { model_call(h, "update"); }
void flexflow_model_zero_gradients(flexflow_model_t h) { model_call(h, "zero_gradients"); }
void flexflow_model_train_step(flexflow_model_t h) { model_call(h, "train_step"); }
void flexflow_model_compile(flexflow_model_t h, int loss_type, int* metrics, int nb_metrics, int comp_mode) {
  FF_VOID("model_compile", "(OiNi)", obj(h.impl), loss_type, int_list(metrics, nb_metrics), comp_mode);
}
flexflow_tensor_t flexflow_model_get_label_tensor(flexflow_model_t h) {
  FF_HANDLE(flexflow_tensor_t, "model_label_tensor", "(O)", obj(h.impl));
}
static float perf(flexflow_model_t h, int what) {
  FF_ENTRY;
  return (float)to_double(call("model_perf", "(Oi)", obj(h.impl), what), -1.0);
}
float flexflow_model_get_accuracy(flexflow_model_t h) { return perf(h, 0); }
float flexflow_model_get_loss(flexflow_model_t h) { return perf(h, 1); }

// ------------------------------------------------------------------------------------ layers
flexflow_tensor_t flexflow_model_add_exp(flexflow_model_t h, const flexflow_tensor_t x, const char* name) {
  return unary(h, "exp", x, name);
}
flexflow_tensor_t flexflow_model_add_sin(flexflow_model_t h, const flexflow_tensor_t x, const char* name) {
  return unary(h, "sin", x, name);
}
flexflow_tensor_t flexflow_model_add_cos(flexflow_model_t h, const flexflow_tensor_t x, const char* name) {
  return unary(h, "cos", x, name);
}
flexflow_tensor_t flexflow_model_add_add(flexflow_model_t h, const flexflow_tensor_t x, const flexflow_tensor_t y, bool,
                                         const char* name) {
  return binary(h, "add", x, y, name);
}
flexflow_tensor_t flexflow_model_add_subtract(flexflow_model_t h, const flexflow_tensor_t x, const flexflow_tensor_t y,
                                              bool, const char* name) {
  return binary(h, "subtract", x, y, name);
}
flexflow_tensor_t flexflow_model_add_multiply(flexflow_model_t h, const flexflow_tensor_t x, const flexflow_tensor_t y,
                                              bool, const char* name) {
  return binary(h, "multiply", x, y, name);
}
flexflow_tensor_t flexflow_model_add_divide(flexflow_model_t h, const flexflow_tensor_t x, const flexflow_tensor_t y,
                                            bool, const char* name) {
  return binary(h, "divide", x, y, name);
}
flexflow_tensor_t flexflow_model_add_max(flexflow_model_t h, const flexflow_tensor_t x, const flexflow_tensor_t y, bool,
                                         const char* name) {
  return binary(h, "max", x, y, name);
}
flexflow_tensor_t flexflow_model_add_min(flexflow_model_t h, const flexflow_tensor_t x, const flexflow_tensor_t y, bool,
                                         const char* name) {
  return binary(h, "min", x, y, name);
}
flexflow_tensor_t flexflow_model_add_reduce_sum(flexflow_model_t h, const flexflow_tensor_t x, int* axes, int n,
                                                bool keepdims, const char* name) {
  FF_HANDLE(flexflow_tensor_t, "add_reduce_ref", "(OsONiz)", obj(h.impl), "reduce_sum", obj(x.impl), int_list(axes, n),
            (int)keepdims, name);
}
flexflow_tensor_t flexflow_model_add_rsqrt(flexflow_model_t h, const flexflow_tensor_t x, const char* name) {
  return unary(h, "rsqrt", x, name);
}
flexflow_tensor_t flexflow_model_add_pow(flexflow_model_t h, const flexflow_tensor_t x, const float e,
                                         const char* name) {
  return scalar(h, "pow", x, e, name);
}
flexflow_tensor_t flexflow_model_add_mean(flexflow_model_t h, const flexflow_tensor_t x, int* dims, int n,
                                          bool keepdims, const char* name) {
  FF_HANDLE(flexflow_tensor_t, "add_reduce_ref", "(OsONiz)", obj(h.impl), "mean", obj(x.impl), int_list(dims, n),
            (int)keepdims, name);
}
flexflow_tensor_t flexflow_model_add_conv2d(flexflow_model_t h, const flexflow_tensor_t x, int oc, int kh, int kw,
                                            int sh, int sw, int ph, int pw, int act, int groups, bool use_bias,
                                            flexflow_op_t shared, flexflow_initializer_t kinit,
                                            flexflow_initializer_t binit, const char* name) {
  FF_HANDLE(flexflow_tensor_t, "add_conv2d_init", "(OOiiiiiiiiiiOOOz)", obj(h.impl), obj(x.impl), oc, kh, kw, sh, sw,
            ph, pw, act, groups, (int)use_bias, obj(shared.impl), obj(kinit.impl), obj(binit.impl), name);
}
flexflow_tensor_t flexflow_model_add_embedding(flexflow_model_t h, const flexflow_tensor_t x, int num, int dim, int aggr,
                                               flexflow_op_t shared, flexflow_initializer_t kinit, const char* name) {
  FF_HANDLE(flexflow_tensor_t, "add_embedding_init", "(OOiiiOOz)", obj(h.impl), obj(x.impl), num, dim, aggr,
            obj(shared.impl), obj(kinit.impl), name);
}
flexflow_tensor_t flexflow_model_add_pool2d(flexflow_model_t h, flexflow_tensor_t x, int kh, int kw, int sh, int sw,
                                            int ph, int pw, int type, int act, const char* name) {
  FF_HANDLE(flexflow_tensor_t, "add_pool2d_ref", "(OOiiiiiiiiz)", obj(h.impl), obj(x.impl), kh, kw, sh, sw, ph, pw,
            type, act, name);
}
flexflow_tensor_t flexflow_model_add_batch_norm(flexflow_model_t h, const flexflow_tensor_t x, bool relu,
                                                const char* name) {
  FF_HANDLE(flexflow_tensor_t, "add_batch_norm", "(OOiz)", obj(h.impl), obj(x.impl), (int)relu, name);
}
flexflow_tensor_t flexflow_model_add_layer_norm(flexflow_model_t h, const flexflow_tensor_t x, int n, int* axes,
                                                bool affine, float eps, const char* name) {
  FF_HANDLE(flexflow_tensor_t, "add_layer_norm", "(OONidz)", obj(h.impl), obj(x.impl), int_list(axes, n), (int)affine,
            (double)eps, name);
}
flexflow_tensor_t flexflow_model_add_batch_matmul(flexflow_model_t h, const flexflow_tensor_t a,
                                                  const flexflow_tensor_t b, int a_seq, int b_seq) {
  FF_HANDLE(flexflow_tensor_t, "add_batch_matmul", "(OOOii)", obj(h.impl), obj(a.impl), obj(b.impl), a_seq, b_seq);
}
flexflow_tensor_t flexflow_model_add_dense(flexflow_model_t h, const flexflow_tensor_t x, int out_dim, int act,
                                           bool use_bias, int data_type, flexflow_op_t shared,
                                           flexflow_initializer_t kinit, flexflow_initializer_t binit, int reg_type,
                                           float reg_lambda, const char* name) {
  FF_HANDLE(flexflow_tensor_t, "add_dense_init", "(OOiiiiOOOidz)", obj(h.impl), obj(x.impl), out_dim, act,
            (int)use_bias, data_type, obj(shared.impl), obj(kinit.impl), obj(binit.impl), reg_type, (double)reg_lambda,
            name);
}
flexflow_tensor_t flexflow_model_add_concat(flexflow_model_t h, int n, flexflow_tensor_t* xs, int axis,
                                            const char* name) {
  FF_HANDLE(flexflow_tensor_t, "add_concat", "(ONiz)", obj(h.impl), tensor_list(n, xs), axis, name);
}
void flexflow_model_add_split(flexflow_model_t h, flexflow_tensor_t x, int n, flexflow_tensor_t* outputs, int* split,
                              int axis, const char* name) {
  FF_ENTRY;
  unpack(call("add_split", "(OONiz)", obj(h.impl), obj(x.impl), int_list(split, n), axis, name), outputs, n);
}
flexflow_tensor_t flexflow_model_add_flat(flexflow_model_t h, flexflow_tensor_t x, const char* name) {
  return unary(h, "flat", x, name);
}
flexflow_tensor_t flexflow_model_add_gather(flexflow_model_t h, const flexflow_tensor_t x, const flexflow_tensor_t index,
                                            int dim, const char* name) {
  FF_HANDLE(flexflow_tensor_t, "add_gather", "(OOOiz)", obj(h.impl), obj(x.impl), obj(index.impl), dim, name);
}
flexflow_tensor_t flexflow_model_add_softmax(flexflow_model_t h, const flexflow_tensor_t x, int dim, const char* name) {
  FF_HANDLE(flexflow_tensor_t, "add_softmax", "(OOiz)", obj(h.impl), obj(x.impl), dim, name);
}
flexflow_tensor_t flexflow_model_add_transpose(flexflow_model_t h, const flexflow_tensor_t x, int n, int* perm,
                                               const char* name) {
  FF_HANDLE(flexflow_tensor_t, "add_transpose", "(OONz)", obj(h.impl), obj(x.impl), int_list(perm, n), name);
}
flexflow_tensor_t flexflow_model_add_reshape(flexflow_model_t h, const flexflow_tensor_t x, int n, int* shape,
                                             const char* name) {
  FF_HANDLE(flexflow_tensor_t, "add_reshape", "(OONz)", obj(h.impl), obj(x.impl), int_list(shape, n), name);
}
flexflow_tensor_t flexflow_model_add_reverse(flexflow_model_t h, const flexflow_tensor_t x, int axis, const char* name) {
  FF_HANDLE(flexflow_tensor_t, "add_reverse", "(OOiz)", obj(h.impl), obj(x.impl), axis, name);
}
flexflow_tensor_t flexflow_model_add_relu(flexflow_model_t h, const flexflow_tensor_t x, bool, const char* name) {
  return unary(h, "relu", x, name);
}
flexflow_tensor_t flexflow_model_add_scalar_multiply(flexflow_model_t h, const flexflow_tensor_t x, const float s,
                                                     bool, const char* name) {
  return scalar(h, "scalar_multiply", x, s, name);
}
flexflow_tensor_t flexflow_model_add_scalar_add(flexflow_model_t h, const flexflow_tensor_t x, const float s, bool,
                                                const char* name) {
  return scalar(h, "scalar_add", x, s, name);
}
flexflow_tensor_t flexflow_model_add_scalar_sub(flexflow_model_t h, const flexflow_tensor_t x, const float s, bool,
                                                const char* name) {
  return scalar(h, "scalar_sub", x, s, name);
}
flexflow_tensor_t flexflow_model_add_scalar_truediv(flexflow_model_t h, const flexflow_tensor_t x, const float s, bool,
                                                    const char* name) {
  return scalar(h, "scalar_true_divide", x, s, name);
}
flexflow_tensor_t flexflow_model_add_gelu(flexflow_model_t h, const flexflow_tensor_t x, const char* name) {
  return unary(h, "gelu", x, name);
}
flexflow_tensor_t flexflow_model_add_identity(flexflow_model_t h, const flexflow_tensor_t x, const char* name) {
  return unary(h, "identity", x, name);
}
flexflow_tensor_t flexflow_model_add_sigmoid(flexflow_model_t h, const flexflow_tensor_t x, const char* name) {
  return unary(h, "sigmoid", x, name);
}
flexflow_tensor_t flexflow_model_add_tanh(flexflow_model_t h, const flexflow_tensor_t x, const char* name) {
  return unary(h, "tanh", x, name);
}
flexflow_tensor_t flexflow_model_add_elu(flexflow_model_t h, const flexflow_tensor_t x, bool, const char* name) {
  return unary(h, "elu", x, name);
}
flexflow_tensor_t flexflow_model_add_dropout(flexflow_model_t h, const flexflow_tensor_t x, float rate,
                                             unsigned long long seed, const char* name) {
  FF_HANDLE(flexflow_tensor_t, "add_dropout", "(OOdKz)", obj(h.impl), obj(x.impl), (double)rate, seed, name);
}
flexflow_tensor_t flexflow_model_add_multihead_attention(flexflow_model_t h, const flexflow_tensor_t q,
                                                         const flexflow_tensor_t k, const flexflow_tensor_t v,
                                                         int embed_dim, int num_heads, int kdim, int vdim,
                                                         float dropout, bool bias, bool add_bias_kv,
                                                         bool add_zero_attn, flexflow_initializer_t kinit,
                                                         const char* name) {
  FF_HANDLE(flexflow_tensor_t, "add_mha_init", "(OOOOiiiidiiiOz)", obj(h.impl), obj(q.impl), obj(k.impl), obj(v.impl),
            embed_dim, num_heads, kdim, vdim, (double)dropout, (int)bias, (int)add_bias_kv, (int)add_zero_attn,
            obj(kinit.impl), name);
}
void flexflow_model_set_sgd_optimizer(flexflow_model_t h, flexflow_sgd_optimizer_t o) {
  FF_VOID("model_set_opt", "(OO)", obj(h.impl), obj(o.impl));
}
void flexflow_model_set_adam_optimizer(flexflow_model_t h, flexflow_adam_optimizer_t o) {
  FF_VOID("model_set_opt", "(OO)", obj(h.impl), obj(o.impl));
}
void flexflow_model_set_optimizer(flexflow_model_t h, flexflow_optimizer_t o) {
  FF_VOID("model_set_opt", "(OO)", obj(h.impl), obj(o.impl));
}
void flexflow_model_print_layers(flexflow_model_t h, int id) {
  FF_VOID("model_print_layers", "(Oi)", obj(h.impl), id);
}
flexflow_op_t flexflow_model_get_layer_by_id(flexflow_model_t h, int id) {
  FF_HANDLE(flexflow_op_t, "model_layer", "(Oi)", obj(h.impl), id);
}
flexflow_op_t flexflow_model_get_last_layer(flexflow_model_t h) {
  FF_HANDLE(flexflow_op_t, "model_last_layer", "(O)", obj(h.impl));
}
flexflow_tensor_t flexflow_model_get_parameter_by_id(flexflow_model_t h, int id) {
  FF_HANDLE(flexflow_tensor_t, "model_parameter", "(Oi)", obj(h.impl), id);
}
flexflow_perf_metrics_t flexflow_model_get_perf_metrics(flexflow_model_t h) {
  FF_HANDLE(flexflow_perf_metrics_t, "model_perf_metrics", "(O)", obj(h.impl));
}
int flexflow_model_get_num_layers(flexflow_model_t h) { FF_INT("model_num_layers", "(O)", obj(h.impl)); }
const char* flexflow_model_get_strategy_name(flexflow_model_t h) {
  FF_ENTRY;
  return cached_str(h.impl, "strategy", call("model_search_algo", "(O)", obj(h.impl)));
}

// ----------------------------------------------------------------------------------- tensors
flexflow_tensor_t flexflow_tensor_create(flexflow_model_t m, int num_dims, const int* dims, int data_type,
                                         bool create_grad) {
  FF_HANDLE(flexflow_tensor_t, "tensor_create", "(ONii)", obj(m.impl), int_list(dims, num_dims), data_type,
            (int)create_grad);
}
void flexflow_tensor_map(flexflow_model_t m, flexflow_tensor_t t, flexflow_op_t op) {
  FF_VOID("tensor_map", "(OOO)", obj(m.impl), obj(t.impl), obj(op.impl));
}
flexflow_tensor_t flexflow_constant_create(flexflow_model_t m, int num_dims, const int* dims, float value,
                                           int data_type) {
  FF_HANDLE(flexflow_tensor_t, "constant_create", "(ONdi)", obj(m.impl), int_list(dims, num_dims), (double)value,
            data_type);
}
void flexflow_tensor_destroy(flexflow_tensor_t h) {
  forget(h.impl);
  drop(h.impl);
}
void flexflow_tensor_inline_map(flexflow_tensor_t h, flexflow_model_t m, flexflow_config_t) {
  FF_VOID("tensor_inline_map", "(OO)", obj(h.impl), obj(m.impl));
}
void flexflow_tensor_inline_unmap(flexflow_tensor_t h, flexflow_model_t m, flexflow_config_t) {
  FF_VOID("tensor_inline_unmap", "(OO)", obj(h.impl), obj(m.impl));
}
float* flexflow_tensor_get_raw_ptr_float(flexflow_tensor_t h, flexflow_model_t m, flexflow_config_t) {
  FF_ENTRY;
  return (float*)to_ptr(call("tensor_raw_ptr", "(OOi)", obj(h.impl), obj(m.impl), 0));
}
int32_t* flexflow_tensor_get_raw_ptr_int32(flexflow_tensor_t h, flexflow_model_t m, flexflow_config_t) {
  FF_ENTRY;
  return (int32_t*)to_ptr(call("tensor_raw_ptr", "(OOi)", obj(h.impl), obj(m.impl), 1));
}
int flexflow_tensor_get_num_dims(flexflow_tensor_t h) {
  FF_ENTRY;
  PyObject* r = call("tensor_dims", "(O)", obj(h.impl));
  if (!r) return -1;
  const int n = (int)PyList_Size(r);
  Py_DECREF(r);
  return n;
}
int* flexflow_tensor_get_dims(flexflow_tensor_t h) {
  FF_ENTRY;
  return cached_ints(h.impl, "dims", call("tensor_dims_legion", "(O)", obj(h.impl)), false);
}
int flexflow_tensor_get_dim(flexflow_tensor_t h, int legion_axis) {
  int* d = flexflow_tensor_get_dims(h);
  const int n = flexflow_tensor_get_num_dims(h);
  if (!d || legion_axis < 0 || legion_axis >= n) return -1;
  return d[legion_axis];
}
int flexflow_tensor_get_data_type(flexflow_tensor_t h) { FF_INT("tensor_dtype", "(O)", obj(h.impl)); }
flexflow_op_t flexflow_tensor_get_owner_op(flexflow_tensor_t h) {
  FF_HANDLE(flexflow_op_t, "tensor_owner", "(O)", obj(h.impl));
}
void flexflow_tensor_attach_raw_ptr(flexflow_tensor_t h, flexflow_model_t m, flexflow_config_t, void* raw_ptr,
                                    bool column_major) {
  FF_VOID("tensor_attach", "(OONi)", obj(h.impl), obj(m.impl), PyLong_FromVoidPtr(raw_ptr), (int)column_major);
}
void flexflow_tensor_detach_raw_ptr(flexflow_tensor_t h, flexflow_model_t m, flexflow_config_t) {
  FF_VOID("tensor_detach", "(OO)", obj(h.impl), obj(m.impl));
}
bool flexflow_tensor_is_mapped(flexflow_tensor_t h) {
  FF_ENTRY;
  return to_int(call("tensor_is_mapped", "(O)", obj(h.impl)), 0) != 0;
}
static bool set_dims(flexflow_tensor_t h, flexflow_model_t m, int num_dim, int* dims, const void* data, int dtype) {
  FF_BOOL("tensor_set_dims", "(OONNi)", obj(h.impl), obj(m.impl), int_list(dims, dims ? num_dim : 0),
          PyLong_FromVoidPtr(const_cast<void*>(data)), dtype);
}
static bool get_into(flexflow_tensor_t h, flexflow_model_t m, void* data, int dtype, bool grads) {
  FF_BOOL("tensor_get_into", "(OONii)", obj(h.impl), obj(m.impl), PyLong_FromVoidPtr(data), dtype, (int)grads);
}
// DataType numeric values (flexflow_amd/type.py, reference ffconst.h)
static const int kDT_INT32 = 41, kDT_INT64 = 42, kDT_FLOAT = 44;
bool flexflow_tensor_set_tensor_float(flexflow_tensor_t h, flexflow_model_t m, int num_dim, int* dims,
                                      const float* data) {
  return set_dims(h, m, num_dim, dims, data, kDT_FLOAT);
}
bool flexflow_tensor_get_tensor_float(flexflow_tensor_t h, flexflow_model_t m, float* data, bool grads) {
  return get_into(h, m, data, kDT_FLOAT, grads);
}
bool flexflow_tensor_set_tensor_int(flexflow_tensor_t h, flexflow_model_t m, int num_dim, int* dims, const int* data) {
  return set_dims(h, m, num_dim, dims, data, kDT_INT32);
}
bool flexflow_tensor_get_tensor_int(flexflow_tensor_t h, flexflow_model_t m, int* data, bool grads) {
  return get_into(h, m, data, kDT_INT32, grads);
}
bool flexflow_tensor_set_tensor_int64(flexflow_tensor_t h, flexflow_model_t m, int num_dim, int* dims,
                                      const int64_t* data, int) {
  return set_dims(h, m, num_dim, dims, data, kDT_INT64);
}
bool flexflow_tensor_get_tensor_int64(flexflow_tensor_t h, flexflow_model_t m, int64_t* data, bool grads) {
  return get_into(h, m, data, kDT_INT64, grads);
}
bool flexflow_model_get_output_tensor_float(flexflow_model_t m, flexflow_tensor_t h, float* data, bool grads) {
  FF_BOOL("model_output_get", "(OONi)", obj(m.impl), obj(h.impl), PyLong_FromVoidPtr(data), (int)grads);
}
// flat host buffers of exactly n elements (extensions)
static bool set_flat(flexflow_tensor_t h, flexflow_model_t m, const void* data, int64_t n, int dtype) {
  FF_BOOL("tensor_set_data", "(OONLi)", obj(m.impl), obj(h.impl), PyLong_FromVoidPtr(const_cast<void*>(data)),
          (long long)n, dtype);
}
bool flexflow_tensor_set_data_float(flexflow_tensor_t h, flexflow_model_t m, const float* data, int64_t n) {
  return set_flat(h, m, data, n, kDT_FLOAT);
}
bool flexflow_tensor_set_data_int(flexflow_tensor_t h, flexflow_model_t m, const int32_t* data, int64_t n) {
  return set_flat(h, m, data, n, kDT_INT32);
}
bool flexflow_tensor_set_data_int64(flexflow_tensor_t h, flexflow_model_t m, const int64_t* data, int64_t n) {
  return set_flat(h, m, data, n, kDT_INT64);
}
bool flexflow_tensor_get_data_float(flexflow_tensor_t h, flexflow_model_t m, float* data, int64_t n) {
  FF_BOOL("tensor_get_data", "(OONL)", obj(m.impl), obj(h.impl), PyLong_FromVoidPtr(data), (long long)n);
}

// -------------------------------------------------------------------------------- parameters
bool flexflow_parameter_set_weights_float(flexflow_parameter_t h, flexflow_model_t m, int num_dim, int* dims,
                                          const float* data) {
  FF_BOOL("param_set", "(OONN)", obj(h.impl), obj(m.impl), int_list(dims, dims ? num_dim : 0),
          PyLong_FromVoidPtr(const_cast<float*>(data)));
}
bool flexflow_parameter_get_weights_float(flexflow_parameter_t h, flexflow_model_t m, float* data) {
  FF_BOOL("param_get", "(OON)", obj(h.impl), obj(m.impl), PyLong_FromVoidPtr(data));
}

// -------------------------------------------------------------------------------- optimizers
flexflow_sgd_optimizer_t flexflow_sgd_optimizer_create(flexflow_model_t m, double lr, double momentum, bool nesterov,
                                                       double wd) {
  FF_HANDLE(flexflow_sgd_optimizer_t, "sgd_create", "(Oddid)", obj(m.impl), lr, momentum, (int)nesterov, wd);
}
void flexflow_sgd_optimizer_destroy(flexflow_sgd_optimizer_t h) { drop(h.impl); }
void flexflow_sgd_optimizer_set_lr(flexflow_sgd_optimizer_t h, double lr) {
  FF_VOID("optimizer_set_lr", "(Od)", obj(h.impl), lr);
}
flexflow_adam_optimizer_t flexflow_adam_optimizer_create(flexflow_model_t m, double alpha, double b1, double b2,
                                                         double wd, double eps) {
  FF_HANDLE(flexflow_adam_optimizer_t, "adam_create", "(Oddddd)", obj(m.impl), alpha, b1, b2, wd, eps);
}
void flexflow_adam_optimizer_destroy(flexflow_adam_optimizer_t h) { drop(h.impl); }
void flexflow_adam_optimizer_set_lr(flexflow_adam_optimizer_t h, double lr) {
  FF_VOID("optimizer_set_lr", "(Od)", obj(h.impl), lr);
}

// ------------------------------------------------------------------------------ initializers
flexflow_initializer_t flexflow_initializer_create_null(void) {
  flexflow_initializer_t h;
  h.impl = nullptr;  // builders read a null handle as "the op's default initializer"
  return h;
}
flexflow_glorot_uniform_initializer_t flexflow_glorot_uniform_initializer_create(int seed) {
  FF_HANDLE(flexflow_glorot_uniform_initializer_t, "init_create", "(sidd)", "glorot", seed, 0.0, 0.0);
}
void flexflow_glorot_uniform_initializer_destroy(flexflow_glorot_uniform_initializer_t h) { drop(h.impl); }
flexflow_zero_initializer_t flexflow_zero_initializer_create(void) {
  FF_HANDLE(flexflow_zero_initializer_t, "init_create", "(sidd)", "zero", 0, 0.0, 0.0);
}
void flexflow_zero_initializer_destroy(flexflow_zero_initializer_t h) { drop(h.impl); }
flexflow_uniform_initializer_t flexflow_uniform_initializer_create(int seed, float mn, float mx) {
  FF_HANDLE(flexflow_uniform_initializer_t, "init_create", "(sidd)", "uniform", seed, (double)mn, (double)mx);
}
void flexflow_uniform_initializer_destroy(flexflow_uniform_initializer_t h) { drop(h.impl); }
flexflow_norm_initializer_t flexflow_norm_initializer_create(int seed, float mean, float stddev) {
  FF_HANDLE(flexflow_norm_initializer_t, "init_create", "(sidd)", "norm", seed, (double)mean, (double)stddev);
}
void flexflow_norm_initializer_destroy(flexflow_norm_initializer_t h) { drop(h.impl); }

// ------------------------------------------------------------------------------- PerfMetrics
void flexflow_per_metrics_destroy(flexflow_perf_metrics_t h) { drop(h.impl); }
float flexflow_per_metrics_get_accuracy(flexflow_perf_metrics_t h) {
  FF_ENTRY;
  return (float)to_double(call("perf_get", "(Oi)", obj(h.impl), 0), -1.0);
}
float flexflow_per_metrics_get_loss(flexflow_perf_metrics_t h) {
  FF_ENTRY;
  return (float)to_double(call("perf_get", "(Oi)", obj(h.impl), 1), -1.0);
}

// --------------------------------------------------------------------------- example configs
flexflow_net_config_t flexflow_net_config_create(void) { FF_HANDLE(flexflow_net_config_t, "net_config_create", "()"); }
void flexflow_net_config_destroy(flexflow_net_config_t h) {
  forget(h.impl);
  drop(h.impl);
}
const char* flexflow_net_config_get_dataset_path(flexflow_net_config_t h) {
  FF_ENTRY;
  return cached_str(h.impl, "dataset_path", call("obj_attr", "(Os)", obj(h.impl), "dataset_path"));
}
flexflow_dlrm_config_t flexflow_dlrm_config_create(void) {
  FF_HANDLE(flexflow_dlrm_config_t, "dlrm_config_create", "()");
}
void flexflow_dlrm_config_destroy(flexflow_dlrm_config_t h) {
  forget(h.impl);
  drop(h.impl);
}
static const char* dlrm_str(flexflow_dlrm_config_t h, const char* key) {
  FF_ENTRY;
  return cached_str(h.impl, key, call("obj_attr", "(Os)", obj(h.impl), key));
}
static int dlrm_int(flexflow_dlrm_config_t h, const char* key) { FF_INT("obj_attr", "(Os)", obj(h.impl), key); }
static int* dlrm_ints(flexflow_dlrm_config_t h, const char* key) {
  FF_ENTRY;
  return cached_ints(h.impl, key, call("obj_attr", "(Os)", obj(h.impl), key), true);
}
const char* flexflow_dlrm_config_get_dataset_path(flexflow_dlrm_config_t h) { return dlrm_str(h, "dataset_path"); }
const char* flexflow_dlrm_config_get_arch_interaction_op(flexflow_dlrm_config_t h) {
  return dlrm_str(h, "arch_interaction_op");
}
int flexflow_dlrm_config_get_sparse_feature_size(flexflow_dlrm_config_t h) {
  return dlrm_int(h, "sparse_feature_size");
}
int flexflow_dlrm_config_get_sigmoid_bot(flexflow_dlrm_config_t h) { return dlrm_int(h, "sigmoid_bot"); }
int flexflow_dlrm_config_get_sigmoid_top(flexflow_dlrm_config_t h) { return dlrm_int(h, "sigmoid_top"); }
int flexflow_dlrm_config_get_embedding_bag_size(flexflow_dlrm_config_t h) {
  return dlrm_int(h, "embedding_bag_size");
}
float flexflow_dlrm_config_get_loss_threshold(flexflow_dlrm_config_t h) {
  FF_ENTRY;
  return (float)to_double(call("obj_attr", "(Os)", obj(h.impl), "loss_threshold"), 0.0);
}
int* flexflow_dlrm_config_get_mlp_bot(flexflow_dlrm_config_t h) { return dlrm_ints(h, "mlp_bot"); }
int* flexflow_dlrm_config_get_mlp_top(flexflow_dlrm_config_t h) { return dlrm_ints(h, "mlp_top"); }
int* flexflow_dlrm_config_get_embedding_size(flexflow_dlrm_config_t h) { return dlrm_ints(h, "embedding_size"); }

// ---------------------------------------------------------------------------- data loaders
flexflow_single_dataloader_t flexflow_single_dataloader_create(flexflow_model_t m, flexflow_tensor_t input,
                                                               flexflow_tensor_t full, int num, int data_type) {
  FF_HANDLE(flexflow_single_dataloader_t, "dataloader_create", "(OOOii)", obj(m.impl), obj(input.impl),
            obj(full.impl), num, data_type);
}
flexflow_single_dataloader_t flexflow_single_dataloader_create2(flexflow_model_t m, flexflow_tensor_t input,
                                                                void* full_ptr, int num, int data_type) {
  FF_HANDLE(flexflow_single_dataloader_t, "dataloader_create_ptr", "(OONii)", obj(m.impl), obj(input.impl),
            PyLong_FromVoidPtr(full_ptr), num, data_type);
}
void flexflow_single_dataloader_destroy(flexflow_single_dataloader_t h) { drop(h.impl); }
void flexflow_single_dataloader_set_num_samples(flexflow_single_dataloader_t h, int n) {
  FF_VOID("dataloader_set_num", "(Oi)", obj(h.impl), n);
}
int flexflow_single_dataloader_get_num_samples(flexflow_single_dataloader_t h) {
  FF_INT("dataloader_get_num", "(O)", obj(h.impl));
}
void flexflow_single_dataloader_reset(flexflow_single_dataloader_t h) {
  FF_VOID("dataloader_reset", "(O)", obj(h.impl));
}
void flexflow_single_dataloader_next_batch(flexflow_single_dataloader_t h, flexflow_model_t m) {
  FF_VOID("dataloader_next", "(OO)", obj(h.impl), obj(m.impl));
}

// ------------------------------------------------------------------- timing / tracing / ops
double flexflow_get_current_time(flexflow_config_t c) {
  FF_ENTRY;
  return to_double(call("current_time_us", "(O)", obj(c.impl)), 0.0);
}
void flexflow_begin_trace(flexflow_config_t c, int id) { FF_VOID("trace", "(Oii)", obj(c.impl), id, 1); }
void flexflow_end_trace(flexflow_config_t c, int id) { FF_VOID("trace", "(Oii)", obj(c.impl), id, 0); }
int flexflow_op_get_num_parameters(flexflow_op_t h) { FF_INT("op_count", "(Oi)", obj(h.impl), 0); }
flexflow_tensor_t flexflow_op_get_parameter_by_id(flexflow_op_t h, int id) {
  FF_HANDLE(flexflow_tensor_t, "op_item", "(Oii)", obj(h.impl), 0, id);
}
int flexflow_op_get_num_inputs(flexflow_op_t h) { FF_INT("op_count", "(Oi)", obj(h.impl), 1); }
flexflow_tensor_t flexflow_op_get_input_by_id(flexflow_op_t h, int id) {
  FF_HANDLE(flexflow_tensor_t, "op_item", "(Oii)", obj(h.impl), 1, id);
}
int flexflow_op_get_num_outputs(flexflow_op_t h) { FF_INT("op_count", "(Oi)", obj(h.impl), 2); }
flexflow_tensor_t flexflow_op_get_output_by_id(flexflow_op_t h, int id) {
  FF_HANDLE(flexflow_tensor_t, "op_item", "(Oii)", obj(h.impl), 2, id);
}
void flexflow_op_init(flexflow_op_t h, flexflow_model_t m) { FF_VOID("op_run", "(OOi)", obj(h.impl), obj(m.impl), 0); }
void flexflow_op_forward(flexflow_op_t h, flexflow_model_t m) {
  FF_VOID("op_run", "(OOi)", obj(h.impl), obj(m.impl), 1);
}
void flexflow_op_destroy(flexflow_op_t h) { drop(h.impl); }
void flexflow_perform_registration(void) { init_once(); }

// ------------------------------------------------------------------------- extension layers
flexflow_tensor_t flexflow_model_add_embedding_typed(flexflow_model_t h, flexflow_tensor_t x, int num, int dim,
                                                     int aggr, int data_type, const char* name) {
  FF_HANDLE(flexflow_tensor_t, "add_embedding_typed", "(OOiiiiz)", obj(h.impl), obj(x.impl), num, dim, aggr, data_type,
            name);
}
flexflow_tensor_t flexflow_model_add_cast(flexflow_model_t h, flexflow_tensor_t x, int data_type, const char* name) {
  FF_HANDLE(flexflow_tensor_t, "add_cast", "(OOiz)", obj(h.impl), obj(x.impl), data_type, name);
}
flexflow_tensor_t flexflow_model_add_rms_norm(flexflow_model_t h, flexflow_tensor_t x, float eps, const char* name) {
  FF_HANDLE(flexflow_tensor_t, "add_rms_norm", "(OOdz)", obj(h.impl), obj(x.impl), (double)eps, name);
}
int flexflow_model_add_top_k(flexflow_model_t h, flexflow_tensor_t x, int k, bool sorted, flexflow_tensor_t* outputs,
                             const char* name) {
  FF_ENTRY;
  return unpack(call("add_top_k", "(OOiiz)", obj(h.impl), obj(x.impl), k, (int)sorted, name), outputs, 2);
}
int flexflow_model_add_group_by(flexflow_model_t h, flexflow_tensor_t data, flexflow_tensor_t assign, int n,
                                float alpha, flexflow_tensor_t* outputs, const char* name) {
  FF_ENTRY;
  return unpack(call("add_group_by", "(OOOidz)", obj(h.impl), obj(data.impl), obj(assign.impl), n, (double)alpha, name),
                outputs, n);
}
static flexflow_tensor_t aggregate(flexflow_model_t h, int ni, const flexflow_tensor_t* xs, int n, float lam, int spec,
                                   const char* name) {
  FF_HANDLE(flexflow_tensor_t, "add_aggregate", "(ONidiz)", obj(h.impl), tensor_list(ni, xs), n, (double)lam, spec,
            name);
}
flexflow_tensor_t flexflow_model_add_aggregate(flexflow_model_t h, int ni, const flexflow_tensor_t* xs, int n, float lam,
                                               const char* name) {
  return aggregate(h, ni, xs, n, lam, 0, name);
}
flexflow_tensor_t flexflow_model_add_aggregate_spec(flexflow_model_t h, int ni, const flexflow_tensor_t* xs, int n,
                                                    float lam, const char* name) {
  return aggregate(h, ni, xs, n, lam, 1, name);
}
flexflow_tensor_t flexflow_model_add_moe(flexflow_model_t h, flexflow_tensor_t x, int num_exp, int num_select,
                                         int hidden, float alpha, float lambda_bal) {
  FF_HANDLE(flexflow_tensor_t, "add_moe", "(OOiiidd)", obj(h.impl), obj(x.impl), num_exp, num_select, hidden,
            (double)alpha, (double)lambda_bal);
}

}  // extern "C"
