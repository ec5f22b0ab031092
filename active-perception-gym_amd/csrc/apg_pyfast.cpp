// apg_pyfast.cpp — CPython METH_FASTCALL entry points for the C-ABI calls made once per env step.
//
// The eager step of a vector env is one C-ABI call (apg_lidar_step / apg_image_step / apg_light_dark_step).  Through
// ctypes, marshalling its 6-8 arguments costs ~2.5 us per call (measured in this container: 2.94 us for an
// apg_image_step that returns at validate(), 0.39 us for a call without arguments), a quarter of the image env's
// host time per step, and the MNIST step loop is host-bound (10 us of host per 12 us kernel).  These wrappers take
// the same arguments as plain Python ints (struct addresses, device pointers, the raw stream) and call the C ABI
// directly, without the GIL, like ctypes does.  Host code only; links libapgym_hip.so next to it ($ORIGIN).
#define PY_SSIZE_T_CLEAN
#include <Python.h>

#include "apgym_capi.h"

namespace {

bool addr_args(PyObject *const *args, const int *which, int count, void **out) {
  for (int i = 0; i < count; i++) {
    out[i] = PyLong_AsVoidPtr(args[which[i]]);
    if (out[i] == nullptr && PyErr_Occurred()) return false;
  }
  return true;
}

bool nargs_ok(Py_ssize_t n, Py_ssize_t want, const char *name) {
  if (n == want) return true;
  PyErr_Format(PyExc_TypeError, "%s takes %zd arguments (%zd given)", name, want, n);
  return false;
}

// lidar_step(cfg, state, action, prediction, outputs, stream) -> rc    (apg_lidar_step)
PyObject *lidar_step(PyObject *, PyObject *const *args, Py_ssize_t n) {
  if (!nargs_ok(n, 6, "lidar_step")) return nullptr;
  static const int w[6] = {0, 1, 2, 3, 4, 5};
  void *v[6];
  if (!addr_args(args, w, 6, v)) return nullptr;
  int rc;
  Py_BEGIN_ALLOW_THREADS
  rc = apg_lidar_step(static_cast<const apg_lidar_config *>(v[0]), static_cast<const apg_lidar_state *>(v[1]),
                      static_cast<const float *>(v[2]), static_cast<const float *>(v[3]),
                      static_cast<const apg_lidar_outputs *>(v[4]), v[5]);
  Py_END_ALLOW_THREADS
  return PyLong_FromLong(rc);
}

// image_step(cfg, state, action, prediction, t, flags, outputs, stream) -> rc    (apg_image_step)
PyObject *image_step(PyObject *, PyObject *const *args, Py_ssize_t n) {
  if (!nargs_ok(n, 8, "image_step")) return nullptr;
  static const int w[6] = {0, 1, 2, 3, 6, 7};
  void *v[6];
  if (!addr_args(args, w, 6, v)) return nullptr;
  const long t = PyLong_AsLong(args[4]), flags = PyLong_AsLong(args[5]);
  if (PyErr_Occurred()) return nullptr;
  int rc;
  Py_BEGIN_ALLOW_THREADS
  rc = apg_image_step(static_cast<const apg_image_config *>(v[0]), static_cast<const apg_image_state *>(v[1]),
                      static_cast<const float *>(v[2]), static_cast<const float *>(v[3]), (int32_t)t, (int32_t)flags,
                      static_cast<const apg_image_outputs *>(v[4]), v[5]);
  Py_END_ALLOW_THREADS
  return PyLong_FromLong(rc);
}

// light_dark_step(cfg, state, action, prediction, outputs, stream) -> rc    (apg_light_dark_step)
PyObject *light_dark_step(PyObject *, PyObject *const *args, Py_ssize_t n) {
  if (!nargs_ok(n, 6, "light_dark_step")) return nullptr;
  static const int w[6] = {0, 1, 2, 3, 4, 5};
  void *v[6];
  if (!addr_args(args, w, 6, v)) return nullptr;
  int rc;
  Py_BEGIN_ALLOW_THREADS
  rc = apg_light_dark_step(static_cast<const apg_light_dark_config *>(v[0]),
                           static_cast<const apg_light_dark_state *>(v[1]), static_cast<const float *>(v[2]),
                           static_cast<const float *>(v[3]), static_cast<const apg_light_dark_outputs *>(v[4]), v[5]);
  Py_END_ALLOW_THREADS
  return PyLong_FromLong(rc);
}

PyMethodDef kMethods[] = {
    {"lidar_step", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)(void)>(lidar_step)), METH_FASTCALL,
     "apg_lidar_step(cfg, state, action, prediction, outputs, stream) with addresses as ints"},
    {"image_step", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)(void)>(image_step)), METH_FASTCALL,
     "apg_image_step(cfg, state, action, prediction, t, flags, outputs, stream) with addresses as ints"},
    {"light_dark_step", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)(void)>(light_dark_step)),
     METH_FASTCALL, "apg_light_dark_step(cfg, state, action, prediction, outputs, stream) with addresses as ints"},
    {nullptr, nullptr, 0, nullptr}};

PyModuleDef kModule = {PyModuleDef_HEAD_INIT, "_apgfast", "fast-call entry points of libapgym_hip.so", -1, kMethods,
                       nullptr, nullptr, nullptr, nullptr};

}  // namespace

PyMODINIT_FUNC PyInit__apgfast(void) { return PyModule_Create(&kModule); }
