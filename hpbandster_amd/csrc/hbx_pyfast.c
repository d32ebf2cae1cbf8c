/* _hbxfast: the drop-in's one-bracket promotion call (promote.advance_mask) without the ctypes hop.
 *
 * HpBandSter's process_results ranks ONE bracket per call (HB_iteration.py:179-182); on the GPU that call
 * is launch-bound (~11 us), so the ~1.2 us a ctypes call with numpy pointer lookups and two numpy slice
 * copies adds is a tenth of it.  This CPython module takes the losses and the output mask through the
 * buffer protocol, copies them to / from the mapped buffers of the caller's staging and calls libhbx's
 * hbx_sh_advance_state (its address handed over once from ctypes: no link-time dependency), with the GIL
 * released while the host spins on the kernel's completion word.  Host marshalling only: the ranking is
 * the GPU kernel's, whatever path reaches it.
 */
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#include <stdint.h>
#include <string.h>

typedef int (*advance_state_fn)(int64_t* state, int64_t n, double k, void* stream);
static advance_state_fn g_advance = NULL;

static PyObject* set_entry(PyObject* self, PyObject* args) {
  unsigned long long addr = 0;
  if (!PyArg_ParseTuple(args, "K", &addr)) return NULL;
  g_advance = (advance_state_fn)(uintptr_t)addr;
  Py_RETURN_NONE;
}

static int is_f64(const Py_buffer* b) {
  const char* f = b->format ? b->format : "B";
  if (*f == '<' || *f == '=' || *f == '@') ++f;
  return b->itemsize == 8 && f[0] == 'd' && f[1] == 0;
}

static int is_u8(const Py_buffer* b) {
  const char* f = b->format ? b->format : "B";
  if (*f == '<' || *f == '=' || *f == '@' || *f == '|') ++f;
  return b->itemsize == 1 && (f[0] == '?' || f[0] == 'B' || f[0] == 'b') && f[1] == 0;
}

/* advance(state_addr, cap, losses, mask, k, stream) -> rc: 0 ok; 1 the buffers do not fit this path (the
 * caller takes the ctypes one); < 0 libhbx's error code.  state = hbx_sh_advance_state's int64[6] block
 * {pin, pout, done, scratch, order_mode, seq}; cap = the mapped buffers' capacity in configurations. */
static PyObject* advance(PyObject* self, PyObject* args) {
  unsigned long long state_addr = 0, stream = 0;
  long long cap = 0;
  PyObject *losses = NULL, *mask = NULL;
  double k = 0.0;
  if (!PyArg_ParseTuple(args, "KLOOdK", &state_addr, &cap, &losses, &mask, &k, &stream)) return NULL;
  if (!g_advance) {
    PyErr_SetString(PyExc_RuntimeError, "_hbxfast: set_entry() was not called");
    return NULL;
  }
  Py_buffer lb, mb;
  if (PyObject_GetBuffer(losses, &lb, PyBUF_C_CONTIGUOUS | PyBUF_FORMAT) != 0) {
    PyErr_Clear();
    return PyLong_FromLong(1);
  }
  if (PyObject_GetBuffer(mask, &mb, PyBUF_C_CONTIGUOUS | PyBUF_FORMAT | PyBUF_WRITABLE) != 0) {
    PyErr_Clear();
    PyBuffer_Release(&lb);
    return PyLong_FromLong(1);
  }
  const Py_ssize_t n = lb.ndim == 1 ? lb.shape[0] : -1;
  int rc = 1;
  if (n > 0 && n <= cap && is_f64(&lb) && is_u8(&mb) && mb.ndim == 1 && mb.shape[0] == n) {
    int64_t* st = (int64_t*)(uintptr_t)state_addr;
    memcpy((void*)(uintptr_t)st[0], lb.buf, (size_t)n * 8);
    Py_BEGIN_ALLOW_THREADS
    rc = g_advance(st, (int64_t)n, k, (void*)(uintptr_t)stream);
    if (rc == 0) memcpy(mb.buf, (const void*)(uintptr_t)st[1], (size_t)n);
    Py_END_ALLOW_THREADS
  }
  PyBuffer_Release(&mb);
  PyBuffer_Release(&lb);
  return PyLong_FromLong(rc);
}

static PyMethodDef methods[] = {
    {"set_entry", set_entry, METH_VARARGS, "set_entry(address of hbx_sh_advance_state)"},
    {"advance", advance, METH_VARARGS, "advance(state_addr, cap, losses, mask, k, stream) -> rc"},
    {NULL, NULL, 0, NULL}};

static struct PyModuleDef module = {PyModuleDef_HEAD_INIT, "_hbxfast", NULL, -1, methods};

PyMODINIT_FUNC PyInit__hbxfast(void) { return PyModule_Create(&module); }
