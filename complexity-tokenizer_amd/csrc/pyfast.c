/* complexity_tokenizer._fast: the Python-object edges of encode_batch (the reference's PyO3
 * `Vec<String>` extraction and `Vec<Vec<u32>>` return, src/bindings/tokenizer.rs:203-210) in C.
 *
 *   pack(texts) -> (bytearray text + 16 zero bytes, bytes of uint64 offsets[D+1])
 *       one pass over the sequence: PyUnicode_AsUTF8AndSize hands out each str's cached UTF-8
 *       (no copy for ASCII strs), then one memcpy per text into the batch buffer.
 *   split(ids_addr, off_addr, n_docs, cache) -> list[list[int]]
 *       ids: uint32[T], off: uint64[D+1] (host addresses); cache: a list whose item i is the int i
 *       for every id of the vocabulary, so no int object is allocated per id (ints are immutable:
 *       sharing them is invisible to the caller); ids past the cache are created.
 * Errors follow pack_texts in __init__.py (TypeError with PyO3's messages).
 */
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#include <stdint.h>
#include <string.h>

static PyObject* fast_pack(PyObject* self, PyObject* arg) {
  (void)self;
  if (PyUnicode_Check(arg) || PyBytes_Check(arg)) {
    PyErr_SetString(PyExc_TypeError, "Can't extract `str` to `Vec`");
    return NULL;
  }
  PyObject* seq = PySequence_Fast(arg, "'object' cannot be converted to 'Sequence'");
  if (!seq) return NULL;
  const Py_ssize_t n = PySequence_Fast_GET_SIZE(seq);
  PyObject** items = PySequence_Fast_ITEMS(seq);
  PyObject* offs = PyBytes_FromStringAndSize(NULL, (n + 1) * (Py_ssize_t)sizeof(uint64_t));
  if (!offs) { Py_DECREF(seq); return NULL; }
  uint64_t* off = (uint64_t*)PyBytes_AS_STRING(offs);
  const char** ptr = (const char**)PyMem_Malloc((n ? n : 1) * sizeof(char*));
  if (!ptr) { Py_DECREF(seq); Py_DECREF(offs); return PyErr_NoMemory(); }
  off[0] = 0;
  for (Py_ssize_t i = 0; i < n; i++) {
    PyObject* t = items[i];
    if (!PyUnicode_Check(t)) {
      PyErr_Format(PyExc_TypeError, "'%.200s' object cannot be converted to 'PyString'", Py_TYPE(t)->tp_name);
      PyMem_Free(ptr); Py_DECREF(seq); Py_DECREF(offs);
      return NULL;
    }
    Py_ssize_t len = 0;
    ptr[i] = PyUnicode_AsUTF8AndSize(t, &len);
    if (!ptr[i]) { PyMem_Free(ptr); Py_DECREF(seq); Py_DECREF(offs); return NULL; }  /* lone surrogates */
    off[i + 1] = off[i] + (uint64_t)len;
  }
  PyObject* buf = PyByteArray_FromStringAndSize(NULL, (Py_ssize_t)off[n] + 16);
  if (!buf) { PyMem_Free(ptr); Py_DECREF(seq); Py_DECREF(offs); return NULL; }
  char* dst = PyByteArray_AS_STRING(buf);
  for (Py_ssize_t i = 0; i < n; i++) memcpy(dst + off[i], ptr[i], off[i + 1] - off[i]);
  memset(dst + off[n], 0, 16);
  PyMem_Free(ptr);
  Py_DECREF(seq);
  PyObject* r = PyTuple_Pack(2, buf, offs);
  Py_DECREF(buf);
  Py_DECREF(offs);
  return r;
}

static PyObject* fast_split(PyObject* self, PyObject* args) {
  (void)self;
  unsigned long long ids_addr, off_addr;
  Py_ssize_t n;
  PyObject* cache;
  if (!PyArg_ParseTuple(args, "KKnO!", &ids_addr, &off_addr, &n, &PyList_Type, &cache)) return NULL;
  const uint32_t* ids = (const uint32_t*)(uintptr_t)ids_addr;
  const uint64_t* off = (const uint64_t*)(uintptr_t)off_addr;
  const Py_ssize_t nc = PyList_GET_SIZE(cache);
  PyObject* out = PyList_New(n);
  if (!out) return NULL;
  for (Py_ssize_t d = 0; d < n; d++) {
    const uint64_t a = off[d], b = off[d + 1];
    PyObject* row = PyList_New((Py_ssize_t)(b - a));
    if (!row) { Py_DECREF(out); return NULL; }
    for (uint64_t k = a; k < b; k++) {
      const uint32_t v = ids[k];
      PyObject* o;
      if ((Py_ssize_t)v < nc) {
        o = PyList_GET_ITEM(cache, v);
        Py_INCREF(o);
      } else {
        o = PyLong_FromUnsignedLong(v);
        if (!o) { Py_DECREF(row); Py_DECREF(out); return NULL; }
      }
      PyList_SET_ITEM(row, (Py_ssize_t)(k - a), o);
    }
    PyList_SET_ITEM(out, d, row);
  }
  return out;
}

static PyMethodDef methods[] = {
    {"pack", fast_pack, METH_O, "list[str] -> (bytearray utf-8 + 16 pad bytes, bytes uint64 offsets)"},
    {"split", fast_split, METH_VARARGS, "(ids addr, offsets addr, n_docs, int cache) -> list[list[int]]"},
    {NULL, NULL, 0, NULL}};

static struct PyModuleDef module = {PyModuleDef_HEAD_INIT, "_fast", NULL, -1, methods, NULL, NULL, NULL, NULL};

PyMODINIT_FUNC PyInit__fast(void) { return PyModule_Create(&module); }
