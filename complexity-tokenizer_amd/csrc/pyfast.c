/* complexity_tokenizer._fast: the Python-object edges of encode_batch (the reference's PyO3
 * `Vec<String>` extraction and `Vec<Vec<u32>>` return, src/bindings/tokenizer.rs:203-210) in C.
 *
 *   pack(texts) -> (bytearray text + 16 zero bytes, bytes of uint64 offsets[D+1])
 *       one pass over the sequence: PyUnicode_AsUTF8AndSize hands out each str's cached UTF-8
 *       (no copy for ASCII strs), then one memcpy per text into the batch buffer.
 *   split(ids_addr, off_addr, n_docs, cache[, threads]) -> list[list[int]]
 *       ids: uint32[T], off: uint64[D+1] (host addresses); cache: a list whose item i is the int i
 *       for every id of the vocabulary, so no int object is allocated per id (ints are immutable:
 *       sharing them is invisible to the caller); ids past the cache are created.  The rows'
 *       items are filled on `threads` threads (see fast_split).
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

/* split: the rows are allocated here (Python API, GIL held), every cached int's reference count
 * is raised once by its number of uses (a histogram of the ids, over threads), and the rows'
 * item pointers are then filled by plain stores on `threads` threads -- no per-id Py_INCREF, no
 * Python API outside this thread.  Ids past the cache (ids >= len(cache): never for a cache
 * covering the vocabulary) take the serial path with a new int per use. */
#include <pthread.h>

typedef struct {
  const uint32_t* ids;
  const uint64_t* off;
  PyObject* out;
  PyObject** table;
  uint32_t* hist; /* this thread's histogram (nc entries), or NULL in the fill phase */
  Py_ssize_t d0, d1, nc;
  int big;        /* an id >= nc was seen */
} split_job;

static void* split_hist(void* p) {
  split_job* j = (split_job*)p;
  const uint64_t a = j->off[j->d0], b = j->off[j->d1];
  for (uint64_t k = a; k < b; k++) {
    const uint32_t v = j->ids[k];
    if ((Py_ssize_t)v < j->nc) j->hist[v]++;
    else j->big = 1;
  }
  return NULL;
}

static void* split_fill(void* p) {
  split_job* j = (split_job*)p;
  for (Py_ssize_t d = j->d0; d < j->d1; d++) {
    PyObject** it = ((PyListObject*)PyList_GET_ITEM(j->out, d))->ob_item;
    const uint64_t a = j->off[d], b = j->off[d + 1];
    for (uint64_t k = a; k < b; k++) it[k - a] = j->table[j->ids[k]];
  }
  return NULL;
}

static int run_jobs(split_job* jobs, int nt, void* (*fn)(void*)) {
  pthread_t th[64];
  int started = 0;
  for (int t = 1; t < nt; t++) {
    if (pthread_create(&th[t], NULL, fn, &jobs[t]) != 0) break;
    started = t;
  }
  fn(&jobs[0]);
  for (int t = started + 1; t < nt; t++) fn(&jobs[t]);  /* (threads that could not start) */
  for (int t = 1; t <= started; t++) pthread_join(th[t], NULL);
  return 0;
}

static PyObject* split_serial(const uint32_t* ids, const uint64_t* off, Py_ssize_t n, PyObject* cache) {
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

static PyObject* fast_split(PyObject* self, PyObject* args) {
  (void)self;
  unsigned long long ids_addr, off_addr;
  Py_ssize_t n;
  PyObject* cache;
  int threads = 1;
  if (!PyArg_ParseTuple(args, "KKnO!|i", &ids_addr, &off_addr, &n, &PyList_Type, &cache, &threads)) return NULL;
  const uint32_t* ids = (const uint32_t*)(uintptr_t)ids_addr;
  const uint64_t* off = (const uint64_t*)(uintptr_t)off_addr;
  const Py_ssize_t nc = PyList_GET_SIZE(cache);
  const uint64_t T = n > 0 ? off[n] : 0;
  if (T < 65536) return split_serial(ids, off, n, cache);  /* (small batches: no histogram to clear) */
#ifdef Py_GIL_DISABLED
  /* free-threaded CPython: the shared int objects' reference counts may be changed by other
   * threads meanwhile, and Py_SET_REFCNT below is not atomic there -- one Py_NewRef per item */
  return split_serial(ids, off, n, cache);
#endif
  /* (per-thread histogram counts are u32: a call holds < 2^32 ids, off[n] < 3.75 GiB of text) */
  if (threads < 1) threads = 1;
  if (threads > 64) threads = 64;
  if (n < (Py_ssize_t)threads) threads = 1;
  /* docs split over the threads by ids (balanced work) */
  split_job jobs[64];
  memset(jobs, 0, sizeof(jobs));
  {
    Py_ssize_t d = 0;
    for (int t = 0; t < threads; t++) {
      const uint64_t target = T * (uint64_t)(t + 1) / (uint64_t)threads;
      jobs[t].d0 = d;
      while (d < n && (t == threads - 1 || off[d + 1] <= target)) d++;
      jobs[t].d1 = t == threads - 1 ? n : d;
      jobs[t].ids = ids;
      jobs[t].off = off;
      jobs[t].nc = nc;
    }
  }
  uint32_t* hist = (uint32_t*)PyMem_Calloc((size_t)threads * (size_t)(nc ? nc : 1), sizeof(uint32_t));
  if (!hist) return PyErr_NoMemory();
  for (int t = 0; t < threads; t++) jobs[t].hist = hist + (size_t)t * (size_t)nc;
  Py_BEGIN_ALLOW_THREADS
  run_jobs(jobs, threads, split_hist);
  Py_END_ALLOW_THREADS
  int big = 0;
  for (int t = 0; t < threads; t++) big |= jobs[t].big;
  if (big) {  /* ids past the cache: the serial path */
    PyMem_Free(hist);
    return split_serial(ids, off, n, cache);
  }
  PyObject** table = (PyObject**)PyMem_Malloc((size_t)(nc ? nc : 1) * sizeof(PyObject*));
  if (!table) { PyMem_Free(hist); return PyErr_NoMemory(); }
  for (Py_ssize_t i = 0; i < nc; i++) table[i] = PyList_GET_ITEM(cache, i);
  PyObject* out = PyList_New(n);
  if (!out) { PyMem_Free(hist); PyMem_Free(table); return NULL; }
  for (Py_ssize_t d = 0; d < n; d++) {  /* rows with NULL items: safe to free on an error */
    PyObject* row = PyList_New((Py_ssize_t)(off[d + 1] - off[d]));
    if (!row) { Py_DECREF(out); PyMem_Free(hist); PyMem_Free(table); return NULL; }
    PyList_SET_ITEM(out, d, row);
  }
  /* every use's reference, taken at once (the histogram), then the plain pointer stores */
  for (Py_ssize_t i = 0; i < nc; i++) {
    Py_ssize_t c = 0;
    for (int t = 0; t < threads; t++) c += hist[(size_t)t * (size_t)nc + (size_t)i];
    if (c) Py_SET_REFCNT(table[i], Py_REFCNT(table[i]) + c);
  }
  PyMem_Free(hist);
  for (int t = 0; t < threads; t++) {
    jobs[t].out = out;
    jobs[t].table = table;
  }
  run_jobs(jobs, threads, split_fill);  /* (GIL held: the rows are not visible to anyone yet) */
  PyMem_Free(table);
  return out;
}

static PyMethodDef methods[] = {
    {"pack", fast_pack, METH_O, "list[str] -> (bytearray utf-8 + 16 pad bytes, bytes uint64 offsets)"},
    {"split", fast_split, METH_VARARGS, "(ids addr, offsets addr, n_docs, int cache[, threads]) -> list[list[int]]"},
    {NULL, NULL, 0, NULL}};

static struct PyModuleDef module = {PyModuleDef_HEAD_INIT, "_fast", NULL, -1, methods, NULL, NULL, NULL, NULL};

PyMODINIT_FUNC PyInit__fast(void) { return PyModule_Create(&module); }
