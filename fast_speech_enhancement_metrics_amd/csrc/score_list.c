/* The drop-in call's result list, built natively: score_list(scores, keys) -> list of dicts.
 *
 * `scores` is a C-contiguous float32 (or float64: the CPU path's) buffer of K x B values (K
 * metrics, one row each; on the GPU path the [3, B] PESQ / STOI / ESTOI block copied once from
 * the device) and `keys` a tuple of K str.
 * Returns [{keys[0]: scores[0][b], ..., keys[K-1]: scores[K-1][b]} for b in range(B)] -- the
 * list the reference's BaseMetric.__call__ returns (fast_se_metrics/base.py, list of
 * dict[str, float]), with the same values as tensor.tolist().
 *
 * Host-side runtime code (no GPU): the Python equivalent, a dict display per row over
 * tensor.tolist(), costs about 80 ns per row on the MI355X box's host (profiles/r3_a/dropin.json,
 * 0.33 ms of an 8.6 ms call at B = 4096); this builds each dict with the key hashes cached and
 * never materialises the K intermediate lists.  Optional: where it cannot be built or loaded
 * (no C compiler or Python headers, a read-only package directory), _native.score_list falls
 * back to the Python form with the same result.
 */
#define PY_SSIZE_T_CLEAN
#include <Python.h>

static PyObject *score_list(PyObject *self, PyObject *args) {
  (void)self;
  PyObject *buf_obj, *keys;
  if (!PyArg_ParseTuple(args, "OO!", &buf_obj, &PyTuple_Type, &keys)) return NULL;
  const Py_ssize_t K = PyTuple_GET_SIZE(keys);
  if (K <= 0) {
    PyErr_SetString(PyExc_ValueError, "score_list: keys must be a non-empty tuple");
    return NULL;
  }
  for (Py_ssize_t k = 0; k < K; ++k) {
    PyObject *key = PyTuple_GET_ITEM(keys, k);
    if (!PyUnicode_Check(key)) {
      PyErr_SetString(PyExc_TypeError, "score_list: keys must be str");
      return NULL;
    }
    if (PyObject_Hash(key) == -1) return NULL; /* cache the hash once */
  }
  Py_buffer view;
  if (PyObject_GetBuffer(buf_obj, &view, PyBUF_C_CONTIGUOUS | PyBUF_FORMAT) != 0) return NULL;
  PyObject *out = NULL;
  const char *fmt = view.format ? view.format : "";
  if (*fmt == '<' || *fmt == '=' || *fmt == '@') ++fmt;
  const int f64 = fmt[0] == 'd' && fmt[1] == 0 && view.itemsize == 8;
  if (!(f64 || (fmt[0] == 'f' && fmt[1] == 0 && view.itemsize == 4)) || view.len % (K * view.itemsize) != 0) {
    PyErr_SetString(PyExc_TypeError, "score_list: scores must be a contiguous float32 / float64 buffer of K x B values");
    goto done;
  }
  const Py_ssize_t B = view.len / (K * view.itemsize);
  const float *v = (const float *)view.buf;
  const double *w = (const double *)view.buf;
  out = PyList_New(B);
  if (!out) goto done;
  for (Py_ssize_t b = 0; b < B; ++b) {
    PyObject *d = PyDict_New(); /* public API; K <= 3 keys fit the minimum table */
    if (!d) goto fail;
    PyList_SET_ITEM(out, b, d); /* owned by the list from here (freed with it on failure) */
    for (Py_ssize_t k = 0; k < K; ++k) {
      PyObject *f = PyFloat_FromDouble(f64 ? w[k * B + b] : (double)v[k * B + b]);
      if (!f) goto fail;
      const int rc = PyDict_SetItem(d, PyTuple_GET_ITEM(keys, k), f);
      Py_DECREF(f);
      if (rc != 0) goto fail;
    }
  }
  goto done;
fail:
  Py_CLEAR(out);
done:
  PyBuffer_Release(&view);
  return out;
}

static PyMethodDef methods[] = {
    {"score_list", score_list, METH_VARARGS, "score_list(scores_f32_KxB, keys) -> list of dicts"},
    {NULL, NULL, 0, NULL},
};

static struct PyModuleDef module = {PyModuleDef_HEAD_INIT, "_score_list", NULL, -1, methods,
                                    NULL, NULL, NULL, NULL};

PyMODINIT_FUNC PyInit__score_list(void) { return PyModule_Create(&module); }
