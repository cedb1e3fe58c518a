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
 *
 * Two-phase form for the GPU path: score_list_alloc(B, keys) builds the B dicts with fresh float
 * objects while the GPU computes (nothing is known yet but the shape) and returns them with a
 * handle holding a reference to every float; score_list_fill(handle, offset, scores, keys)
 * writes the values into them once a chunk's scores reach the host -- a few ns per dict instead
 * of ~100, so the list no longer trails the GPU.  The floats are private until the list is
 * returned (created here, referenced by their dict and the handle only), so setting their value
 * in place is the same as creating them with it, as a fresh tuple is filled with
 * PyTuple_SET_ITEM; a float referenced anywhere else (a list the caller touched) is left alone
 * and its dict gets a new one through PyDict_SetItem.
 */
#define PY_SSIZE_T_CLEAN
#include <Python.h>

/* The in-place fill relies on the refcount semantics of GIL builds of CPython up to 3.13: a
 * float whose count is 2 is referenced by its dict and the handle only.  Free-threaded builds
 * (Py_GIL_DISABLED: biased, shared counts) and later versions (deferred reference counting) may
 * report other counts, so there every value goes in through PyDict_SetItem -- the same list, a
 * few ns more per value.  `inplace_fill` also switches it off at run time (set_inplace: the
 * tests compare the two forms). */
#if !defined(Py_GIL_DISABLED) && PY_VERSION_HEX < 0x030E0000
#define FSEM_INPLACE_FLOATS 1
#else
#define FSEM_INPLACE_FLOATS 0
#endif
static int inplace_fill = FSEM_INPLACE_FLOATS;

/* keys: a non-empty tuple of str (hashes cached once); returns K or -1 with an exception set */
static Py_ssize_t check_keys(PyObject *keys) {
  const Py_ssize_t K = PyTuple_GET_SIZE(keys);
  if (K <= 0) {
    PyErr_SetString(PyExc_ValueError, "score_list: keys must be a non-empty tuple");
    return -1;
  }
  for (Py_ssize_t k = 0; k < K; ++k) {
    PyObject *key = PyTuple_GET_ITEM(keys, k);
    if (!PyUnicode_Check(key)) {
      PyErr_SetString(PyExc_TypeError, "score_list: keys must be str");
      return -1;
    }
    if (PyObject_Hash(key) == -1) return -1; /* cache the hash once */
  }
  return K;
}

/* the K x B float32 / float64 scores of buf_obj (view released by the caller on success);
 * returns B or -1 with an exception set */
static Py_ssize_t get_scores(PyObject *buf_obj, Py_ssize_t K, Py_buffer *view, int *f64) {
  if (PyObject_GetBuffer(buf_obj, view, PyBUF_C_CONTIGUOUS | PyBUF_FORMAT) != 0) return -1;
  const char *fmt = view->format ? view->format : "";
  if (*fmt == '<' || *fmt == '=' || *fmt == '@') ++fmt;
  *f64 = fmt[0] == 'd' && fmt[1] == 0 && view->itemsize == 8;
  if (!(*f64 || (fmt[0] == 'f' && fmt[1] == 0 && view->itemsize == 4)) || view->len % (K * view->itemsize) != 0) {
    PyErr_SetString(PyExc_TypeError, "score_list: scores must be a contiguous float32 / float64 buffer of K x B values");
    PyBuffer_Release(view);
    return -1;
  }
  return view->len / (K * view->itemsize);
}

static PyObject *score_list(PyObject *self, PyObject *args) {
  (void)self;
  PyObject *buf_obj, *keys;
  if (!PyArg_ParseTuple(args, "OO!", &buf_obj, &PyTuple_Type, &keys)) return NULL;
  const Py_ssize_t K = check_keys(keys);
  if (K < 0) return NULL;
  Py_buffer view;
  int f64;
  const Py_ssize_t B = get_scores(buf_obj, K, &view, &f64);
  if (B < 0) return NULL;
  PyObject *out = NULL;
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

/* The two-phase form's handle: the list and, per row and key, its float object (one extra
 * reference each, so none can be freed behind the handle's back). */
typedef struct {
  PyObject *lst;
  PyObject *keys; /* the allocation's keys: score_list_fill must pass equal ones */
  Py_ssize_t B, K;
  PyObject **f; /* B x K */
} Pending;

static void pending_free(PyObject *cap) {
  Pending *p = (Pending *)PyCapsule_GetPointer(cap, "fsem.score_list");
  if (!p) return;
  if (p->f) {
    for (Py_ssize_t i = 0; i < p->B * p->K; ++i) Py_XDECREF(p->f[i]);
    PyMem_Free(p->f);
  }
  Py_XDECREF(p->lst);
  Py_XDECREF(p->keys);
  PyMem_Free(p);
}

/* score_list_alloc(B, keys) -> (list, handle): [{keys[0]: nan, ...} x B], every value a fresh
 * float object, and the handle score_list_fill writes the scores through */
static PyObject *score_list_alloc(PyObject *self, PyObject *args) {
  (void)self;
  Py_ssize_t B;
  PyObject *keys;
  if (!PyArg_ParseTuple(args, "nO!", &B, &PyTuple_Type, &keys)) return NULL;
  if (B < 0) {
    PyErr_SetString(PyExc_ValueError, "score_list_alloc: negative length");
    return NULL;
  }
  const Py_ssize_t K = check_keys(keys);
  if (K < 0) return NULL;
  Pending *p = (Pending *)PyMem_Calloc(1, sizeof(Pending));
  if (!p) return PyErr_NoMemory();
  PyObject *cap = PyCapsule_New(p, "fsem.score_list", pending_free);
  if (!cap) {
    PyMem_Free(p);
    return NULL;
  }
  p->f = (PyObject **)PyMem_Calloc((size_t)(B * K) + 1, sizeof(PyObject *));
  p->lst = PyList_New(B);
  if (!p->f || !p->lst) {
    const int oom = !p->f;
    Py_DECREF(cap); /* frees p */
    return oom ? PyErr_NoMemory() : NULL;
  }
  p->B = B;
  p->K = K;
  Py_INCREF(keys);
  p->keys = keys;
  for (Py_ssize_t b = 0; b < B; ++b) {
    PyObject *d = PyDict_New();
    if (!d) goto fail;
    PyList_SET_ITEM(p->lst, b, d);
    for (Py_ssize_t k = 0; k < K; ++k) {
      PyObject *f = PyFloat_FromDouble(Py_NAN);
      if (!f) goto fail;
      p->f[b * K + k] = f; /* the handle's reference */
      if (PyDict_SetItem(d, PyTuple_GET_ITEM(keys, k), f) != 0) goto fail;
    }
  }
  return Py_BuildValue("(ON)", p->lst, cap);
fail:
  Py_DECREF(cap);
  return NULL;
}

/* score_list_fill(handle, offset, scores_KxB, keys): lst[offset + b][keys[k]] = scores[k][b] */
static PyObject *score_list_fill(PyObject *self, PyObject *args) {
  (void)self;
  PyObject *cap, *buf_obj, *keys;
  Py_ssize_t off;
  if (!PyArg_ParseTuple(args, "OnOO!", &cap, &off, &buf_obj, &PyTuple_Type, &keys)) return NULL;
  Pending *p = (Pending *)PyCapsule_GetPointer(cap, "fsem.score_list");
  if (!p) return NULL;
  const Py_ssize_t K = check_keys(keys);
  if (K < 0) return NULL;
  /* the same keys, element by element (as the Python form's tuple comparison): the in-place
   * path writes through the allocation's float objects, which belong to the allocation's keys */
  int same = K == p->K;
  for (Py_ssize_t k = 0; same && k < K; ++k) {
    const int eq = PyObject_RichCompareBool(PyTuple_GET_ITEM(keys, k), PyTuple_GET_ITEM(p->keys, k), Py_EQ);
    if (eq < 0) return NULL;
    same = eq;
  }
  if (!same) {
    PyErr_SetString(PyExc_ValueError, "score_list_fill: keys differ from the allocation's");
    return NULL;
  }
  Py_buffer view;
  int f64;
  const Py_ssize_t B = get_scores(buf_obj, K, &view, &f64);
  if (B < 0) return NULL;
  PyObject *ret = NULL;
  if (off < 0 || off > p->B - B) {
    PyErr_SetString(PyExc_IndexError, "score_list_fill: rows past the list's end");
    goto done;
  }
  const float *v = (const float *)view.buf;
  const double *w = (const double *)view.buf;
  for (Py_ssize_t b = 0; b < B; ++b) {
    for (Py_ssize_t k = 0; k < K; ++k) {
      const double x = f64 ? w[k * B + b] : (double)v[k * B + b];
      PyObject *f = p->f[(off + b) * K + k];
#if FSEM_INPLACE_FLOATS
      if (inplace_fill && Py_REFCNT(f) == 2) {
        /* referenced by its dict and the handle only: not yet visible to anyone else */
        ((PyFloatObject *)f)->ob_fval = x;
        continue;
      }
#else
      (void)f;
#endif
      /* replaced or shared since the allocation: a new float through the dict API */
      PyObject *d = PyList_GET_ITEM(p->lst, off + b);
      if (!PyDict_Check(d)) {
        PyErr_SetString(PyExc_TypeError, "score_list_fill: list items must be dicts");
        goto done;
      }
      PyObject *nf = PyFloat_FromDouble(x);
      if (!nf) goto done;
      const int rc = PyDict_SetItem(d, PyTuple_GET_ITEM(keys, k), nf);
      Py_DECREF(nf);
      if (rc != 0) goto done;
    }
  }
  ret = Py_None;
  Py_INCREF(ret);
done:
  PyBuffer_Release(&view);
  return ret;
}

/* set_inplace(flag) -> previous flag: the in-place fill on (where compiled in) or off */
static PyObject *set_inplace(PyObject *self, PyObject *arg) {
  (void)self;
  const int on = PyObject_IsTrue(arg);
  if (on < 0) return NULL;
  const int prev = inplace_fill;
  inplace_fill = on && FSEM_INPLACE_FLOATS;
  return PyBool_FromLong(prev);
}

static PyMethodDef methods[] = {
    {"set_inplace", set_inplace, METH_O,
     "set_inplace(flag) -> previous: fill fresh floats in place (GIL builds <= 3.13 only) or by PyDict_SetItem"},
    {"score_list", score_list, METH_VARARGS, "score_list(scores_f32_KxB, keys) -> list of dicts"},
    {"score_list_alloc", score_list_alloc, METH_VARARGS,
     "score_list_alloc(B, keys) -> (list of B dicts with nan values, handle)"},
    {"score_list_fill", score_list_fill, METH_VARARGS,
     "score_list_fill(handle, offset, scores_f32_KxB, keys): write the scores into list[offset:offset+B]"},
    {NULL, NULL, 0, NULL},
};

static struct PyModuleDef module = {PyModuleDef_HEAD_INIT, "_score_list", NULL, -1, methods,
                                    NULL, NULL, NULL, NULL};

PyMODINIT_FUNC PyInit__score_list(void) {
  PyObject *m = PyModule_Create(&module);
  if (m && PyModule_AddIntConstant(m, "INPLACE_COMPILED", FSEM_INPLACE_FLOATS) != 0) Py_CLEAR(m);
  return m;
}
