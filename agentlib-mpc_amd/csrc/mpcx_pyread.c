/* Host-side reader of the agents' MPCVariable attributes for the plugin batch
 * (agentlib_mpc_amd/optimization_backends/plugin_batch.py, ResidentBatch.read).
 *
 * The reference marshals every agent's variables one agent at a time
 * (core/casadi_backend.py:141-253: for each variable, ``var_ref`` name -> ``value`` /
 * ``lb`` / ``ub`` of the MPCVariable in ``current_vars``).  The batched plugin call reads
 * the same attributes of every agent of the fleet once per call; done with Python
 * iterators that is ~90 ns per attribute read, 3-6 ms per 4096-agent call -- more than
 * the kernel.  This CPython extension reads all (variable, attribute) columns in one C
 * pass over the agents (dict lookup + attribute lookup + float unpack) into one float64
 * buffer.
 *
 *   read_columns(batch_vars, specs, out) -> (status, bad_type_spec)
 *
 * batch_vars: list of mappings (one per agent); specs: sequence of
 * (name, attrs, check_type) with attrs a tuple of attribute names; out: writable
 * C-contiguous float64 buffer of sum(len(attrs)) * n doubles, column c of the result at
 * out[c * n : (c + 1) * n].  status: bytes, one per column: 0 = every agent holds a Python
 * float / int that is not NaN (the column is in out), 1 = not (the caller takes its
 * checked Python path for that column, which also produces the reference's errors).
 * bad_type_spec: index of the first spec with check_type whose variable has a type
 * without ``interpolation_method`` (the reference's TypeError), or -1; reading stops
 * there.  A missing variable raises the mapping's KeyError, as ``current_vars[name]``
 * does in the reference.
 */
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#include <math.h>

static PyObject* read_columns(PyObject* self, PyObject* args) {
  PyObject *vars, *specs, *outobj;
  if (!PyArg_ParseTuple(args, "O!OO", &PyList_Type, &vars, &specs, &outobj)) return NULL;
  PyObject* spec_seq = PySequence_Fast(specs, "specs must be a sequence");
  if (spec_seq == NULL) return NULL;
  const Py_ssize_t n = PyList_GET_SIZE(vars);
  const Py_ssize_t ns = PySequence_Fast_GET_SIZE(spec_seq);
  Py_ssize_t ncol = 0;
  for (Py_ssize_t s = 0; s < ns; ++s) {
    PyObject* sp = PySequence_Fast_GET_ITEM(spec_seq, s);
    if (!PyTuple_Check(sp) || PyTuple_GET_SIZE(sp) != 3 || !PyTuple_Check(PyTuple_GET_ITEM(sp, 1))) {
      Py_DECREF(spec_seq);
      PyErr_SetString(PyExc_TypeError, "spec must be (name, attrs tuple, check_type)");
      return NULL;
    }
    ncol += PyTuple_GET_SIZE(PyTuple_GET_ITEM(sp, 1));
  }
  Py_buffer buf;
  if (PyObject_GetBuffer(outobj, &buf, PyBUF_WRITABLE | PyBUF_C_CONTIGUOUS) != 0) {
    Py_DECREF(spec_seq);
    return NULL;
  }
  if (buf.len < (Py_ssize_t)(ncol * n * sizeof(double))) {
    PyBuffer_Release(&buf);
    Py_DECREF(spec_seq);
    PyErr_SetString(PyExc_ValueError, "output buffer too small");
    return NULL;
  }
  double* out = (double*)buf.buf;
  PyObject* status = PyBytes_FromStringAndSize(NULL, ncol);
  if (status == NULL) goto fail;
  char* st = PyBytes_AS_STRING(status);
  memset(st, 0, (size_t)ncol);
  PyObject* interp = PyUnicode_InternFromString("interpolation_method");
  if (interp == NULL) goto fail_status;
  Py_ssize_t bad_type = -1;
  /* agents outer, variables inner: one agent's dict and variable objects are visited
     together (the fleet's objects do not fit the host caches; a column-by-column walk
     re-fetches every agent dict once per variable) */
  PyTypeObject* last_type[64];
  Py_ssize_t first_col[65];
  if (ns > 64) {
    PyErr_SetString(PyExc_ValueError, "at most 64 variables per read");
    goto fail_interp;
  }
  first_col[0] = 0;
  for (Py_ssize_t s = 0; s < ns; ++s) {
    last_type[s] = NULL;
    first_col[s + 1] = first_col[s] + PyTuple_GET_SIZE(PyTuple_GET_ITEM(PySequence_Fast_GET_ITEM(spec_seq, s), 1));
  }
  Py_ssize_t ns_live = ns;  /* variables before a failed type check */
  for (Py_ssize_t i = 0; i < n; ++i) {
    PyObject* d = PyList_GET_ITEM(vars, i);
    const int exact = PyDict_CheckExact(d);
    for (Py_ssize_t s = 0; s < ns_live; ++s) {
      PyObject* sp = PySequence_Fast_GET_ITEM(spec_seq, s);
      PyObject* name = PyTuple_GET_ITEM(sp, 0);
      PyObject* attrs = PyTuple_GET_ITEM(sp, 1);
      PyObject* v;
      if (exact) {
        v = PyDict_GetItemWithError(d, name);  /* borrowed */
        if (v == NULL) {
          if (!PyErr_Occurred()) PyErr_SetObject(PyExc_KeyError, name);
          goto fail_interp;
        }
        Py_INCREF(v);
      } else {
        v = PyObject_GetItem(d, name);
        if (v == NULL) goto fail_interp;
      }
      if (Py_TYPE(v) != last_type[s] && PyTuple_GET_ITEM(sp, 2) == Py_True) {
        last_type[s] = Py_TYPE(v);  /* one check per type, as the Python reader */
        if (!PyObject_HasAttr(v, interp)) {
          Py_DECREF(v);
          bad_type = s;
          ns_live = s;  /* stop reading this variable and the later ones */
          break;
        }
      }
      const Py_ssize_t na = PyTuple_GET_SIZE(attrs);
      for (Py_ssize_t a = 0; a < na; ++a) {
        const Py_ssize_t c = first_col[s] + a;
        if (st[c]) continue;
        PyObject* x = PyObject_GetAttr(v, PyTuple_GET_ITEM(attrs, a));
        if (x == NULL) {
          Py_DECREF(v);
          goto fail_interp;
        }
        double val;
        if (PyFloat_CheckExact(x)) {
          val = PyFloat_AS_DOUBLE(x);
        } else if (PyLong_CheckExact(x)) {
          val = PyLong_AsDouble(x);
          if (val == -1.0 && PyErr_Occurred()) { PyErr_Clear(); st[c] = 1; }
        } else {
          st[c] = 1;  /* anything else (None, lists, series, numpy scalars): Python path */
          val = 0.0;
        }
        Py_DECREF(x);
        if (isnan(val)) st[c] = 1;
        out[c * n + i] = val;
      }
      Py_DECREF(v);
    }
  }
  Py_DECREF(interp);
  PyBuffer_Release(&buf);
  Py_DECREF(spec_seq);
  return Py_BuildValue("(Nn)", status, bad_type);

fail_interp:
  Py_DECREF(interp);
fail_status:
  Py_DECREF(status);
fail:
  PyBuffer_Release(&buf);
  Py_DECREF(spec_seq);
  return NULL;
}

static PyMethodDef methods[] = {
    {"read_columns", read_columns, METH_VARARGS,
     "read_columns(batch_vars, specs, out) -> (status bytes, bad_type_spec)"},
    {NULL, NULL, 0, NULL},
};

static struct PyModuleDef module = {PyModuleDef_HEAD_INIT, "_mpcx_pyread", NULL, -1, methods};

PyMODINIT_FUNC PyInit__mpcx_pyread(void) { return PyModule_Create(&module); }
