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
 *   read_columns(batch_vars, specs, out[, cache]) -> (status, bad_type_spec)
 *   new_cache() -> cache
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
 *
 * cache (r05): the numbers of the last call per (agent, variable), valid while the agent's
 * mapping, the variable object, its type and its instance dict are the same objects and
 * neither dict has changed since (CPython's per-dict version tag, PEP 509: every insertion
 * or replacement of a value bumps it; floats and ints are immutable).  A control step that
 * sets one measurement per agent then re-reads one variable per agent: the other variables
 * cost a pointer and a version comparison instead of two hash lookups per attribute.
 * Python >= 3.12 deprecates the version tag: there the cache is never used.
 */
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#include <math.h>
#include <stdint.h>
#include <string.h>

#if PY_VERSION_HEX < 0x030C0000
#define MPCX_DICT_VERSIONS 1
static inline uint64_t dict_version(PyObject* d) { return ((PyDictObject*)d)->ma_version_tag; }
#else
#define MPCX_DICT_VERSIONS 0
static inline uint64_t dict_version(PyObject* d) { (void)d; return 0; }
#endif

/* attribute reads of instances of ``tp`` may skip the type walk of PyObject_GetAttr: the type
   uses the generic lookup, and none of ``attrs`` names a data descriptor on it (those take
   precedence over the instance dict); every name must be an exact str */
static int fast_attrs_ok(PyTypeObject* tp, PyObject* attrs) {
  if (tp->tp_getattro != PyObject_GenericGetAttr || tp->tp_dictoffset == 0) return 0;
  for (Py_ssize_t a = 0; a < PyTuple_GET_SIZE(attrs); ++a) {
    PyObject* an = PyTuple_GET_ITEM(attrs, a);
    if (!PyUnicode_CheckExact(an)) return 0;
    PyObject* descr = _PyType_Lookup(tp, an); /* borrowed */
    if (descr != NULL && Py_TYPE(descr)->tp_descr_set != NULL) return 0;
  }
  return 1;
}

/* ---- the read cache ------------------------------------------------------------------- */
typedef struct {
  PyObject* var;       /* strong: the variable object the mapping held */
  PyObject* idict;     /* strong: its instance dict */
  PyTypeObject* tp;    /* its type (kept alive by var) */
  uint64_t iver;       /* version of idict when the values were read */
  unsigned int tver;   /* tp_version_tag then (a changed class invalidates) */
  int valid;
} VarEntry;

typedef struct {
  Py_ssize_t n, ns, ncol;
  PyObject* specs;     /* strong: the specs object the layout belongs to */
  PyObject** dicts;    /* [n] strong: the agents' mappings */
  uint64_t* dver;      /* [n] their versions after the variable lookups */
  VarEntry* ent;       /* [n * ns] */
  double* vals;        /* [ncol * n] the numbers read (column-major, as out) */
} ReadCache;

static void cache_clear(ReadCache* rc) {
  if (rc->dicts) {
    for (Py_ssize_t i = 0; i < rc->n; ++i) Py_XDECREF(rc->dicts[i]);
  }
  if (rc->ent) {
    for (Py_ssize_t k = 0; k < rc->n * rc->ns; ++k) {
      Py_XDECREF(rc->ent[k].var);
      Py_XDECREF(rc->ent[k].idict);
    }
  }
  Py_XDECREF(rc->specs);
  PyMem_Free(rc->dicts);
  PyMem_Free(rc->dver);
  PyMem_Free(rc->ent);
  PyMem_Free(rc->vals);
  memset(rc, 0, sizeof(*rc));
}

static int cache_reset(ReadCache* rc, Py_ssize_t n, Py_ssize_t ns, Py_ssize_t ncol, PyObject* specs) {
  cache_clear(rc);
  rc->dicts = PyMem_Calloc((size_t)(n ? n : 1), sizeof(PyObject*));
  rc->dver = PyMem_Calloc((size_t)(n ? n : 1), sizeof(uint64_t));
  rc->ent = PyMem_Calloc((size_t)(n * ns ? n * ns : 1), sizeof(VarEntry));
  rc->vals = PyMem_Calloc((size_t)(n * ncol ? n * ncol : 1), sizeof(double));
  if (!rc->dicts || !rc->dver || !rc->ent || !rc->vals) {
    cache_clear(rc);
    PyErr_NoMemory();
    return -1;
  }
  rc->n = n;
  rc->ns = ns;
  rc->ncol = ncol;
  Py_INCREF(specs);
  rc->specs = specs;
  return 0;
}

static void cache_capsule_free(PyObject* cap) {
  ReadCache* rc = (ReadCache*)PyCapsule_GetPointer(cap, "mpcx_read_cache");
  if (rc) {
    cache_clear(rc);
    PyMem_Free(rc);
  }
}

static PyObject* new_cache(PyObject* self, PyObject* noargs) {
  ReadCache* rc = PyMem_Calloc(1, sizeof(ReadCache));
  if (rc == NULL) return PyErr_NoMemory();
  PyObject* cap = PyCapsule_New(rc, "mpcx_read_cache", cache_capsule_free);
  if (cap == NULL) PyMem_Free(rc);
  return cap;
}

/* agents ahead whose cached objects are prefetched */
#ifndef PREFETCH_AHEAD
#define PREFETCH_AHEAD 4
#endif

/* the cached numbers of (agent, variable) still hold */
static inline int entry_current(const VarEntry* e) {
  if (!e->valid) return 0;
  PyObject* v = e->var;
  if (Py_TYPE(v) != e->tp || !PyType_HasFeature(e->tp, Py_TPFLAGS_VALID_VERSION_TAG) || e->tp->tp_version_tag != e->tver)
    return 0;
  PyObject** dp = _PyObject_GetDictPtr(v);
  return dp != NULL && *dp == e->idict && dict_version(e->idict) == e->iver;
}

static PyObject* read_columns(PyObject* self, PyObject* args) {
  PyObject *vars, *specs, *outobj, *capobj = Py_None;
  if (!PyArg_ParseTuple(args, "O!OO|O", &PyList_Type, &vars, &specs, &outobj, &capobj)) return NULL;
  ReadCache* rc = NULL;
  if (capobj != Py_None) {
    rc = (ReadCache*)PyCapsule_GetPointer(capobj, "mpcx_read_cache");
    if (rc == NULL) return NULL;
  }
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
  PyTypeObject* fast_type[64]; /* the type whose attributes come straight from the instance dict */
  Py_ssize_t first_col[65];
  if (ns > 64) {
    PyErr_SetString(PyExc_ValueError, "at most 64 variables per read");
    goto fail_interp;
  }
  first_col[0] = 0;
  for (Py_ssize_t s = 0; s < ns; ++s) {
    last_type[s] = NULL;
    fast_type[s] = NULL;
    first_col[s + 1] = first_col[s] + PyTuple_GET_SIZE(PyTuple_GET_ITEM(PySequence_Fast_GET_ITEM(spec_seq, s), 1));
  }
  if (!MPCX_DICT_VERSIONS) rc = NULL;
  if (rc != NULL && (rc->n != n || rc->ns != ns || rc->ncol != ncol || rc->specs != specs)) {
    if (cache_reset(rc, n, ns, ncol, specs) != 0) goto fail_interp;
  }
  Py_ssize_t ns_live = ns;  /* variables before a failed type check */
  for (Py_ssize_t i = 0; i < n; ++i) {
    PyObject* d = PyList_GET_ITEM(vars, i);
    if (PREFETCH_AHEAD > 0 && rc != NULL && i + PREFETCH_AHEAD < n) {
      /* the objects the version checks of a later agent touch: independent loads the core
         overlaps, instead of one dependent miss after another */
      const Py_ssize_t k = i + PREFETCH_AHEAD;
      __builtin_prefetch(PyList_GET_ITEM(vars, k));
      for (Py_ssize_t s = 0; s < ns; ++s) {
        const VarEntry* f = &rc->ent[k * ns + s];
        if (f->var != NULL) {
          __builtin_prefetch(f->var);
          __builtin_prefetch(f->idict);
        }
      }
    }
    const int exact = PyDict_CheckExact(d);
    /* the mapping is the one of the last call, unchanged: it holds the same variable objects */
    const int same_map = rc != NULL && exact && rc->dicts[i] == d && dict_version(d) == rc->dver[i];
    const uint64_t dver0 = exact ? dict_version(d) : 0;
    for (Py_ssize_t s = 0; s < ns_live; ++s) {
      PyObject* sp = PySequence_Fast_GET_ITEM(spec_seq, s);
      PyObject* name = PyTuple_GET_ITEM(sp, 0);
      PyObject* attrs = PyTuple_GET_ITEM(sp, 1);
      const Py_ssize_t na = PyTuple_GET_SIZE(attrs);
      VarEntry* e = rc != NULL ? &rc->ent[i * ns + s] : NULL;
      PyObject* v;
      if (same_map && e->valid) {
        v = e->var;
        Py_INCREF(v);
      } else if (exact) {
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
      if (e != NULL && e->var == v && entry_current(e)) {
        for (Py_ssize_t a = 0; a < na; ++a) {
          const Py_ssize_t c = first_col[s] + a;
          out[c * n + i] = rc->vals[c * n + i];
        }
        Py_DECREF(v);
        continue;
      }
      if (fast_type[s] != Py_TYPE(v) && fast_attrs_ok(Py_TYPE(v), attrs)) fast_type[s] = Py_TYPE(v);
      PyObject* idict = NULL;
      if (fast_type[s] == Py_TYPE(v)) {
        PyObject** dp = _PyObject_GetDictPtr(v);
        if (dp != NULL && *dp != NULL && PyDict_CheckExact(*dp)) idict = *dp;
      }
      /* the entry is refreshed only if every attribute came from the instance dict as a
         number (nothing else ran in between: the dict's version covers all of them) */
      int cacheable = e != NULL && idict != NULL;
      const uint64_t iver0 = idict != NULL ? dict_version(idict) : 0;
      for (Py_ssize_t a = 0; a < na; ++a) {
        const Py_ssize_t c = first_col[s] + a;
        if (st[c]) {
          cacheable = 0;
          continue;
        }
        PyObject* an = PyTuple_GET_ITEM(attrs, a);
        /* generic attribute lookup without the type walk: the type has no data descriptor of
           that name (fast_attrs_ok), so an instance-dict entry is what getattr returns */
        PyObject* x = idict != NULL ? PyDict_GetItemWithError(idict, an) : NULL;
        if (x != NULL) {
          Py_INCREF(x);
        } else {
          if (PyErr_Occurred()) {
            Py_DECREF(v);
            goto fail_interp;
          }
          cacheable = 0;
          x = PyObject_GetAttr(v, an);
        }
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
        if (st[c]) cacheable = 0;
        out[c * n + i] = val;
      }
      if (e != NULL) {
        if (cacheable && PyType_HasFeature(Py_TYPE(v), Py_TPFLAGS_VALID_VERSION_TAG) &&
            dict_version(idict) == iver0) {
          for (Py_ssize_t a = 0; a < na; ++a) {
            const Py_ssize_t c = first_col[s] + a;
            rc->vals[c * n + i] = out[c * n + i];
          }
          Py_INCREF(v);
          Py_XSETREF(e->var, v);
          Py_INCREF(idict);
          Py_XSETREF(e->idict, idict);
          e->tp = Py_TYPE(v);
          e->tver = Py_TYPE(v)->tp_version_tag;
          e->iver = iver0;
          e->valid = 1;
        } else {
          e->valid = 0;
        }
      }
      Py_DECREF(v);
    }
    if (rc != NULL) {
      if (exact && ns_live == ns && dict_version(d) == dver0) {
        if (rc->dicts[i] != d) {
          Py_INCREF(d);
          Py_XSETREF(rc->dicts[i], d);
        }
        rc->dver[i] = dver0;
      } else {
        Py_CLEAR(rc->dicts[i]);  /* a mapping that changed while it was read: look up again */
      }
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
     "read_columns(batch_vars, specs, out[, cache]) -> (status bytes, bad_type_spec)"},
    {"new_cache", new_cache, METH_NOARGS, "new_cache() -> an empty read cache for read_columns"},
    {NULL, NULL, 0, NULL},
};

static struct PyModuleDef module = {PyModuleDef_HEAD_INIT, "_mpcx_pyread", NULL, -1, methods};

PyMODINIT_FUNC PyInit__mpcx_pyread(void) { return PyModule_Create(&module); }
