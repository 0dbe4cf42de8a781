/* come_pyext.c -- the per-call drop-ins' host route as a CPython extension (_come_pyext).
 *
 * The reference's train_o2 / train_o1 (utils/training_sdg_inner.pyx:407-509) are Cython functions:
 * a few microseconds of Python-level work per call (two global-RNG draws, pyx:427,477; the path's
 * Vocab.index reads, pyx:483-490), then the update loop with the GIL released (pyx:443,493).  The
 * reference's trainers call them once per walk / edge from `workers` threads
 * (context_embeddings.py:72-98, node_embeddings.py:58-83), so per-call overhead and GIL release are
 * both part of the contract.  These two functions do the same Python-level work in C and run
 * libcome's host twins (come_cpu_sgns_o2 / _o1, sequential mode, include/come.h) on the caller's
 * numpy arrays in place, with the GIL released whenever the call's update work is worth more than
 * a GIL hand-over (GIL_RELEASE_WORK: a C3 walk releases it, a d = 128 edge keeps it).  libcome is not linked: training_sdg_inner passes
 * the twins' addresses (ctypes) to init(), after loading the library its usual way.
 *
 *   init(o2_fn, o1_fn, last_error_fn, randint)   addresses of come_cpu_sgns_o2 / _o1 /
 *                                                come_last_error, and numpy.random.randint
 *   train_o2(node, ctx, path, lr, negative, window, table, alpha) -> non-None count
 *   train_o1(node, edge, lr, negative, table) -> non-None count
 *
 * Argument errors raise TypeError before the RNG is drawn (so a caller may convert and retry). */
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#include <stdint.h>
#include <string.h>

#define COME_PYEXT_VERSION 1
#define MAX_SENTENCE_LEN 10000 /* pyx:18 */
#define MODE_SEQUENTIAL 1
/* row-element products below which a call keeps the GIL (see train_o1) */
#define GIL_RELEASE_WORK 16384

typedef int (*o2_fn_t)(float *, float *, int64_t, int, const int32_t *, int64_t, int,
                       const uint64_t *, int, int, const uint32_t *, uint64_t, float, float, int,
                       int, int64_t *);
typedef int (*o1_fn_t)(float *, int64_t, int, const int32_t *, int64_t, const uint64_t *, int,
                       const uint32_t *, uint64_t, float, int, int, int64_t *);
typedef const char *(*err_fn_t)(void);

static o2_fn_t g_o2;
static o1_fn_t g_o1;
static err_fn_t g_err;
static PyObject *g_randint;    /* numpy.random.randint (the global RandomState) */
static PyObject *g_draw_args;  /* (0, 2**24) */
static PyObject *g_index;      /* "index" */

static PyObject *py_init(PyObject *self, PyObject *args) {
    unsigned long long o2, o1, err;
    PyObject *randint;
    (void)self;
    if (!PyArg_ParseTuple(args, "KKKO", &o2, &o1, &err, &randint)) return NULL;
    if (!o2 || !o1 || !err || !PyCallable_Check(randint)) {
        PyErr_SetString(PyExc_ValueError, "init needs three function addresses and a callable");
        return NULL;
    }
    g_o2 = (o2_fn_t)(uintptr_t)o2;
    g_o1 = (o1_fn_t)(uintptr_t)o1;
    g_err = (err_fn_t)(uintptr_t)err;
    Py_INCREF(randint);
    Py_XSETREF(g_randint, randint);
    Py_RETURN_NONE;
}

/* A float32 [V, d] C-contiguous writable buffer (a numpy embedding table). */
static int get_table(PyObject *o, Py_buffer *b, const char *name) {
    if (PyObject_GetBuffer(o, b, PyBUF_WRITABLE | PyBUF_C_CONTIGUOUS | PyBUF_FORMAT) != 0) {
        PyErr_Clear();
        PyErr_Format(PyExc_TypeError, "%s must be a writable C-contiguous float32 [V, d] array",
                     name);
        return -1;
    }
    const char *f = b->format ? b->format : "B";
    if (*f == '=' || *f == '<' || *f == '@') ++f;
    if (b->ndim != 2 || b->itemsize != 4 || strcmp(f, "f") != 0) {
        PyBuffer_Release(b);
        PyErr_Format(PyExc_TypeError, "%s must be a writable C-contiguous float32 [V, d] array",
                     name);
        return -1;
    }
    return 0;
}

/* The negative table: a C-contiguous 1-D buffer of 4-byte integers (np.uint32, pyx:421,472). */
static int get_neg(PyObject *o, Py_buffer *b) {
    if (PyObject_GetBuffer(o, b, PyBUF_C_CONTIGUOUS | PyBUF_FORMAT) != 0) {
        PyErr_Clear();
        PyErr_SetString(PyExc_TypeError, "py_table must be a C-contiguous uint32 array");
        return -1;
    }
    const char *f = b->format ? b->format : "B";
    if (*f == '=' || *f == '<' || *f == '@') ++f;
    if (b->ndim != 1 || b->itemsize != 4 || !(strcmp(f, "I") == 0 || strcmp(f, "i") == 0 ||
                                              strcmp(f, "L") == 0 || strcmp(f, "l") == 0)) {
        PyBuffer_Release(b);
        PyErr_SetString(PyExc_TypeError, "py_table must be a C-contiguous uint32 array");
        return -1;
    }
    return 0;
}

/* pyx:427,477: next_random = 2**24 * randint(0, 2**24) + randint(0, 2**24), left draw first. */
static int draw_seed(uint64_t *out) {
    uint64_t v[2];
    for (int i = 0; i < 2; ++i) {
        PyObject *r = PyObject_Call(g_randint, g_draw_args, NULL);
        if (!r) return -1;
        v[i] = PyLong_AsUnsignedLongLong(r);
        Py_DECREF(r);
        if (PyErr_Occurred()) return -1;
    }
    *out = (v[0] << 24) + v[1];
    return 0;
}

/* Items (Vocab-like objects with .index, or None) -> rows, -1 for None (pyx:483-490). */
static Py_ssize_t read_rows(PyObject *seq, int32_t *rows, Py_ssize_t cap, long *result) {
    PyObject *fast = PySequence_Fast(seq, "the path must be a sequence");
    if (!fast) return -1;
    Py_ssize_t n = PySequence_Fast_GET_SIZE(fast);
    if (n > cap) n = cap;
    PyObject **items = PySequence_Fast_ITEMS(fast);
    long count = 0;
    for (Py_ssize_t i = 0; i < n; ++i) {
        if (items[i] == Py_None) {
            rows[i] = -1;
            continue;
        }
        PyObject *ix = PyObject_GetAttr(items[i], g_index);
        if (!ix) {
            Py_DECREF(fast);
            return -1;
        }
        long long v = PyLong_AsLongLong(ix);
        Py_DECREF(ix);
        if (v == -1 && PyErr_Occurred()) {
            Py_DECREF(fast);
            return -1;
        }
        rows[i] = (v < 0 || v > INT32_MAX) ? -1 : (int32_t)v;  /* outside the table: None */
        ++count;
    }
    Py_DECREF(fast);
    *result = count;
    return n;
}

static PyObject *twin_error(int rc, const char *what) {
    PyErr_Format(PyExc_RuntimeError, "%s failed (rc=%d): %s", what, rc, g_err ? g_err() : "");
    return NULL;
}

static int ready(void) {
    if (!g_o2 || !g_randint) {
        PyErr_SetString(PyExc_RuntimeError, "_come_pyext.init() was not called");
        return 0;
    }
    return 1;
}

static PyObject *py_train_o2(PyObject *self, PyObject *args) {
    PyObject *node_o, *ctx_o, *path, *table_o;
    float lr, alpha = 1.0f;
    int negative, window;
    (void)self;
    if (!ready()) return NULL;
    if (!PyArg_ParseTuple(args, "OOOfiiO|f", &node_o, &ctx_o, &path, &lr, &negative, &window,
                          &table_o, &alpha))
        return NULL;
    Py_buffer nb, cb, tb;
    if (get_table(node_o, &nb, "py_node_embedding")) return NULL;
    if (get_table(ctx_o, &cb, "py_context_embedding")) {
        PyBuffer_Release(&nb);
        return NULL;
    }
    if (get_neg(table_o, &tb)) {
        PyBuffer_Release(&nb);
        PyBuffer_Release(&cb);
        return NULL;
    }
    PyObject *ret = NULL;
    if (nb.shape[0] != cb.shape[0] || nb.shape[1] != cb.shape[1]) {
        PyErr_SetString(PyExc_TypeError, "node and context embeddings must have the same shape");
        goto done;
    }
    uint64_t seed;
    if (draw_seed(&seed)) goto done;
    static __thread int32_t rows[MAX_SENTENCE_LEN];
    long result = 0;
    const Py_ssize_t L = read_rows(path, rows, MAX_SENTENCE_LEN, &result);
    if (L < 0) goto done;
    int rc = 0;
    if (L > 0) {
        /* at most 2 * window pairs per entry, each (1 + negative) row products of d elements */
        const int64_t work = (int64_t)L * 2 * (window > 0 ? window : 0) *
                             (1 + (negative > 0 ? negative : 0)) * nb.shape[1];
        if (work >= GIL_RELEASE_WORK) {
            Py_BEGIN_ALLOW_THREADS
            rc = g_o2((float *)nb.buf, (float *)cb.buf, nb.shape[0], (int)nb.shape[1], rows, 1,
                      (int)L, &seed, window, negative, (const uint32_t *)tb.buf,
                      (uint64_t)tb.shape[0], lr, alpha, MODE_SEQUENTIAL, 1, NULL);
            Py_END_ALLOW_THREADS
        } else {
            rc = g_o2((float *)nb.buf, (float *)cb.buf, nb.shape[0], (int)nb.shape[1], rows, 1,
                      (int)L, &seed, window, negative, (const uint32_t *)tb.buf,
                      (uint64_t)tb.shape[0], lr, alpha, MODE_SEQUENTIAL, 1, NULL);
        }
    }
    ret = rc ? twin_error(rc, "come_cpu_sgns_o2") : PyLong_FromLong(result);
done:
    PyBuffer_Release(&nb);
    PyBuffer_Release(&cb);
    PyBuffer_Release(&tb);
    return ret;
}

static PyObject *py_train_o1(PyObject *self, PyObject *args) {
    PyObject *node_o, *edge, *table_o;
    float lr;
    int negative;
    (void)self;
    if (!ready()) return NULL;
    if (!PyArg_ParseTuple(args, "OOfiO", &node_o, &edge, &lr, &negative, &table_o)) return NULL;
    Py_buffer nb, tb;
    if (get_table(node_o, &nb, "py_node_embedding")) return NULL;
    if (get_neg(table_o, &tb)) {
        PyBuffer_Release(&nb);
        return NULL;
    }
    PyObject *ret = NULL;
    uint64_t seed;
    int32_t rows[2];
    long result = 0;
    int rc = 0;
    if (draw_seed(&seed)) goto done;
    const Py_ssize_t n = read_rows(edge, rows, 2, &result);
    if (n < 0) goto done;
    if (n == 2) {
        /* One edge is 2 (1 + negative) row products of d elements: at the reference's sizes a
         * couple of microseconds, less than handing the GIL to a waiting worker and taking it back
         * (measured: 8 workers, d = 128, n = 5 -- 0.54e5 pair-updates/s releasing, see
         * scripts/dropin_rate.py).  The GIL is released only when an edge is worth it. */
        const int64_t work = 2 * (int64_t)(1 + (negative > 0 ? negative : 0)) * nb.shape[1];
        if (work >= GIL_RELEASE_WORK) {
            Py_BEGIN_ALLOW_THREADS
            rc = g_o1((float *)nb.buf, nb.shape[0], (int)nb.shape[1], rows, 1, &seed, negative,
                      (const uint32_t *)tb.buf, (uint64_t)tb.shape[0], lr, MODE_SEQUENTIAL, 1,
                      NULL);
            Py_END_ALLOW_THREADS
        } else {
            rc = g_o1((float *)nb.buf, nb.shape[0], (int)nb.shape[1], rows, 1, &seed, negative,
                      (const uint32_t *)tb.buf, (uint64_t)tb.shape[0], lr, MODE_SEQUENTIAL, 1,
                      NULL);
        }
    }
    ret = rc ? twin_error(rc, "come_cpu_sgns_o1") : PyLong_FromLong(result);
done:
    PyBuffer_Release(&nb);
    PyBuffer_Release(&tb);
    return ret;
}

static PyMethodDef methods[] = {
    {"init", py_init, METH_VARARGS, "init(o2_addr, o1_addr, last_error_addr, randint)"},
    {"train_o2", py_train_o2, METH_VARARGS,
     "train_o2(node, ctx, path, lr, negative, window, table, alpha=1.0) -> int"},
    {"train_o1", py_train_o1, METH_VARARGS, "train_o1(node, edge, lr, negative, table) -> int"},
    {NULL, NULL, 0, NULL}};

static struct PyModuleDef module = {PyModuleDef_HEAD_INIT, "_come_pyext",
                                    "Host route of the per-call drop-ins (csrc/come_pyext.c).", -1,
                                    methods, NULL, NULL, NULL, NULL};

PyMODINIT_FUNC PyInit__come_pyext(void) {
    PyObject *m = PyModule_Create(&module);
    if (!m) return NULL;
    g_index = PyUnicode_InternFromString("index");
    g_draw_args = Py_BuildValue("(ii)", 0, 1 << 24);
    if (!g_index || !g_draw_args || PyModule_AddIntConstant(m, "VERSION", COME_PYEXT_VERSION)) {
        Py_DECREF(m);
        return NULL;
    }
    return m;
}
