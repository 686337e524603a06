/* pandas object columns of Python str -> Arrow string layout (n + 1 int64 offsets + UTF-8 bytes), for the boundary's
 * device column path (mobheat.stream.ArrowColumns -> hm_arrow_columns; reference heatmap_stream.py:51-61,150: provider
 * and vehicleId are StringType).  pyarrow's conversion of an object column visits every row under the GIL (~0.3 s per
 * 1e7-row column, most of a pandas micro-batch's host time); here the compact-ASCII strings -- CPython keeps their
 * bytes right after the object header -- are measured and copied by several threads with the GIL released, and the
 * rest (None, non-ASCII str, other objects) are left to the caller.
 *
 * lengths(ptrs, n, lens, threads): ptrs = the address of the object array's n PyObject pointers, lens = int64[n] out:
 *   the byte length of a compact-ASCII str, -1 for None, -2 for anything else (the caller encodes or rejects it).
 * copy(ptrs, n, offsets, data, threads): the bytes of every row with lens >= 0 to data[offsets[i], offsets[i+1]).
 * floats(ptrs, n, values, kinds, threads): an object column of Python float / None (a nullable double column as pandas
 *   holds it): values[i] = the float, kinds[i] = 1 float, 0 None, 2 anything else (the caller converts those).
 * measure(ptrs, n, offs, threads) -> (bytes, nulls, others, [per-block bytes]): the fused form's first pass -- offs
 *   = int64[n + 1], offs[i + 1] = the byte length of row i (-1 None, -2 anything else); the rows split into blocks of
 *   whole bytes of the validity bitmap (multiples of 64 rows), one per thread.
 * fill(ptrs, n, offs, data, bitmap, block_bytes, threads): its second pass over the same blocks -- offs becomes the
 *   exclusive offsets (offs[0] = 0, a null row adds 0), every compact-ASCII row's bytes are copied to data, and the
 *   validity bitmap (Arrow: LSB first; bitmap may be 0) written: two threaded passes instead of lengths, a numpy
 *   cumsum, copy and packbits (only when others == 0: the caller converts such a column another way).
 * The object array must stay alive (it holds the references) and unchanged during both calls. */
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#include <pthread.h>
#include <stdint.h>
#include <string.h>

typedef struct {
    PyObject *const *obj;
    int64_t lo, hi;
    int64_t *lens;
    const int64_t *offs;
    uint8_t *data;
    double *vals;
} Job;

static int is_ascii_str(PyObject *o) {
    return PyUnicode_Check(o) && PyUnicode_IS_READY(o) && PyUnicode_IS_COMPACT_ASCII(o);
}

static void *len_job(void *p) {
    Job *j = (Job *)p;
    for (int64_t i = j->lo; i < j->hi; i++) {
        PyObject *o = j->obj[i];
        j->lens[i] = o == Py_None ? -1 : is_ascii_str(o) ? (int64_t)PyUnicode_GET_LENGTH(o) : -2;
    }
    return NULL;
}

static void *copy_job(void *p) {
    Job *j = (Job *)p;
    for (int64_t i = j->lo; i < j->hi; i++) {
        PyObject *o = j->obj[i];
        const int64_t a = j->offs[i], b = j->offs[i + 1];
        if (b > a && is_ascii_str(o) && PyUnicode_GET_LENGTH(o) == b - a) memcpy(j->data + a, PyUnicode_DATA(o), (size_t)(b - a));
    }
    return NULL;
}

/* object column of Python float / None: the value (exact float objects only), data[i] = 1 valid, 0 None, 2 other */
static void *float_job(void *p) {
    Job *j = (Job *)p;
    for (int64_t i = j->lo; i < j->hi; i++) {
        PyObject *o = j->obj[i];
        if (PyFloat_CheckExact(o)) {
            j->vals[i] = PyFloat_AS_DOUBLE(o);
            j->data[i] = 1;
        } else {
            j->vals[i] = 0.0;
            j->data[i] = o == Py_None ? 0 : 2;
        }
    }
    return NULL;
}

static void run(void *(*fn)(void *), Job base, int64_t n, int threads) {
    if (threads < 1) threads = 1;
    if (threads > 64) threads = 64;
    if (n < 65536) threads = 1;
    pthread_t th[64];
    Job jobs[64];
    int started[64] = {0};
    for (int t = 0; t < threads; t++) {
        jobs[t] = base;
        jobs[t].lo = n * t / threads;
        jobs[t].hi = n * (t + 1) / threads;
    }
    for (int t = 1; t < threads; t++) {
        started[t] = pthread_create(&th[t], NULL, fn, &jobs[t]) == 0;
        if (!started[t]) fn(&jobs[t]);   /* (no thread: done here) */
    }
    fn(&jobs[0]);
    for (int t = 1; t < threads; t++)
        if (started[t]) pthread_join(th[t], NULL);
}

static PyObject *py_lengths(PyObject *self, PyObject *args) {
    unsigned long long ptrs, lens;
    long long n;
    int threads;
    if (!PyArg_ParseTuple(args, "KLKi", &ptrs, &n, &lens, &threads)) return NULL;
    Job j = {(PyObject *const *)(uintptr_t)ptrs, 0, 0, (int64_t *)(uintptr_t)lens, NULL, NULL, NULL};
    Py_BEGIN_ALLOW_THREADS
    run(len_job, j, n, threads);
    Py_END_ALLOW_THREADS
    Py_RETURN_NONE;
}

static PyObject *py_copy(PyObject *self, PyObject *args) {
    unsigned long long ptrs, offs, data;
    long long n;
    int threads;
    if (!PyArg_ParseTuple(args, "KLKKi", &ptrs, &n, &offs, &data, &threads)) return NULL;
    Job j = {(PyObject *const *)(uintptr_t)ptrs, 0, 0, NULL, (const int64_t *)(uintptr_t)offs, (uint8_t *)(uintptr_t)data, NULL};
    Py_BEGIN_ALLOW_THREADS
    run(copy_job, j, n, threads);
    Py_END_ALLOW_THREADS
    Py_RETURN_NONE;
}

static PyObject *py_floats(PyObject *self, PyObject *args) {
    unsigned long long ptrs, vals, kinds;
    long long n;
    int threads;
    if (!PyArg_ParseTuple(args, "KLKKi", &ptrs, &n, &vals, &kinds, &threads)) return NULL;
    Job j = {(PyObject *const *)(uintptr_t)ptrs, 0, 0, NULL, NULL, (uint8_t *)(uintptr_t)kinds, (double *)(uintptr_t)vals};
    Py_BEGIN_ALLOW_THREADS
    run(float_job, j, n, threads);
    Py_END_ALLOW_THREADS
    Py_RETURN_NONE;
}

/* blocks of whole 64-row groups (so that no two threads share a byte of the bitmap): block t = [lo(t), lo(t + 1)) */
static int64_t block_lo(int64_t n, int t, int threads) {
    const int64_t g = (n + 63) / 64;
    const int64_t lo = g * t / threads * 64;
    return lo < n ? lo : n;
}
typedef struct {
    PyObject *const *obj;
    int64_t lo, hi;
    int64_t *offs;
    uint8_t *data, *bitmap;
    int64_t base, bytes, nulls, others;
} Blk;
static void *measure_job(void *p) {
    Blk *b = (Blk *)p;
    int64_t bytes = 0, nulls = 0, others = 0;
    for (int64_t i = b->lo; i < b->hi; i++) {
        PyObject *o = b->obj[i];
        int64_t l;
        if (o == Py_None) { l = -1; nulls++; }
        else if (is_ascii_str(o)) { l = (int64_t)PyUnicode_GET_LENGTH(o); bytes += l; }
        else { l = -2; others++; }
        b->offs[i + 1] = l;
    }
    b->bytes = bytes;
    b->nulls = nulls;
    b->others = others;
    return NULL;
}
static void *fill_job(void *p) {
    Blk *b = (Blk *)p;
    int64_t run = b->base;
    for (int64_t i = b->lo; i < b->hi; i++) {
        const int64_t l = b->offs[i + 1];
        if (l > 0) memcpy(b->data + run, PyUnicode_DATA(b->obj[i]), (size_t)l);
        if (l > 0) run += l;
        b->offs[i + 1] = run;
        if (b->bitmap) {
            if ((i & 7) == 0) b->bitmap[i >> 3] = 0;
            if (l >= 0) b->bitmap[i >> 3] |= (uint8_t)(1u << (i & 7));
        }
    }
    return NULL;
}
static void run_blocks(void *(*fn)(void *), Blk *blk, int threads) {
    pthread_t th[64];
    int started[64] = {0};
    for (int t = 1; t < threads; t++) {
        started[t] = pthread_create(&th[t], NULL, fn, &blk[t]) == 0;
        if (!started[t]) fn(&blk[t]);
    }
    fn(&blk[0]);
    for (int t = 1; t < threads; t++)
        if (started[t]) pthread_join(th[t], NULL);
}
static int clamp_threads(int threads, int64_t n) {
    if (threads < 1) threads = 1;
    if (threads > 64) threads = 64;
    if (n < 65536) threads = 1;
    return threads;
}
static PyObject *py_measure(PyObject *self, PyObject *args) {
    unsigned long long ptrs, offs;
    long long n;
    int threads;
    if (!PyArg_ParseTuple(args, "KLKi", &ptrs, &n, &offs, &threads)) return NULL;
    threads = clamp_threads(threads, n);
    Blk blk[64];
    for (int t = 0; t < threads; t++) {
        memset(&blk[t], 0, sizeof blk[t]);
        blk[t].obj = (PyObject *const *)(uintptr_t)ptrs;
        blk[t].offs = (int64_t *)(uintptr_t)offs;
        blk[t].lo = block_lo(n, t, threads);
        blk[t].hi = block_lo(n, t + 1, threads);
    }
    Py_BEGIN_ALLOW_THREADS
    run_blocks(measure_job, blk, threads);
    Py_END_ALLOW_THREADS
    long long bytes = 0, nulls = 0, others = 0;
    PyObject *per = PyList_New(threads);
    if (!per) return NULL;
    for (int t = 0; t < threads; t++) {
        bytes += blk[t].bytes;
        nulls += blk[t].nulls;
        others += blk[t].others;
        PyList_SET_ITEM(per, t, PyLong_FromLongLong(blk[t].bytes));
    }
    return Py_BuildValue("LLLN", bytes, nulls, others, per);
}
static PyObject *py_fill(PyObject *self, PyObject *args) {
    unsigned long long ptrs, offs, data, bitmap;
    long long n;
    PyObject *per;
    int threads;
    if (!PyArg_ParseTuple(args, "KLKKKOi", &ptrs, &n, &offs, &data, &bitmap, &per, &threads)) return NULL;
    threads = clamp_threads(threads, n);
    if (!PyList_Check(per) || PyList_GET_SIZE(per) != threads) {
        PyErr_SetString(PyExc_ValueError, "fill: block_bytes must be measure's list (same n and threads)");
        return NULL;
    }
    Blk blk[64];
    int64_t base = 0;
    for (int t = 0; t < threads; t++) {
        memset(&blk[t], 0, sizeof blk[t]);
        blk[t].obj = (PyObject *const *)(uintptr_t)ptrs;
        blk[t].offs = (int64_t *)(uintptr_t)offs;
        blk[t].data = (uint8_t *)(uintptr_t)data;
        blk[t].bitmap = (uint8_t *)(uintptr_t)bitmap;
        blk[t].lo = block_lo(n, t, threads);
        blk[t].hi = block_lo(n, t + 1, threads);
        blk[t].base = base;
        base += PyLong_AsLongLong(PyList_GET_ITEM(per, t));
    }
    ((int64_t *)(uintptr_t)offs)[0] = 0;
    Py_BEGIN_ALLOW_THREADS
    run_blocks(fill_job, blk, threads);
    Py_END_ALLOW_THREADS
    Py_RETURN_NONE;
}

static PyMethodDef methods[] = {
    {"measure", py_measure, METH_VARARGS, "fused pass 1: lengths into offs[1..n], totals and per-block bytes"},
    {"fill", py_fill, METH_VARARGS, "fused pass 2: exclusive offsets, the bytes and the validity bitmap"},
    {"floats", py_floats, METH_VARARGS, "values of float objects (kinds: 1 float, 0 None, 2 other)"},
    {"lengths", py_lengths, METH_VARARGS, "byte lengths of compact-ASCII str objects (-1 None, -2 other)"},
    {"copy", py_copy, METH_VARARGS, "copy the compact-ASCII strings' bytes to their offsets"},
    {NULL, NULL, 0, NULL}};

static struct PyModuleDef mod = {PyModuleDef_HEAD_INIT, "_strcols", NULL, -1, methods};

PyMODINIT_FUNC PyInit__strcols(void) { return PyModule_Create(&mod); }
