/* bmpow_pyext.c -- CPython marshalling for the batched receive-side verification
 * (pybitmessage_amd.verify.isProofOfWorkSufficient_batch).
 *
 * The reference checks each received object with protocol.isProofOfWorkSufficient
 * (src/protocol.py:258-286) as it arrives; the batched path hands a whole inventory flood to
 * bmpow_verify_batch_ptrs (include/bmpow.h) in one call.  Gathering the addresses and lengths of
 * 500,000 Python bytes objects costs ~0.1 s in Python (map(id), map(len), numpy) -- as much as the
 * padding, the PCIe upload and the kernel together.  This module walks the list in C
 * (PyList_GET_ITEM / PyBytes_AS_STRING, no copies), releases the GIL and calls the library entry
 * point whose address the caller passes (taken from the ctypes handle, so this module does not
 * link against libbmpow_hip.so).  Pure marshalling: every hash is computed on the GPU.
 */
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef int (*verify_ptrs_fn)(size_t n, const uint8_t *const *objs, const uint64_t *lens, const uint64_t *ntpb,
                              const uint64_t *extra, const int64_t *recv_time, uint8_t *ok_out);

/* Grow-only scratch reused across calls: a flood's arrays are MBs, and fresh pages cost a fault per
 * 4 KB.  Taken under the GIL; a call that finds it busy (another thread inside the library with
 * the GIL released) allocates its own. */
typedef struct {
    const uint8_t **ptrs;
    uint64_t *lens, *vn, *ve;
    int64_t *vr;
    PyObject **held;
    size_t cap;
    int busy;
} scratch_t;

static scratch_t g_scratch;

static void scratch_free(scratch_t *s) {
    free(s->ptrs); free(s->lens); free(s->vn); free(s->ve); free(s->vr); free(s->held);
    memset(s, 0, sizeof(*s));
}

static int scratch_reserve(scratch_t *s, size_t n) {
    if (n <= s->cap) return 0;
    scratch_t t;
    memset(&t, 0, sizeof(t));
    t.ptrs = (const uint8_t **)malloc(sizeof(*t.ptrs) * n);
    t.lens = (uint64_t *)malloc(sizeof(*t.lens) * n);
    t.vn = (uint64_t *)malloc(sizeof(*t.vn) * n);
    t.ve = (uint64_t *)malloc(sizeof(*t.ve) * n);
    t.vr = (int64_t *)malloc(sizeof(*t.vr) * n);
    t.held = (PyObject **)malloc(sizeof(*t.held) * n);
    if (!t.ptrs || !t.lens || !t.vn || !t.ve || !t.vr || !t.held) {
        scratch_free(&t);
        return -1;
    }
    t.cap = n;
    t.busy = s->busy;
    scratch_free(s);
    *s = t;
    return 0;
}

/* verify_list(fn_address, objects: list of bytes, ntpb: int, extra: int, recv: int) -> (rc, bytes ok)
 * rc < 0: the library's error code (the caller reads bmpow_last_error).  TypeError when an item
 * is not a bytes object (the caller converts those first).  A zero ntpb / extra / recv is passed
 * as a null array: the library reads it as 0 (the network minimum, "now"), as the reference does. */
static PyObject *verify_list(PyObject *self, PyObject *args) {
    unsigned long long fn_addr, ntpb, extra;
    long long recv;
    PyObject *list;
    (void)self;
    if (!PyArg_ParseTuple(args, "KO!KKL", &fn_addr, &PyList_Type, &list, &ntpb, &extra, &recv)) return NULL;
    const Py_ssize_t n = PyList_GET_SIZE(list);
    const size_t cap = (size_t)(n ? n : 1);
    scratch_t own;
    memset(&own, 0, sizeof(own));
    scratch_t *sc = g_scratch.busy ? &own : &g_scratch;
    if (scratch_reserve(sc, cap) < 0) {
        scratch_free(&own);
        return PyErr_NoMemory();
    }
    sc->busy = 1;
    PyObject *ok = PyBytes_FromStringAndSize(NULL, n);
    if (!ok) {
        sc->busy = 0;
        scratch_free(&own);
        return PyErr_NoMemory();
    }
    for (Py_ssize_t i = 0; i < n; ++i) {
        /* the objects' headers are scattered over the heap: one cache miss each, so ask early */
        if (i + 16 < n) __builtin_prefetch(PyList_GET_ITEM(list, i + 16), 1);
        PyObject *o = PyList_GET_ITEM(list, i);
        if (!PyBytes_CheckExact(o)) {
            for (Py_ssize_t j = 0; j < i; ++j) Py_DECREF(sc->held[j]);
            sc->busy = 0;
            scratch_free(&own);
            Py_DECREF(ok);
            return PyErr_Format(PyExc_TypeError, "object %zd is not bytes", i);
        }
        /* a reference of our own: another thread may change the list while the GIL is released */
        Py_INCREF(o);
        sc->held[i] = o;
        sc->ptrs[i] = (const uint8_t *)PyBytes_AS_STRING(o);
        sc->lens[i] = (uint64_t)PyBytes_GET_SIZE(o);
    }
    const uint64_t *vn = NULL, *ve = NULL;
    const int64_t *vr = NULL;
    if (ntpb) { for (Py_ssize_t i = 0; i < n; ++i) sc->vn[i] = ntpb; vn = sc->vn; }
    if (extra) { for (Py_ssize_t i = 0; i < n; ++i) sc->ve[i] = extra; ve = sc->ve; }
    if (recv) { for (Py_ssize_t i = 0; i < n; ++i) sc->vr[i] = recv; vr = sc->vr; }
    int rc;
    Py_BEGIN_ALLOW_THREADS
    rc = ((verify_ptrs_fn)(uintptr_t)fn_addr)((size_t)n, sc->ptrs, sc->lens, vn, ve, vr,
                                              (uint8_t *)PyBytes_AS_STRING(ok));
    Py_END_ALLOW_THREADS
    /* the headers were evicted by the payload pass meanwhile: ask for them ahead again */
    for (Py_ssize_t i = 0; i < n; ++i) {
        if (i + 16 < n) __builtin_prefetch(sc->held[i + 16], 1);
        Py_DECREF(sc->held[i]);
    }
    sc->busy = 0;
    scratch_free(&own);
    PyObject *res = Py_BuildValue("(iO)", rc, ok);
    Py_DECREF(ok);
    return res;
}

/* verdicts(ok: bytes of 0/1) -> list of bool.  numpy's bool tolist() costs ~16 ns per object (8 ms for a
 * 500k flood, a fifth of the whole call); the two singletons referenced directly cost a few ns. */
static PyObject *verdicts(PyObject *self, PyObject *arg) {
    (void)self;
    if (!PyBytes_Check(arg)) return PyErr_Format(PyExc_TypeError, "verdicts() takes bytes");
    const Py_ssize_t n = PyBytes_GET_SIZE(arg);
    const unsigned char *ok = (const unsigned char *)PyBytes_AS_STRING(arg);
    PyObject *list = PyList_New(n);
    if (!list) return NULL;
    PyObject **items = ((PyListObject *)list)->ob_item;
    Py_ssize_t nt = 0;
    for (Py_ssize_t i = 0; i < n; ++i) {
        const int t = ok[i] != 0;
        nt += t;
        items[i] = t ? Py_True : Py_False;
    }
    /* one reference per slot, added in two sums instead of n increments of two shared counters (on
     * an interpreter with immortal singletons, 3.12+, Py_SET_REFCNT leaves them alone, as Py_INCREF
     * would) */
    Py_SET_REFCNT(Py_True, Py_REFCNT(Py_True) + nt);
    Py_SET_REFCNT(Py_False, Py_REFCNT(Py_False) + (n - nt));
    return list;
}

static PyMethodDef methods[] = {
    {"verify_list", verify_list, METH_VARARGS, "bmpow_verify_batch_ptrs over a list of bytes (see module doc)"},
    {"verdicts", verdicts, METH_O, "bytes of 0/1 -> list of bool"},
    {NULL, NULL, 0, NULL}};

static struct PyModuleDef module = {PyModuleDef_HEAD_INIT, "_bmpow_fast",
                                    "CPython marshalling for libbmpow_hip.so's batched verification", -1, methods,
                                    NULL, NULL, NULL, NULL};

PyMODINIT_FUNC PyInit__bmpow_fast(void) { return PyModule_Create(&module); }
