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

typedef int (*verify_ptrs_fn)(size_t n, const uint8_t *const *objs, const uint64_t *lens, const uint64_t *ntpb,
                              const uint64_t *extra, const int64_t *recv_time, uint8_t *ok_out);

/* verify_list(fn_address, objects: list of bytes, ntpb: int, extra: int, recv: int) -> (rc, bytes ok)
 * rc < 0: the library's error code (the caller reads bmpow_last_error).  TypeError when an item
 * is not a bytes object (the caller converts those first). */
static PyObject *verify_list(PyObject *self, PyObject *args) {
    unsigned long long fn_addr, ntpb, extra;
    long long recv;
    PyObject *list;
    (void)self;
    if (!PyArg_ParseTuple(args, "KO!KKL", &fn_addr, &PyList_Type, &list, &ntpb, &extra, &recv)) return NULL;
    const Py_ssize_t n = PyList_GET_SIZE(list);
    const uint8_t **ptrs = (const uint8_t **)malloc(sizeof(*ptrs) * (size_t)(n ? n : 1));
    uint64_t *lens = (uint64_t *)malloc(sizeof(*lens) * (size_t)(n ? n : 1));
    uint64_t *vn = (uint64_t *)malloc(sizeof(*vn) * (size_t)(n ? n : 1));
    uint64_t *ve = (uint64_t *)malloc(sizeof(*ve) * (size_t)(n ? n : 1));
    int64_t *vr = (int64_t *)malloc(sizeof(*vr) * (size_t)(n ? n : 1));
    PyObject *ok = PyBytes_FromStringAndSize(NULL, n);
    if (!ptrs || !lens || !vn || !ve || !vr || !ok) {
        free(ptrs); free(lens); free(vn); free(ve); free(vr);
        Py_XDECREF(ok);
        return PyErr_NoMemory();
    }
    PyObject **held = (PyObject **)malloc(sizeof(*held) * (size_t)(n ? n : 1));
    if (!held) {
        free(ptrs); free(lens); free(vn); free(ve); free(vr);
        Py_DECREF(ok);
        return PyErr_NoMemory();
    }
    for (Py_ssize_t i = 0; i < n; ++i) {
        PyObject *o = PyList_GET_ITEM(list, i);
        if (!PyBytes_CheckExact(o)) {
            for (Py_ssize_t j = 0; j < i; ++j) Py_DECREF(held[j]);
            free(held); free(ptrs); free(lens); free(vn); free(ve); free(vr);
            Py_DECREF(ok);
            return PyErr_Format(PyExc_TypeError, "object %zd is not bytes", i);
        }
        /* a reference of our own: another thread may change the list while the GIL is released */
        Py_INCREF(o);
        held[i] = o;
        ptrs[i] = (const uint8_t *)PyBytes_AS_STRING(o);
        lens[i] = (uint64_t)PyBytes_GET_SIZE(o);
        vn[i] = ntpb;
        ve[i] = extra;
        vr[i] = recv;
    }
    int rc;
    Py_BEGIN_ALLOW_THREADS
    rc = ((verify_ptrs_fn)(uintptr_t)fn_addr)((size_t)n, ptrs, lens, vn, ve, vr, (uint8_t *)PyBytes_AS_STRING(ok));
    Py_END_ALLOW_THREADS
    for (Py_ssize_t i = 0; i < n; ++i) Py_DECREF(held[i]);
    free(held); free(ptrs); free(lens); free(vn); free(ve); free(vr);
    PyObject *res = Py_BuildValue("(iO)", rc, ok);
    Py_DECREF(ok);
    return res;
}

static PyMethodDef methods[] = {
    {"verify_list", verify_list, METH_VARARGS, "bmpow_verify_batch_ptrs over a list of bytes (see module doc)"},
    {NULL, NULL, 0, NULL}};

static struct PyModuleDef module = {PyModuleDef_HEAD_INIT, "_bmpow_fast",
                                    "CPython marshalling for libbmpow_hip.so's batched verification", -1, methods,
                                    NULL, NULL, NULL, NULL};

PyMODINIT_FUNC PyInit__bmpow_fast(void) { return PyModule_Create(&module); }
