/*
 * _pebblefast — the per-key calls of the drop-in class without ctypes.
 *
 * LsmStorage.get calls `sstable.bloom_filter.may_contain(key)` once per SSTable and key
 * (reference src/lsm_storage.py:164-179, bloom_filter.py:67-74).  Through ctypes each call pays
 * argument conversion, a byref and the foreign-call machinery (~2 us) around a 3 us bus round trip
 * to the device's resident reader wave.  Here the str goes straight to the C-ABI entry point
 * (include/pebblebloom.h pbf_may_contain / pbf_may_contain_set), whose addresses the Python layer
 * takes from the loaded libpebblebloom.so once (bind); the key's UTF-8 bytes are CPython's cached
 * form (what key.encode("utf-8") produces, bloom_filter.py:43), and the GIL is released while the
 * device answers, so reader threads overlap their waits.
 *
 * Host code; every GPU operation happens inside the library call.
 */
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#include <stdint.h>

typedef int (*may_contain_fn)(void*, const uint8_t*, uint64_t, int*);
typedef int (*may_contain_set_fn)(void* const*, uint32_t, const uint8_t*, uint64_t, uint8_t*);

static may_contain_fn g_may_contain;
static may_contain_set_fn g_may_contain_set;

/* Result codes the Python layer handles (the library's own are PBF_ERR_* < 0). */
#define FAST_NOT_STR (-100) /* key is not a str: the caller's slow path raises what the reference raises */

static PyObject* py_bind(PyObject* self, PyObject* args) {
    unsigned long long mc, mcs;
    if (!PyArg_ParseTuple(args, "KK", &mc, &mcs)) return NULL;
    g_may_contain = (may_contain_fn)(uintptr_t)mc;
    g_may_contain_set = (may_contain_set_fn)(uintptr_t)mcs;
    Py_RETURN_NONE;
}

/* may_contain(handle, key) -> True / False, or an int result code (< 0). */
static PyObject* py_may_contain(PyObject* self, PyObject* const* args, Py_ssize_t nargs) {
    if (nargs != 2) {
        PyErr_SetString(PyExc_TypeError, "may_contain(handle, key)");
        return NULL;
    }
    if (!g_may_contain) {
        PyErr_SetString(PyExc_RuntimeError, "_pebblefast is not bound to libpebblebloom.so");
        return NULL;
    }
    void* h = PyLong_AsVoidPtr(args[0]);
    if (!h && PyErr_Occurred()) return NULL;
    if (!PyUnicode_Check(args[1])) return PyLong_FromLong(FAST_NOT_STR);
    Py_ssize_t len;
    const char* s = PyUnicode_AsUTF8AndSize(args[1], &len);
    if (!s) return NULL; /* UnicodeEncodeError, as key.encode("utf-8") raises */
    int out = 0, rc;
    Py_BEGIN_ALLOW_THREADS
    rc = g_may_contain(h, (const uint8_t*)s, (uint64_t)len, &out);
    Py_END_ALLOW_THREADS
    if (rc) return PyLong_FromLong(rc);
    if (out) Py_RETURN_TRUE;
    Py_RETURN_FALSE;
}

/* may_contain_set(handles, key) -> (0, bits) with bit i = filters[i].may_contain(key), or
 * (result code < 0, 0).  handles: a list or tuple of at most 64 handle ints. */
static PyObject* py_may_contain_set(PyObject* self, PyObject* const* args, Py_ssize_t nargs) {
    if (nargs != 2) {
        PyErr_SetString(PyExc_TypeError, "may_contain_set(handles, key)");
        return NULL;
    }
    if (!g_may_contain_set) {
        PyErr_SetString(PyExc_RuntimeError, "_pebblefast is not bound to libpebblebloom.so");
        return NULL;
    }
    PyObject* seq = PySequence_Fast(args[0], "handles must be a sequence");
    if (!seq) return NULL;
    const Py_ssize_t nf = PySequence_Fast_GET_SIZE(seq);
    if (nf > 64) {
        Py_DECREF(seq);
        PyErr_SetString(PyExc_ValueError, "at most 64 filters per call");
        return NULL;
    }
    void* hs[64];
    PyObject** items = PySequence_Fast_ITEMS(seq);
    for (Py_ssize_t i = 0; i < nf; ++i) {
        hs[i] = PyLong_AsVoidPtr(items[i]);
        if (!hs[i] && PyErr_Occurred()) {
            Py_DECREF(seq);
            return NULL;
        }
    }
    Py_DECREF(seq);
    if (!PyUnicode_Check(args[1])) return Py_BuildValue("(ii)", FAST_NOT_STR, 0);
    Py_ssize_t len;
    const char* s = PyUnicode_AsUTF8AndSize(args[1], &len);
    if (!s) return NULL;
    uint8_t bits[8] = {0};
    int rc = 0;
    if (nf) {
        Py_BEGIN_ALLOW_THREADS
        rc = g_may_contain_set(hs, (uint32_t)nf, (const uint8_t*)s, (uint64_t)len, bits);
        Py_END_ALLOW_THREADS
    }
    if (rc) return Py_BuildValue("(ii)", rc, 0);
    uint64_t v = 0;
    for (int i = 0; i < 8; ++i) v |= (uint64_t)bits[i] << (8 * i);
    return Py_BuildValue("(iK)", 0, (unsigned long long)v);
}

/* candidates_one(key, level0, levels) -> the list lsm_get.candidates_one returns, or None when
 * the Python path must take the call (a non-str key, a filter with buffered adds or another
 * device, more than 64 filters, a comparison that raised, any library error: that path
 * reproduces the reference's exceptions and raises the library's).  One LsmStorage.get(key)'s
 * filter stage (reference src/lsm_storage.py:164-179): every L0 filter, newest first, then per
 * level the tables with first_key <= key <= last_key (:173), all tested in ONE
 * pbf_may_contain_set call; the result numbers the tables as candidate_masks rows. */
static PyObject* s_fast, *s_first, *s_last, *s_bf;

static int handle_of(PyObject* bf, void** out) { /* 1 ok, 0 fall back, -1 error */
    PyObject* v = PyObject_GetAttr(bf, s_fast);
    if (!v) {
        PyErr_Clear();
        return 0;
    }
    void* h = PyLong_Check(v) ? PyLong_AsVoidPtr(v) : NULL;
    Py_DECREF(v);
    if (!h) {
        PyErr_Clear();
        return 0;
    }
    *out = h;
    return 1;
}

static PyObject* py_candidates_one(PyObject* self, PyObject* const* args, Py_ssize_t nargs) {
    if (nargs != 3) {
        PyErr_SetString(PyExc_TypeError, "candidates_one(key, level0, levels)");
        return NULL;
    }
    if (!g_may_contain_set) {
        PyErr_SetString(PyExc_RuntimeError, "_pebblefast is not bound to libpebblebloom.so");
        return NULL;
    }
    PyObject* key = args[0];
    if (!PyUnicode_Check(key)) Py_RETURN_NONE;
    void* hs[64];
    int32_t in_range[64];
    uint32_t nt = 0, ni = 0;
    PyObject* l0 = PySequence_Fast(args[1], "level0 must be a sequence");
    if (!l0) {
        PyErr_Clear();
        Py_RETURN_NONE;
    }
    const Py_ssize_t n0 = PySequence_Fast_GET_SIZE(l0);
    int ok = n0 <= 64;
    for (Py_ssize_t i = 0; ok && i < n0; ++i) ok = handle_of(PySequence_Fast_GET_ITEM(l0, i), &hs[nt++]);
    Py_DECREF(l0);
    if (!ok) Py_RETURN_NONE;
    PyObject* lv = PySequence_Fast(args[2], "levels must be a sequence");
    if (!lv) {
        PyErr_Clear();
        Py_RETURN_NONE;
    }
    int32_t j = (int32_t)n0;
    for (Py_ssize_t a = 0; ok && a < PySequence_Fast_GET_SIZE(lv); ++a) {
        PyObject* lvl = PySequence_Fast(PySequence_Fast_GET_ITEM(lv, a), "a level must be a sequence");
        if (!lvl) {
            ok = 0;
            break;
        }
        for (Py_ssize_t b = 0; ok && b < PySequence_Fast_GET_SIZE(lvl); ++b, ++j) {
            PyObject* t = PySequence_Fast_GET_ITEM(lvl, b);
            PyObject* first = PyObject_GetAttr(t, s_first);
            PyObject* last = first ? PyObject_GetAttr(t, s_last) : NULL;
            int in = -1;
            if (last) {
                in = PyObject_RichCompareBool(first, key, Py_LE);
                if (in == 1) in = PyObject_RichCompareBool(key, last, Py_LE);
            }
            Py_XDECREF(first);
            Py_XDECREF(last);
            if (in < 0) {
                ok = 0;
                break;
            }
            if (!in) continue;
            if (nt == 64) {
                ok = 0;
                break;
            }
            PyObject* bf = PyObject_GetAttr(t, s_bf);
            ok = bf ? handle_of(bf, &hs[nt]) : 0;
            Py_XDECREF(bf);
            ++nt;
            in_range[ni++] = j;
        }
        Py_DECREF(lvl);
    }
    Py_DECREF(lv);
    if (!ok) {
        PyErr_Clear();
        Py_RETURN_NONE;
    }
    if (nt == 0) return PyList_New(0);
    Py_ssize_t len;
    const char* s = PyUnicode_AsUTF8AndSize(key, &len);
    if (!s) {
        PyErr_Clear();
        Py_RETURN_NONE;
    }
    uint8_t bits[8] = {0};
    int rc;
    Py_BEGIN_ALLOW_THREADS
    rc = g_may_contain_set(hs, nt, (const uint8_t*)s, (uint64_t)len, bits);
    Py_END_ALLOW_THREADS
    if (rc) Py_RETURN_NONE;
    uint64_t v = 0;
    for (int i = 0; i < 8; ++i) v |= (uint64_t)bits[i] << (8 * i);
    PyObject* out = PyList_New(0);
    if (!out) return NULL;
    for (uint32_t i = 0; i < nt; ++i) {
        if (!((v >> i) & 1u)) continue;
        PyObject* x = PyLong_FromLong(i < (uint32_t)n0 ? (long)i : (long)in_range[i - (uint32_t)n0]);
        if (!x || PyList_Append(out, x)) {
            Py_XDECREF(x);
            Py_DECREF(out);
            return NULL;
        }
        Py_DECREF(x);
    }
    return out;
}

static PyMethodDef methods[] = {
    {"bind", py_bind, METH_VARARGS, "bind(pbf_may_contain address, pbf_may_contain_set address)"},
    {"may_contain", (PyCFunction)(void (*)(void))py_may_contain, METH_FASTCALL,
     "may_contain(handle, key) -> bool, or a negative result code"},
    {"may_contain_set", (PyCFunction)(void (*)(void))py_may_contain_set, METH_FASTCALL,
     "may_contain_set(handles, key) -> (rc, bits)"},
    {"candidates_one", (PyCFunction)(void (*)(void))py_candidates_one, METH_FASTCALL,
     "candidates_one(key, level0, levels) -> list of candidate rows, or None (take the Python path)"},
    {NULL, NULL, 0, NULL},
};

static struct PyModuleDef module = {PyModuleDef_HEAD_INIT, "_pebblefast", NULL, -1, methods};

PyMODINIT_FUNC PyInit__pebblefast(void) {
    s_fast = PyUnicode_InternFromString("_fast");
    s_first = PyUnicode_InternFromString("first_key");
    s_last = PyUnicode_InternFromString("last_key");
    s_bf = PyUnicode_InternFromString("bloom_filter");
    if (!s_fast || !s_first || !s_last || !s_bf) return NULL;
    return PyModule_Create(&module);
}
