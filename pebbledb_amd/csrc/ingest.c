/*
 * _pebbleingest — packed-key ingestion straight from the flush / compaction iterators
 * (reference src/sstable.py:224-244 SSTableBuilder.add, which appends
 * every key to a Python list, and src/iterators.py:24-55,144-190, which yield the records).
 *
 * One C loop drains any iterable and appends each record's UTF-8 key bytes, value bytes and
 * u64 end offsets to growing buffers — the boundary layout of include/pebblebloom.h — with no
 * list[str] / list[bytes] materialised and no Python bytecode per record.  Accepted items:
 *   str / bytes                      a key (pack_keys)
 *   (key, value) tuple or list       a record
 *   any object with .key and .value  a Record (src/record.py:4, what the iterators yield)
 * Keys are encoded exactly as bloom_filter.py:43 does (str.encode("utf-8"); CPython's cached
 * UTF-8 form, no copy for ASCII strings).  Values are any buffer-protocol object (bytes).
 * Host-side code: it never touches a GPU.
 */
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>

/* Growing output buffers are anonymous mappings (mremap to grow, transparent huge pages asked
 * for): a flush-sized run is hundreds of MB, and first-touch faults of 4 KiB pages, not the
 * copying, would otherwise bound the packing rate.  The finished mapping is handed to Python
 * without a copy, owned by a PackedBuffer object (buffer protocol; np.frombuffer keeps it). */
typedef struct {
    char* p;
    size_t n, cap;
} Buf;

static int buf_grow(Buf* b, size_t want) {
    size_t c = b->cap ? b->cap : ((size_t)1 << 21);
    while (c < want) c *= 2;
    void* q = b->p ? mremap(b->p, b->cap, c, MREMAP_MAYMOVE)
                   : mmap(NULL, c, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (q == MAP_FAILED) {
        PyErr_NoMemory();
        return -1;
    }
#ifdef MADV_HUGEPAGE
    (void)madvise(q, c, MADV_HUGEPAGE);
#endif
    b->p = (char*)q;
    b->cap = c;
    return 0;
}

static inline int buf_put(Buf* b, const void* s, size_t len) {
    if (b->n + len > b->cap && buf_grow(b, b->n + len)) return -1;
    if (len) memcpy(b->p + b->n, s, len);
    b->n += len;
    return 0;
}

static inline int buf_u64(Buf* b, uint64_t v) { return buf_put(b, &v, 8); }

static void buf_free(Buf* b) {
    if (b->p) munmap(b->p, b->cap);
    b->p = NULL;
    b->n = b->cap = 0;
}

typedef struct {
    PyObject_HEAD Buf b;
} PackedBuffer;

static int pb_getbuffer(PyObject* self, Py_buffer* view, int flags) {
    PackedBuffer* o = (PackedBuffer*)self;
    static char empty[1];
    return PyBuffer_FillInfo(view, self, o->b.p ? o->b.p : empty, (Py_ssize_t)o->b.n, 0, flags);
}

static void pb_dealloc(PyObject* self) {
    buf_free(&((PackedBuffer*)self)->b);
    Py_TYPE(self)->tp_free(self);
}

static Py_ssize_t pb_len(PyObject* self) { return (Py_ssize_t)((PackedBuffer*)self)->b.n; }

static PyBufferProcs pb_as_buffer = {pb_getbuffer, NULL};
static PySequenceMethods pb_as_seq = {pb_len};

static PyTypeObject PackedBufferType = {
    PyVarObject_HEAD_INIT(NULL, 0).tp_name = "_pebbleingest.PackedBuffer",
    .tp_basicsize = sizeof(PackedBuffer),
    .tp_dealloc = pb_dealloc,
    .tp_as_sequence = &pb_as_seq,
    .tp_as_buffer = &pb_as_buffer,
    .tp_flags = Py_TPFLAGS_DEFAULT,
    .tp_doc = "packed key / value / offset bytes (an anonymous mapping; buffer protocol)",
};

/* Hand the mapping to a PackedBuffer (no copy); b is left empty. */
static PyObject* buf_release(Buf* b) {
    PackedBuffer* o = PyObject_New(PackedBuffer, &PackedBufferType);
    if (!o) {
        buf_free(b);
        return NULL;
    }
    o->b = *b;
    b->p = NULL;
    b->n = b->cap = 0;
    return (PyObject*)o;
}

static PyObject* s_key;
static PyObject* s_value;
static PyObject* s_struct_error;

/* UTF-8 bytes of a key object (str or bytes); *ascii cleared for a non-ASCII str. */
static int key_view(PyObject* k, const char** s, Py_ssize_t* len, int* ascii) {
    if (PyUnicode_Check(k)) {
        *s = PyUnicode_AsUTF8AndSize(k, len);
        if (!*s) return -1;
        if (!PyUnicode_IS_ASCII(k)) *ascii = 0;
        return 0;
    }
    if (PyBytes_Check(k)) {
        *s = PyBytes_AS_STRING(k);
        *len = PyBytes_GET_SIZE(k);
        return 0;
    }
    PyErr_Format(PyExc_TypeError, "key must be str or bytes, not %.100s", Py_TYPE(k)->tp_name);
    return -1;
}

/* Split an item into borrowed-or-new (key, value) references.  *kv_owned tells whether the two
 * references must be released. */
static int split_item(PyObject* item, int with_values, PyObject** k, PyObject** v, int* owned) {
    *owned = 0;
    *v = NULL;
    if (PyUnicode_Check(item) || PyBytes_Check(item)) {
        if (with_values) {
            PyErr_SetString(PyExc_TypeError, "pack_records: a bare key has no value");
            return -1;
        }
        *k = item;
        return 0;
    }
    if ((PyTuple_Check(item) && PyTuple_GET_SIZE(item) == 2) || (PyList_Check(item) && PyList_GET_SIZE(item) == 2)) {
        *k = PySequence_Fast_GET_ITEM(item, 0);
        *v = PySequence_Fast_GET_ITEM(item, 1);
        return 0;
    }
    *k = PyObject_GetAttr(item, s_key);
    if (!*k) {
        if (PyErr_ExceptionMatches(PyExc_AttributeError)) {
            PyErr_Clear();
            PyErr_Format(PyExc_TypeError, "expected str, bytes, a (key, value) pair or a record with .key, not %.100s",
                         Py_TYPE(item)->tp_name);
        }
        return -1;
    }
    if (with_values) {
        *v = PyObject_GetAttr(item, s_value);
        if (!*v) {
            Py_DECREF(*k);
            return -1;
        }
    }
    *owned = 1;
    return 0;
}

/* One item of a list / tuple (borrowed) or of an iterator (new reference). */
static PyObject* next_item(PyObject* seq, PyObject* it, Py_ssize_t* i) {
    if (seq) {
        if (*i >= PySequence_Fast_GET_SIZE(seq)) return NULL;
        PyObject* o = PySequence_Fast_GET_ITEM(seq, *i);
        ++*i;
        Py_INCREF(o);
        return o;
    }
    return PyIter_Next(it);
}

/* pack(iterable, with_values) -> (key_bytes, key_offsets, value_bytes, value_offsets, n, ascii,
 * min_len, max_len); offsets are little-endian u64 [n+1] in bytearrays, starting at 0.  A list
 * or tuple is walked by index (no iterator protocol) with its buffers sized up front. */
static PyObject* pack_impl(PyObject* iterable, int with_values) {
    PyObject* seq = (PyList_CheckExact(iterable) || PyTuple_CheckExact(iterable)) ? iterable : NULL;
    PyObject* it = seq ? NULL : PyObject_GetIter(iterable);
    if (!seq && !it) return NULL;
    Py_ssize_t idx = 0;
    Buf kb = {0}, ko = {0}, vb = {0}, vo = {0};
    uint64_t n = 0, min_len = UINT64_MAX, max_len = 0;
    int ascii = 1;
    if (seq) {  // reserve: offsets exactly, key bytes at 16 per key (grown on demand)
        const size_t cnt = (size_t)PySequence_Fast_GET_SIZE(seq);
        if (buf_grow(&ko, (cnt + 1) * 8) || buf_grow(&kb, cnt * 16 + 64)) goto fail;
        if (with_values && buf_grow(&vo, (cnt + 1) * 8)) goto fail;
    }
    if (buf_u64(&ko, 0) || (with_values && buf_u64(&vo, 0))) goto fail;
    PyObject* item;
    while ((item = next_item(seq, it, &idx))) {
        PyObject *k, *v;
        int owned;
        if (split_item(item, with_values, &k, &v, &owned)) {
            Py_DECREF(item);
            goto fail;
        }
        const char* s;
        Py_ssize_t len;
        int rc = key_view(k, &s, &len, &ascii);
        if (!rc) rc = buf_put(&kb, s, (size_t)len);
        if (!rc) rc = buf_u64(&ko, kb.n);
        if (!rc && with_values) {
            Py_buffer view;
            rc = PyObject_GetBuffer(v, &view, PyBUF_SIMPLE);
            if (!rc) {
                rc = buf_put(&vb, view.buf, (size_t)view.len);
                PyBuffer_Release(&view);
            }
            if (!rc) rc = buf_u64(&vo, vb.n);
        }
        if ((uint64_t)len < min_len) min_len = (uint64_t)len;
        if ((uint64_t)len > max_len) max_len = (uint64_t)len;
        if (owned) {
            Py_DECREF(k);
            Py_XDECREF(v);
        }
        Py_DECREF(item);
        if (rc) goto fail;
        ++n;
    }
    if (PyErr_Occurred()) goto fail;
    Py_XDECREF(it);
    if (n == 0) min_len = 0;
    PyObject* a = buf_release(&kb);
    PyObject* b = buf_release(&ko);
    PyObject* c = buf_release(&vb);
    PyObject* d = buf_release(&vo);
    if (!a || !b || !c || !d) {
        Py_XDECREF(a);
        Py_XDECREF(b);
        Py_XDECREF(c);
        Py_XDECREF(d);
        return NULL;
    }
    return Py_BuildValue("(NNNNKiKK)", a, b, c, d, (unsigned long long)n, ascii, (unsigned long long)min_len,
                         (unsigned long long)max_len);
fail:
    Py_XDECREF(it);
    buf_free(&kb);
    buf_free(&ko);
    buf_free(&vb);
    buf_free(&vo);
    return NULL;
}

/* pack_encoded(iterable of bytes-like) — records as the memtable stores them (the values of
 * memtable.map, Record.to_bytes record.py:66-72: i32 key_size | key | i32 value_size | value),
 * split exactly as Record._from_bytes does (record.py:77-88): key = the key_size bytes after
 * the first i32 (the reference slices BYTES by key_size), value = the value_size bytes after the
 * second, both clipped to the data as Python slicing clips them.  A key that is not valid UTF-8
 * raises UnicodeDecodeError and a size field cut short raises struct.error, as the reference's
 * decoder would; a negative size raises ValueError (the reference would slice backwards). */
/* Strict UTF-8 check, the rules of CPython's decoder (what key.decode("utf-8") accepts): no
 * continuation or 0xC0/0xC1/0xF5+ lead bytes, no overlong 3- and 4-byte forms, no surrogates
 * (ED A0..BF), nothing above U+10FFFF (F4 90+), no truncated sequence. */
static int utf8_valid(const unsigned char* s, size_t n) {
    size_t i = 0;
    while (i < n) {
        const unsigned c = s[i];
        if (c < 0x80) {
            ++i;
            continue;
        }
        size_t len;
        unsigned lo = 0x80, hi = 0xBF;  // range of the first continuation byte
        if (c >= 0xC2 && c <= 0xDF) {
            len = 2;
        } else if (c >= 0xE0 && c <= 0xEF) {
            len = 3;
            if (c == 0xE0) lo = 0xA0;
            if (c == 0xED) hi = 0x9F;
        } else if (c >= 0xF0 && c <= 0xF4) {
            len = 4;
            if (c == 0xF0) lo = 0x90;
            if (c == 0xF4) hi = 0x8F;
        } else {
            return 0;
        }
        if (i + len > n) return 0;
        if (s[i + 1] < lo || s[i + 1] > hi) return 0;
        for (size_t j = 2; j < len; ++j)
            if ((s[i + j] & 0xC0) != 0x80) return 0;
        i += len;
    }
    return 1;
}

/* The parallel form of pack_encoded for a list / tuple of exact bytes objects (the memtable's
 * records as they come out of memtable.map.values()).  Pass 1 (threads) splits every record
 * and validates non-ASCII keys; a prefix sum places them; pass 2 (threads) copies keys and
 * values to their final offsets.  The calling thread keeps the GIL throughout, so no Python
 * code can change the list or free a record while the worker threads (plain memory reads, no
 * Python API) look at them; touching the million scattered objects in parallel is the point.
 * Returns Py_None (no exception) when an item is not an exact bytes object or a record is
 * malformed: the serial loop below then runs from the start and raises exactly what the
 * reference's decoder would, in its order. */
typedef struct {
    const unsigned char* d;   // the record's bytes
    uint32_t kl, vo, vl, ok;  // clipped key length (key at d + 4), value start and length
} RecSplit;

static PyObject* pack_encoded_parallel(PyObject* seq) {
    const Py_ssize_t n = PySequence_Fast_GET_SIZE(seq);
    PyObject** items = PySequence_Fast_ITEMS(seq);
    RecSplit* rs = (RecSplit*)malloc(sizeof(*rs) * (size_t)(n ? n : 1));
    if (!rs) return PyErr_NoMemory();
    int bad = 0, ascii = 1;
    uint64_t min_len = UINT64_MAX, max_len = 0, kt = 0, vt = 0;
#pragma omp parallel for schedule(static) reduction(| : bad) reduction(& : ascii) reduction(min : min_len) \
    reduction(max : max_len)
    for (Py_ssize_t i = 0; i < n; ++i) {
        PyObject* o = items[i];
        rs[i].ok = 0;
        if (Py_TYPE(o) != &PyBytes_Type) {
            bad = 1;
            continue;
        }
        const unsigned char* r = (const unsigned char*)PyBytes_AS_STRING(o);
        const size_t len = (size_t)PyBytes_GET_SIZE(o);
        int32_t ks, vs;
        if (len < 4) {
            bad = 1;
            continue;
        }
        memcpy(&ks, r, 4);
        const size_t key_end = 4 + (size_t)(uint32_t)ks;
        if (ks < 0 || key_end + 4 > len) {
            bad = 1;
            continue;
        }
        const size_t kl = (size_t)ks;
        int a = 1;
        for (size_t c = 0; c < kl; ++c)
            if (r[4 + c] & 0x80) {
                a = 0;
                break;
            }
        if (!a) {
            ascii = 0;
            if (!utf8_valid(r + 4, kl)) {
                bad = 1;
                continue;
            }
        }
        memcpy(&vs, r + key_end, 4);
        if (vs < 0) {
            bad = 1;
            continue;
        }
        const size_t v0 = key_end + 4;
        rs[i].d = r;
        rs[i].kl = (uint32_t)kl;
        rs[i].vo = (uint32_t)v0;
        rs[i].vl = (uint32_t)(v0 + (size_t)vs <= len ? (size_t)vs : len - v0);
        rs[i].ok = 1;
        if ((uint64_t)kl < min_len) min_len = (uint64_t)kl;
        if ((uint64_t)kl > max_len) max_len = (uint64_t)kl;
    }
    Buf kb = {0}, ko = {0}, vb = {0}, vo = {0};
    PyObject* ret = NULL;
    if (bad) {  // let the serial loop raise the reference's exception
        Py_INCREF(Py_None);
        ret = Py_None;
        goto done;
    }
    if (buf_grow(&ko, ((size_t)n + 1) * 8) || buf_grow(&vo, ((size_t)n + 1) * 8)) goto done;
    {
        uint64_t* kof = (uint64_t*)ko.p;
        uint64_t* vof = (uint64_t*)vo.p;
        kof[0] = vof[0] = 0;
        for (Py_ssize_t i = 0; i < n; ++i) {
            kt += rs[i].kl;
            vt += rs[i].vl;
            kof[i + 1] = kt;
            vof[i + 1] = vt;
        }
        ko.n = vo.n = ((size_t)n + 1) * 8;
        if (buf_grow(&kb, kt ? kt : 1) || buf_grow(&vb, vt ? vt : 1)) goto done;
        kb.n = kt;
        vb.n = vt;
        char* kp = kb.p;
        char* vp = vb.p;
#pragma omp parallel for schedule(static)
        for (Py_ssize_t i = 0; i < n; ++i) {
            memcpy(kp + kof[i], rs[i].d + 4, rs[i].kl);
            memcpy(vp + vof[i], rs[i].d + rs[i].vo, rs[i].vl);
        }
    }
    if (n == 0) min_len = 0;
    {
        PyObject* a = buf_release(&kb);
        PyObject* b = buf_release(&ko);
        PyObject* c = buf_release(&vb);
        PyObject* e = buf_release(&vo);
        if (a && b && c && e)
            ret = Py_BuildValue("(NNNNKiKK)", a, b, c, e, (unsigned long long)n, ascii, (unsigned long long)min_len,
                                (unsigned long long)max_len);
        else {
            Py_XDECREF(a);
            Py_XDECREF(b);
            Py_XDECREF(c);
            Py_XDECREF(e);
        }
    }
done:
    buf_free(&kb);
    buf_free(&ko);
    buf_free(&vb);
    buf_free(&vo);
    free(rs);
    return ret;
}

static PyObject* py_pack_encoded(PyObject* self, PyObject* args) {
    PyObject* iterable;
    if (!PyArg_ParseTuple(args, "O", &iterable)) return NULL;
    if ((PyList_CheckExact(iterable) || PyTuple_CheckExact(iterable)) && PySequence_Fast_GET_SIZE(iterable) > 4096) {
        PyObject* r = pack_encoded_parallel(iterable);
        if (r != Py_None) return r;  // packed, or an exception (out of memory)
        Py_DECREF(r);
    }
    PyObject* seq = (PyList_CheckExact(iterable) || PyTuple_CheckExact(iterable)) ? iterable : NULL;
    PyObject* it = seq ? NULL : PyObject_GetIter(iterable);
    if (!seq && !it) return NULL;
    Py_ssize_t idx = 0;
    Buf kb = {0}, ko = {0}, vb = {0}, vo = {0};
    uint64_t n = 0, min_len = UINT64_MAX, max_len = 0;
    int ascii = 1;
    if (seq) {
        const size_t cnt = (size_t)PySequence_Fast_GET_SIZE(seq);
        if (buf_grow(&ko, (cnt + 1) * 8) || buf_grow(&vo, (cnt + 1) * 8)) goto fail;
    }
    if (buf_u64(&ko, 0) || buf_u64(&vo, 0)) goto fail;
    PyObject* item;
    while ((item = next_item(seq, it, &idx))) {
        Py_buffer view;
        view.obj = NULL;
        const unsigned char* d;
        size_t L;
        if (PyBytes_CheckExact(item)) {  // the memtable's records are bytes: no buffer request
            d = (const unsigned char*)PyBytes_AS_STRING(item);
            L = (size_t)PyBytes_GET_SIZE(item);
        } else {
            if (PyObject_GetBuffer(item, &view, PyBUF_SIMPLE)) {
                Py_DECREF(item);
                goto fail;
            }
            d = (const unsigned char*)view.buf;
            L = (size_t)view.len;
        }
        int32_t ks, vs;
        int rc = -1;
        // Record._from_bytes, step by step: struct.unpack needs 4 bytes; the key and value
        // slices are clipped to the data (Python slicing); the key is decoded before the value
        // size is read
        if (L < 4) goto bad;
        memcpy(&ks, d, 4);
        if (ks < 0) goto neg;
        {
            const size_t key_end = 4 + (size_t)ks;
            const size_t kl = key_end <= L ? (size_t)ks : L - 4;
            const unsigned char* key = d + 4;
            int all_ascii = 1;
            for (size_t c = 0; c < kl; ++c)
                if (key[c] & 0x80) {
                    all_ascii = 0;
                    break;
                }
            if (!all_ascii) {  // the reference decodes: invalid UTF-8 raises there too
                ascii = 0;
                PyObject* u = PyUnicode_DecodeUTF8((const char*)key, (Py_ssize_t)kl, NULL);
                if (!u) goto out;
                Py_DECREF(u);
            }
            if (key_end + 4 > L) goto bad;
            memcpy(&vs, d + key_end, 4);
            if (vs < 0) goto neg;
            const size_t v0 = key_end + 4;
            const size_t vl = v0 + (size_t)vs <= L ? (size_t)vs : L - v0;
            rc = buf_put(&kb, key, kl);
            if (!rc) rc = buf_u64(&ko, kb.n);
            if (!rc) rc = buf_put(&vb, d + v0, vl);
            if (!rc) rc = buf_u64(&vo, vb.n);
            if ((uint64_t)kl < min_len) min_len = (uint64_t)kl;
            if ((uint64_t)kl > max_len) max_len = (uint64_t)kl;
            goto out;
        }
    neg:
        PyErr_SetString(PyExc_ValueError, "pack_encoded: negative key or value size");
        goto out;
    bad:
        // struct.unpack("i", ...) of fewer than 4 bytes: struct.error, as in the reference
        PyErr_SetString(s_struct_error, "unpack requires a buffer of 4 bytes");
    out:
        if (view.obj) PyBuffer_Release(&view);
        Py_DECREF(item);
        if (rc) goto fail;
        ++n;
    }
    if (PyErr_Occurred()) goto fail;
    Py_XDECREF(it);
    if (n == 0) min_len = 0;
    {
        PyObject* a = buf_release(&kb);
        PyObject* b = buf_release(&ko);
        PyObject* c = buf_release(&vb);
        PyObject* e = buf_release(&vo);
        if (!a || !b || !c || !e) {
            Py_XDECREF(a);
            Py_XDECREF(b);
            Py_XDECREF(c);
            Py_XDECREF(e);
            return NULL;
        }
        return Py_BuildValue("(NNNNKiKK)", a, b, c, e, (unsigned long long)n, ascii, (unsigned long long)min_len,
                             (unsigned long long)max_len);
    }
fail:
    Py_XDECREF(it);
    buf_free(&kb);
    buf_free(&ko);
    buf_free(&vb);
    buf_free(&vo);
    return NULL;
}

static PyObject* py_pack_keys(PyObject* self, PyObject* args) {
    PyObject* iterable;
    if (!PyArg_ParseTuple(args, "O", &iterable)) return NULL;
    return pack_impl(iterable, 0);
}

static PyObject* py_pack_records(PyObject* self, PyObject* args) {
    PyObject* iterable;
    if (!PyArg_ParseTuple(args, "O", &iterable)) return NULL;
    return pack_impl(iterable, 1);
}

static PyMethodDef methods[] = {
    {"pack_keys", py_pack_keys, METH_VARARGS,
     "pack_keys(iterable) -> (key_bytes, key_offsets_u64, b'', b'', n, ascii, min_len, max_len)"},
    {"pack_records", py_pack_records, METH_VARARGS,
     "pack_records(iterable) -> (key_bytes, key_offsets_u64, value_bytes, value_offsets_u64, n, ascii, min_len, "
     "max_len)"},
    {"pack_encoded", py_pack_encoded, METH_VARARGS,
     "pack_encoded(iterable of Record.to_bytes() bytes) -> as pack_records (split as Record._from_bytes)"},
    {NULL, NULL, 0, NULL},
};

static struct PyModuleDef module = {PyModuleDef_HEAD_INIT, "_pebbleingest", NULL, -1, methods};

PyMODINIT_FUNC PyInit__pebbleingest(void) {
    if (PyType_Ready(&PackedBufferType) < 0) return NULL;
    s_key = PyUnicode_InternFromString("key");
    s_value = PyUnicode_InternFromString("value");
    if (!s_key || !s_value) return NULL;
    PyObject* st = PyImport_ImportModule("struct");
    if (!st) return NULL;
    s_struct_error = PyObject_GetAttrString(st, "error");
    Py_DECREF(st);
    if (!s_struct_error) return NULL;
    return PyModule_Create(&module);
}
