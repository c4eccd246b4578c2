// Native host preprocessing for the request-authentication path (SURVEY.md
// §8 row f2): base58 and the canonical signing serializer, the two host-side
// costs in front of every verify (client_authn.py:97-102,
// plenum/common/verifier.py:25-51, common/serializers/signing_serializer.py:35-92).
//
// CPython extension `plenum_gpu._host`.  Contract: identical results to the
// pure-Python restatements in plenum_gpu/base58.py and serialization.py.  On
// any input those restatements would REJECT (bad base58 character, an
// unacceptable type, unsortable dict keys) or treat differently (container
// subclasses, memoryviews) the native function raises _host.Fallback and the
// Python wrapper re-runs the restatement, so results, exception types and
// texts are exactly the reference's.  Common inputs never go through Python.
#define PY_SSIZE_T_CLEAN
#include <Python.h>

#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

namespace {

PyObject* g_fallback = nullptr;  // _host.Fallback

const char kAlphabet[] = "123456789ABCDEFGHJKLMNPQRSTUVWXYZabcdefghijkmnopqrstuvwxyz";
int8_t g_index[256];

void init_index() {
  memset(g_index, -1, sizeof g_index);
  for (int i = 0; i < 58; ++i) g_index[(uint8_t)kAlphabet[i]] = (int8_t)i;
}

// borrowed view of str (ASCII/UTF-8) or bytes-like; false if neither
bool view(PyObject* o, const char** p, Py_ssize_t* n, Py_buffer* buf, bool* release) {
  *release = false;
  if (PyUnicode_Check(o)) {
    if (!PyUnicode_IS_ASCII(o)) return false;  // the restatement raises (ascii encode)
    *p = (const char*)PyUnicode_DATA(o);
    *n = PyUnicode_GET_LENGTH(o);
    return true;
  }
  // bytes / bytearray only: other buffers (memoryview, ...) and other types
  // behave differently in the restatement (v.rstrip(), bytes(v)) -> fallback
  if ((PyBytes_Check(o) || PyByteArray_Check(o)) && PyObject_GetBuffer(o, buf, PyBUF_SIMPLE) == 0) {
    *p = (const char*)buf->buf;
    *n = buf->len;
    *release = true;
    return true;
  }
  PyErr_Clear();
  return false;
}

PyObject* fallback() {
  PyErr_SetNone(g_fallback);
  return nullptr;
}

bool is_space(unsigned char c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == '\v' || c == '\f'; }

// b58decode(v) -> bytes  (base58 2.x: trailing whitespace stripped, leading '1' -> 0x00)
PyObject* b58decode(PyObject*, PyObject* arg) {
  const char* p;
  Py_ssize_t n;
  Py_buffer buf;
  bool rel;
  if (!view(arg, &p, &n, &buf, &rel)) return fallback();
  // str.rstrip() also strips \x1c-\x1f and \x85 etc.; those are not base58
  // characters either, so any such byte simply takes the fallback path.
  while (n > 0 && is_space((unsigned char)p[n - 1])) --n;
  Py_ssize_t zeros = 0;
  while (zeros < n && p[zeros] == '1') ++zeros;
  // value in little-endian 32-bit limbs, 5 digits (58^5 < 2^32) per step
  std::vector<uint32_t> limb;
  limb.reserve((size_t)(n / 5 + 2));
  for (Py_ssize_t i = zeros; i < n;) {
    uint64_t mul = 1, val = 0;
    for (int k = 0; k < 5 && i < n; ++k, ++i) {
      const int d = g_index[(uint8_t)p[i]];
      if (d < 0) {
        if (rel) PyBuffer_Release(&buf);
        return fallback();
      }
      val = val * 58 + (uint64_t)d;
      mul *= 58;
    }
    uint64_t carry = val;
    for (auto& l : limb) {
      const uint64_t t = (uint64_t)l * mul + carry;
      l = (uint32_t)t;
      carry = t >> 32;
    }
    if (carry) limb.push_back((uint32_t)carry);
  }
  if (rel) PyBuffer_Release(&buf);
  // significant bytes: drop the top limb's leading zero bytes
  size_t nbytes = limb.size() * 4;
  while (nbytes > 0 && ((limb[(nbytes - 1) / 4] >> (8 * ((nbytes - 1) % 4))) & 0xffu) == 0) --nbytes;
  PyObject* out = PyBytes_FromStringAndSize(nullptr, zeros + (Py_ssize_t)nbytes);
  if (!out) return nullptr;
  char* q = PyBytes_AS_STRING(out);
  memset(q, 0, (size_t)zeros);
  q += zeros;
  for (size_t b = 0; b < nbytes; ++b) {
    const size_t bit = (nbytes - 1 - b);  // byte index from the least significant end
    q[b] = (char)(limb[bit / 4] >> (8 * (bit % 4)));
  }
  return out;
}

// b58encode(v) -> bytes
PyObject* b58encode(PyObject*, PyObject* arg) {
  const char* p;
  Py_ssize_t n;
  Py_buffer buf;
  bool rel;
  if (!view(arg, &p, &n, &buf, &rel)) return fallback();
  Py_ssize_t zeros = 0;
  while (zeros < n && p[zeros] == 0) ++zeros;
  // big-endian bytes -> little-endian 32-bit limbs
  const size_t nb = (size_t)(n - zeros);
  std::vector<uint32_t> limb((nb + 3) / 4, 0u);
  for (size_t b = 0; b < nb; ++b) {
    const size_t bit = nb - 1 - b;
    limb[bit / 4] |= (uint32_t)(uint8_t)p[zeros + b] << (8 * (bit % 4));
  }
  if (rel) PyBuffer_Release(&buf);
  // repeated division by 58^5, 5 digits per pass (little-endian digits)
  std::vector<uint8_t> dig;
  dig.reserve(nb * 138 / 100 + 6);
  size_t top = limb.size();
  while (top > 0) {
    uint64_t rem = 0;
    for (size_t k = top; k-- > 0;) {
      const uint64_t cur = (rem << 32) | limb[k];
      limb[k] = (uint32_t)(cur / 656356768u);
      rem = cur % 656356768u;
    }
    while (top > 0 && limb[top - 1] == 0) --top;
    for (int k = 0; k < 5; ++k) {
      dig.push_back((uint8_t)(rem % 58));
      rem /= 58;
    }
  }
  while (!dig.empty() && dig.back() == 0) dig.pop_back();  // the last pass pads with zero digits
  PyObject* out = PyBytes_FromStringAndSize(nullptr, zeros + (Py_ssize_t)dig.size());
  if (!out) return nullptr;
  char* q = PyBytes_AS_STRING(out);
  memset(q, '1', (size_t)zeros);
  for (size_t k = 0; k < dig.size(); ++k) q[zeros + k] = kAlphabet[dig[dig.size() - 1 - k]];
  return out;
}

// ---------------------------------------------------------------- serializer
// SigningSerializer._ser: str -> itself; dict -> sorted "k:v" joined by "|"
// (level-0 keys in `ignore` dropped); list -> items joined by ","; None -> "";
// int/float (and bool) -> str().  Returns false to request the Python path.
bool ser(PyObject* obj, int level, PyObject* ignore, std::string& out) {
  if (PyUnicode_Check(obj)) {
    Py_ssize_t n;
    const char* s = PyUnicode_AsUTF8AndSize(obj, &n);
    if (!s) {
      PyErr_Clear();
      return false;  // lone surrogates: let Python raise
    }
    out.append(s, (size_t)n);
    return true;
  }
  if (PyDict_CheckExact(obj)) {
    PyObject* keys = PyDict_Keys(obj);
    if (!keys) return false;
    // exact reference semantics: sorted(k for k in keys if k not in set(ignore or ()))
    if (level == 0 && ignore && PyObject_IsTrue(ignore) == 1) {
      PyObject* skip = PySet_New(ignore);
      PyObject* kept = skip ? PyList_New(0) : nullptr;
      if (!kept) {
        Py_XDECREF(skip);
        Py_DECREF(keys);
        PyErr_Clear();
        return false;
      }
      const Py_ssize_t m = PyList_GET_SIZE(keys);
      for (Py_ssize_t i = 0; i < m; ++i) {
        PyObject* k = PyList_GET_ITEM(keys, i);
        const int c = PySet_Contains(skip, k);
        if (c < 0 || (c == 0 && PyList_Append(kept, k) < 0)) {
          Py_DECREF(kept);
          Py_DECREF(skip);
          Py_DECREF(keys);
          PyErr_Clear();
          return false;
        }
      }
      Py_DECREF(skip);
      Py_DECREF(keys);
      keys = kept;
    }
    if (PyList_Sort(keys) < 0) {  // Python ordering (mixed key types raise -> fallback)
      PyErr_Clear();
      Py_DECREF(keys);
      return false;
    }
    const Py_ssize_t m = PyList_GET_SIZE(keys);
    for (Py_ssize_t i = 0; i < m; ++i) {
      PyObject* k = PyList_GET_ITEM(keys, i);
      if (i) out.push_back('|');
      PyObject* ks = PyObject_Str(k);
      if (!ks) {
        PyErr_Clear();
        Py_DECREF(keys);
        return false;
      }
      Py_ssize_t kn;
      const char* kc = PyUnicode_AsUTF8AndSize(ks, &kn);
      if (!kc) {
        PyErr_Clear();
        Py_DECREF(ks);
        Py_DECREF(keys);
        return false;
      }
      out.append(kc, (size_t)kn);
      Py_DECREF(ks);
      out.push_back(':');
      PyObject* v = PyDict_GetItemWithError(obj, k);
      if (!v || !ser(v, level + 1, nullptr, out)) {
        PyErr_Clear();
        Py_DECREF(keys);
        return false;
      }
    }
    Py_DECREF(keys);
    return true;
  }
  if (PyList_CheckExact(obj)) {
    const Py_ssize_t m = PyList_GET_SIZE(obj);
    for (Py_ssize_t i = 0; i < m; ++i) {
      if (i) out.push_back(',');
      if (!ser(PyList_GET_ITEM(obj, i), level + 1, nullptr, out)) return false;
    }
    return true;
  }
  if (obj == Py_None) return true;
  // exact int/float (bool is an int subclass) -> str(); anything else is not
  // an ACCEPTABLE type (or a subclass with its own __str__): Python path
  if (PyLong_CheckExact(obj) || PyFloat_CheckExact(obj) || PyBool_Check(obj)) {
    PyObject* s = PyObject_Str(obj);
    if (!s) {
      PyErr_Clear();
      return false;
    }
    Py_ssize_t n;
    const char* c = PyUnicode_AsUTF8AndSize(s, &n);
    if (c) out.append(c, (size_t)n);
    Py_DECREF(s);
    return c != nullptr;
  }
  return false;
}

// serialize(msg, topLevelKeysToIgnore=None) -> bytes (UTF-8)
PyObject* serialize(PyObject*, PyObject* args) {
  PyObject* obj;
  PyObject* ignore = Py_None;
  if (!PyArg_ParseTuple(args, "O|O", &obj, &ignore)) return nullptr;
  std::string out;
  out.reserve(512);
  if (!ser(obj, 0, ignore, out)) return fallback();
  return PyBytes_FromStringAndSize(out.data(), (Py_ssize_t)out.size());
}

// pack(list|tuple of bytes-like) -> (blob bytes, offsets bytes: n+1 little-endian u64)
// the message layout of pv_verify_batch / pv_sha256_batch / pv_merkle_root.  Any
// item without a C-contiguous buffer raises Fallback (the Python packer runs).
// The items are snapshotted into a tuple holding strong references first: a
// buffer provider (PyObject_GetBuffer) may run Python code that mutates the
// caller's list, and the packer must never read a borrowed pointer after that.
PyObject* pack_items(PyObject* snap);

PyObject* pack(PyObject*, PyObject* seq) {
  if (!PyList_CheckExact(seq) && !PyTuple_CheckExact(seq)) return fallback();
  PyObject* snap = PySequence_Tuple(seq);
  if (!snap) return nullptr;
  PyObject* r = pack_items(snap);
  Py_DECREF(snap);
  return r;
}

PyObject* pack_items(PyObject* snap) {
  const Py_ssize_t n = PyTuple_GET_SIZE(snap);
  PyObject** items = &PyTuple_GET_ITEM(snap, 0);
  PyObject* off = PyBytes_FromStringAndSize(nullptr, (n + 1) * 8);
  if (!off) return nullptr;
  uint64_t* o = reinterpret_cast<uint64_t*>(PyBytes_AS_STRING(off));
  o[0] = 0;
  bool all_bytes = true;
  for (Py_ssize_t i = 0; i < n; ++i) {
    Py_ssize_t len;
    if (PyBytes_CheckExact(items[i])) {
      len = PyBytes_GET_SIZE(items[i]);
    } else {
      all_bytes = false;
      Py_buffer b;
      if (PyObject_GetBuffer(items[i], &b, PyBUF_C_CONTIGUOUS) < 0) {
        PyErr_Clear();
        Py_DECREF(off);
        return fallback();
      }
      len = b.len;
      PyBuffer_Release(&b);
    }
    o[i + 1] = o[i] + (uint64_t)len;
  }
  PyObject* blob = PyBytes_FromStringAndSize(nullptr, (Py_ssize_t)o[n]);
  if (!blob) {
    Py_DECREF(off);
    return nullptr;
  }
  char* dst = PyBytes_AS_STRING(blob);
  for (Py_ssize_t i = 0; i < n; ++i) {
    if (all_bytes || PyBytes_CheckExact(items[i])) {
      memcpy(dst + o[i], PyBytes_AS_STRING(items[i]), o[i + 1] - o[i]);
      continue;
    }
    Py_buffer b;
    // a buffer whose size changed since the first pass is not packed here
    if (PyObject_GetBuffer(items[i], &b, PyBUF_C_CONTIGUOUS) < 0 || (uint64_t)b.len != o[i + 1] - o[i]) {
      if (PyErr_Occurred()) PyErr_Clear();
      else PyBuffer_Release(&b);
      Py_DECREF(off);
      Py_DECREF(blob);
      return fallback();
    }
    memcpy(dst + o[i], b.buf, (size_t)b.len);
    PyBuffer_Release(&b);
  }
  PyObject* r = PyTuple_Pack(2, blob, off);
  Py_DECREF(blob);
  Py_DECREF(off);
  return r;
}

// verify_batch(fn, pk, sig, blob, off, verdict, device_mask, flags) -> rc:
// pv_verify_batch (include/plenum_verify.h; `fn` = its address, from the ctypes
// binding) called on the buffers of C-contiguous arrays, the GIL released.  The
// ctypes call converts five pointers at ~0.6 us each; a lone cached verify is
// ~80 us, so the plenum_gpu wrapper takes this path when the module is built.
using verify_fn = int (*)(const uint8_t*, const uint8_t*, const uint8_t*, const uint64_t*, uint64_t, uint8_t*,
                          uint32_t, uint32_t);
PyObject* verify_batch(PyObject*, PyObject* args) {
  unsigned long long fn = 0;
  PyObject *o[5];
  unsigned int mask = 0, flags = 0;
  if (!PyArg_ParseTuple(args, "KOOOOOII", &fn, &o[0], &o[1], &o[2], &o[3], &o[4], &mask, &flags)) return nullptr;
  if (!fn) return fallback();
  Py_buffer b[5];
  int got = 0;
  for (; got < 5; ++got) {
    const int req = got == 4 ? (PyBUF_SIMPLE | PyBUF_WRITABLE) : PyBUF_SIMPLE;
    if (PyObject_GetBuffer(o[got], &b[got], req) != 0) break;
  }
  if (got < 5) {
    for (int i = 0; i < got; ++i) PyBuffer_Release(&b[i]);
    PyErr_Clear();
    return fallback();
  }
  const uint64_t n = (uint64_t)b[4].len;   // one verdict byte per signature
  // every input must cover n signatures and off[n] the blob: a caller that skipped
  // the Python shape checks gets the ValueError of the ctypes path, never a read
  // past a buffer with the GIL released
  const uint64_t* offp = static_cast<const uint64_t*>(b[3].buf);
  const bool sized = (uint64_t)b[0].len >= 32 * n && (uint64_t)b[1].len >= 64 * n &&
                     (uint64_t)b[3].len >= 8 * (n + 1) && offp[n] <= (uint64_t)b[2].len;
  if (!sized) {
    for (int i = 0; i < 5; ++i) PyBuffer_Release(&b[i]);
    PyErr_SetString(PyExc_ValueError, "verify_batch: pk / sig / off / blob smaller than the verdict count needs");
    return nullptr;
  }
  int rc;
  Py_BEGIN_ALLOW_THREADS
  rc = reinterpret_cast<verify_fn>((uintptr_t)fn)(static_cast<const uint8_t*>(b[0].buf),
                                                  static_cast<const uint8_t*>(b[1].buf),
                                                  static_cast<const uint8_t*>(b[2].buf),
                                                  static_cast<const uint64_t*>(b[3].buf), n,
                                                  static_cast<uint8_t*>(b[4].buf), mask, flags);
  Py_END_ALLOW_THREADS
  for (int i = 0; i < 5; ++i) PyBuffer_Release(&b[i]);
  return PyLong_FromLong(rc);
}

PyMethodDef kMethods[] = {
    {"verify_batch", verify_batch, METH_VARARGS, "pv_verify_batch(fn address, pk, sig, blob, off, verdict, mask, flags) -> rc"},
    {"pack", pack, METH_O, "pack a list of bytes-like messages -> (blob, u64 offsets)"},
    {"b58decode", b58decode, METH_O, "base58 decode (str or bytes) -> bytes"},
    {"b58encode", b58encode, METH_O, "base58 encode (bytes or str) -> bytes"},
    {"serialize", serialize, METH_VARARGS, "canonical signing serialization -> UTF-8 bytes"},
    {nullptr, nullptr, 0, nullptr},
};

PyModuleDef kModule = {PyModuleDef_HEAD_INIT, "_host", "native host preprocessing (base58, signing serializer)", -1,
                       kMethods};

}  // namespace

PyMODINIT_FUNC PyInit__host(void) {
  init_index();
  PyObject* m = PyModule_Create(&kModule);
  if (!m) return nullptr;
  g_fallback = PyErr_NewException("_host.Fallback", PyExc_Exception, nullptr);
  if (!g_fallback || PyModule_AddObject(m, "Fallback", g_fallback) < 0) {
    Py_DECREF(m);
    return nullptr;
  }
  Py_INCREF(g_fallback);
  return m;
}
