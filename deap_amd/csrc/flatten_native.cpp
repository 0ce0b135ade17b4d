// flatten_native.cpp — native host flattener (CPython extension _flatnative).
//
// The same lowering as deap_amd/flatten.py (Flattener._build/_emit/_encode),
// word for word, for whole generations: PrimitiveTree (prefix list of node
// objects, reference deap/gp.py:44-184) -> postfix programs for the F / B
// machines of gpeval.hip.  The Python flattener stays the specification and
// the fallback for the rare trees this code declines (a constant it cannot
// fold with Python semantics, e.g. integers beyond int64); tests compare the
// two on every golden set.
//
// Node identification: shared pset nodes (primitives, argument and constant
// terminals — PrimitiveTree.__deepcopy__ keeps them shared, gp.py:58-61) by
// object identity; after pickling, by name; any other leaf is an ephemeral
// constant whose `value` is read here (gp.py:243-257).
#include <Python.h>
#include <structmember.h>

#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <cstring>
#include <string>
#include <unordered_map>
#include <vector>

#include "host_pool.h"
#include "lower_core.h"

namespace {

using namespace lowering;

// Identity map of the shared pset nodes (a few dozen objects), probed once
// per tree node: a multiplicative hash on the object address whose multiplier
// is searched at build time until no two keys share a slot, so a lookup is
// one slot and one compare (no probe loop, no mispredicted branches on the
// population's node stream).  Linear probing remains for a key set no tried
// multiplier separates.
struct PtrMap {
  std::vector<uintptr_t> keys;
  std::vector<int> vals;
  int shift = 63;
  uint64_t mul = 0x9E3779B97F4A7C15ull;
  bool perfect = false;
  void build(const std::vector<std::pair<uintptr_t, int>>& kv) {
    size_t cap = 16;
    while (cap < kv.size() * 4) cap <<= 1;
    uint64_t seed = 0x9E3779B97F4A7C15ull;
    for (int attempt = 0; attempt < 4096; ++attempt) {
      if (attempt && attempt % 512 == 0) cap <<= 1;   // sparser table
      shift = 64;
      for (size_t c = cap; c > 1; c >>= 1) --shift;
      mul = seed | 1;
      seed = seed * 6364136223846793005ull + 1442695040888963407ull;
      std::vector<uint8_t> used(cap, 0);
      bool clash = false;
      for (const auto& e : kv) {
        uint8_t& u = used[slot(e.first)];
        clash |= u != 0;
        u = 1;
      }
      if (!clash) {
        perfect = true;
        break;
      }
    }
    if (!perfect) {
      cap = 16;
      while (cap < kv.size() * 4) cap <<= 1;
      shift = 64;
      for (size_t c = cap; c > 1; c >>= 1) --shift;
      mul = 0x9E3779B97F4A7C15ull;
    }
    keys.assign(cap, 0);
    vals.assign(cap, -1);
    for (const auto& e : kv) {
      size_t h = slot(e.first);
      while (keys[h] && keys[h] != e.first) h = (h + 1) & (cap - 1);
      keys[h] = e.first;
      vals[h] = e.second;
    }
  }
  size_t slot(uintptr_t k) const { return (size_t)(((uint64_t)k * mul) >> shift); }
  // the perfect map's fields as a value: held in registers by a loop that
  // stores bytes (through which the compiler would otherwise reload them)
  struct Probe {
    const uintptr_t* keys;
    const int* vals;
    uint64_t mul;
    int shift;
    int find(uintptr_t k) const {
      const size_t h = (size_t)(((uint64_t)k * mul) >> shift);
      return keys[h] == k ? vals[h] : -1;
    }
  };
  Probe probe() const { return Probe{keys.data(), vals.data(), mul, shift}; }
  int find(uintptr_t k) const {
    size_t h = slot(k);
    if (perfect) return keys[h] == k ? vals[h] : -1;
    const size_t mask = keys.size() - 1;
    for (;; h = (h + 1) & mask) {
      if (keys[h] == k) return vals[h];
      if (!keys[h]) return -1;
    }
  }
};

struct Fl {
  int machine = 0;     // 0 F, 1 B
  int nv = 0;
  std::vector<uint8_t> leaf;               // per argument: trig leaf column
  std::vector<Entry> entries;
  PtrMap by_id;
  PyObject* by_name = nullptr;             // dict name -> entry index
  PyObject* s_name = nullptr;
  PyObject* s_value = nullptr;
  std::vector<PyTypeObject*> eph_types;    // ephemeral constant classes
  Py_ssize_t value_off = -1;               // offset of the `value` slot
  // per-tree scratch (grown, never shrunk)
  std::vector<Rec> recs;
  std::vector<lowering::PRec> precs;       // the device's packed records
  std::vector<double> ibs;                 // int bounds (F machine)
  std::vector<uint32_t> wscr;              // interleaved word scratch (lower_codes)
  std::vector<int32_t> stack;
  std::vector<Val> cvals;                  // constants of the tree's records
};

bool to_val(PyObject* o, Val& v) {
  if (PyBool_Check(o)) {
    v.t = 'b';
    v.i = (o == Py_True) ? 1 : 0;
    return true;
  }
  if (PyLong_Check(o)) {
    int overflow = 0;
    long long x = PyLong_AsLongLongAndOverflow(o, &overflow);
    if (overflow || (x == -1 && PyErr_Occurred())) {
      PyErr_Clear();
      v.t = 'x';
      return false;
    }
    v.t = 'i';
    v.i = x;
    return true;
  }
  if (PyFloat_Check(o)) {
    v.t = 'f';
    v.f = PyFloat_AS_DOUBLE(o);
    return true;
  }
  v.t = 'x';
  return false;
}

int lookup(Fl& F, PyObject* node) {
  const int hit = F.by_id.find((uintptr_t)node);
  if (hit >= 0) return hit;
  for (PyTypeObject* t : F.eph_types)
    if (Py_TYPE(node) == t) return -1;                     // ephemeral leaf
  PyObject* name = PyObject_GetAttr(node, F.s_name);
  if (!name) { PyErr_Clear(); return -2; }
  PyObject* e = PyDict_GetItemWithError(F.by_name, name);   // borrowed
  Py_DECREF(name);
  if (e) return (int)PyLong_AsLong(e);
  if (PyErr_Occurred()) PyErr_Clear();
  return -1;                                               // ephemeral leaf
}

void cap_free(PyObject* cap) {
  Fl* F = (Fl*)PyCapsule_GetPointer(cap, "_flatnative.Fl");
  if (!F) return;
  Py_XDECREF(F->by_name);
  Py_XDECREF(F->s_name);
  Py_XDECREF(F->s_value);
  delete F;
}

// new(machine, nv, leaves(bytes, 1 per arg), ids(list[int]), entries(list of
// (kind, arity, sem, var, value)), by_name(dict)) -> capsule
PyObject* py_new(PyObject*, PyObject* args) {
  int machine, nv;
  Py_buffer leaves;
  PyObject *ids, *entries, *by_name, *eph, *value_descr;
  if (!PyArg_ParseTuple(args, "iiy*O!O!O!O!O", &machine, &nv, &leaves,
                        &PyList_Type, &ids, &PyList_Type, &entries, &PyDict_Type,
                        &by_name, &PyList_Type, &eph, &value_descr))
    return nullptr;
  Fl* F = new Fl();
  for (Py_ssize_t i = 0; i < PyList_GET_SIZE(eph); ++i) {
    PyObject* t = PyList_GET_ITEM(eph, i);
    if (PyType_Check(t)) F->eph_types.push_back((PyTypeObject*)t);
  }
  // the `value` slot of Terminal (a member descriptor of an object slot)
  if (Py_TYPE(value_descr) == &PyMemberDescr_Type) {
    PyMemberDef* m = ((PyMemberDescrObject*)value_descr)->d_member;
    if (m->type == T_OBJECT_EX || m->type == T_OBJECT) F->value_off = m->offset;
  }
  F->machine = machine;
  F->nv = nv;
  F->leaf.assign((const uint8_t*)leaves.buf, (const uint8_t*)leaves.buf + leaves.len);
  PyBuffer_Release(&leaves);
  const Py_ssize_t ne = PyList_GET_SIZE(entries);
  if (PyList_GET_SIZE(ids) != ne) {
    delete F;
    PyErr_SetString(PyExc_ValueError, "ids/entries length mismatch");
    return nullptr;
  }
  std::vector<std::pair<uintptr_t, int>> kv;
  for (Py_ssize_t i = 0; i < ne; ++i) {
    PyObject* t = PyList_GET_ITEM(entries, i);
    Entry e;
    PyObject* value;
    if (!PyArg_ParseTuple(t, "iiiiO", &e.kind, &e.arity, &e.sem, &e.var, &value)) {
      delete F;
      return nullptr;
    }
    if (e.kind == K_CONST) to_val(value, e.c);
    F->entries.push_back(e);
    kv.emplace_back((uintptr_t)PyLong_AsUnsignedLongLong(PyList_GET_ITEM(ids, i)), (int)i);
  }
  F->by_id.build(kv);
  if (PyErr_Occurred()) { delete F; return nullptr; }
  Py_INCREF(by_name);
  F->by_name = by_name;
  F->s_name = PyUnicode_InternFromString("name");
  F->s_value = PyUnicode_InternFromString("value");
  return PyCapsule_New(F, "_flatnative.Fl", cap_free);
}

// Per-tree outcome of the GIL-free pass.
struct TreeOut {
  int32_t depth = 0;
  uint8_t err = 0;
  bool declined = false, inexact = false, verr = false;
};

// Lower one tree from its node codes (reversed prefix: entry index, or
// -1 - i for the ephemeral value evals[i]); Python-free, so it runs without
// the GIL.  Appends the program words (or one END) to `words`.
// the host's sin/cos for folded constants: glibc, as math.sin/cos
struct HostTrig {
  static double sin(double x) { return std::sin(x); }
  static double cos(double x) { return std::cos(x); }
};
struct VecEnts {
  const int32_t* e;
  int32_t operator()(int64_t k) const { return e[k]; }
};

// Lower one tree from its node codes (reversed prefix: entry index, or
// -1 - i for the ephemeral value evals[i]; lower_core.h); Python-free, so it
// runs without the GIL.  Appends the program words (or one END) to `words`.
// packed: the device kernel's storage — packed records, and every scratch
// array interleaved as lower_trees<true> lays it out (element k of the tree
// of lane `lane` at k·64 + lane) — for lower_codes' check of the device path
// on the host.
void lower_tree(Fl& F, const int32_t* ent, int64_t len, const Val* evals,
                std::vector<uint32_t>& words, TreeOut& o, bool packed = false,
                int lane = 0) {
  const size_t base = words.size();
  static const int neg_fold = [] {
    const char* e = std::getenv("GPE_NEG_PEEPHOLE");
    return e && e[0] == '0' ? 0 : 1;
  }();
  const Tables T{F.entries.data(), F.leaf.data(), (int)F.leaf.size(), F.nv, F.machine,
                 neg_fold};
  VecEnts E{ent};
  Result r;
  if (packed) {
    // (a declined tree past the 16-bit indices writes its one END only)
    const size_t rows = len <= lowering::PackedRecs::kMaxLen ? (size_t)len : 1;
    const size_t m = 64 * rows + 64;
    if (F.precs.size() < m) F.precs.resize(m);
    if (F.stack.size() < m) F.stack.resize(m);
    if (F.cvals.size() < m) F.cvals.resize(m);
    if (F.ibs.size() < m) F.ibs.resize(m);
    if (F.wscr.size() < 64 * (3 * rows + 1) + 64) F.wscr.resize(64 * (3 * rows + 1) + 64);
    lowering::lower<HostTrig>(T, E, len, evals, lowering::PackedRecsS<64>{F.precs.data() + lane},
                              lowering::Strided<int32_t, 64>{F.stack.data() + lane},
                              lowering::Strided<Val, 64>{F.cvals.data() + lane},
                              lowering::Strided<double, 64>{F.ibs.data() + lane},
                              lowering::Strided<uint32_t, 64>{F.wscr.data() + lane}, r);
    words.resize(base + (size_t)r.n_words);
    for (int32_t j = 0; j < r.n_words; ++j) words[base + (size_t)j] = F.wscr[(size_t)j * 64 + lane];
  } else {
    if ((int64_t)F.stack.size() < len) {
      F.stack.resize((size_t)len);
      F.cvals.resize((size_t)len);
      F.ibs.resize((size_t)len);
    }
    if ((int64_t)F.recs.size() < len) F.recs.resize((size_t)len);
    words.resize(base + 3 * (size_t)len + 1);
    lowering::lower<HostTrig>(T, E, len, evals, lowering::PlainRecs{F.recs.data()},
                              F.stack.data(), F.cvals.data(), F.ibs.data(),
                              words.data() + base, r);
    words.resize(base + (size_t)r.n_words);
  }
  o.depth = r.depth;
  o.err = r.err;
  o.declined = r.declined;
  o.inexact = r.inexact;
  o.verr = r.verr;
}

int flatten_threads(int64_t n_trees) {
  // the GPU box sets OMP_NUM_THREADS to its CPU share; default 8, at most 16
  const int t = hostpool::threads();
  return (int)std::max<int64_t>(1, std::min<int64_t>(t, n_trees / 4096));
}

enum Read { RD_OK = 0, RD_DECLINE = 1, RD_NEED_GIL = 2 };

// A population's trees are separate list objects, each with its own item
// array: a worker walking them is bound by the two dependent cache misses per
// tree (list header, then items), not by the per-node lookup.  Prefetch the
// header of tree i + kPfHead and the item array of tree i + kPfItems (whose
// header was prefetched kPfHead - kPfItems trees earlier).  Reads only, as
// the workers' other accesses (the calling thread holds the GIL).
constexpr int64_t kPfHead = 24, kPfItems = 12;
inline void prefetch_trees(PyObject* const* tv, int64_t i, int64_t end) {
  if (i + kPfHead < end) __builtin_prefetch(tv[i + kPfHead]);
  if (i + kPfItems < end) {
    PyObject* t = tv[i + kPfItems];
    if (PyList_Check(t)) {
      const char* it = (const char*)((PyListObject*)t)->ob_item;
      const Py_ssize_t bytes = PyList_GET_SIZE(t) * (Py_ssize_t)sizeof(PyObject*);
      for (Py_ssize_t o = 0; o < bytes; o += 64) __builtin_prefetch(it + o);
    }
  }
}

// Node objects of one tree -> codes (reversed prefix; see lower_tree).
// Without the GIL (gil = false) only plain reads are allowed: list items,
// object addresses, the `value` slot of ephemerals and the payload of
// int/float/bool objects; anything that needs the interpreter (a node found
// by name after pickling, a non-list tree, a value without the slot) is
// reported as RD_NEED_GIL and read again by the calling thread.  The calling
// thread holds the GIL throughout, so no Python code mutates the trees.
int read_tree(const Fl& F, PyObject* tree, bool gil, std::vector<int32_t>& ent,
              std::vector<Val>& evals, int64_t& len) {
  PyObject** items;
  PyObject* fast = nullptr;
  if (PyList_Check(tree)) {
    len = PyList_GET_SIZE(tree);
    items = ((PyListObject*)tree)->ob_item;
  } else {
    if (!gil) return RD_NEED_GIL;
    fast = PySequence_Fast(tree, "a tree must be a sequence");
    if (!fast) { PyErr_Clear(); return RD_DECLINE; }
    len = PySequence_Fast_GET_SIZE(fast);
    items = PySequence_Fast_ITEMS(fast);
  }
  int rc = RD_OK;
  for (int64_t k = len - 1; k >= 0; --k) {
    PyObject* node = items[k];
    int ei = F.by_id.find((uintptr_t)node);
    if (ei < 0) {
      bool eph = false;
      for (PyTypeObject* t : F.eph_types) eph |= Py_TYPE(node) == t;
      if (!eph) {
        if (!gil) { rc = RD_NEED_GIL; break; }
        ei = lookup(const_cast<Fl&>(F), node);
        if (ei == -2) { rc = RD_DECLINE; break; }
      }
    }
    if (ei >= 0) {
      ent.push_back(ei);
      continue;
    }
    // ephemeral constant
    PyObject* v = nullptr;
    if (F.value_off > 0 && Py_TYPE(node)->tp_basicsize > F.value_off) {
      v = *(PyObject**)((char*)node + F.value_off);    // __slots__ value
      if (!v) { rc = RD_DECLINE; break; }
      if (gil) Py_INCREF(v);               // workers never touch refcounts
    } else if (gil) {
      v = PyObject_GetAttr(node, F.s_value);
      if (!v) { PyErr_Clear(); rc = RD_DECLINE; break; }
    } else {
      rc = RD_NEED_GIL;
      break;
    }
    Val c;
    bool ok;
    if (gil) {
      ok = to_val(v, c);
      Py_DECREF(v);
    } else {
      // the same conversions as to_val, without touching refcounts or
      // the error indicator
      if (PyBool_Check(v)) {
        c.t = 'b';
        c.i = v == Py_True;
        ok = true;
      } else if (PyFloat_Check(v)) {
        c.t = 'f';
        c.f = PyFloat_AS_DOUBLE(v);
        ok = true;
      } else if (PyLong_CheckExact(v) && Py_SIZE(v) >= -1 && Py_SIZE(v) <= 1) {
        c.t = 'i';
        c.i = Py_SIZE(v) == 0 ? 0
              : (int64_t)((PyLongObject*)v)->ob_digit[0] * Py_SIZE(v);
        ok = true;
      } else {
        rc = RD_NEED_GIL;
        break;
      }
    }
    if (!ok) { rc = RD_DECLINE; break; }
    evals.push_back(c);
    ent.push_back(-1 - (int32_t)(evals.size() - 1));
  }
  Py_XDECREF(fast);
  return rc;
}

// flatten(capsule, trees) -> (code, offsets, depth, length, err, inexact,
//                             declined, value_errors)
// Worker threads read and lower contiguous ranges of trees; the calling
// thread keeps the GIL and afterwards handles the trees a worker could not
// read without it.
PyObject* py_flatten(PyObject*, PyObject* args) {
  PyObject *cap, *trees;
  if (!PyArg_ParseTuple(args, "OO", &cap, &trees)) return nullptr;
  Fl* F = (Fl*)PyCapsule_GetPointer(cap, "_flatnative.Fl");
  if (!F) return nullptr;
  PyObject* seq = PySequence_Fast(trees, "trees must be a sequence");
  if (!seq) return nullptr;
  const Py_ssize_t n = PySequence_Fast_GET_SIZE(seq);
  PyObject** tv = PySequence_Fast_ITEMS(seq);
  const auto t_p0 = std::chrono::steady_clock::now();
  std::vector<int64_t> length((size_t)n, 0);
  std::vector<TreeOut> outs((size_t)n);
  std::vector<uint8_t> need_gil((size_t)n, 0);
  const int T = flatten_threads(n);
  std::vector<std::vector<uint32_t>> tw((size_t)T);
  std::vector<std::vector<int64_t>> trel((size_t)T);
  auto lower_one = [&](Fl& fl, PyObject* tree, bool gil, std::vector<int32_t>& ent,
                       std::vector<Val>& evals, std::vector<uint32_t>& w,
                       int64_t i) -> bool {
    ent.clear();
    evals.clear();
    int64_t len = 0;
    const int rc = read_tree(fl, tree, gil, ent, evals, len);
    if (rc == RD_NEED_GIL) return false;
    length[i] = len;
    if (rc == RD_DECLINE) {
      outs[i].declined = true;
      w.push_back(OP_END);
      return true;
    }
    lower_tree(fl, ent.data(), (int64_t)ent.size(), evals.data(), w, outs[i]);
    return true;
  };
  auto work = [&](int t) {
    Fl local = *F;                         // tables + private scratch
    std::vector<int32_t> ent;
    std::vector<Val> evals;
    const int64_t a = n * t / T, b = n * (t + 1) / T;
    std::vector<uint32_t>& w = tw[(size_t)t];
    std::vector<int64_t>& rel = trel[(size_t)t];
    rel.reserve((size_t)(b - a) + 1);
    {
      size_t est = 0;
      for (int64_t i = a; i < b; ++i)
        est += PyList_Check(tv[i]) ? (size_t)PyList_GET_SIZE(tv[i]) * 3 + 1 : 64;
      w.reserve(est);
    }
    for (int64_t i = a; i < b; ++i) {
      prefetch_trees(tv, i, b);
      rel.push_back((int64_t)w.size());
      if (!lower_one(local, tv[i], false, ent, evals, w, i)) {
        need_gil[i] = 1;
        w.push_back(OP_END);
      }
    }
    rel.push_back((int64_t)w.size());
  };
  if (T == 1) {
    work(0);
  } else {
    hostpool::par_run(T, work);
  }
  const auto t_p1 = std::chrono::steady_clock::now();
  // trees that need the interpreter: read and lowered here, with the GIL
  std::vector<uint32_t> wg;
  std::vector<int64_t> gstart((size_t)n, -1), gend((size_t)n, -1);
  {
    Fl local = *F;
    std::vector<int32_t> ent;
    std::vector<Val> evals;
    for (Py_ssize_t i = 0; i < n; ++i) {
      if (!need_gil[i]) continue;
      gstart[i] = (int64_t)wg.size();
      lower_one(local, tv[i], true, ent, evals, wg, i);
      gend[i] = (int64_t)wg.size();
    }
  }
  Py_DECREF(seq);
  const auto t_p2 = std::chrono::steady_clock::now();

  // merge: per-tree sizes (a tree lowered with the GIL replaces its
  // worker placeholder), per-thread totals, then every thread writes its
  // offsets and copies its words straight into the result bytes object
  std::vector<int64_t> tbase((size_t)T + 1, 0);
  auto range = [&](int t, int64_t& a, int64_t& b) {
    a = n * t / T;
    b = n * (t + 1) / T;
  };
  auto tree_words = [&](int t, int64_t i, const uint32_t*& src) -> int64_t {
    if (need_gil[i]) {
      src = wg.data() + gstart[i];
      return gend[i] - gstart[i];
    }
    int64_t a, b;
    range(t, a, b);
    const std::vector<int64_t>& rel = trel[(size_t)t];
    src = tw[(size_t)t].data() + rel[i - a];
    return rel[i - a + 1] - rel[i - a];
  };
  for (int t = 0; t < T; ++t) {
    int64_t a, b, sz = 0;
    range(t, a, b);
    const std::vector<int64_t>& rel = trel[(size_t)t];
    sz = rel[b - a] - rel[0];
    for (int64_t i = a; i < b; ++i)
      if (need_gil[i]) sz += (gend[i] - gstart[i]) - (rel[i - a + 1] - rel[i - a]);
    tbase[(size_t)t + 1] = tbase[(size_t)t] + sz;
  }
  const int64_t total = tbase[(size_t)T];
  PyObject* words_b = PyBytes_FromStringAndSize(nullptr, (Py_ssize_t)(total * 4));
  PyObject* off_b = PyBytes_FromStringAndSize(nullptr, (Py_ssize_t)((n + 1) * 8));
  if (!words_b || !off_b) {
    Py_XDECREF(words_b);
    Py_XDECREF(off_b);
    return nullptr;
  }
  uint32_t* words = (uint32_t*)PyBytes_AS_STRING(words_b);
  int64_t* off = (int64_t*)PyBytes_AS_STRING(off_b);
  auto copy = [&](int t) {
    int64_t a, b;
    range(t, a, b);
    int64_t pos = tbase[(size_t)t];
    for (int64_t i = a; i < b; ++i) {
      const uint32_t* src;
      const int64_t m = tree_words(t, i, src);
      off[i] = pos;
      std::memcpy(words + pos, src, (size_t)m * 4);
      pos += m;
    }
  };
  if (T == 1) {
    copy(0);
  } else {
    hostpool::par_run(T, copy);
  }
  off[n] = total;
  std::vector<int32_t> depth((size_t)n, 0);
  std::vector<uint8_t> err((size_t)n, 0);
  std::vector<int64_t> inexact, declined, verr;
  for (Py_ssize_t i = 0; i < n; ++i) {
    const TreeOut& o = outs[i];
    depth[i] = o.depth;
    err[i] = o.err;
    if (o.declined) declined.push_back(i);
    if (o.inexact) inexact.push_back(i);
    if (o.verr) verr.push_back(i);
  }
  auto bytes = [](const void* p, size_t nb) {
    return PyBytes_FromStringAndSize((const char*)p, (Py_ssize_t)nb);
  };
  auto ilist = [](const std::vector<int64_t>& v) {
    PyObject* l = PyList_New((Py_ssize_t)v.size());
    for (size_t i = 0; i < v.size(); ++i)
      PyList_SET_ITEM(l, (Py_ssize_t)i, PyLong_FromLongLong(v[i]));
    return l;
  };
  if (std::getenv("DEAP_AMD_FLAT_TIMING")) {
    const auto t_p3 = std::chrono::steady_clock::now();
    auto ms = [](auto a, auto b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
    std::fprintf(stderr, "flatten: threads %.1f ms (%d), gil pass %.1f ms, merge %.1f ms\n",
                 ms(t_p0, t_p1), T, ms(t_p1, t_p2), ms(t_p2, t_p3));
  }
  return Py_BuildValue("(NNNNNNNN)", words_b, off_b,
                       bytes(depth.data(), depth.size() * 4),
                       bytes(length.data(), length.size() * 8),
                       bytes(err.data(), err.size()), ilist(inexact),
                       ilist(declined), ilist(verr));
}

// tuples1(buffer of float64, as_int) -> [(v,), ...]: the fitness 1-tuples
// toolbox.map returns, built in one pass (no intermediate list of numbers).
// as_int: hit counts (the reference's sum of bools), exact in a double; a
// population has few distinct counts, so equal counts share one (immutable)
// tuple object.
PyObject* py_tuples1(PyObject*, PyObject* args) {
  Py_buffer b;
  int as_int = 0;
  if (!PyArg_ParseTuple(args, "y*p", &b, &as_int)) return nullptr;
  const Py_ssize_t n = b.len / (Py_ssize_t)sizeof(double);
  const double* v = (const double*)b.buf;
  PyObject* out = PyList_New(n);
  if (!out) {
    PyBuffer_Release(&b);
    return nullptr;
  }
  constexpr long long kShared = 1 << 16;
  std::vector<PyObject*> shared;
  bool ok = true;
  if (as_int && n >= 65536) {
    // hit counts: every value an integer count below kShared (checked and
    // counted on host threads), so the list is filled in parallel with
    // borrowed pointers to one tuple per count, whose reference counts are
    // then raised once per count (no Python call off the calling thread)
    const int T = hostpool::threads();
    std::vector<std::vector<Py_ssize_t>> cnt((size_t)T);
    std::vector<uint8_t> bad((size_t)T, 0);
    hostpool::par_run(T, [&](int t) {
      std::vector<Py_ssize_t>& c = cnt[(size_t)t];
      for (Py_ssize_t i = n * t / T, e = n * (t + 1) / T; i < e; ++i) {
        const double x = v[i];
        if (!(x >= 0.0 && x < (double)kShared) || x != (double)(long long)x) {
          bad[(size_t)t] = 1;
          return;
        }
        const size_t k = (size_t)x;
        if (k >= c.size()) c.resize(k + 1, 0);
        ++c[k];
      }
    });
    bool fast = true;
    size_t kmax = 0;
    for (int t = 0; t < T; ++t) {
      fast &= !bad[(size_t)t];
      kmax = std::max(kmax, cnt[(size_t)t].size());
    }
    if (fast) {
      std::vector<Py_ssize_t> total(kmax, 0);
      for (const auto& c : cnt)
        for (size_t k = 0; k < c.size(); ++k) total[k] += c[k];
      shared.assign(kmax, nullptr);
      for (size_t k = 0; k < kmax && ok; ++k) {
        if (!total[k]) continue;
        PyObject* x = PyLong_FromLongLong((long long)k);
        PyObject* t = x ? PyTuple_New(1) : nullptr;
        if (!t) {
          Py_XDECREF(x);
          ok = false;
          break;
        }
        PyTuple_SET_ITEM(t, 0, x);
        shared[k] = t;                       // our reference, dropped below
      }
      if (ok) {
        PyObject** items = ((PyListObject*)out)->ob_item;
        hostpool::par_run(T, [&](int t) {
          for (Py_ssize_t i = n * t / T, e = n * (t + 1) / T; i < e; ++i)
            items[i] = shared[(size_t)v[i]];
        });
        for (size_t k = 0; k < kmax; ++k)
          if (shared[k]) Py_SET_REFCNT(shared[k], Py_REFCNT(shared[k]) + total[k]);
      }
      for (PyObject* t : shared) Py_XDECREF(t);
      PyBuffer_Release(&b);
      if (!ok) {
        Py_DECREF(out);
        return nullptr;
      }
      return out;
    }
  }
  for (Py_ssize_t i = 0; i < n && ok; ++i) {
    PyObject* t = nullptr;
    const long long k = as_int ? (long long)v[i] : -1;
    if (k >= 0 && k < kShared) {
      if ((size_t)k >= shared.size()) shared.resize((size_t)k + 1, nullptr);
      t = shared[(size_t)k];
      if (t) {
        Py_INCREF(t);
        PyList_SET_ITEM(out, i, t);
        continue;
      }
    }
    PyObject* x = as_int ? PyLong_FromLongLong((long long)v[i]) : PyFloat_FromDouble(v[i]);
    t = x ? PyTuple_New(1) : nullptr;
    if (!t) {
      Py_XDECREF(x);
      ok = false;
      break;
    }
    PyTuple_SET_ITEM(t, 0, x);
    if (k >= 0 && k < kShared) {
      Py_INCREF(t);
      shared[(size_t)k] = t;
    }
    PyList_SET_ITEM(out, i, t);
  }
  for (PyObject* t : shared) Py_XDECREF(t);
  PyBuffer_Release(&b);
  if (!ok) {
    Py_DECREF(out);     // unset items are NULL; list_dealloc skips them
    return nullptr;
  }
  return out;
}

// One list tree's nodes -> codes (prefix order: out[j] its entry, 255 an
// ephemeral whose value goes to ev).  False: a node only the general path
// reads (an unknown object, an ephemeral without a plain value slot).
inline bool read_nodes(const Fl& F, const PtrMap::Probe& P, bool perfect,
                       PyObject* const* items, int64_t len, uint8_t* __restrict out,
                       std::vector<Val>& ev) {
  int64_t j = 0;
  if (perfect)             // the common tree: pset entries only
    for (; j < len; ++j) {
      const int ei = P.find((uintptr_t)items[j]);
      if (ei < 0) break;
      out[j] = (uint8_t)ei;
    }
  for (; j < len; ++j) {
    PyObject* node = items[j];
    const int ei = F.by_id.find((uintptr_t)node);
    if (ei >= 0) {
      out[j] = (uint8_t)ei;
      continue;
    }
    // an ephemeral: its value slot read without the interpreter
    bool eph = false;
    for (PyTypeObject* ty : F.eph_types) eph |= Py_TYPE(node) == ty;
    PyObject* v = nullptr;
    if (eph && F.value_off > 0 && Py_TYPE(node)->tp_basicsize > F.value_off)
      v = *(PyObject**)((char*)node + F.value_off);
    Val c;
    if (v && PyBool_Check(v)) {
      c.t = 'b';
      c.i = v == Py_True;
    } else if (v && PyFloat_Check(v)) {
      c.t = 'f';
      c.f = PyFloat_AS_DOUBLE(v);
    } else if (v && PyLong_CheckExact(v) && Py_SIZE(v) >= -1 && Py_SIZE(v) <= 1) {
      c.t = 'i';
      c.i = Py_SIZE(v) == 0 ? 0
            : (int64_t)((PyLongObject*)v)->ob_digit[0] * Py_SIZE(v);
    } else {
      return false;                      // the general path decides
    }
    ev.push_back(c);
    out[j] = 255;
  }
  return true;
}

// read_codes' common case, straight into the output buffers: every tree a
// list whose nodes are pset entries or ephemerals with a value slot.  Pass 1
// sums each thread's node count (list sizes), the codes buffer is allocated
// once, pass 2 writes each tree's codes and offsets in place (no per-thread
// copies to merge); only the ephemeral values go through per-thread vectors.
// Returns the result tuple, Py_None (with a Python error set) on an
// allocation failure, or nullptr when a tree needs the general path.
PyObject* read_codes_direct(const Fl& F, PyObject* const* tv, Py_ssize_t n, int T) {
  std::vector<int64_t> tot((size_t)T + 1, 0);
  std::vector<uint8_t> ok((size_t)T, 1);
  auto range = [&](int t, int64_t& a, int64_t& b) {
    a = n * t / T;
    b = n * (t + 1) / T;
  };
  auto pass1 = [&](int t) {
    int64_t a, b, sum = 0;
    range(t, a, b);
    for (int64_t i = a; i < b; ++i) {
      if (i + kPfHead < b) __builtin_prefetch(tv[i + kPfHead]);
      if (!PyList_Check(tv[i])) {
        ok[(size_t)t] = 0;
        return;
      }
      sum += PyList_GET_SIZE(tv[i]);
    }
    tot[(size_t)t + 1] = sum;
  };
  auto run = [&](auto fn) {
    if (T == 1) {
      fn(0);
      return;
    }
    hostpool::par_run(T, fn);
  };
  run(pass1);
  for (int t = 0; t < T; ++t)
    if (!ok[(size_t)t]) return nullptr;
  for (int t = 0; t < T; ++t) tot[(size_t)t + 1] += tot[(size_t)t];
  PyObject* codes_b = PyBytes_FromStringAndSize(nullptr, (Py_ssize_t)tot[(size_t)T]);
  PyObject* off_b = PyBytes_FromStringAndSize(nullptr, (Py_ssize_t)((n + 1) * 8));
  PyObject* eoff_b = PyBytes_FromStringAndSize(nullptr, (Py_ssize_t)((n + 1) * 8));
  if (!codes_b || !off_b || !eoff_b) {
    Py_XDECREF(codes_b);
    Py_XDECREF(off_b);
    Py_XDECREF(eoff_b);
    Py_INCREF(Py_None);
    return Py_None;
  }
  uint8_t* cd = (uint8_t*)PyBytes_AS_STRING(codes_b);
  int64_t* off = (int64_t*)PyBytes_AS_STRING(off_b);
  int64_t* eoff = (int64_t*)PyBytes_AS_STRING(eoff_b);
  std::vector<std::vector<Val>> te((size_t)T);
  auto pass2 = [&](int t) {
    int64_t a, b;
    range(t, a, b);
    int64_t pos = tot[(size_t)t];
    std::vector<Val>& ev = te[(size_t)t];
    const bool perfect = F.by_id.perfect;
    const PtrMap::Probe P = F.by_id.probe();
    for (int64_t i = a; i < b; ++i) {
      prefetch_trees(tv, i, b);
      const int64_t len = PyList_GET_SIZE(tv[i]);
      PyObject* const* items = ((PyListObject*)tv[i])->ob_item;
      if (!read_nodes(F, P, perfect, items, len, cd + pos, ev)) {
        ok[(size_t)t] = 0;                   // the general path decides
        return;
      }
      off[i + 1] = pos + len;                // (thread-absolute: fixed below)
      eoff[i + 1] = (int64_t)ev.size();      // (thread-relative)
      pos += len;
    }
  };
  run(pass2);
  bool all_ok = true;
  for (int t = 0; t < T; ++t) all_ok &= ok[(size_t)t] != 0;
  if (!all_ok) {
    Py_DECREF(codes_b);
    Py_DECREF(off_b);
    Py_DECREF(eoff_b);
    return nullptr;
  }
  off[0] = eoff[0] = 0;
  size_t total_e = 0;
  std::vector<size_t> ebase((size_t)T, 0);
  for (int t = 0; t < T; ++t) {
    ebase[(size_t)t] = total_e;
    total_e += te[(size_t)t].size();
  }
  for (int t = 0; t < T; ++t) {               // eph offsets: thread base
    int64_t a, b;
    range(t, a, b);
    if (ebase[(size_t)t])
      for (int64_t i = a; i < b; ++i) eoff[i + 1] += (int64_t)ebase[(size_t)t];
  }
  PyObject* ev_b = PyBytes_FromStringAndSize(nullptr, (Py_ssize_t)(total_e * sizeof(Val)));
  if (!ev_b) {
    Py_DECREF(codes_b);
    Py_DECREF(off_b);
    Py_DECREF(eoff_b);
    Py_INCREF(Py_None);
    return Py_None;
  }
  Val* evp = (Val*)PyBytes_AS_STRING(ev_b);
  for (int t = 0; t < T; ++t)
    if (!te[(size_t)t].empty())
      std::memcpy((void*)(evp + ebase[(size_t)t]), te[(size_t)t].data(),
                  te[(size_t)t].size() * sizeof(Val));
  return Py_BuildValue("(NNNN)", codes_b, off_b, ev_b, eoff_b);
}

// read_lower's chunk reader: the same arrays as read_codes_direct, into a
// slot of reused buffers (a chunk's arrays live only until gpe_lower_add has
// staged them; fresh bytes objects per chunk were ~40 MB of first-touch pages
// and frees per evaluate at C3's pop 1M), in ONE pass over the trees: each
// thread appends its trees' codes to its own kept buffer (no pass over the
// list headers for the lengths first), then the threads copy their parts
// into the slot's contiguous codes and turn their lengths into offsets.
// Py_True, Py_None (MemoryError set), or nullptr (the general path).
struct RawBuf {                        // grown, never shrunk or zeroed
  char* p = nullptr;
  size_t cap = 0;
  char* get(size_t n) {
    if (n > cap || !p) {
      const size_t c = std::max<size_t>(std::max<size_t>(n, 64), cap + cap / 4);
      char* q = (char*)realloc(p, c);
      if (!q) return nullptr;
      p = q;
      cap = c;
    }
    return p;
  }
};
struct ReadSlot {
  RawBuf codes, off, evals, eoff;
  std::vector<RawBuf> tc;              // per thread: its codes (kept)
  std::vector<std::vector<Val>> te;    // per thread: its ephemerals (kept)
};
PyObject* read_codes_slot(const Fl& F, PyObject* const* tv, Py_ssize_t n, int T,
                          ReadSlot& sl) {
  if (sl.tc.size() < (size_t)T) sl.tc.resize((size_t)T);
  if (sl.te.size() < (size_t)T) sl.te.resize((size_t)T);
  int64_t* off = (int64_t*)sl.off.get((size_t)(n + 1) * 8);
  int64_t* eoff = (int64_t*)sl.eoff.get((size_t)(n + 1) * 8);
  if (!off || !eoff) {
    PyErr_NoMemory();
    Py_INCREF(Py_None);
    return Py_None;
  }
  std::vector<uint8_t> ok((size_t)T, 1);
  std::vector<int64_t> nc((size_t)T + 1, 0), ne((size_t)T + 1, 0);
  auto range = [&](int t, int64_t& a, int64_t& b) {
    a = n * t / T;
    b = n * (t + 1) / T;
  };
  auto run = [&](auto fn) {
    if (T == 1) {
      fn(0);
      return;
    }
    hostpool::par_run(T, fn);
  };
  run([&](int t) {
    int64_t a, b;
    range(t, a, b);
    RawBuf& c = sl.tc[(size_t)t];
    std::vector<Val>& ev = sl.te[(size_t)t];
    ev.clear();
    size_t pos = 0;
    const bool perfect = F.by_id.perfect;
    const PtrMap::Probe P = F.by_id.probe();
    for (int64_t i = a; i < b; ++i) {
      prefetch_trees(tv, i, b);
      if (!PyList_Check(tv[i])) {
        ok[(size_t)t] = 0;
        return;
      }
      const int64_t len = PyList_GET_SIZE(tv[i]);
      if (pos + (size_t)len > c.cap && !c.get(std::max<size_t>(pos + (size_t)len, 4096))) {
        ok[(size_t)t] = 2;                   // out of memory
        return;
      }
      const size_t e0 = ev.size();
      if (!read_nodes(F, P, perfect, ((PyListObject*)tv[i])->ob_item, len,
                      (uint8_t*)c.p + pos, ev)) {
        ok[(size_t)t] = 0;
        return;
      }
      off[i + 1] = len;                      // (lengths: offsets below)
      eoff[i + 1] = (int64_t)(ev.size() - e0);
      pos += (size_t)len;
    }
    nc[(size_t)t + 1] = (int64_t)pos;
    ne[(size_t)t + 1] = (int64_t)ev.size();
  });
  for (int t = 0; t < T; ++t) {
    if (ok[(size_t)t] == 2) {
      PyErr_NoMemory();
      Py_INCREF(Py_None);
      return Py_None;
    }
    if (!ok[(size_t)t]) return nullptr;
  }
  for (int t = 0; t < T; ++t) {
    nc[(size_t)t + 1] += nc[(size_t)t];
    ne[(size_t)t + 1] += ne[(size_t)t];
  }
  uint8_t* cd = (uint8_t*)sl.codes.get((size_t)nc[(size_t)T]);
  Val* evp = (Val*)sl.evals.get((size_t)ne[(size_t)T] * sizeof(Val));
  if (!cd || !evp) {
    PyErr_NoMemory();
    Py_INCREF(Py_None);
    return Py_None;
  }
  off[0] = eoff[0] = 0;
  run([&](int t) {
    int64_t a, b;
    range(t, a, b);
    const size_t bytes = (size_t)(nc[(size_t)t + 1] - nc[(size_t)t]);
    if (bytes) std::memcpy(cd + nc[(size_t)t], sl.tc[(size_t)t].p, bytes);
    const std::vector<Val>& ev = sl.te[(size_t)t];
    if (!ev.empty())
      std::memcpy((void*)(evp + ne[(size_t)t]), ev.data(), ev.size() * sizeof(Val));
    int64_t c = nc[(size_t)t], e = ne[(size_t)t];
    for (int64_t i = a; i < b; ++i) {
      c += off[i + 1];
      off[i + 1] = c;
      e += eoff[i + 1];
      eoff[i + 1] = e;
    }
  });
  Py_RETURN_TRUE;
}

// read_codes(capsule, trees) -> (codes, node_off, evals, eph_off) or None
// The host half of device lowering (gpe_lower_programs): each node object
// becomes its entry index (one byte, prefix order; 255 = an ephemeral, its
// value appended to evals as lowering::Val), read by worker threads without
// the GIL; trees a worker cannot read without the interpreter (nodes found by
// name, e.g. after from_string or pickling) are read again by the calling
// thread.  None when a tree is declined or the pset has 255 or more entries:
// the caller flattens the batch on the host instead.
PyObject* py_read_codes(PyObject*, PyObject* args) {
  PyObject *cap, *trees;
  Py_ssize_t start = 0, stop = -1;     // trees[start:stop] (no slice copy)
  if (!PyArg_ParseTuple(args, "OO|nn", &cap, &trees, &start, &stop)) return nullptr;
  Fl* F = (Fl*)PyCapsule_GetPointer(cap, "_flatnative.Fl");
  if (!F) return nullptr;
  if (F->entries.size() >= 255) Py_RETURN_NONE;
  PyObject* seq = PySequence_Fast(trees, "trees must be a sequence");
  if (!seq) return nullptr;
  const Py_ssize_t len_all = PySequence_Fast_GET_SIZE(seq);
  if (stop < 0 || stop > len_all) stop = len_all;
  if (start < 0 || start > stop) {
    Py_DECREF(seq);
    PyErr_SetString(PyExc_ValueError, "bad tree range");
    return nullptr;
  }
  const Py_ssize_t n = stop - start;
  PyObject** tv = PySequence_Fast_ITEMS(seq) + start;
  const int T = flatten_threads(n);
  if (PyObject* r = read_codes_direct(*F, tv, n, T)) {
    Py_DECREF(seq);
    return r == Py_None ? (Py_DECREF(r), nullptr) : r;
  }
  std::vector<std::vector<uint8_t>> tc((size_t)T);
  std::vector<std::vector<Val>> te((size_t)T);
  std::vector<int64_t> nodes((size_t)n, 0), neph((size_t)n, 0);
  std::vector<uint8_t> bad((size_t)T, 0), need_gil((size_t)n, 0);
  // one tree's codes (reversed prefix entries -> prefix bytes) and its
  // ephemeral values (in prefix order) appended to c / e
  auto put = [](const std::vector<int32_t>& ent, const std::vector<Val>& evals,
                int64_t len, std::vector<uint8_t>& c, std::vector<Val>& e) {
    const size_t base = c.size();
    c.resize(base + (size_t)len);
    for (int64_t k = 0; k < len; ++k) {
      const int32_t v = ent[(size_t)k];
      c[base + (size_t)(len - 1 - k)] = v >= 0 ? (uint8_t)v : (uint8_t)255;
    }
    for (size_t q = evals.size(); q-- > 0;) e.push_back(evals[q]);
  };
  auto work = [&](int t) {
    std::vector<int32_t> ent;
    std::vector<Val> evals;
    const int64_t a = n * t / T, b = n * (t + 1) / T;
    tc[(size_t)t].reserve((size_t)(b - a) * 32);
    for (int64_t i = a; i < b; ++i) {
      prefetch_trees(tv, i, b);
      // fast path: a list tree whose nodes are all pset entries (no
      // ephemerals) is written straight into the codes, prefix order
      if (PyList_Check(tv[i])) {
        const int64_t len = PyList_GET_SIZE(tv[i]);
        PyObject** items = ((PyListObject*)tv[i])->ob_item;
        std::vector<uint8_t>& c = tc[(size_t)t];
        const size_t base = c.size();
        c.resize(base + (size_t)len);
        uint8_t* out = c.data() + base;
        int64_t j = 0;
        for (; j < len; ++j) {
          const int ei = F->by_id.find((uintptr_t)items[j]);
          if (ei < 0) break;
          out[j] = (uint8_t)ei;
        }
        if (j == len) {
          nodes[(size_t)i] = len;
          continue;
        }
        c.resize(base);                    // an ephemeral (or unknown) node
      }
      ent.clear();
      evals.clear();
      int64_t len = 0;
      const int rc = read_tree(*F, tv[i], false, ent, evals, len);
      if (rc == RD_NEED_GIL) {
        need_gil[(size_t)i] = 1;
        continue;
      }
      if (rc != RD_OK) {
        bad[(size_t)t] = 1;
        return;
      }
      put(ent, evals, len, tc[(size_t)t], te[(size_t)t]);
      nodes[(size_t)i] = len;
      neph[(size_t)i] = (int64_t)evals.size();
    }
  };
  if (T == 1) {
    work(0);
  } else {
    hostpool::par_run(T, work);
  }
  for (uint8_t b : bad)
    if (b) {
      Py_DECREF(seq);
      Py_RETURN_NONE;
    }
  // trees the workers left to the interpreter, read here with the GIL; the
  // merge below then goes tree by tree
  bool any_gil = false;
  std::vector<uint8_t> gc;
  std::vector<Val> ge;
  {
    std::vector<int32_t> ent;
    std::vector<Val> evals;
    for (Py_ssize_t i = 0; i < n; ++i) {
      if (!need_gil[(size_t)i]) continue;
      any_gil = true;
      ent.clear();
      evals.clear();
      int64_t len = 0;
      if (read_tree(*F, tv[i], true, ent, evals, len) != RD_OK) {
        Py_DECREF(seq);
        if (PyErr_Occurred()) PyErr_Clear();
        Py_RETURN_NONE;
      }
      put(ent, evals, len, gc, ge);
      nodes[(size_t)i] = len;
      neph[(size_t)i] = (int64_t)evals.size();
    }
  }
  Py_DECREF(seq);
  size_t total = gc.size(), total_e = ge.size();
  for (int t = 0; t < T; ++t) {
    total += tc[(size_t)t].size();
    total_e += te[(size_t)t].size();
  }
  PyObject* codes_b = PyBytes_FromStringAndSize(nullptr, (Py_ssize_t)total);
  PyObject* off_b = PyBytes_FromStringAndSize(nullptr, (Py_ssize_t)((n + 1) * 8));
  PyObject* ev_b = PyBytes_FromStringAndSize(nullptr, (Py_ssize_t)(total_e * sizeof(Val)));
  PyObject* eoff_b = PyBytes_FromStringAndSize(nullptr, (Py_ssize_t)((n + 1) * 8));
  if (!codes_b || !off_b || !ev_b || !eoff_b) {
    Py_XDECREF(codes_b);
    Py_XDECREF(off_b);
    Py_XDECREF(ev_b);
    Py_XDECREF(eoff_b);
    return nullptr;
  }
  uint8_t* cd = (uint8_t*)PyBytes_AS_STRING(codes_b);
  Val* ev = (Val*)PyBytes_AS_STRING(ev_b);
  size_t pc = 0, pe = 0;
  if (any_gil) {
    size_t gcp = 0, gep = 0;
    for (int t = 0; t < T; ++t) {
      size_t tcp = 0, tep = 0;
      for (int64_t i = n * t / T, b = n * (t + 1) / T; i < b; ++i) {
        const size_t nc = (size_t)nodes[(size_t)i], ne = (size_t)neph[(size_t)i];
        const bool g = need_gil[(size_t)i];
        std::memcpy(cd + pc, g ? gc.data() + gcp : tc[(size_t)t].data() + tcp, nc);
        if (ne)
          std::memcpy((void*)(ev + pe), g ? ge.data() + gep : te[(size_t)t].data() + tep,
                      ne * sizeof(Val));
        (g ? gcp : tcp) += nc;
        (g ? gep : tep) += ne;
        pc += nc;
        pe += ne;
      }
    }
  } else for (int t = 0; t < T; ++t) {
    std::memcpy(cd + pc, tc[(size_t)t].data(), tc[(size_t)t].size());
    pc += tc[(size_t)t].size();
    if (!te[(size_t)t].empty())
      std::memcpy((void*)(ev + pe), te[(size_t)t].data(), te[(size_t)t].size() * sizeof(Val));
    pe += te[(size_t)t].size();
  }
  int64_t* off = (int64_t*)PyBytes_AS_STRING(off_b);
  int64_t* eoff = (int64_t*)PyBytes_AS_STRING(eoff_b);
  off[0] = eoff[0] = 0;
  for (Py_ssize_t i = 0; i < n; ++i) {
    off[i + 1] = off[i] + nodes[(size_t)i];
    eoff[i + 1] = eoff[i] + neph[(size_t)i];
  }
  return Py_BuildValue("(NNNN)", codes_b, off_b, ev_b, eoff_b);
}

// read_lower(capsule, trees, ends, lower_add, ctx, off_out[, start]) -> 0,
// the lowering's error code, or None (a chunk the reader declines: nothing
// more is added).  The chunked device lowering as one pipeline: the trees
// [start, ends[-1]) are read in chunks [ends[k-1], ends[k]) (the first from
// start; read_codes) while, on a thread of its
// own, the previous chunk goes to `lower_add` (the library's gpe_lower_add,
// by address: it stages the chunk into pinned memory, so the chunk's buffers
// can go once it returns).  The reads need the GIL (the calling thread holds
// it); gpe_lower_add is plain C.  off_out (int64[n + 1], writable buffer):
// the node offsets of the n trees read, from 0.
typedef int (*LowerAddFn)(void*, const uint8_t*, const int64_t*, int64_t, const void*,
                          const int64_t*);

// The helper thread of read_lower: one per process, kept (a fresh
// std::thread per chunk exited after its gpe_lower_add, and the HIP
// runtime's per-thread teardown at exit waited for the device — the
// pipeline's last join took 1-4 ms at C3's pop 1M).  One job at a time.
class LowerWorker {
 public:
  LowerWorker() : pid_(getpid()) { std::thread([this] { loop(); }).detach(); }
  pid_t pid() const { return pid_; }
  void submit(std::function<void()> fn) {
    std::lock_guard<std::mutex> lk(mu_);
    job_ = std::move(fn);
    busy_ = true;
    cv_.notify_all();
  }
  void wait() {
    std::unique_lock<std::mutex> lk(mu_);
    done_.wait(lk, [&] { return !busy_; });
  }

 private:
  void loop() {
    std::unique_lock<std::mutex> lk(mu_);
    for (;;) {
      cv_.wait(lk, [&] { return busy_ && job_; });
      std::function<void()> fn = std::move(job_);
      job_ = nullptr;
      lk.unlock();
      fn();
      lk.lock();
      busy_ = false;
      done_.notify_all();
    }
  }
  pid_t pid_;
  std::mutex mu_;
  std::condition_variable cv_, done_;
  std::function<void()> job_;
  bool busy_ = false;
};

LowerWorker& lower_worker() {
  // never destroyed (its thread sleeps in cv_ at exit); a forked child gets
  // its own
  static std::mutex mu;
  static LowerWorker* w = nullptr;
  std::lock_guard<std::mutex> lk(mu);
  if (!w || w->pid() != getpid()) w = new LowerWorker();
  return *w;
}
PyObject* py_read_lower(PyObject*, PyObject* args) {
  PyObject *cap, *trees, *ends_obj;
  unsigned long long fn_addr, ctx_addr;
  Py_buffer ob;
  Py_ssize_t start = 0;
  if (!PyArg_ParseTuple(args, "OOOKKw*|n", &cap, &trees, &ends_obj, &fn_addr, &ctx_addr, &ob,
                        &start))
    return nullptr;
  LowerAddFn fn = (LowerAddFn)(uintptr_t)fn_addr;
  void* ctxp = (void*)(uintptr_t)ctx_addr;
  int64_t* off = (int64_t*)ob.buf - start;   // indexed by tree: off[start] is 0
  PyObject* ends = PySequence_Fast(ends_obj, "ends must be a sequence");
  if (!ends) {
    PyBuffer_Release(&ob);
    return nullptr;
  }
  const Py_ssize_t nk = PySequence_Fast_GET_SIZE(ends);
  {
    // the ends rise from start within the trees, and off_out holds their offsets
    Py_ssize_t prev = start;
    bool ok = start >= 0;
    for (Py_ssize_t k = 0; k < nk && ok; ++k) {
      const Py_ssize_t e = PyLong_AsSsize_t(PySequence_Fast_GET_ITEM(ends, k));
      ok = !(e == -1 && PyErr_Occurred()) && e >= prev;
      prev = e;
    }
    if (ok && (Py_ssize_t)(ob.len / (Py_ssize_t)sizeof(int64_t)) < prev - start + 1) ok = false;
    const Py_ssize_t n_trees = ok ? PySequence_Size(trees) : -1;
    if (ok && (n_trees < 0 || prev > n_trees)) ok = false;
    if (!ok) {
      Py_DECREF(ends);
      PyBuffer_Release(&ob);
      if (!PyErr_Occurred()) PyErr_SetString(PyExc_ValueError, "bad chunk ends or offsets buffer");
      return nullptr;
    }
  }
  Fl* F = (Fl*)PyCapsule_GetPointer(cap, "_flatnative.Fl");
  PyObject* seq = F ? PySequence_Fast(trees, "trees must be a sequence") : nullptr;
  if (!seq) {
    Py_DECREF(ends);
    PyBuffer_Release(&ob);
    return nullptr;
  }
  PyObject** tv = PySequence_Fast_ITEMS(seq);
  // one read_lower at a time per process: the helper thread and the chunk
  // slots are shared (taken with the GIL released: the holder may wait on
  // a lower_add that is a Python callback)
  static std::mutex rl_mu;
  static ReadSlot slots[2];            // chunk k's arrays: slots[k & 1]
  std::unique_lock<std::mutex> guard(rl_mu, std::defer_lock);
  Py_BEGIN_ALLOW_THREADS
  guard.lock();
  Py_END_ALLOW_THREADS
  LowerWorker& worker = lower_worker();
  bool in_flight = false;
  int wrc = 0;
  PyObject* held = nullptr;            // the chunk in flight (its four buffers)
  auto join = [&]() {
    if (in_flight) {
      Py_BEGIN_ALLOW_THREADS               // (a lower_add that is a Python
      worker.wait();                       //  callback needs the GIL)
      Py_END_ALLOW_THREADS
      in_flight = false;
    }
    Py_XDECREF(held);
    held = nullptr;
  };
  PyObject* result = nullptr;
  Py_ssize_t a = start;
  off[start] = 0;
  bool declined = false;
  // GPE_DIAG: the reads' and the joins' time on the calling thread
  static const bool diag = getenv("GPE_DIAG") != nullptr;
  using clk = std::chrono::steady_clock;
  double t_read = 0, t_join = 0;
  for (Py_ssize_t k = 0; k < nk; ++k) {
    const Py_ssize_t b = PyLong_AsSsize_t(PySequence_Fast_GET_ITEM(ends, k));
    if (b < 0 && PyErr_Occurred()) break;
    const auto t0 = clk::now();
    const int64_t nn = b - a;
    // the common case straight into this chunk's slot; trees it declines
    // (not lists, nodes that need the interpreter) through read_codes
    PyObject* r = nullptr;
    ReadSlot& sl = slots[k & 1];
    if (F->entries.size() < 255)
      r = read_codes_slot(*F, tv + a, nn, flatten_threads(nn), sl);
    if (r == Py_None) {                 // out of memory (error set)
      Py_DECREF(r);
      break;
    }
    if (!r) {
      PyObject* rargs = Py_BuildValue("(OOnn)", cap, trees, a, b);
      r = rargs ? py_read_codes(nullptr, rargs) : nullptr;
      Py_XDECREF(rargs);
    }
    t_read += std::chrono::duration<double, std::milli>(clk::now() - t0).count();
    if (!r) break;                      // an exception
    if (r == Py_None) {                 // the host flattener's batch
      Py_DECREF(r);
      declined = true;
      break;
    }
    const uint8_t* codes;
    const void* evals;
    const int64_t *no, *eph;
    PyObject* keep = nullptr;           // a read_codes result: its bytes
    if (r == Py_True) {
      Py_DECREF(r);
      codes = (const uint8_t*)sl.codes.p;
      no = (const int64_t*)sl.off.p;
      evals = sl.evals.p;
      eph = (const int64_t*)sl.eoff.p;
    } else {
      // (the buffers stay valid while `held` does: bytes objects)
      codes = (const uint8_t*)PyBytes_AS_STRING(PyTuple_GET_ITEM(r, 0));
      no = (const int64_t*)PyBytes_AS_STRING(PyTuple_GET_ITEM(r, 1));
      evals = PyBytes_AS_STRING(PyTuple_GET_ITEM(r, 2));
      eph = (const int64_t*)PyBytes_AS_STRING(PyTuple_GET_ITEM(r, 3));
      keep = r;
    }
    for (int64_t i = 0; i < nn; ++i) off[a + i + 1] = off[a] + no[i + 1];
    const auto t1 = clk::now();
    join();                             // the previous chunk is staged
    t_join += std::chrono::duration<double, std::milli>(clk::now() - t1).count();
    if (wrc) {
      Py_XDECREF(keep);
      break;
    }
    held = keep;
    worker.submit([&wrc, fn, ctxp, codes, no, nn, evals, eph] {
      wrc = fn(ctxp, codes, no, nn, evals, eph);
    });
    in_flight = true;
    a = b;
  }
  const auto t2 = clk::now();
  join();
  if (diag)
    fprintf(stderr, "read_lower chunks %zd read %.3f ms joins %.3f ms @%.3f last join %.3f ms\n",
            nk, t_read, t_join,
            [&] {
              const double ms = std::chrono::duration<double, std::milli>(
                                    t2.time_since_epoch()).count();
              return ms - 1e8 * (double)(int64_t)(ms / 1e8);
            }(),
            std::chrono::duration<double, std::milli>(clk::now() - t2).count());
  guard.unlock();
  Py_DECREF(seq);
  Py_DECREF(ends);
  PyBuffer_Release(&ob);
  if (PyErr_Occurred()) return nullptr;
  if (declined) Py_RETURN_NONE;
  result = PyLong_FromLong(wrc);
  return result;
}

// lower_codes(capsule, codes, node_off, evals, eph_off) -> (code, offsets,
// depth, err, status): read_codes' output lowered on the host through the same
// lowering::lower the device kernel (gpeval.hip lower_trees) runs, on the
// kernel's packed record storage; status per
// program = declined | inexact << 1 | value error << 2 as gpe_lower_programs
// reports it.  Test support: device lowering checked on machines without a GPU.
PyObject* py_lower_codes(PyObject*, PyObject* args) {
  PyObject* cap;
  Py_buffer cb, ob, eb, eob;
  if (!PyArg_ParseTuple(args, "Oy*y*y*y*", &cap, &cb, &ob, &eb, &eob)) return nullptr;
  struct Rel {
    Py_buffer* b[4];
    ~Rel() { for (Py_buffer* x : b) PyBuffer_Release(x); }
  } rel{{&cb, &ob, &eb, &eob}};
  Fl* F = (Fl*)PyCapsule_GetPointer(cap, "_flatnative.Fl");
  if (!F) return nullptr;
  const int64_t* off = (const int64_t*)ob.buf;
  const int64_t* eoff = (const int64_t*)eob.buf;
  const int64_t n = ob.len / 8 - 1;
  if (n < 0 || eob.len != ob.len || off[n] != cb.len ||
      eoff[n] * (int64_t)sizeof(Val) != eb.len) {
    PyErr_SetString(PyExc_ValueError, "inconsistent lowering arrays");
    return nullptr;
  }
  const uint8_t* codes = (const uint8_t*)cb.buf;
  const Val* evals = (const Val*)eb.buf;
  std::vector<uint32_t> words;
  std::vector<int64_t> woff((size_t)n + 1, 0);
  std::vector<int32_t> depth((size_t)n);
  std::vector<uint8_t> err((size_t)n), status((size_t)n);
  std::vector<int32_t> ent;
  for (int64_t i = 0; i < n; ++i) {
    const int64_t len = off[i + 1] - off[i];
    ent.assign((size_t)len, 0);
    int32_t e = (int32_t)(eoff[i + 1] - eoff[i]) - 1;
    for (int64_t k = 0; k < len; ++k) {           // reversed prefix
      const uint8_t v = codes[off[i] + len - 1 - k];
      ent[(size_t)k] = v != 255 ? (int32_t)v : -1 - (e--);
    }
    TreeOut o;
    lower_tree(*F, ent.data(), len, evals + eoff[i], words, o, true, (int)(i & 63));
    woff[(size_t)i + 1] = (int64_t)words.size();
    depth[(size_t)i] = o.depth;
    err[(size_t)i] = (uint8_t)o.err;
    status[(size_t)i] = (uint8_t)((o.declined ? 1 : 0) | (o.inexact ? 2 : 0) | (o.verr ? 4 : 0));
  }
  auto B = [](const void* p, size_t nb) {
    return PyBytes_FromStringAndSize((const char*)p, (Py_ssize_t)nb);
  };
  return Py_BuildValue("(NNNNN)", B(words.data(), words.size() * 4),
                       B(woff.data(), woff.size() * 8), B(depth.data(), depth.size() * 4),
                       B(err.data(), err.size()), B(status.data(), status.size()));
}

// entries(capsule) -> bytes: the pset entries as lowering::Entry (= the C
// ABI's gpe_entry), for gpe_set_lowering
PyObject* py_entries(PyObject*, PyObject* args) {
  PyObject* cap;
  if (!PyArg_ParseTuple(args, "O", &cap)) return nullptr;
  Fl* F = (Fl*)PyCapsule_GetPointer(cap, "_flatnative.Fl");
  if (!F) return nullptr;
  return PyBytes_FromStringAndSize((const char*)F->entries.data(),
                                   (Py_ssize_t)(F->entries.size() * sizeof(Entry)));
}

// lengths(trees) -> bytes (int64 per tree): len(tree), read by worker threads
// for list trees (the population sharder balances ranks by total length,
// SURVEY 8e; len() over a million lists in Python costs tens of ms); None
// when an item is not a list (the caller then uses len()).
PyObject* py_lengths(PyObject*, PyObject* args) {
  PyObject* trees;
  if (!PyArg_ParseTuple(args, "O", &trees)) return nullptr;
  PyObject* seq = PySequence_Fast(trees, "trees must be a sequence");
  if (!seq) return nullptr;
  const Py_ssize_t n = PySequence_Fast_GET_SIZE(seq);
  PyObject* const* tv = PySequence_Fast_ITEMS(seq);
  PyObject* out = PyBytes_FromStringAndSize(nullptr, (Py_ssize_t)(n * 8));
  if (!out) {
    Py_DECREF(seq);
    return nullptr;
  }
  int64_t* len = (int64_t*)PyBytes_AS_STRING(out);
  const int T = flatten_threads(n);
  std::vector<uint8_t> ok((size_t)T, 1);
  auto work = [&](int t) {
    const int64_t a = n * t / T, b = n * (t + 1) / T;
    for (int64_t i = a; i < b; ++i) {
      if (i + kPfHead < b) __builtin_prefetch(tv[i + kPfHead]);
      if (!PyList_Check(tv[i])) {
        ok[(size_t)t] = 0;
        return;
      }
      len[i] = PyList_GET_SIZE(tv[i]);
    }
  };
  if (T == 1) {
    work(0);
  } else {
    hostpool::par_run(T, work);
  }
  Py_DECREF(seq);
  for (uint8_t o : ok)
    if (!o) {
      Py_DECREF(out);
      Py_RETURN_NONE;
    }
  return out;
}

PyMethodDef methods[] = {
    {"tuples1", py_tuples1, METH_VARARGS, "tuples1(float64 buffer, as_int)"},
    {"lengths", py_lengths, METH_VARARGS, "lengths(trees) -> int64 bytes"},
    {"new", py_new, METH_VARARGS,
     "new(machine, nv, leaves, ids, entries, by_name, eph_types, value_descr)"},
    {"flatten", py_flatten, METH_VARARGS, "flatten(capsule, trees)"},
    {"read_codes", py_read_codes, METH_VARARGS, "read_codes(capsule, trees[, start, stop])"},
    {"read_lower", py_read_lower, METH_VARARGS,
     "read_lower(capsule, trees, ends, lower_add_addr, ctx_addr, off_out)"},
    {"entries", py_entries, METH_VARARGS, "entries(capsule)"},
    {"lower_codes", py_lower_codes, METH_VARARGS,
     "lower_codes(capsule, codes, node_off, evals, eph_off)"},
    {nullptr, nullptr, 0, nullptr}};

PyModuleDef module = {PyModuleDef_HEAD_INIT, "_flatnative",
                      "Native PrimitiveTree flattener (see flatten_native.cpp)",
                      -1, methods};

}  // namespace

PyMODINIT_FUNC PyInit__flatnative(void) { return PyModule_Create(&module); }
