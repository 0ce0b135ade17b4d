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

namespace {

// opcodes — keep in sync with deap_amd/flatten.py:Op
enum : uint32_t {
  OP_END = 0, OP_LDV = 1, OP_LDC = 2, OP_PUSH = 3, OP_PUSHV = 4, OP_PUSHC = 5,
  OP_ADD = 8, OP_SUB = 11, OP_RSUB = 14, OP_MUL = 17, OP_DIV = 20,
  OP_RDIV = 23, OP_LT = 26, OP_GT = 29, OP_EQ = 32, OP_AND = 35, OP_OR = 38,
  OP_XOR = 41, OP_NEG = 48, OP_SIN = 49, OP_COS = 50, OP_NOT = 51,
  OP_ITE = 52, OP_NPDIV = 56, OP_RNPDIV = 59
};
// semantic codes passed from Python (flatten.py: _NATIVE_SEM)
enum Sem : int {
  S_ADD = 0, S_SUB, S_MUL, S_PDIV, S_NEG, S_SIN, S_COS, S_AND, S_OR, S_XOR,
  S_NOT, S_LT, S_EQ, S_ITE, S_NPDIV, S_NPSIN, S_NPCOS
};
enum Kind : int { K_PRIM = 0, K_ARG = 1, K_CONST = 2 };
constexpr int MAX_COMPILE_HEIGHT = 200;
constexpr uint8_t ERR_SYNTAX = 3, ERR_CONST = 4;

// a Python number as the fold sees it
struct Val {
  char t = 'f';        // 'f' float, 'i' int, 'b' bool, 'x' unsupported
  double f = 0.0;
  int64_t i = 0;
  bool err_value = false;  // the fold raised ValueError (sin/cos of inf)
  double as_f() const { return t == 'f' ? f : (double)i; }
  bool truth() const { return t == 'f' ? f != 0.0 : i != 0; }
};

struct Entry {
  int kind = K_CONST;
  int arity = 0;
  int sem = 0;
  int var = 0;
  Val c;
};

// One lowered node (24 bytes; records of a tree live in Fl::recs in
// reversed-prefix order, children before parents).
struct Rec {
  uint8_t kind;        // 'v' variable column, 'c' constant, 'p' primitive
  uint8_t nk;          // children
  uint16_t height;     // gp.compile's nesting height of the subtree
  int32_t payload;     // var index, sem, or constant index into Fl::cvals
  int32_t need;        // stack slots the subtree needs (flatten.py _need)
  int32_t kid[3];
};

// Identity map of the shared pset nodes (a few dozen objects): open
// addressing on the object address, probed once per tree node.
struct PtrMap {
  std::vector<uintptr_t> keys;
  std::vector<int> vals;
  int shift = 63;
  void build(const std::vector<std::pair<uintptr_t, int>>& kv) {
    size_t cap = 16;
    while (cap < kv.size() * 4) cap <<= 1;
    shift = 64;
    for (size_t c = cap; c > 1; c >>= 1) --shift;
    keys.assign(cap, 0);
    vals.assign(cap, -1);
    for (const auto& e : kv) {
      size_t h = slot(e.first);
      while (keys[h] && keys[h] != e.first) h = (h + 1) & (cap - 1);
      keys[h] = e.first;
      vals[h] = e.second;
    }
  }
  size_t slot(uintptr_t k) const {
    return (size_t)(((uint64_t)k * 0x9E3779B97F4A7C15ull) >> shift);
  }
  int find(uintptr_t k) const {
    const size_t mask = keys.size() - 1;
    for (size_t h = slot(k);; h = (h + 1) & mask) {
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

// Python semantics of the fold (flatten.py Flattener._fold with the pset's
// own callables: operator.*, protectedDiv, math.sin/cos, if_then_else).
// Returns false to decline (the Python flattener then handles the tree).
bool fold(int sem, const Val* k, int n, Val& r) {
  for (int i = 0; i < n; ++i) {
    if (k[i].err_value) { r.err_value = true; return true; }
    if (k[i].t == 'x') return false;
  }
  const bool ints = (n < 1 || k[0].t != 'f') && (n < 2 || k[1].t != 'f');
  switch (sem) {
    case S_ADD: case S_SUB: case S_MUL: {
      if (ints) {
        long long o;
        bool ov = sem == S_ADD ? __builtin_add_overflow(k[0].i, k[1].i, &o)
                : sem == S_SUB ? __builtin_sub_overflow(k[0].i, k[1].i, &o)
                               : __builtin_mul_overflow(k[0].i, k[1].i, &o);
        if (ov) return false;
        r.t = 'i'; r.i = o;
        return true;
      }
      const double a = k[0].as_f(), b = k[1].as_f();
      r.t = 'f';
      r.f = sem == S_ADD ? a + b : sem == S_SUB ? a - b : a * b;
      return true;
    }
    case S_PDIV: {
      // true division; ZeroDivisionError -> int 1 (symbreg.py:29-33)
      if (k[1].as_f() == 0.0) { r.t = 'i'; r.i = 1; return true; }
      if (ints && (std::llabs(k[0].i) > (1LL << 53) || std::llabs(k[1].i) > (1LL << 53)))
        return false;          // Python rounds the exact quotient
      r.t = 'f';
      r.f = k[0].as_f() / k[1].as_f();
      return true;
    }
    case S_NEG:
      if (k[0].t == 'f') { r.t = 'f'; r.f = -k[0].f; return true; }
      if (k[0].i == INT64_MIN) return false;
      r.t = 'i'; r.i = -k[0].i;
      return true;
    case S_SIN: case S_COS: {
      const double x = k[0].as_f();
      if (std::isinf(x)) { r.err_value = true; return true; }
      r.t = 'f';
      r.f = sem == S_SIN ? std::sin(x) : std::cos(x);   // glibc, as math.*
      return true;
    }
    case S_NPSIN: case S_NPCOS: {            // numpy: sin(inf) = nan
      const double x = k[0].as_f();
      r.t = 'f';
      r.f = std::isinf(x) ? std::nan("") : sem == S_NPSIN ? std::sin(x) : std::cos(x);
      return true;
    }
    case S_NPDIV: {                          // symbreg_numpy.py:28-36
      const double q = k[0].as_f() / k[1].as_f();
      if (std::isinf(q) || std::isnan(q)) { r.t = 'i'; r.i = 1; return true; }
      r.t = 'f';
      r.f = q;
      return true;
    }
    case S_AND: case S_OR: case S_XOR: {
      if (k[0].t == 'f' || k[1].t == 'f') return false;   // TypeError
      const int64_t a = k[0].i, b = k[1].i;
      r.i = sem == S_AND ? (a & b) : sem == S_OR ? (a | b) : (a ^ b);
      r.t = (k[0].t == 'b' && k[1].t == 'b') ? 'b' : 'i';
      return true;
    }
    case S_NOT:
      r.t = 'b'; r.i = k[0].truth() ? 0 : 1;
      return true;
    case S_LT: case S_EQ: {
      bool v;
      if (ints) v = sem == S_LT ? k[0].i < k[1].i : k[0].i == k[1].i;
      else {
        const double a = k[0].as_f(), b = k[1].as_f();
        if ((k[0].t != 'f' && std::llabs(k[0].i) > (1LL << 53)) ||
            (k[1].t != 'f' && std::llabs(k[1].i) > (1LL << 53)))
          return false;        // Python compares int/float exactly
        v = sem == S_LT ? a < b : a == b;
      }
      r.t = 'b'; r.i = v ? 1 : 0;
      return true;
    }
    case S_ITE:
      r = k[0].truth() ? k[1] : k[2];
      return true;
  }
  return false;
}

int need_of(const Rec* R, const Rec& p) {
  if (p.nk == 1) return R[p.kid[0]].need;
  if (p.nk == 3)
    return std::max(R[p.kid[0]].need,
                    std::max(1 + R[p.kid[1]].need, 2 + R[p.kid[2]].need));
  const Rec& l = R[p.kid[0]];
  const Rec& r = R[p.kid[1]];
  if (r.kind != 'p') return l.need;
  if (l.kind != 'p') return r.need;
  return l.need == r.need ? l.need + 1 : std::max(l.need, r.need);
}

void binary_ops(int sem, uint32_t& fwd, uint32_t& rev) {
  switch (sem) {
    case S_ADD: fwd = rev = OP_ADD; return;
    case S_SUB: fwd = OP_SUB; rev = OP_RSUB; return;
    case S_MUL: fwd = rev = OP_MUL; return;
    case S_PDIV: fwd = OP_DIV; rev = OP_RDIV; return;
    case S_LT: fwd = OP_LT; rev = OP_GT; return;
    case S_EQ: fwd = rev = OP_EQ; return;
    case S_AND: fwd = rev = OP_AND; return;
    case S_OR: fwd = rev = OP_OR; return;
    case S_XOR: fwd = rev = OP_XOR; return;
    case S_NPDIV: fwd = OP_NPDIV; rev = OP_RNPDIV; return;
  }
  fwd = rev = 0xff;
}

uint32_t unary_op(int sem) {
  return sem == S_NEG ? OP_NEG
       : (sem == S_SIN || sem == S_NPSIN) ? OP_SIN
       : (sem == S_COS || sem == S_NPCOS) ? OP_COS : OP_NOT;
}

// flatten.py Flattener._emit + _encode in one pass: instruction words are
// written straight to `o`.  _encode's peephole (PUSH followed by LDV/LDC ->
// PUSHV/PUSHC carrying the PUSH's slot) is a pending PUSH that the next
// leaf load absorbs; _check_consts (F machine) is tallied per constant word.
struct Emitter {
  const Rec* R;
  const Val* cv;
  uint32_t* o;
  int pend = -1;       // slot of a PUSH not yet written
  bool fm;             // F machine: constants as two fp64 words
  bool bad = false;    // a constant whose fold raised
  bool big = false;    // an int constant beyond 2**53

  void flush() {
    if (pend >= 0) {
      *o++ = OP_PUSH | ((uint32_t)pend << 8);
      pend = -1;
    }
  }
  void konst(uint32_t op, uint32_t d, const Val& c) {
    if (fm) {
      if (c.err_value) bad = true;
      else if (c.t == 'i' && std::llabs(c.i) > (1LL << 53)) big = true;
      const double v = c.as_f();
      uint64_t bits;
      std::memcpy(&bits, &v, 8);
      o[0] = op | (d << 8);
      o[1] = (uint32_t)(bits & 0xffffffffu);
      o[2] = (uint32_t)(bits >> 32);
      o += 3;
    } else {
      *o++ = op | (d << 8) | ((c.truth() ? 1u : 0u) << 16);
    }
  }
  void leaf(const Rec& L, uint32_t d) {          // LDV / LDC (or fused)
    uint32_t op = L.kind == 'v' ? OP_LDV : OP_LDC;
    if (pend >= 0) {
      op = L.kind == 'v' ? OP_PUSHV : OP_PUSHC;
      d = (uint32_t)pend;
      pend = -1;
    }
    if (L.kind == 'v') *o++ = op | (d << 8) | ((uint32_t)L.payload << 16);
    else konst(op, d, cv[L.payload]);
  }
  void operand(uint32_t op, const Rec& L, uint32_t d) {   // op+1 / op+2
    flush();
    if (L.kind == 'v') *o++ = (op + 1) | (d << 8) | ((uint32_t)L.payload << 16);
    else konst(op + 2, d, cv[L.payload]);
  }
  void plain(uint32_t op, uint32_t d) {
    flush();
    *o++ = op | (d << 8);
  }
  void push(uint32_t d) {
    flush();
    pend = (int)d;
  }
  uint32_t emit(int ri, uint32_t d) {
    const Rec& rec = R[ri];
    if (rec.kind != 'p') {
      leaf(rec, d);
      return d;
    }
    const int sem = rec.payload;
    if (rec.nk == 1) {
      const uint32_t top = emit(rec.kid[0], d);
      plain(unary_op(sem), d);
      return top;
    }
    if (rec.nk == 3) {
      const uint32_t t0 = emit(rec.kid[0], d);
      push(d);
      const uint32_t t1 = emit(rec.kid[1], d + 1);
      push(d + 1);
      const uint32_t t2 = emit(rec.kid[2], d + 2);
      plain(OP_ITE, d);
      return std::max(std::max(t0, t1), std::max(t2, d + 2));
    }
    uint32_t fwd, rev;
    binary_ops(sem, fwd, rev);
    const int left = rec.kid[0], right = rec.kid[1];
    const Rec& L = R[left];
    const Rec& Rr = R[right];
    if (Rr.kind != 'p') {
      const uint32_t top = emit(left, d);
      operand(rev, Rr, d);
      return top;
    }
    if (L.kind != 'p') {
      const uint32_t top = emit(right, d);
      operand(fwd, L, d);
      return top;
    }
    const bool lfirst = L.need >= Rr.need;
    const uint32_t t0 = emit(lfirst ? left : right, d);
    push(d);
    const uint32_t t1 = emit(lfirst ? right : left, d + 1);
    plain(lfirst ? fwd : rev, d);
    return std::max(std::max(t0, t1), d + 1);
  }
};

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
void lower_tree(Fl& F, const int32_t* ent, int64_t len, const Val* evals,
                std::vector<uint32_t>& words, TreeOut& o) {
  if ((int64_t)F.recs.size() < len) {
    F.recs.resize((size_t)len);
    F.stack.resize((size_t)len);
  }
  F.cvals.clear();
  Rec* R = F.recs.data();
  int32_t* stk = F.stack.data();
  int64_t sp = 0;
  bool decline = false;
  for (int64_t k = 0; k < len; ++k) {
    const int32_t ei = ent[k];
    Rec& r = R[k];
    r.nk = 0;
    r.height = 0;
    r.need = 1;
    if (ei < 0) {                          // ephemeral constant
      r.kind = 'c';
      r.payload = (int32_t)F.cvals.size();
      F.cvals.push_back(evals[-1 - ei]);
      stk[sp++] = (int32_t)k;
      continue;
    }
    const Entry& e = F.entries[ei];
    if (e.kind == K_ARG) {
      r.kind = 'v';
      r.payload = e.var;
      stk[sp++] = (int32_t)k;
      continue;
    }
    if (e.kind == K_CONST) {
      if (e.c.t == 'x') { decline = true; break; }
      r.kind = 'c';
      r.payload = (int32_t)F.cvals.size();
      F.cvals.push_back(e.c);
      stk[sp++] = (int32_t)k;
      continue;
    }
    const int ar = e.arity;
    if (sp < ar || ar > 3) { decline = true; break; }
    int h = 0;
    for (int q = 0; q < ar; ++q) {
      const int32_t c = stk[--sp];
      r.kid[q] = c;
      h = std::max(h, (int)R[c].height + 1);
    }
    r.height = (uint16_t)std::min(h, 65535);
    const Rec& k0 = R[r.kid[0]];
    const bool trig = e.sem == S_SIN || e.sem == S_COS ||
                      e.sem == S_NPSIN || e.sem == S_NPCOS;
    if (trig && k0.kind == 'v' && k0.payload < (int)F.leaf.size() &&
        F.leaf[k0.payload]) {
      r.kind = 'v';                        // a trig-leaf column
      r.payload = ((e.sem == S_SIN || e.sem == S_NPSIN) ? 1 : 2) * F.nv +
                  k0.payload;
    } else {
      bool all_c = true;
      for (int q = 0; q < ar; ++q) all_c &= R[r.kid[q]].kind == 'c';
      if (all_c) {
        Val kv[3];
        for (int q = 0; q < ar; ++q) kv[q] = F.cvals[R[r.kid[q]].payload];
        Val out;
        if (!fold(e.sem, kv, ar, out)) { decline = true; break; }
        r.kind = 'c';
        r.payload = (int32_t)F.cvals.size();
        F.cvals.push_back(out);
      } else {
        r.kind = 'p';
        r.nk = (uint8_t)ar;
        r.payload = e.sem;
        r.need = need_of(R, r);
      }
    }
    stk[sp++] = (int32_t)k;
  }
  if (decline || sp != 1) {
    o.declined = true;
    words.push_back(OP_END);
    return;
  }
  const int root = stk[0];
  const Rec& rr = R[root];
  if (len > MAX_COMPILE_HEIGHT && rr.height > MAX_COMPILE_HEIGHT) {
    o.err = ERR_SYNTAX;
    words.push_back(OP_END);
    return;
  }
  if (rr.kind == 'c' && F.cvals[rr.payload].err_value) {
    o.err = ERR_CONST;
    o.verr = true;
    words.push_back(OP_END);
    return;
  }
  // at most 3 words per node (an F-machine constant) plus END
  const size_t base = words.size();
  words.resize(base + 3 * (size_t)len + 1);
  Emitter em{R, F.cvals.data(), words.data() + base};
  em.fm = F.machine == 0;
  o.depth = (int32_t)em.emit(root, 0);
  em.flush();
  *em.o++ = OP_END;
  if (em.bad) {                            // _check_consts: a raising fold
    words.resize(base);
    o.err = ERR_CONST;
    o.verr = true;
    words.push_back(OP_END);
    return;
  }
  o.inexact = em.big;
  words.resize((size_t)(em.o - words.data()));
}

int flatten_threads(int64_t n_trees) {
  // the GPU box sets OMP_NUM_THREADS to its CPU share; default 8, at most 16
  int t = 8;
  if (const char* env = std::getenv("OMP_NUM_THREADS")) t = std::atoi(env);
  const unsigned hw = std::thread::hardware_concurrency();
  if (hw) t = std::min<int>(t, (int)hw);
  t = std::max(1, std::min(t, 16));
  return (int)std::max<int64_t>(1, std::min<int64_t>(t, n_trees / 4096));
}

enum Read { RD_OK = 0, RD_DECLINE = 1, RD_NEED_GIL = 2 };

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
    std::vector<std::thread> pool;
    for (int t = 0; t < T; ++t) pool.emplace_back(work, t);
    for (auto& th : pool) th.join();
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
    std::vector<std::thread> pool;
    for (int t = 0; t < T; ++t) pool.emplace_back(copy, t);
    for (auto& th : pool) th.join();
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
// as_int: hit counts (the reference's sum of bools), exact in a double.
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
  for (Py_ssize_t i = 0; i < n; ++i) {
    PyObject* x = as_int ? PyLong_FromLongLong((long long)v[i]) : PyFloat_FromDouble(v[i]);
    PyObject* t = x ? PyTuple_New(1) : nullptr;
    if (!t) {
      Py_XDECREF(x);
      Py_DECREF(out);
      PyBuffer_Release(&b);
      return nullptr;
    }
    PyTuple_SET_ITEM(t, 0, x);
    PyList_SET_ITEM(out, i, t);
  }
  PyBuffer_Release(&b);
  return out;
}

PyMethodDef methods[] = {
    {"tuples1", py_tuples1, METH_VARARGS, "tuples1(float64 buffer, as_int)"},
    {"new", py_new, METH_VARARGS,
     "new(machine, nv, leaves, ids, entries, by_name, eph_types, value_descr)"},
    {"flatten", py_flatten, METH_VARARGS, "flatten(capsule, trees)"},
    {nullptr, nullptr, 0, nullptr}};

PyModuleDef module = {PyModuleDef_HEAD_INIT, "_flatnative",
                      "Native PrimitiveTree flattener (see flatten_native.cpp)",
                      -1, methods};

}  // namespace

PyMODINIT_FUNC PyInit__flatnative(void) { return PyModule_Create(&module); }
