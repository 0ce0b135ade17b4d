// lower_core.h — the PrimitiveTree → postfix lowering shared by the host
// flattener (flatten_native.cpp, g++) and the device lowering kernel
// (gpeval.hip, hipcc): flatten.py's Flattener._build/_emit/_encode, word for
// word.  Plain structs and raw arrays only; LC_HD marks what both compilers
// build.  The fold's sin/cos come in as a template parameter (the host
// libm, or the device's bit-identical restatement of glibc).
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define LC_HD __host__ __device__
#define LC_UNROLL _Pragma("unroll")
#else
#define LC_HD
#define LC_UNROLL _Pragma("GCC unroll 3")
#endif

namespace lowering {

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

// a Python number as the fold sees it (the same layout on host and device)
struct Val {
  char t = 'f';        // 'f' float, 'i' int, 'b' bool, 'x' unsupported
  double f = 0.0;
  int64_t i = 0;
  bool err_value = false;  // the fold raised ValueError (sin/cos of inf)
  LC_HD double as_f() const { return t == 'f' ? f : (double)i; }
  LC_HD bool truth() const { return t == 'f' ? f != 0.0 : i != 0; }
};

struct Entry {
  int kind = K_CONST;
  int arity = 0;
  int sem = 0;
  int var = 0;
  Val c;
};

// One lowered node (a tree's records in reversed-prefix order, children
// before parents).  The bound of |value| (flatten.py _int_bounds, F machine
// only) is kept beside the records, in its own array.
struct Rec {
  uint8_t kind = 0;    // 'v' variable column, 'c' constant, 'p' primitive
  uint8_t nk = 0;      // children
  uint16_t height = 0; // gp.compile's nesting height of the subtree
  int32_t payload = 0; // var index, sem, or constant index into cvals
  int32_t need = 1;    // stack slots the subtree needs (flatten.py _need)
  int32_t kid[3] = {0, 0, 0};
};

// A tree's record storage.  The algorithm below reads a record whole, works
// on the copy and writes it back whole: the host keeps Rec arrays; the
// device packs a record into 16 bytes (one dwordx4 per access — the lowering
// kernel is bound by its scattered per-lane memory instructions, and a
// field-by-field Rec cost several per access).
struct PlainRecs {
  Rec* R;
  LC_HD Rec get(int64_t k) const { return R[k]; }
  LC_HD void put(int64_t k, const Rec& r) const { R[k] = r; }
  static constexpr int64_t kMaxLen = 0x7fffffff;
};
struct alignas(16) PRec {
  uint32_t w0, w1, w2, w3;   // kind | nk << 8 | height << 16, payload,
};                           // need | kid0 << 16, kid1 | kid2 << 16
// S: the distance between a tree's consecutive records, in records — 1, or 64
// on the device, where record k of the tree of lane l lies at k·64 + l of its
// wave's region: the lanes' accesses to one node index are then adjacent.
template <int S>
struct PackedRecsS {
  PRec* P;
  LC_HD Rec get(int64_t k) const {
    const PRec p = P[k * S];
    Rec r;
    r.kind = (uint8_t)(p.w0 & 0xffu);
    r.nk = (uint8_t)((p.w0 >> 8) & 0xffu);
    r.height = (uint16_t)(p.w0 >> 16);
    r.payload = (int32_t)p.w1;
    r.need = (int32_t)(p.w2 & 0xffffu);
    r.kid[0] = (int32_t)(p.w2 >> 16);
    r.kid[1] = (int32_t)(p.w3 & 0xffffu);
    r.kid[2] = (int32_t)(p.w3 >> 16);
    return r;
  }
  LC_HD void put(int64_t k, const Rec& r) const {
    PRec p;
    p.w0 = (uint32_t)r.kind | ((uint32_t)r.nk << 8) | ((uint32_t)r.height << 16);
    p.w1 = (uint32_t)r.payload;
    p.w2 = ((uint32_t)r.need & 0xffffu) | ((uint32_t)r.kid[0] << 16);
    p.w3 = ((uint32_t)r.kid[1] & 0xffffu) | ((uint32_t)r.kid[2] << 16);
    P[k * S] = p;
  }
  // node indices and stack needs in 16 bits: longer trees are declined
  // (the batch is then lowered on the host)
  static constexpr int64_t kMaxLen = 0xffff;
};
using PackedRecs = PackedRecsS<1>;

// A pointer whose consecutive elements lie S apart (the device's interleaved
// scratch: the stack, constants, int bounds and output words of the tree of
// lane l at element k·S + l).  With S = 1 it behaves as T*.
template <class T, int S>
struct Strided {
  T* p;
  LC_HD T& operator[](int64_t k) const { return p[k * S]; }
  LC_HD T& operator*() const { return *p; }
  LC_HD Strided operator++(int) {
    Strided t = *this;
    p += S;
    return t;
  }
  LC_HD Strided& operator+=(int64_t k) {
    p += k * S;
    return *this;
  }
  LC_HD int64_t operator-(const Strided& b) const { return (p - b.p) / S; }
};

// Python ints beyond 2**53 (flatten.py _int_bounds): a float64 no longer
// holds them exactly, so a program that computes such an int at run time (an
// int constant meeting protectedDiv's per-case int 1, say) is a candidate for
// the exact-integer pass.  Bounds are doubles; the test is made at 2**52 so
// that their rounding can only over-report (Python decides exactly).
constexpr double kXintCandidate = 4503599627370496.0;   // 2**52
LC_HD inline double val_ib(const Val& c) {
  if (c.err_value || c.t == 'f' || c.t == 'x') return -1.0;
  if (c.t == 'b') return 1.0;
  return c.i < 0 ? -(double)c.i : (double)c.i;
}
// The bound of a primitive's result from its children's; *cand is set when
// the primitive computes with an int past the float64 range of exact ints.
LC_HD inline double prim_ib(int sem, const double* b, int n, bool* cand) {
  auto big = [](double v) { return v > kXintCandidate; };
  switch (sem) {
    case S_ADD: case S_SUB: case S_MUL: {
      if (b[0] < 0.0 || b[1] < 0.0) return -1.0;
      const double r = sem == S_MUL ? b[0] * b[1] : b[0] + b[1];
      if (big(r)) *cand = true;
      return r;
    }
    case S_NEG:
      if (big(b[0])) *cand = true;
      return b[0];
    case S_PDIV:                 // the int is protectedDiv's 1; the quotient
      if (b[0] >= 0.0 && b[1] >= 0.0 && (big(b[0]) || big(b[1]))) *cand = true;
      return 1.0;                // of two ints rounds the exact ratio
    case S_LT: case S_EQ:        // exact int/float comparisons
      if (big(b[0]) || big(b[1])) *cand = true;
      return 1.0;
    case S_AND: case S_OR: case S_XOR: case S_NOT:
      return 1.0;
    case S_ITE:
      return b[1] > b[2] ? b[1] : b[2];
    default:                     // sin/cos (float), numpy semantics
      return -1.0;
  }
}

// |i| > 2**53 (Python ints a float cannot hold exactly; INT64_MIN included)
LC_HD inline bool big53(int64_t i) {
  const uint64_t a = i < 0 ? (uint64_t)0 - (uint64_t)i : (uint64_t)i;
  return a > (1ULL << 53);
}
LC_HD inline int lc_max(int a, int b) { return a > b ? a : b; }

// Python semantics of the fold (flatten.py Flattener._fold with the pset's
// own callables: operator.*, protectedDiv, math.sin/cos, if_then_else).
// Returns false to decline (the Python flattener then handles the tree).
template <class Trig>
LC_HD bool fold(int sem, const Val* k, int n, Val& r) {
LC_UNROLL
  for (int i = 0; i < 3; ++i) {
    if (i >= n) break;
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
      if (ints && (big53(k[0].i) || big53(k[1].i)))
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
      if (__builtin_isinf(x)) { r.err_value = true; return true; }
      r.t = 'f';
      r.f = sem == S_SIN ? Trig::sin(x) : Trig::cos(x);   // glibc, as math.*
      return true;
    }
    case S_NPSIN: case S_NPCOS: {            // numpy: sin(inf) = nan
      const double x = k[0].as_f();
      r.t = 'f';
      r.f = __builtin_isinf(x) ? __builtin_nan("") : sem == S_NPSIN ? Trig::sin(x) : Trig::cos(x);
      return true;
    }
    case S_NPDIV: {                          // symbreg_numpy.py:28-36
      const double q = k[0].as_f() / k[1].as_f();
      if (__builtin_isinf(q) || __builtin_isnan(q)) { r.t = 'i'; r.i = 1; return true; }
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
        if ((k[0].t != 'f' && big53(k[0].i)) ||
            (k[1].t != 'f' && big53(k[1].i)))
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

// the stack slots a primitive needs, from its children's records
LC_HD inline int need_of(const Rec* k, int nk) {
  if (nk == 1) return k[0].need;
  if (nk == 3) return lc_max(k[0].need, lc_max(1 + k[1].need, 2 + k[2].need));
  if (k[1].kind != 'p') return k[0].need;
  if (k[0].kind != 'p') return k[1].need;
  return k[0].need == k[1].need ? k[0].need + 1 : lc_max(k[0].need, k[1].need);
}

LC_HD inline void binary_ops(int sem, uint32_t& fwd, uint32_t& rev) {
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

LC_HD inline uint32_t unary_op(int sem) {
  return sem == S_NEG ? OP_NEG
       : (sem == S_SIN || sem == S_NPSIN) ? OP_SIN
       : (sem == S_COS || sem == S_NPCOS) ? OP_COS : OP_NOT;
}

// flatten.py Flattener._emit + _encode in one pass: instruction words are
// written straight to `o`.  _encode's peephole (PUSH followed by LDV/LDC ->
// PUSHV/PUSHC carrying the PUSH's slot) is a pending PUSH that the next
// leaf load absorbs; _check_consts (F machine) is tallied per constant word.
// _emit's recursion runs on an explicit stack of node indices (the parse
// stack, free by then) so the device kernel needs no call stack: once a
// primitive's frame starts, its own `height` holds the slot d, `need` the
// running top and nk's upper bits the resume phase (the parent read the
// child's need and kind before the child started).  Records are read and
// written whole through the storage R (PlainRecs / PackedRecs).
template <class Recs, class CvP, class OutP>
struct Emitter {
  Recs R;
  CvP cv;
  OutP o;
  int pend = -1;       // slot of a PUSH not yet written
  bool fm;             // F machine: constants as two fp64 words
  bool bad = false;    // a constant whose fold raised
  bool big = false;    // an int constant beyond 2**53
  // _encode's second peephole: a NEG not yet written.  The next instruction
  // absorbs it when it is an add or sub (a + -T = a - T, a - -T = a + T,
  // exactly, signed zeros included), a mul passes it on (a * -T = -(a * T)),
  // a second NEG cancels it.
  bool pneg = false;
  bool neg_fold = true;

  LC_HD void negate() {                     // the pending NEG, written
    if (pneg) {
      *o++ = OP_NEG;
      pneg = false;
    }
  }
  // family base op (ADD, SUB, ...) with the pending NEG absorbed, carried
  // past a mul (a * -T is -(a * T) exactly), or written
  LC_HD uint32_t fam_op(uint32_t op) {
    if (pneg && (op == OP_ADD || op == OP_SUB)) {
      pneg = false;
      return op == OP_ADD ? OP_SUB : OP_ADD;
    }
    if (op != OP_MUL) negate();
    return op;
  }
  LC_HD void flush() {
    if (pend >= 0) {
      negate();
      *o++ = OP_PUSH | ((uint32_t)pend << 8);
      pend = -1;
    }
  }
  LC_HD void konst(uint32_t op, uint32_t d, const Val& c) {
    if (fm) {
      if (c.err_value) bad = true;
      else if (c.t == 'i' && big53(c.i)) big = true;
      const double v = c.as_f();
      uint64_t bits;
      __builtin_memcpy(&bits, &v, 8);
      o[0] = op | (d << 8);
      o[1] = (uint32_t)(bits & 0xffffffffu);
      o[2] = (uint32_t)(bits >> 32);
      o += 3;
    } else {
      *o++ = op | (d << 8) | ((c.truth() ? 1u : 0u) << 16);
    }
  }
  LC_HD void leaf(const Rec& L, uint32_t d) {          // LDV / LDC (or fused)
    negate();
    uint32_t op = L.kind == 'v' ? OP_LDV : OP_LDC;
    if (pend >= 0) {
      op = L.kind == 'v' ? OP_PUSHV : OP_PUSHC;
      d = (uint32_t)pend;
      pend = -1;
    }
    if (L.kind == 'v') *o++ = op | (d << 8) | ((uint32_t)L.payload << 16);
    else konst(op, d, cv[L.payload]);
  }
  LC_HD void operand(uint32_t op, const Rec& L, uint32_t d) {   // op+1 / op+2
    flush();
    op = fm ? fam_op(op) : op;
    if (L.kind == 'v') *o++ = (op + 1) | (d << 8) | ((uint32_t)L.payload << 16);
    else konst(op + 2, d, cv[L.payload]);
  }
  LC_HD void plain(uint32_t op, uint32_t d) {
    flush();
    if (fm && neg_fold && op == OP_NEG) {
      pneg = !pneg;
      return;
    }
    if (fm && op >= OP_ADD && op < OP_XOR && (op - OP_ADD) % 3 == 0) op = fam_op(op);
    else negate();
    *o++ = op | (d << 8);
  }
  LC_HD void push(uint32_t d) {
    flush();
    pend = (int)d;
  }
  // Emit the subtree at `root` into slots d = 0..; S is scratch for one
  // node index per tree level.  Returns the highest slot used.
  template <class StkP>
  LC_HD uint32_t emit(int32_t root, StkP S) {
    const Rec rt = R.get(root);
    if (rt.kind != 'p') {
      leaf(rt, 0);
      return 0;
    }
    int64_t sp = 0;
    uint32_t ret = 0;                      // the last finished subtree's top
    auto start = [&](int32_t ri, Rec x, uint32_t d) {
      x.height = (uint16_t)d;
      R.put(ri, x);
      S[sp++] = ri;
    };
    // a child: a leaf is emitted at once (ret = its slot); a primitive gets
    // a frame.  The caller has already set its own resume phase.
    auto child = [&](int32_t ci, const Rec& c, uint32_t d) {
      if (c.kind != 'p') {
        leaf(c, d);
        ret = d;
      } else {
        start(ci, c, d);
      }
    };
    start(root, rt, 0);
    while (sp > 0) {
      const int32_t ri = S[sp - 1];
      Rec r = R.get(ri);
      const uint32_t d = r.height;
      const int nk = r.nk & 3, phase = r.nk >> 2;
      auto next = [&](int ph) {            // the resume phase, stored
        r.nk = (uint8_t)(nk | (ph << 2));
        R.put(ri, r);
      };
      auto finish = [&](uint32_t top) {
        ret = top;
        --sp;
      };
      const int sem = r.payload;
      if (nk == 1) {
        if (phase == 0) {
          next(1);
          child(r.kid[0], R.get(r.kid[0]), d);
        } else {
          plain(unary_op(sem), d);
          finish(ret);
        }
        continue;
      }
      if (nk == 3) {                       // if_then_else(cond, a, b)
        switch (phase) {
          case 0:
            next(1);
            child(r.kid[0], R.get(r.kid[0]), d);
            break;
          case 1:
            r.need = (int32_t)ret;
            push(d);
            next(2);
            child(r.kid[1], R.get(r.kid[1]), d + 1);
            break;
          case 2:
            r.need = lc_max(r.need, (int)ret);
            push(d + 1);
            next(3);
            child(r.kid[2], R.get(r.kid[2]), d + 2);
            break;
          default:
            plain(OP_ITE, d);
            finish((uint32_t)lc_max(lc_max(r.need, (int)ret), (int)d + 2));
        }
        continue;
      }
      uint32_t fwd, rev;
      binary_ops(sem, fwd, rev);
      const int32_t left = r.kid[0], right = r.kid[1];
      switch (phase) {
        case 0: {
          const Rec L = R.get(left);
          const Rec Rr = R.get(right);
          if (Rr.kind != 'p') {            // T = left; T = T op right
            next(1);
            child(left, L, d);
          } else if (L.kind != 'p') {      // T = right; T = left op T
            next(2);
            child(right, Rr, d);
          } else {
            const bool lfirst = L.need >= Rr.need;
            next(lfirst ? 3 : 4);
            child(lfirst ? left : right, lfirst ? L : Rr, d);
          }
          break;
        }
        case 1:
          operand(rev, R.get(right), d);
          finish(ret);
          break;
        case 2:
          operand(fwd, R.get(left), d);
          finish(ret);
          break;
        case 3:
        case 4: {
          r.need = (int32_t)ret;
          push(d);
          next(phase + 2);
          const int32_t c = phase == 3 ? right : left;
          child(c, R.get(c), d + 1);
          break;
        }
        default:                           // 5: R[d] op T, 6: T op R[d]
          plain(phase == 5 ? fwd : rev, d);
          finish((uint32_t)lc_max(lc_max(r.need, (int)ret), (int)d + 1));
      }
    }
    return ret;
  }
};


// the pset tables a lowering needs
struct Tables {
  const Entry* entries;
  const uint8_t* leaf;   // per argument: 1 = sin/cos of it read from a column
  int n_leaf;
  int nv;
  int machine;           // 0 F, 1 B
  int neg_fold = 1;      // the NEG peephole (0: GPE_NEG_PEEPHOLE=0, A/B runs)
};
struct Result {
  int32_t depth = 0;
  int32_t n_words = 0;
  uint8_t err = 0;
  bool declined = false, inexact = false, verr = false;   // inexact: a
                       // candidate for the exact-integer pass (kXintCandidate)
};

// Lower one tree.  ent(k), k = 0 .. len-1, yields the node codes in
// reversed prefix order: an entry index, or -1 - i for the ephemeral value
// evals[i].  Scratch: R (len records), stk[len], cv[len], ib[len] (the F
// machine's int bounds; unused, may be null, for B); out[3 * len + 1]
// receives the program words (or one END); o.n_words their count.
template <class Trig, class Ents, class Recs, class StkP, class CvP, class IbP, class OutP>
LC_HD void lower(const Tables& T, Ents& ent, int64_t len, const Val* evals,
                 Recs R, StkP stk, CvP cv, IbP ib, OutP out, Result& o) {
  int32_t ncv = 0;
  int64_t sp = 0;
  bool decline = len > Recs::kMaxLen;
  bool xint = false;
  const bool fm = T.machine == 0;
  for (int64_t k = 0; k < len && !decline; ++k) {
    const int32_t ei = ent(k);
    Rec r;
    double rib = -1.0;
    if (ei < 0) {                          // ephemeral constant
      r.kind = 'c';
      r.payload = ncv;
      cv[ncv] = evals[-1 - ei];
      rib = val_ib(cv[ncv++]);
    } else {
      const Entry& e = T.entries[ei];
      if (e.kind == K_ARG) {
        r.kind = 'v';
        r.payload = e.var;
      } else if (e.kind == K_CONST) {
        if (e.c.t == 'x') { decline = true; break; }
        r.kind = 'c';
        r.payload = ncv;
        cv[ncv++] = e.c;
        rib = val_ib(e.c);
      } else {
        const int ar = e.arity;
        if (sp < ar || ar > 3) { decline = true; break; }
        Rec kr[3];                         // the children, read once each
        int h = 0;
        // (fixed trip counts, unrolled: the arrays stay in registers — a
        // loop to `ar` made the device compiler move them to LDS)
LC_UNROLL
        for (int q = 0; q < 3; ++q)
          if (q < ar) {
            const int32_t c = stk[--sp];
            r.kid[q] = c;
            kr[q] = R.get(c);
            h = lc_max(h, (int)kr[q].height + 1);
          }
        r.height = (uint16_t)(h < 65535 ? h : 65535);
        const bool trig = e.sem == S_SIN || e.sem == S_COS ||
                          e.sem == S_NPSIN || e.sem == S_NPCOS;
        if (trig && kr[0].kind == 'v' && kr[0].payload < T.n_leaf && T.leaf[kr[0].payload]) {
          r.kind = 'v';                    // a trig-leaf column
          r.payload = ((e.sem == S_SIN || e.sem == S_NPSIN) ? 1 : 2) * T.nv +
                      kr[0].payload;
        } else {
          bool all_c = true;
LC_UNROLL
          for (int q = 0; q < 3; ++q)
            if (q < ar) all_c &= kr[q].kind == 'c';
          if (all_c) {
            Val kv[3];
LC_UNROLL
            for (int q = 0; q < 3; ++q)
              if (q < ar) kv[q] = cv[kr[q].payload];
            Val res;
            if (!fold<Trig>(e.sem, kv, ar, res)) { decline = true; break; }
            r.kind = 'c';
            r.payload = ncv;
            cv[ncv++] = res;
            rib = val_ib(res);
          } else {
            r.kind = 'p';
            r.nk = (uint8_t)ar;
            r.payload = e.sem;
            r.need = need_of(kr, ar);
            if (fm) {
              double kb[3];
LC_UNROLL
              for (int q = 0; q < 3; ++q) kb[q] = q < ar ? ib[r.kid[q]] : -1.0;
              rib = prim_ib(e.sem, kb, ar, &xint);
            }
          }
        }
      }
    }
    R.put(k, r);
    if (fm) ib[k] = rib;
    stk[sp++] = (int32_t)k;
  }
  o.n_words = 1;
  out[0] = OP_END;
  if (decline || sp != 1) {
    o.declined = true;
    return;
  }
  const Rec rr = R.get(stk[0]);
  if (len > MAX_COMPILE_HEIGHT && rr.height > MAX_COMPILE_HEIGHT) {
    o.err = ERR_SYNTAX;
    return;
  }
  if (rr.kind == 'c' && cv[rr.payload].err_value) {
    o.err = ERR_CONST;
    o.verr = true;
    return;
  }
  Emitter<Recs, CvP, OutP> em{R, cv, out};
  em.fm = fm;
  em.neg_fold = T.neg_fold != 0;
  o.depth = (int32_t)em.emit(stk[0], stk);
  em.negate();
  em.flush();
  *em.o++ = OP_END;
  if (em.bad) {                            // _check_consts: a raising fold
    out[0] = OP_END;
    o.err = ERR_CONST;
    o.verr = true;
    return;
  }
  o.inexact = em.big || xint;
  o.n_words = (int32_t)(em.o - out);
}

}  // namespace lowering
